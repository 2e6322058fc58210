"""ELBO-head cost split at cfg2: the forward entry with need_grad = 0 (head phases L/A/B only,
no MLP backward / gradient stores) vs need_grad = 1, timed with HIP events over 20 calls each;
the difference is what the gradient half of the head costs.  usage: python tools/head_ab.py [B]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vq-vae-hmm-model_amd"))


def main():
    import vqhmm
    from vqhmm import _ext
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    T = 200
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128).cuda()
    st = vqhmm.TrainState(m, lr=1e-3)
    g = torch.Generator(device="cuda").manual_seed(1234)
    x = torch.randn(B, 5, T, device="cuda", generator=g)
    u = torch.randn(B, 4, T, device="cuda", generator=g)
    L = torch.full((B,), T, dtype=torch.int64, device="cuda")
    lib = st.lib
    ws = st.workspace(B, T)
    d = ctypes.byref(st.dims)
    sp = _ext.stream_ptr()
    s = torch.cuda.current_stream()
    res = {}
    for ng in (0, 1, 0, 1):
        run = lambda: lib.vqhmm_elbo_fwd_f32(d, st.ptrs, _ext.ptr(x), _ext.ptr(u), 0, _ext.ptr(L), None, B, T, 1.0,  # noqa
                                             ng, _ext.ptr(ws), ws.numel(), _ext.ptr(st.loss), None, sp)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            run()
        e1.record(s)
        torch.cuda.synchronize()
        res[ng] = e0.elapsed_time(e1) / 20 * 1e3
    print(f"B={B} forward need_grad=0 {res[0]:.1f} us  need_grad=1 {res[1]:.1f} us  gradient half {res[1]-res[0]:.1f} us")


if __name__ == "__main__":
    main()
