"""Phase split of the parallel-in-time forward-backward (hmm_seg.hip; profiling build, VQHMM_FB_PROF=1):
per-wave shader cycles of load issue + emission rows, phase 1 (segment matrices), barrier + phase 2
(boundary vectors) + barrier, phase 3 (vector chains), gamma; and the workgroups' wall-clock spread.
    VQHMM_LIB_PATH=vqhmm/libvqhmm_prof.so VQHMM_FB_PROF=1 python tools/fbseg_prof.py [B] [T]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vq-vae-hmm-model_amd"))


def main():
    from vqhmm import _ext
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    K = 8
    g = torch.Generator(device="cuda").manual_seed(7)
    log_pi = torch.log_softmax(torch.randn(K, device="cuda", generator=g), -1)
    log_A = torch.log_softmax(torch.randn(B, T, K, K, device="cuda", generator=g), -1)
    em = torch.log_softmax(torch.randn(B, T, K, device="cuda", generator=g), -1)
    lengths = torch.full((B,), T, dtype=torch.int64, device="cuda")
    gamma = torch.empty(B, T, K, device="cuda")
    logZ = torch.empty(B, device="cuda")
    lib = _ext.load()
    nb = lib.vqhmm_fwdbwd_workspace_size(B, T, K)
    ws = torch.zeros(nb // 8, dtype=torch.int64, device="cuda")
    for _ in range(3):
        _ext.check(lib.vqhmm_fwdbwd_f32(_ext.ptr(log_pi), _ext.ptr(log_A), _ext.ptr(em), _ext.ptr(lengths), B, T, K,
                                        _ext.ptr(gamma), _ext.ptr(logZ), _ext.ptr(ws), nb, _ext.stream_ptr(em.device)),
                   "fwdbwd")
    torch.cuda.synchronize()
    nw = (T + 63) // 64
    p = ws[:B * 16 * 8].view(B, 16, 8)[:, :nw].double().cpu()
    names = ["issue+em", "phase1", "bar+ph2+bar", "chains", "gamma"]
    cols = [(2, 3), (3, 4), (4, 5), (5, 6), (6, 7)]
    for w in (0, 1, nw - 1):
        parts = [(p[:, w, b] - p[:, w, a]).mean().item() for a, b in cols]
        tot = (p[:, w, 7] - p[:, w, 2]).mean().item()
        print(f"wave {w:2d}: total {tot:8.0f} cyc | " + " | ".join(f"{n} {v:7.0f}" for n, v in zip(names, parts)))
    t0 = p[:, :, 0].min().item()
    st = (p[:, 0, 0] - t0) / 100.0  # us (100 MHz)
    en = (p[:, 0, 1] - t0) / 100.0
    print(f"workgroups: start spread {st.min().item():.2f}..{st.max().item():.2f} us, end {en.min().item():.2f}.."
          f"{en.max().item():.2f} us, mean duration {(en - st).mean().item():.2f} us")
    clk = (p[:, 0, 7] - p[:, 0, 2]).mean().item() / ((en - st).mean().item() * 1e3)
    print(f"in-kernel clock ~{clk:.2f} GHz")


if __name__ == "__main__":
    main()
