"""Per-wave cycle split of the LDS-resident forward-backward (run with VQHMM_FB_PROF=1): total cycles,
busy cycles between barriers, and the helpers' linearisation share.   usage: python tools/fb_prof.py [B] [T]"""
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
    g = torch.Generator(device="cuda").manual_seed(0)
    log_pi = torch.log_softmax(torch.randn(K, device="cuda", generator=g), -1)
    log_A = torch.log_softmax(1.5 * torch.randn(B, T, K, K, device="cuda", generator=g), -1)
    em = torch.log_softmax(2.0 * torch.randn(B, T, K, device="cuda", generator=g), -1)
    lengths = torch.full((B,), T, dtype=torch.int64, device="cuda")
    gamma = torch.empty(B, T, K, device="cuda")
    logZ = torch.empty(B, device="cuda")
    lib = _ext.load()
    nb = lib.vqhmm_fwdbwd_workspace_size(B, T, K)
    ws = torch.zeros(nb // 8, dtype=torch.int64, device="cuda")
    for _ in range(2):
        _ext.check(lib.vqhmm_fwdbwd_f32(_ext.ptr(log_pi), _ext.ptr(log_A), _ext.ptr(em), _ext.ptr(lengths), B, T, K,
                                        _ext.ptr(gamma), _ext.ptr(logZ), _ext.ptr(ws), nb, _ext.stream_ptr(em.device)),
                   "fwdbwd")
    torch.cuda.synchronize()
    p = ws[:B * 16].view(B, 4, 4).double().cpu()
    names = ["alpha", "beta", "helper-up", "helper-down"]
    nch = p[0, 0, 3].item()
    for w in range(4):
        tot, busy, lin = p[:, w, 0].mean().item(), p[:, w, 1].mean().item(), p[:, w, 2].mean().item()
        print(f"{names[w]:12s} total {tot:9.0f}  busy {busy:9.0f} ({busy / tot:5.1%})  linearise {lin:8.0f}  "
              f"per chunk busy {busy / (nch + 1):7.0f}  per step {busy / max(nch, 1) / 16:6.1f} cycles")


if __name__ == "__main__":
    main()
