"""Phase timings of a profiled kernel family from its prof.h stamps, medians over workgroups:
the conv2 pair kernel (conv2f_kernel; the last one of a training step to run it; VQHMM_CONV_PROF=1) or,
with --head, the cooperative ELBO head (VQHMM_HEAD_PROF=1).
usage: VQHMM_CONV_PROF=1 python tools/conv_prof.py [B ...];  VQHMM_HEAD_PROF=1 python tools/conv_prof.py --head [B ...]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vq-vae-hmm-model_amd"))
import vqhmm  # noqa: E402
from vqhmm import _ext  # noqa: E402


HEAD = "--head" in sys.argv


def run(B, T=200, D=5, H=64, K=3, H2=32):
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(B, D, T, generator=gen).cuda()
    u = torch.randn(B, 4, T, generator=gen).cuda()
    L = torch.full((B,), T, dtype=torch.int64)
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=4, trans_hidden=128).cuda()
    st = vqhmm.TrainState(m, lr=1e-3)
    xs, us, Ls = st.prepare(x, u, L)
    for _ in range(5):
        st.forward_backward(xs, us, Ls, 1.0)
    torch.cuda.synchronize()
    buf = np.zeros(256 * 16, dtype=np.uint64)
    _ext.check(_ext.load().vqhmm_debug_prof(2 if HEAD else 1, buf.ctypes.data_as(ctypes.c_void_p), buf.size), "debug_prof")
    t = buf.reshape(256, 16).astype(np.int64)
    t = t[t[:, 8] > 0]
    t0 = t[:, 0].min()
    print(f"B={B}: {len(t)} workgroups, wave-0 {'windows' if HEAD else 'tiles'} {t[:, 8].min()}..{t[:, 8].max()}, span {(t[:, 7].max() - t0) * 0.01:.2f} us, "
          f"start skew {(t[:, 0].max() - t0) * 0.01:.2f} us")
    ph = ((0, 1, "staging"), (1, 2, "first window"), (1, 9, "  u' to LDS / pipe: A(0)"), (9, 10, "  A: transition logits / pipe: step 0"),
          (10, 11, "  pipe step 1: C(0)"), (11, 12, "  pipe step 1: A(2)"), (12, 2, "  pipe step 1: barrier wait"), (2, 13, "  pipe step 1: row waves done (vs its end)"),
          (10, 11, "  B: rows"), (11, 12, "  B2: dq + prefetch"), (12, 2, "  C: MLP backward"),
          (2, 3, "other windows"), (3, 7, "slab epilogue")) if HEAD else \
        ((0, 1, "staging"), (1, 2, "first tile (wave 0)"), (2, 7, "rest + drain"))
    for a, b, n in ph:
        if not (t[:, a].all() and t[:, b].all()):
            continue  # a stamp this kernel does not write (the pipelined head: 0, 1, 10, 2, 3, 7)
        d = (t[:, b] - t[:, a]) * 0.01
        print(f"  {n:22s} median {np.median(d):7.2f}  max {d.max():7.2f} us")


if __name__ == "__main__":
    for b in ([v for v in sys.argv[1:] if v != "--head"] or ["128", "1024"]):
        run(int(b))
