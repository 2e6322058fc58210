"""Phase timings of the backward strip with the folded weight gradients (strip_bwdw.hip; profiling build:
VQHMM_LIB_PATH=vqhmm/libvqhmm_prof.so VQHMM_STRIP_PROF=1): per-workgroup s_memrealtime stamps (100 MHz) of
the first strip's phases, medians / maxima over workgroups, and the in-kernel clock (s_memtime).
usage: VQHMM_STRIP_PROF=1 [VQHMM_STRIP_PROF_IT=n] python tools/bwdw_prof.py [B ...]  (strip n of each workgroup, default 0)"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vq-vae-hmm-model_amd"))
import vqhmm  # noqa: E402
from vqhmm import _ext  # noqa: E402

NAMES = ["P1 staging + front (1x1 dgrad), G1 / Q", "P2 dec_conv2 dgrad + wgrad", "P3 D1 / G2 / DP, image DMA",
         "P4 dec_conv1 dgrad + epilogue, wgrad to_params / dec_conv1'", "P5 H1 / H2 staging",
         "P6 enc_conv2 dgrad + wgrad, to_logits wgrad", "P7 DH1 / XX + P8 enc_conv1 wgrad", "slabs + dE share"]


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
    _ext.check(_ext.load().vqhmm_debug_prof(3, buf.ctypes.data_as(ctypes.c_void_p), buf.size), "debug_prof")
    t = buf.reshape(256, 16).astype(np.int64)
    t = t[t[:, 9] > 0]
    pit = int(os.environ.get("VQHMM_STRIP_PROF_IT", "0"))
    if pit > 0:  # a later strip (VQHMM_STRIP_PROF_IT): its phases from its own start stamp; "slabs" = the rest
        t = t[t[:, 9] > pit]
        t[:, 0] = t[:, 15]
    d = np.diff(t[:, :9], axis=1) * 0.01  # us
    t0 = t[:, 0].min()
    ghz = (t[:, 14] - t[:, 13]) / ((t[:, 8] - t[:, 0]) * 10.0)
    print(f"B={B}: {len(t)} workgroups, strips/wg {t[:, 9].min()}..{t[:, 9].max()}, kernel span "
          f"{(t[:, 8].max() - t0) * 0.01:.2f} us, start skew {(t[:, 0].max() - t0) * 0.01:.2f} us, "
          f"clock {np.median(ghz):.3f} GHz")
    for i, n in enumerate(NAMES):
        print(f"  {n:62s} median {np.median(d[:, i]):7.2f}  max {d[:, i].max():7.2f} us")
    if t[:, 12].max() > 0:  # P1 of the first strip, wave 0: loads issued, front MFMAs done, slots / G1 / Q written
        p1 = np.median((t[:, [10, 11, 12, 1]] - t[:, [0]]) * 0.01, axis=0)
        print("  P1 (wave 0, from the start): loads issued %.2f, front MFMAs %.2f, LDS writes %.2f, B1 %.2f us" % tuple(p1))


if __name__ == "__main__":
    for b in (sys.argv[1:] or ["128", "256"]):
        run(int(b))
