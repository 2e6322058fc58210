"""Phase timings of the strip kernel (strip.hip, VQHMM_STRIP_PROF=1 builds its profiling variant):
per-workgroup s_memrealtime stamps (100 MHz) of the first strip's phases, medians over workgroups.
usage: VQHMM_STRIP_PROF=1 python tools/strip_prof.py [B ...]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vq-vae-hmm-model_amd"))
import vqhmm  # noqa: E402
from vqhmm import _ext  # noqa: E402

NAMES = ["staging", "enc_conv1+enc_conv2+logits", "dec_conv1+dec_conv2+params", "-", "-", "-", "other strips"]
# the non-folded backward strip (VQHMM_STRIP_WGRAD=0: it is then the step's last strip launch)
NAMES_BWD = ["DMA issue", "params+dec2 dgrad, dg1 swap", "dec1 dgrad+logits bwd", "-", "-", "-", "enc2 dgrad + rest"]


def run(B, T=200, D=5, H=64, K=3, H2=32):
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(B, D, T, generator=gen).cuda()
    u = torch.randn(B, 4, T, generator=gen).cuda()
    L = torch.full((B,), T, dtype=torch.int64)
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=4, trans_hidden=128).cuda()
    st = vqhmm.TrainState(m, lr=1e-3)
    xs, us, Ls = st.prepare(x, u, L)
    for _ in range(int(os.environ.get("STRIP_PROF_STEPS", "5"))):
        st.forward_backward(xs, us, Ls, 1.0)
    torch.cuda.synchronize()
    buf = np.zeros(256 * 16, dtype=np.uint64)
    _ext.check(_ext.load().vqhmm_debug_prof(0, buf.ctypes.data_as(ctypes.c_void_p), buf.size), "debug_prof")
    t = buf.reshape(256, 16).astype(np.int64)
    used = t[:, 8] > 0
    t = t[used]
    w0 = t[:, [2, 4, 5, 6, 3]].astype(np.int64)  # wave 0 in the second phase: start, front, loop, tail, barrier
    t[:, 4:7] = t[:, 3:4]  # stamps 0, 1, 2, 3, 7
    d = np.diff(t[:, :8], axis=1) * 10 / 1000.0  # us
    t0 = t[:, 0].min()
    print(f"B={B}: {used.sum()} workgroups, strips/wg {t[:, 8].min()}..{t[:, 8].max()}, "
          f"kernel span {(t[:, 7].max() - t0) * 0.01:.2f} us, start skew {(t[:, 0].max() - t0) * 0.01:.2f} us")
    # buffer 0 holds the forward strip's stamps unless the non-folded backward strip ran after it
    # (VQHMM_STRIP_WGRAD=0 with VQHMM_STRIP_BWD on)
    bwd = os.environ.get("VQHMM_STRIP_WGRAD", "1") == "0" and os.environ.get("VQHMM_STRIP_BWD", "1") != "0"
    names = NAMES_BWD if bwd else NAMES
    for i, n in enumerate(names):
        if n != "-":
            print(f"  {n:28s} median {np.median(d[:, i]):7.2f}  max {d[:, i].max():7.2f} us")
    if names is NAMES:
        dw = np.median(np.diff(w0, axis=1), axis=0) * 0.01
        print("  wave 0, second phase: front %.2f, dec_conv2 loop %.2f, tail %.2f, to barrier %.2f us" % tuple(dw))
        fw = np.median(np.diff(t[:, [2, 10, 11, 4]].astype(np.int64), axis=1), axis=0) * 0.01
        print("    front: LDS reads + 32 MFMAs %.2f, epilogue A %.2f, epilogue B + wave barrier %.2f us" % tuple(fw))
    if names is NAMES and t[:, 14].max() > 0:  # s_memtime around the launch: the in-kernel clock
        ghz = (t[:, 14] - t[:, 13]) / ((t[:, 7] - t[:, 0]) * 10.0)
        print(f"  in-kernel clock median {np.median(ghz):.3f} GHz (min {ghz.min():.3f}, max {ghz.max():.3f})")
    if t[:, 9].max() > 0:  # VQHMM_STRIP_PROF=2: serialised latency probes from the kernel's start
        for k, n in ((9, "x load"), (10, "+ constants"), (11, "+ front weights"), (12, "+ image DMA")):
            print(f"  {n:18s} at {np.median(t[:, k] - t[:, 0]) * 0.01:7.2f} us")


if __name__ == "__main__":
    for b in (sys.argv[1:] or ["128", "1024"]):
        run(int(b))
