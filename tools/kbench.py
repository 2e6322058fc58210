"""Kernel micro-benchmarks (HIP events on the launch stream).

    python tools/kbench.py vq [--B 2048 --Dv 64 --T 200 --K 32]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vq-vae-hmm-model_amd"))
import vqhmm  # noqa: E402

HBM_PEAK = 8.0e12


def time_fn(fn, iters=50, warmup=10):
    for _ in range(warmup):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def bench_vq(a):
    g = torch.Generator(device="cuda").manual_seed(1234)
    z = torch.randn(a.B, a.Dv, a.T, device="cuda", generator=g)
    cb = torch.randn(a.K, a.Dv, device="cuda", generator=g)
    idx = torch.empty(a.B, a.T, dtype=torch.int32, device="cuda")
    lib = vqhmm._ext.load()
    P = vqhmm._ext.ptr
    st = vqhmm._ext.stream_ptr()

    def fn():
        lib.vqhmm_vq_argmin_f32(P(z), a.B, a.Dv, a.T, P(cb), a.K, P(idx), None, st)

    t = time_fn(fn)
    N = a.B * a.T
    byts = 4 * N * a.Dv + 4 * a.K * a.Dv + 4 * N
    print(json.dumps({"kernel": "vq_argmin", "B": a.B, "Dv": a.Dv, "T": a.T, "K": a.K, "us": t * 1e6,
                      "GBps": byts / t / 1e9, "frac_hbm": byts / t / HBM_PEAK}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what")
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--Dv", type=int, default=64)
    ap.add_argument("--T", type=int, default=200)
    ap.add_argument("--K", type=int, default=32)
    a = ap.parse_args()
    {"vq": bench_vq}[a.what](a)
