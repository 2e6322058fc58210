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


def bench_stream(a):
    """Bandwidth references on the VQ input size: torch read-reduce and copy of z."""
    z = torch.randn(a.B, a.Dv, a.T, device="cuda")
    out = torch.empty_like(z)
    nb = z.numel() * 4
    t_sum = time_fn(lambda: z.sum())
    t_cp = time_fn(lambda: out.copy_(z))
    print(json.dumps({"kernel": "torch_stream", "bytes": nb, "sum_us": t_sum * 1e6, "sum_GBps": nb / t_sum / 1e9,
                      "copy_us": t_cp * 1e6, "copy_GBps": 2 * nb / t_cp / 1e9}))


def hmm_tables(B, T, K, seed=7):
    g = torch.Generator(device="cuda").manual_seed(seed)
    log_pi = torch.log_softmax(torch.randn(K, device="cuda", generator=g), -1)
    log_A = torch.log_softmax(torch.randn(B, T, K, K, device="cuda", generator=g), -1)
    em = torch.log_softmax(torch.randn(B, T, K, device="cuda", generator=g), -1)
    L = torch.full((B,), T, dtype=torch.int64, device="cuda")
    return log_pi, log_A, em, L


def bench_viterbi(a):
    B, T, K = a.B, a.T, a.K
    log_pi, log_A, em, L = hmm_tables(B, T, K)
    lib = vqhmm._ext.load()
    P = vqhmm._ext.ptr
    st = vqhmm._ext.stream_ptr()
    path = torch.empty(B, T, dtype=torch.int32, device="cuda")
    score = torch.empty(B, device="cuda")
    nb = lib.vqhmm_viterbi_workspace_size(B, T, K)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")

    def fn():
        lib.vqhmm_viterbi_f32(P(log_pi), P(log_A), P(em), P(L), B, T, K, P(path), P(score), P(ws), nb, st)

    t = time_fn(fn, iters=5, warmup=2)
    byts = B * (4 * T * K * K + 4 * T * K + 4 * T) + 4 * K
    print(json.dumps({"kernel": "viterbi", "B": B, "T": T, "K": K, "us": t * 1e6, "GBps": byts / t / 1e9,
                      "frac_hbm": byts / t / HBM_PEAK}))


def bench_fwdbwd(a):
    B, T, K = a.B, a.T, a.K
    log_pi, log_A, em, L = hmm_tables(B, T, K)
    lib = vqhmm._ext.load()
    P = vqhmm._ext.ptr
    st = vqhmm._ext.stream_ptr()
    gamma = torch.empty(B, T, K, device="cuda")
    logZ = torch.empty(B, device="cuda")
    nb = lib.vqhmm_fwdbwd_workspace_size(B, T, K)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")

    def fn():
        lib.vqhmm_fwdbwd_f32(P(log_pi), P(log_A), P(em), P(L), B, T, K, P(gamma), P(logZ), P(ws), nb, st)

    t = time_fn(fn, iters=20, warmup=3)
    byts = B * (4 * T * K * K + 4 * T * K + 4 * T * K) + 4 * K
    print(json.dumps({"kernel": "fwdbwd", "B": B, "T": T, "K": K, "us": t * 1e6, "GBps": byts / t / 1e9,
                      "frac_hbm": byts / t / HBM_PEAK}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what")
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--Dv", type=int, default=64)
    ap.add_argument("--T", type=int, default=200)
    ap.add_argument("--K", type=int, default=32)
    a = ap.parse_args()
    {"vq": bench_vq, "stream": bench_stream, "viterbi": bench_viterbi, "fwdbwd": bench_fwdbwd}[a.what](a)
