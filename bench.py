#!/usr/bin/env python3
"""Headline benchmark: VAE_HMM train-step sequences/sec on MI355X.

    python bench.py [--gpus N --steps K --warmup W --scaling strong|weak]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1], "cfg2"): VAE_HMM(K=3, input_dim=5,
hidden_dim=64, hidden_dim2=32, u_dim=4, trans_hidden=128), T=200, synthetic
x/u ~ N(0,1) already resident in HBM, lengths = T, beta=1, Adam lr=1e-3.  A
step = zero_grad + compute_loss + backward + [RCCL all-reduce of the flat
gradient] + Adam, exactly the reference's train_model inner loop
(VQ_VAE_HMM_fixed.py:154-157).

Scaling: "strong" (default) keeps the GLOBAL batch at the
config's 1024 sequences (cfg4: 4096) and splits it over the N ranks (128 per
GPU at N=8); "weak" gives every rank the full batch.  `value` = sequences of
all ranks per step * K / max-over-ranks wall time of K steps.

Multi-GPU: one process per GPU over RCCL.  Under torchrun the world comes from
its env (it must equal --gpus); a bare `python bench.py --gpus N` spawns the N
rank processes itself (fresh interpreters; the parent never touches the GPU).

Also reported (rank 0):
  roofline      dominant kernel of the step, timed live with HIP events on the
                launch stream over instrumented steps; achieved = algorithmic
                FLOPs (or bytes) per launch / average launch duration
                (vqhmm_elbo_stage_info); traffic = PMC HBM bytes per launch from
                profiles/ when a matching measurement is committed, else null.
  cpu_baseline  the CPU oracle (oracle/ref_model.py, a from-scratch restatement
                pinned bit-exact to the reference) timed on this host's cores on
                the same workload shape (N=1 only).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

# The HIP runtime pre-captures a graph's kernel packets by default; on this step (5 dependent launches)
# that replays ~0.7 us per node slower than with it off (B = 128 one-graph DP step 0.1041 -> 0.1005 ms,
# tools/gpu_graph_ab.sh).  Read once at HIP initialisation, so it is set before torch touches the GPU.
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
# Kernel arguments in device memory (vqhmm sets the same default on import; here it must precede torch's
# first GPU call): B = 128 0.1082 -> 0.0939 ms, cfg2 0.4342 -> 0.4199 ms (tools/gpu_kernarg_ab.sh).
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vq-vae-hmm-model_amd"))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (global B, T, D, H, H2, K, U, TH)
    "cfg2": (1024, 200, 5, 64, 32, 3, 4, 128),
    "cfg4": (4096, 512, 16, 64, 32, 8, 4, 128),
    # BASELINE configs[2]'s model dims (H2 = H/2 as the reference's default ratio): the
    # training step at K=32, D=64, H=256 (BASELINE frames this config as the VQ stress: vq_cfg3 leg)
    "cfg3": (2048, 200, 64, 256, 128, 32, 4, 128),
}
MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense FP32 (matrix = vector peak)
HBM_PEAK_GBPS = 8000.0         # MI355X_MICROARCH.md: HBM3E spec peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default="strong", choices=("strong", "weak"),
                    help="strong: the config's global batch split over the ranks; weak: the full batch per rank")
    ap.add_argument("--batch", type=int, default=0, help="override the global batch (strong) / per-rank batch (weak)")
    ap.add_argument("--launch", default="auto", choices=("auto", "graph", "eager"),
                    help="how the step reaches the GPU: auto = eager launches for the fused single-process step "
                         "(its 5 launches: 0.0945 vs 0.0994 ms as a graph at B = 128), one HIP graph for the "
                         "data-parallel form (the all-reduce captured: 0.1005 vs 0.1069 ms eager)")
    ap.add_argument("--no-graph", action="store_true", help="same as --launch eager")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--profile-steps", type=int, default=5)
    ap.add_argument("--no-hmm", action="store_true", help="skip the Viterbi / forward-backward kernel lines")
    ap.add_argument("--dp-form", action="store_true",
                    help="N=1: run the data-parallel step form (fwd+bwd graph, RCCL all-reduce over a 1-rank "
                         "process group, Adam graph) instead of the fused single-process step")
    return ap.parse_args()


def stage_timings(lib, st, x, u, L, B, T, beta, nsteps):
    """Per-stage device time (us) inside real steps: events around each stage on the launch stream."""
    from vqhmm import _ext
    d = ctypes.byref(st.dims)
    ws = st.workspace(B, T)
    lay = st.model.prior.u_layout(u)
    n = lib.vqhmm_elbo_num_stages()
    stream = torch.cuda.current_stream()
    sp = _ext.stream_ptr()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(n + 1)] for _ in range(nsteps)]
    for k in range(nsteps):
        for s in range(n):
            ev[k][s].record(stream)
            _ext.check(lib.vqhmm_elbo_stage_f32(d, st.ptrs, _ext.ptr(x), _ext.ptr(u), lay, _ext.ptr(L), None, B,
                                                T, float(beta), _ext.ptr(ws), ws.numel(), _ext.ptr(st.grad), s, sp),
                       "stage")
        ev[k][n].record(stream)
        st.apply_adam()
    torch.cuda.synchronize()
    out = []
    name = ctypes.create_string_buffer(256)
    fl, by, mf = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    for s in range(n):
        us = statistics.median(ev[k][s].elapsed_time(ev[k][s + 1]) * 1e3 for k in range(nsteps))
        lib.vqhmm_elbo_stage_info(d, B, T, s, name, len(name), ctypes.byref(fl), ctypes.byref(by), ctypes.byref(mf))
        out.append(dict(stage=s, name=name.value.decode(), us=us, flops=fl.value, bytes=by.value,
                        mfma=bool(mf.value)))
    return out


def traffic_for(kernel_name, cfg, batch=None):
    """PMC-measured HBM bytes per launch, if committed under profiles/ for this kernel at this config AND
    batch (training-step sections are keyed "cfg/B<batch>"; the fixed-shape kernel legs by name): null when
    no PMC pass ran at this shape, never another batch's figure."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            tab = json.load(f)
        sec = f"{cfg}/B{batch}" if batch is not None else cfg
        return tab.get(sec, {}).get(kernel_name)
    except (OSError, ValueError):
        return None


def traffic_checked(traffic, avg_us, where=""):
    """A PMC byte count is kept only if it is physically possible for the launch it is quoted with
    (traffic / duration <= the 8 TB/s HBM peak); otherwise null, with the rejected figure reported by
    traffic_rejected() and on stderr (a stale profiles/pmc_traffic.json or a wrong kernel match: regenerate
    it with tools/gpu_pmc_r6.sh), so 'rejected' is not mistaken for 'not profiled'."""
    if traffic is None or avg_us is None or avg_us <= 0:
        return traffic
    if traffic / (avg_us * 1e-6) <= HBM_PEAK_GBPS * 1e9:
        return traffic
    print(f"bench.py: PMC traffic {traffic} B for {where or 'a launch'} implies "
          f"{traffic / (avg_us * 1e-6) / 1e9:.0f} GB/s at {avg_us:.2f} us (> peak): reported as null",
          file=sys.stderr)
    return None


def traffic_rejected(traffic, avg_us):
    """The raw figure traffic_checked() nulled (bytes and the implied GB/s), or None."""
    if traffic is None or avg_us is None or avg_us <= 0 or traffic / (avg_us * 1e-6) <= HBM_PEAK_GBPS * 1e9:
        return None
    return {"bytes": traffic, "implied_GBps": round(traffic / (avg_us * 1e-6) / 1e9, 1)}


def vq_cfg3(lib):
    """VQ L2-argmin at BASELINE cfg3 shape (K=32, Dv=64, B=2048, T=200): HBM roofline."""
    from vqhmm import _ext
    g = torch.Generator(device="cuda").manual_seed(1234)
    B, Dv, T, K = 2048, 64, 200, 32
    z = torch.randn(B, Dv, T, device="cuda", generator=g)
    cb = torch.randn(K, Dv, device="cuda", generator=g)
    idx = torch.empty(B, T, dtype=torch.int32, device="cuda")
    sp = _ext.stream_ptr()
    run = lambda: lib.vqhmm_vq_argmin_f32(_ext.ptr(z), B, Dv, T, _ext.ptr(cb), K, _ext.ptr(idx), None, sp)
    for _ in range(5):
        run()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    byts = 4.0 * B * T * Dv + 4.0 * K * Dv + 4.0 * B * T
    gbps = byts / (us * 1e-6) / 1e9
    out = {"kernel": "vq_rows_kernel (vqhmm_vq_argmin_f32)", "bound": "hbm", "avg_us": round(us, 2),
           "achieved": round(gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(gbps / HBM_PEAK_GBPS, 4),
           "traffic": traffic_checked(traffic_for("vq_argmin", "vq_cfg3"), us, "vq_cfg3"),
           "shape": "B2048 Dv64 T200 K32"}
    # the fused quantize (pseudocode.txt:12-18): argmin + z_q gather + straight-through value written +
    # squared-error partials, then the fixed-order partial sum: z read once, z_q_st and idx written
    zq = torch.empty_like(z)
    sse = torch.zeros((), dtype=torch.float64, device="cuda")
    nb = lib.vqhmm_vq_quantize_workspace_size(B, Dv, T, K)
    ws = torch.empty(max(nb, 8), dtype=torch.uint8, device="cuda")
    runq = lambda: lib.vqhmm_vq_quantize_f32(_ext.ptr(z), B, Dv, T, _ext.ptr(cb), K, _ext.ptr(idx), _ext.ptr(zq),  # noqa: E731
                                             _ext.ptr(sse), _ext.ptr(ws), ws.numel(), sp)
    for _ in range(5):
        runq()
    e0.record(s)
    for _ in range(20):
        runq()
    e1.record(s)
    torch.cuda.synchronize()
    usq = e0.elapsed_time(e1) / 20 * 1e3
    byq = 8.0 * B * T * Dv + 4.0 * K * Dv + 4.0 * B * T
    gq = byq / (usq * 1e-6) / 1e9
    out["quantize"] = {"kernel": "vq_rows_kernel<.., QUANT> + vq_sse_finalize_kernel (vqhmm_vq_quantize_f32)",
                       "bound": "hbm", "avg_us": round(usq, 2), "achieved": round(gq, 1), "peak": HBM_PEAK_GBPS,
                       "unit": "GB/s", "frac": round(gq / HBM_PEAK_GBPS, 4)}
    del z, zq
    return out


def hmm_kernels(lib):
    """Viterbi at the cfg5 per-GPU shard (K=8, T=4096, 1024 sequences = 8192 / 8 GPUs) and
    forward-backward at the cfg4 per-GPU shard (K=8, T=512, 512 sequences = 4096 / 8), HBM roofline.
    Tables are log_softmax(N(0,1)) over the last dim."""
    from vqhmm import _ext
    out = {}
    sp = _ext.stream_ptr()
    for name, (B, T, K) in (("viterbi_cfg5", (1024, 4096, 8)), ("fwdbwd_cfg4", (512, 512, 8))):
        g = torch.Generator(device="cuda").manual_seed(7)
        log_pi = torch.log_softmax(torch.randn(K, device="cuda", generator=g), -1)
        log_A = torch.log_softmax(torch.randn(B, T, K, K, device="cuda", generator=g), -1)
        em = torch.log_softmax(torch.randn(B, T, K, device="cuda", generator=g), -1)
        L = torch.full((B,), T, dtype=torch.int64, device="cuda")
        P = _ext.ptr
        if name.startswith("viterbi"):
            path = torch.empty(B, T, dtype=torch.int32, device="cuda")
            score = torch.empty(B, device="cuda")
            nb = lib.vqhmm_viterbi_workspace_size(B, T, K)
            ws = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")
            run = lambda: lib.vqhmm_viterbi_f32(P(log_pi), P(log_A), P(em), P(L), B, T, K, P(path), P(score),  # noqa: E731
                                                P(ws), nb, sp)
            byts = B * (4.0 * T * K * K + 4.0 * T * K + 4.0 * T) + 4.0 * K
            kern = "viterbi_kernel<8, true>"
        else:
            gamma = torch.empty(B, T, K, device="cuda")
            logZ = torch.empty(B, device="cuda")
            nb = lib.vqhmm_fwdbwd_workspace_size(B, T, K)
            ws = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")
            run = lambda: lib.vqhmm_fwdbwd_f32(P(log_pi), P(log_A), P(em), P(L), B, T, K, P(gamma), P(logZ),  # noqa: E731
                                               P(ws), nb, sp)
            byts = B * (4.0 * T * K * K + 4.0 * T * K + 4.0 * T * K) + 4.0 * K
            kern = "fwdbwd_seg_kernel"
        for _ in range(3):
            run()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            run()
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        gbps = byts / (us * 1e-6) / 1e9
        out[name] = {"kernel": kern, "bound": "hbm", "avg_us": round(us, 2), "achieved": round(gbps, 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(gbps / HBM_PEAK_GBPS, 4),
                     "traffic": traffic_checked(traffic_for(name, name), us, name), "shape": f"B{B} T{T} K{K}"}
        del log_A, em, ws
    # the fused Prior-MLP -> Viterbi at the same cfg5 shard: log_A is built on the chip
    # from u, so the kernel is bound by the MLP on the f32 MFMA: 2 (U + K^2) TH flops per position
    import vqhmm
    B, T, K, U, TH = 1024, 4096, 8, 4, 128
    torch.manual_seed(0)
    prior = vqhmm.Prior(K, u_dim=U, trans_hidden=TH).cuda()
    g = torch.Generator(device="cuda").manual_seed(9)
    u = torch.randn(B, U, T, device="cuda", generator=g)
    em = torch.log_softmax(torch.randn(B, T, K, device="cuda", generator=g), -1)
    L = torch.full((B,), T, dtype=torch.int64, device="cuda")
    run = lambda: vqhmm.prior_viterbi(prior, u, em, L)  # noqa: E731
    for _ in range(2):
        run()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(5):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 5 * 1e3
    tf = B * T * 2.0 * (U + K * K) * TH / (us * 1e-6) / 1e12
    out["prior_viterbi_cfg5"] = {"kernel": "prior_viterbi_kernel<8, 8, 8, 32> (vqhmm_prior_viterbi_f32)",
                                 "bound": "mfma", "avg_us": round(us, 2), "achieved": round(tf, 2),
                                 "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                                 "frac": round(tf / MFMA_F32_PEAK_TFLOPS, 4), "shape": f"B{B} T{T} K{K} TH{TH} U{U}",
                                 "note": "per call incl. log_pi + workspace allocation; the unfused Prior.forward "
                                         "+ Viterbi writes and reads the 1.07 GB log_A"}
    return out


def host_threads():
    """Threads for the CPU baseline: the CPUs this process may run on
    (len(os.sched_getaffinity(0))), capped by the cgroup CPU quota and OMP_NUM_THREADS when
    those are set (a GPU box's affinity mask can list the whole machine while its share is
    smaller).  Returns (threads, affinity_cpus)."""
    n_aff = len(os.sched_getaffinity(0))
    n = n_aff
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n, n_aff


def _oracle_step_times(cfg, B, threads, seconds, min_steps, warmup):
    from oracle import ref_model as RM
    import vqhmm
    _, T, D, H, H2, K, U, TH = cfg
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=U, trans_hidden=TH)  # same init as the GPU run (CPU tensors)
    p = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    gen = torch.Generator().manual_seed(1234)
    x = torch.randn(B, D, T, generator=gen)
    u = torch.randn(B, U, T, generator=gen)
    L = torch.full((B,), T, dtype=torch.long)
    opt = torch.optim.Adam([p[k] for k in RM.PARAM_ORDER], lr=1e-3)

    def step():
        opt.zero_grad()
        RM.elbo(p, x, u, L, 1.0, K, U).backward()
        opt.step()

    for _ in range(warmup):
        step()
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < min_steps:
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    return statistics.median(times), len(times)


def cpu_baseline(cfg, B, seconds):
    """CPU oracle (oracle/ref_model.py, pinned bit-exact to the reference) train step on the
    same shape.  First a thread sweep (1, 2, 4, ... up to the host threads this process may
    use; 1 warm-up + 2 timed full-batch steps each), then ~`seconds` of full-batch steps
    (>= 3 warm-up) at the sweep's fastest thread count, which is what `cores` states."""
    nthr, n_aff = host_threads()
    saved = torch.get_num_threads()
    counts = sorted({c for c in (1, 2, 4, 8, 16, 32, 64) if c <= nthr} | {nthr})
    sweep = {}
    try:
        for c in counts:
            med, _ = _oracle_step_times(cfg, B, c, 0.0, 2, 1)
            sweep[c] = B / med
        best = max(sweep, key=sweep.get)
        med, n = _oracle_step_times(cfg, B, best, seconds, 3, 3)
    finally:
        torch.set_num_threads(saved)
    _, T = cfg[0], cfg[1]
    scales = sweep[best] >= 1.2 * sweep[1]
    return {"value": round(B / med, 1), "unit": "sequences/s", "cores": best, "kind": "port",
            "sample": f"{n} full train steps (B={B}, T={T}) of the torch-CPU oracle after 3 warm-up steps at "
                      f"the thread sweep's fastest count ({best} of {nthr} usable threads; {n_aff} CPUs in the "
                      f"affinity mask, capped by the cgroup quota / OMP_NUM_THREADS), median {med*1e3:.1f} ms/step",
            "thread_sweep": {"batch": B, "seq_per_s": {str(c): round(v, 1) for c, v in sweep.items()},
                             "interop_threads": torch.get_num_interop_threads()},
            "note": None if scales else
            f"the host does not scale this workload: {best} threads give {sweep[best] / sweep[1]:.2f}x one thread"}


def spawn_ranks(n):
    """`python bench.py --gpus N` without torchrun: start N fresh rank processes (this
    parent never touches the GPU) on 127.0.0.1; report every rank's exit code or signal
    and return the worst one."""
    import signal
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    if any(codes):
        def describe(c):
            if c < 0:
                try:
                    return f"signal {signal.Signals(-c).name}"
                except ValueError:
                    return f"signal {-c}"
            return f"exit {c}"
        print("bench.py: rank exits: " + ", ".join(f"rank {r}: {describe(c)}" for r, c in enumerate(codes)),
              file=sys.stderr)
    return max(abs(c) for c in codes)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0:
        if a.gpus > 1:
            sys.exit(spawn_ranks(a.gpus))
        world = 1
    if world != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but the launcher's WORLD_SIZE is {world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rank 0's one JSON line must stand alone on stdout, but RCCL writes its version line and warnings there
    # even at NCCL_DEBUG=WARN (VQHMM_NCCL_DEBUG picks another level): the JSON gets a private handle on the
    # real stdout and file descriptor 1 goes to stderr for everything else, native libraries included
    os.environ["NCCL_DEBUG"] = os.environ.get("VQHMM_NCCL_DEBUG", "WARN")
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if world > 1:
        # VQHMM_BENCH_BACKEND=gloo rehearses the N-rank path on a box with fewer GPUs (ranks share
        # devices round-robin; the all-reduce then goes through host memory): never a measurement
        backend = os.environ.get("VQHMM_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            torch.distributed.init_process_group(backend)
        if torch.distributed.get_world_size() != world:
            sys.exit("bench.py: process group size disagrees with WORLD_SIZE")
    else:
        torch.cuda.set_device(0)
        if a.dp_form:  # a 1-rank RCCL group: the DP step's collective runs for real, on one GPU
            torch.distributed.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(),
                                                 world_size=1, rank=0, device_id=torch.device("cuda", 0))
    import vqhmm
    from vqhmm import _ext
    lib = _ext.load()

    cfg = CONFIGS[a.config]
    Bglob, T, D, H, H2, K, U, TH = cfg
    if a.batch:
        Bglob = a.batch
    if a.scaling == "strong":
        if Bglob % world:
            sys.exit(f"bench.py: global batch {Bglob} does not split over {world} ranks")
        B = Bglob // world
    else:
        B = Bglob
        Bglob = B * world
    torch.manual_seed(0)
    model = vqhmm.VAE_HMM(D, H, K, H2, u_dim=U, trans_hidden=TH).cuda()
    st = vqhmm.TrainState(model, lr=1e-3, dp_form=True if a.dp_form else None)
    g = torch.Generator(device="cuda").manual_seed(1234 + rank)
    x = torch.randn(B, D, T, device="cuda", generator=g)
    u = torch.randn(B, U, T, device="cuda", generator=g)
    L = torch.full((B,), T, dtype=torch.int64, device="cuda")
    beta = 1.0

    launch = "eager" if a.no_graph else a.launch
    if launch == "auto":
        launch = "graph" if st.dp_form else "eager"
    use_graph = launch == "graph"  # the DP form: fwd+bwd, RCCL all-reduce and Adam as one graph
    if use_graph:
        step = st.capture(x, u, L, beta)
    else:
        step = lambda: st.step(x, u, L, beta)  # noqa: E731

    for _ in range(a.warmup):
        step()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()
    ms_per_step = elapsed / a.steps * 1e3
    value = Bglob * a.steps / elapsed
    st.check_status()  # any device-side error word set during the timed steps raises here

    roof = None
    kernels = None
    stage_roof = None
    if rank == 0 and a.profile_steps > 0:
        stages = stage_timings(lib, st, x, u, L, B, T, beta, a.profile_steps)
        dom = max(stages, key=lambda s: s["us"])
        dur = dom["us"] * 1e-6
        if dom["mfma"]:
            ach = dom["flops"] / dur / 1e12
            roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(ach / MFMA_F32_PEAK_TFLOPS, 4)}
        else:
            ach = dom["bytes"] / dur / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBPS, 4)}
        raw = traffic_for(dom["name"], a.config, B)
        roof.update({"traffic": traffic_checked(raw, dom["us"], dom["name"]),
                     "kernel": dom["name"], "avg_us": round(dom["us"], 2)})
        if traffic_rejected(raw, dom["us"]):
            roof["traffic_rejected"] = traffic_rejected(raw, dom["us"])
        # per launch only: the stages that launch nothing of their own (named "(... in ...)": their work
        # rides in a neighbour's launch) are left out; they would read ~5 us of event overhead each
        kernels = {s["name"]: round(s["us"], 2) for s in stages if not s["name"].startswith("(")}
        # every launch's own roofline (SURVEY 8d asks for the H->H convs' MFMA fraction, not only the
        # dominant stage's): algorithmic flops (MFMA-bound) or bytes (HBM-bound) over the event-timed
        # stage duration (which includes ~5 us of event overhead: an empty stage reads ~5 us)
        stage_roof = {}
        for sd in stages:
            if sd["name"].startswith("(") or sd["us"] <= 0 or (sd["flops"] <= 0 and sd["bytes"] <= 0):
                continue
            dur = sd["us"] * 1e-6
            if sd["mfma"]:
                ach = sd["flops"] / dur / 1e12
                stage_roof[sd["name"]] = {"bound": "mfma", "us": round(sd["us"], 2), "achieved": round(ach, 2),
                                          "unit": "TFLOP/s", "frac": round(ach / MFMA_F32_PEAK_TFLOPS, 4)}
            else:
                ach = sd["bytes"] / dur / 1e9
                stage_roof[sd["name"]] = {"bound": "hbm", "us": round(sd["us"], 2), "achieved": round(ach, 1),
                                          "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4)}
    vq = vq_cfg3(lib) if rank == 0 and world == 1 else None
    hmm = hmm_kernels(lib) if rank == 0 and world == 1 and not a.no_hmm else {}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(cfg, B, a.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "VAE_HMM train-step sequences/sec (K=3, T=200, D=5) at 1/2/4/8 MI355X",
            # (BASELINE.json's metric names cfg2; --config cfg3 / cfg4 report the same quantity at those shapes)
            "value": round(value, 1), "unit": "sequences/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": a.scaling, "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{a.config}: VAE_HMM train step (compute_loss+backward+Adam)",
                       "global_batch": Bglob, "per_gpu_batch": B, "seq_len": T, "K": K, "input_dim": D,
                       "hidden_dim": H, "hidden_dim2": H2, "u_dim": U, "trans_hidden": TH,
                       "parallelism": f"dp{world}" if world > 1 else "single", "hip_graph": use_graph,
                       # HIP runtime settings this process ran with (bench.py sets the graph packet-capture
                       # switch before HIP starts; it changes only the DP form's graph replay, ~0.7 us/node)
                       "hip_env": {k: os.environ[k] for k in ("DEBUG_CLR_GRAPH_PACKET_CAPTURE",
                                                              "HIP_FORCE_DEV_KERNARG") if k in os.environ},
                       "step_form": _step_form(st, use_graph),
                       "collective": ({"backend": _backend_name(), "ranks": torch.distributed.get_world_size()}
                                      if torch.distributed.is_initialized() else None)},
            "roofline": roof, "cpu_baseline": cpu,
            "step_kernels_us": kernels,
            "step_kernels_note": ("HIP-event time of each launch of the step run stage by stage (the forward "
                                  "finalizing its own loss: need_grad=1, one launch the timed step does not "
                                  "have); each includes ~5 us of event overhead"),
            "stage_roofline": stage_roof, "vq_cfg3": vq, **hmm,
        }
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), file=json_out, flush=True)
    # ordered teardown: drop the captured graphs (and with them their memory pools) while the
    # device and the communicator are alive, drain the device, then leave the process group
    del step, st, model
    torch.cuda.synchronize()
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def _step_form(st, use_graph):
    if not st.dp_form:
        return "fused (Adam in the backward's tail launch)" + (", one graph" if use_graph else ", eager")
    if not use_graph:
        return "dp, eager (fwd+bwd, all-reduce, Adam)"
    if getattr(st, "step_graphs", 2) == 1:
        return "dp, one graph (fwd+bwd, RCCL all-reduce and Adam captured together)"
    return "dp, split graphs (fwd+bwd graph, host-issued all-reduce, Adam graph)"


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _backend_name():
    """The collective library the step's all-reduce actually runs on ("rccl" for the nccl backend
    on ROCm; "gloo" in the CPU-side rehearsal)."""
    b = str(torch.distributed.get_backend())
    return "rccl" if b == "nccl" else b


if __name__ == "__main__":
    main()
