"""Data-parallel path.

CPU (gloo, world_size 2, spawned processes): the DP math and plumbing —
  the SUM all-reduce of per-shard flat gradients / world equals the full-batch
  gradient of the reference objective (CPU oracle), and per-rank sampling
  draws different chunks.
GPU (gloo over 2 processes on cuda:0): TrainState with the all-reduce gives
  the same parameters after 3 Adam steps as one process on the full batch.
"""
import math
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    for p in (ROOT, PKG_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)


def _cpu_worker(rank, world, port, out):
    _setup(rank, world, port)
    torch.set_num_threads(1)
    from oracle import ref_model as RM
    from vqhmm import dist
    torch.manual_seed(0)
    shapes = RM.param_shapes(5, 16, 3, 8, 4, 16)
    p = {k: (torch.randn(shapes[k]) * 0.3).requires_grad_(True) for k in RM.PARAM_ORDER}
    g = torch.Generator().manual_seed(7)
    B, T = 8, 30
    x, u = torch.randn(B, 5, T, generator=g), torch.randn(B, 4, T, generator=g)
    L = torch.full((B,), T)
    xs, us, Ls = dist.shard_batch(x, u, L, rank, world)
    RM.elbo(p, xs, us, Ls, 1.0, 3, 4).backward()
    flat = torch.cat([p[k].grad.reshape(-1) for k in RM.PARAM_ORDER])
    dist.allreduce_sum_(flat)
    flat /= world
    dist.seed_rank_sampling(11, rank)
    import random
    draws = [random.random() for _ in range(3)]
    if rank == 0:
        torch.save({"flat": flat, "draws": draws}, out)
    else:
        torch.save({"draws": draws}, out + ".r1")
    torch.distributed.destroy_process_group()


def test_gloo_allreduce_equals_full_batch(tmp_path):
    from oracle import ref_model as RM
    out = str(tmp_path / "r0.pt")
    mp.start_processes(_cpu_worker, args=(2, free_port(), out), nprocs=2, join=True, start_method="spawn")
    torch.manual_seed(0)
    shapes = RM.param_shapes(5, 16, 3, 8, 4, 16)
    p = {k: (torch.randn(shapes[k]) * 0.3).requires_grad_(True) for k in RM.PARAM_ORDER}
    g = torch.Generator().manual_seed(7)
    x, u = torch.randn(8, 5, 30, generator=g), torch.randn(8, 4, 30, generator=g)
    RM.elbo(p, x, u, torch.full((8,), 30), 1.0, 3, 4).backward()
    ref = torch.cat([p[k].grad.reshape(-1) for k in RM.PARAM_ORDER])
    got = torch.load(out)["flat"]
    assert torch.linalg.norm(got - ref) <= 1e-5 * torch.linalg.norm(ref)
    d0 = torch.load(out)["draws"]
    d1 = torch.load(out + ".r1")["draws"]
    assert d0 != d1


def test_shard_batch_rejects_uneven():
    from vqhmm import dist
    with pytest.raises(ValueError):
        dist.shard_batch(torch.zeros(5, 2, 3), torch.zeros(5, 1, 3), torch.zeros(5), 0, 2)


def _gpu_worker(rank, world, port, out, graph=False):
    _setup(rank, world, port)
    import vqhmm
    from vqhmm import dist
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128).cuda()
    g = torch.Generator().manual_seed(3)
    B, T = 64, 120
    x, u = torch.randn(B, 5, T, generator=g), torch.randn(B, 4, T, generator=g)
    L = torch.full((B,), T)
    xs, us, Ls = dist.shard_batch(x, u, L, rank, world)
    st = vqhmm.TrainState(m, lr=1e-3, distributed=True)
    if graph:  # 2 warm-up steps + 1 replay of the split graphs (fwd+bwd graph, all-reduce, Adam graph)
        st.capture(xs.cuda(), us.cuda(), Ls, 1.0, warmup=2)()
    else:
        for _ in range(3):
            st.step(xs.cuda(), us.cuda(), Ls, 1.0)
    torch.cuda.synchronize()
    if rank == 0:
        torch.save(st.flat.cpu(), out)
    torch.distributed.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_gpu_two_ranks_match_one(tmp_path, graph):
    import vqhmm
    out = str(tmp_path / "dp.pt")
    mp.start_processes(_gpu_worker, args=(2, free_port(), out, graph), nprocs=2, join=True, start_method="spawn")
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128).cuda()
    g = torch.Generator().manual_seed(3)
    B, T = 64, 120
    x, u = torch.randn(B, 5, T, generator=g), torch.randn(B, 4, T, generator=g)
    st = vqhmm.TrainState(m, lr=1e-3)
    for _ in range(3):
        st.step(x.cuda(), u.cuda(), torch.full((B,), T), 1.0)
    ref = st.flat.cpu()
    got = torch.load(out)
    # Adam moves each element by <= lr per step: compare trajectories at 1% of 3*lr
    assert (got - ref).abs().max().item() <= 1e-2 * 3e-3
    assert (got - ref).abs().mean().item() <= 1e-4 * 3e-3
