"""Data-parallel path.

CPU (gloo, world_size 2, spawned processes): the DP math and plumbing —
  the SUM all-reduce of per-shard flat gradients / world equals the full-batch
  gradient of the reference objective (CPU oracle), and per-rank sampling
  draws different chunks.
  Ragged batches with global normalisers (vqhmm.dist.global_norm): the SUM of
  the shard gradients equals the full-batch gradient, both for shards of one
  collated batch and for independently drawn per-rank batches padded to a
  common T (pad_to_common_T), which is also shown to be necessary.
GPU (gloo over 2 processes on cuda:0): TrainState with the all-reduce gives
  the same parameters after 3 Adam steps as one process on the full batch;
  with ragged lengths and global normalisers too.  Single process: the HIP
  kernels' per-shard losses / gradients with `norm` sum to the full batch's.
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


def _ragged_case():
    from oracle import ref_model as RM
    torch.manual_seed(0)
    shapes = RM.param_shapes(5, 16, 3, 8, 4, 16)
    p = {k: (torch.randn(shapes[k]) * 0.3).requires_grad_(True) for k in RM.PARAM_ORDER}
    g = torch.Generator().manual_seed(9)
    B, T = 8, 30
    L = torch.tensor([30, 7, 19, 25, 1, 28, 12, 22])  # shard 1 alone would pad to 28
    x, u = torch.randn(B, 5, T, generator=g), torch.randn(B, 4, T, generator=g)
    valid = (torch.arange(T)[None, :] < L[:, None]).float()
    return RM, p, x * valid[:, None], u * valid[:, None], L


def _flat_grad(RM, p, loss):
    for k in RM.PARAM_ORDER:
        p[k].grad = None
    loss.backward()
    return torch.cat([p[k].grad.reshape(-1) for k in RM.PARAM_ORDER])


def _cpu_ragged_worker(rank, world, port, out):
    _setup(rank, world, port)
    torch.set_num_threads(1)
    from vqhmm import dist
    RM, p, x, u, L = _ragged_case()
    T = x.shape[-1]
    res = {}
    # (a) shards of one collated global batch: normalisers from the global lengths, no exchange
    xs, us, Ls = dist.shard_batch(x, u, L, rank, world)
    n_glob = dist.global_norm(L, T, reduce=False)
    n_red = dist.global_norm(Ls, T)  # (b) the same numbers by an all-reduce of the local lengths
    assert n_glob.tolist() == n_red.tolist() == [int(L.clamp(0, T).sum()), 8]
    loss = RM.elbo(p, xs, us, Ls, 0.7, 3, 4, norm=n_glob.tolist())
    flat = _flat_grad(RM, p, loss)
    dist.allreduce_sum_(flat)
    lsum = loss.detach().clone().reshape(1)
    dist.allreduce_sum_(lsum)
    res["shard"] = (flat, lsum)
    # (c) independently drawn per-rank batches of different T: pad to the common T
    Tr = int(Ls.max())
    xr, ur = xs[..., :Tr].contiguous(), us[..., :Tr].contiguous()
    xp, up, Tg = dist.pad_to_common_T(xr, ur)
    nr = dist.global_norm(Ls, Tg)
    res["padded"] = _flat_grad(RM, p, RM.elbo(p, xp, up, Ls, 0.7, 3, 4, norm=nr.tolist()))
    dist.allreduce_sum_(res["padded"])
    res["Tg"] = Tg
    res["unpadded"] = _flat_grad(RM, p, RM.elbo(p, xr, ur, Ls, 0.7, 3, 4, norm=nr.tolist()))
    dist.allreduce_sum_(res["unpadded"])
    if rank == 0:
        torch.save(res, out)
    torch.distributed.destroy_process_group()


def test_gloo_ragged_global_norm_sums_to_full_batch(tmp_path):
    out = str(tmp_path / "rag.pt")
    mp.start_processes(_cpu_ragged_worker, args=(2, free_port(), out), nprocs=2, join=True, start_method="spawn")
    RM, p, x, u, L = _ragged_case()
    full = RM.elbo(p, x, u, L, 0.7, 3, 4)
    ref = _flat_grad(RM, p, full)
    res = torch.load(out)
    flat, lsum = res["shard"]
    assert torch.linalg.norm(flat - ref) <= 1e-5 * torch.linalg.norm(ref)
    assert abs(lsum.item() - full.item()) <= 1e-5 * abs(full.item())
    assert res["Tg"] == 30
    assert torch.linalg.norm(res["padded"] - ref) <= 1e-5 * torch.linalg.norm(ref)
    # without the common padding, the longest sequence of the shorter shard sees
    # conv zero-padding instead of relu(bias) activations: not the global batch
    assert torch.linalg.norm(res["unpadded"] - ref) > 1e-4 * torch.linalg.norm(ref)


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
    grads = []
    st.step(xs.cuda(), us.cuda(), Ls, 1.0)  # the first step eagerly: its all-reduced gradient is compared
    grads.append(st.grad.cpu() * st.grad_scale())  # the SUM over ranks / world: the batch gradient Adam applies
    if graph:  # 1 warm-up step + 1 replay of the captured DP step (fwd+bwd, all-reduce, Adam)
        st.capture(xs.cuda(), us.cuda(), Ls, 1.0, warmup=1)()
    else:
        for _ in range(2):
            st.step(xs.cuda(), us.cuda(), Ls, 1.0)
    torch.cuda.synchronize()
    grads.append(st.grad.cpu() * st.grad_scale())
    if rank == 0:
        torch.save({"flat": st.flat.cpu(), "grads": grads}, out)
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
    ref_grads = []
    for _ in range(3):
        st.step(x.cuda(), u.cuda(), torch.full((B,), T), 1.0)
        ref_grads.append(st.grad.cpu())
    check_trajectories(st, torch.load(out), ref_grads)


@pytest.mark.gpu
def test_gpu_global_norm_shards_sum_to_full_batch():
    """HIP path, one process: per-shard losses/grads with the global normalisers
    (vqhmm_elbo_fwd/bwd_f32 `norm`) sum to the full ragged batch's."""
    import vqhmm
    from vqhmm import dist
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128).cuda()
    g = torch.Generator().manual_seed(5)
    B, T = 64, 120
    L = torch.randint(1, T + 1, (B,), generator=g)
    L[3] = T
    x, u = torch.randn(B, 5, T, generator=g), torch.randn(B, 4, T, generator=g)
    st = vqhmm.TrainState(m, lr=1e-3)
    xc, uc, Lc = st.prepare(x, u, L)
    st.forward_backward(xc, uc, Lc, 0.6)
    ref_g, ref_l = st.grad.clone(), st.loss.clone()
    norm = dist.global_norm(Lc, T, reduce=False)
    assert norm.tolist() == [int(L.sum()), B]
    acc_g, acc_l = torch.zeros_like(ref_g), torch.zeros_like(ref_l)
    for r in range(4):
        xs, us, Ls = dist.shard_batch(xc, uc, Lc, r, 4)
        st.forward_backward(xs.contiguous(), us.contiguous(), Ls.contiguous(), 0.6, norm)
        acc_g += st.grad
        acc_l += st.loss
    torch.cuda.synchronize()
    assert torch.linalg.norm(acc_g - ref_g) <= 1e-5 * torch.linalg.norm(ref_g)
    assert abs(acc_l.item() - ref_l.item()) <= 1e-5 * abs(ref_l.item())


def _gpu_ragged_worker(rank, world, port, out):
    _setup(rank, world, port)
    import vqhmm
    from vqhmm import dist
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128).cuda()
    g = torch.Generator().manual_seed(4)
    B, T = 64, 120
    L = torch.randint(1, T + 1, (B,), generator=g)
    x, u = torch.randn(B, 5, T, generator=g), torch.randn(B, 4, T, generator=g)
    xs, us, Ls = dist.shard_batch(x, u, L, rank, world)
    st = vqhmm.TrainState(m, lr=1e-3, distributed=True)
    grads = []
    for _ in range(3):
        xc, uc, Lc = st.prepare(xs, us, Ls)
        st.step(xc, uc, Lc, 1.0, dist.global_norm(Lc, T))
        grads.append(st.grad.cpu())  # the all-reduced gradient the step's Adam applied
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({"flat": st.flat.cpu(), "grads": grads}, out)
    torch.distributed.destroy_process_group()


def check_trajectories(st, got, ref_grads, lr=1e-3, steps=3):
    """DP run vs one process: the first step's gradient (same parameters on both sides; later steps start
    from slightly different ones) per parameter tensor normwise within 1e-5, and the Adam trajectories:
    all elements on average within 1e-4 of steps * lr, every element within a quarter of steps * lr.
    The max is loose on purpose: Adam moves an element by lr * m / (sqrt(v) + eps), so where a gradient is
    near 0, or changes sign between steps (m ~ 0), an fp32 summation difference moves it by a visible
    fraction of lr (one decoder.conv2 element parts by 0.14 lr over 3 steps).  A wrong DP scale or a
    missing shard would move every element by ~lr, which the mean catches.  Elements whose gradient is
    firm (the same sign on all steps and at least a tenth of the tensor's RMS gradient on each) keep the
    tight bound, 1% of steps * lr, so an error confined to a few tensors cannot hide under the loose one."""
    ref = st.flat.cpu()
    got_grads = got.get("grads") or []
    assert len(got_grads) > 0, "the DP worker must save its all-reduced gradients"
    ga, gb = ref_grads[0], got_grads[0]
    for i in range(len(st.off) - 1):
        a, b = ga[st.off[i]:st.off[i + 1]], gb[st.off[i]:st.off[i + 1]]
        assert (a - b).norm() <= 1e-5 * a.norm() + 1e-12, (i, float((a - b).norm() / a.norm()))
    d = (got["flat"] - ref).abs()
    assert d.mean().item() <= 1e-4 * steps * lr
    assert d.max().item() <= 0.25 * steps * lr, d.max().item()
    G = torch.stack(ref_grads[:steps])
    rms = torch.cat([ga[st.off[i]:st.off[i + 1]].pow(2).mean().sqrt().expand(st.off[i + 1] - st.off[i])
                     for i in range(len(st.off) - 1)])
    firm = ((G > 0).all(0) | (G < 0).all(0)) & (G.abs().min(0).values >= 0.1 * rms)
    assert firm.sum().item() > 0.05 * firm.numel(), firm.sum().item()  # 13% of this case's elements
    assert d[firm].max().item() <= 1e-2 * steps * lr, d[firm].max().item()


@pytest.mark.gpu
def test_gpu_two_ranks_ragged_global_norm_match_one(tmp_path):
    import vqhmm
    out = str(tmp_path / "dpr.pt")
    mp.start_processes(_gpu_ragged_worker, args=(2, free_port(), out), nprocs=2, join=True, start_method="spawn")
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128).cuda()
    g = torch.Generator().manual_seed(4)
    B, T = 64, 120
    L = torch.randint(1, T + 1, (B,), generator=g)
    x, u = torch.randn(B, 5, T, generator=g), torch.randn(B, 4, T, generator=g)
    st = vqhmm.TrainState(m, lr=1e-3)
    ref_grads = []
    for _ in range(3):
        st.step(x.cuda(), u.cuda(), L, 1.0)
        ref_grads.append(st.grad.cpu())
    check_trajectories(st, torch.load(out), ref_grads)
