"""Data step: DeviceChunkLoader vs the reference loop
DataLoader(RandomChunkDataset(...), batch_size, collate_fn=collate_fn)
(VQ_VAE_HMM_fixed.py:10-29, 164-179).  Same `random` seed -> same batches,
bit for bit."""
import random

import numpy as np
import pytest
import torch

from vqhmm.data import DeviceChunkLoader, RandomChunkDataset, _bases, collate_fn


def make_sequences(seed, n_seq=7, C=5, U=4):
    g = torch.Generator().manual_seed(seed)
    lens = [60, 250, 199, 1000, 20, 333, 201][:n_seq]
    xs = [torch.randn(C, n, generator=g) for n in lens]
    us = [torch.randn(U, n, generator=g) for n in lens]
    return xs, us


def reference_batches(ds, batch_size, seed):
    random.seed(seed)
    n = len(ds)
    out = []
    for b0 in range(0, n, batch_size):
        batch = [ds[i] for i in range(b0, min(n, b0 + batch_size))]
        out.append(collate_fn(batch, device="cpu"))
    return out


def test_draw_matches_getitem():
    xs, us = make_sequences(0)
    ds = RandomChunkDataset(xs, us, min_len=20, max_len=200)
    random.seed(11)
    items = [ds[i] for i in range(50)]
    random.seed(11)
    draws = [ds.draw() for _ in range(50)]
    for (x, u, L), (k, s, L2) in zip(items, draws):
        assert L == L2
        assert torch.equal(x, xs[k][:, s:s + L]) and torch.equal(u, us[k][:, s:s + L])


def test_plan_meta_reproduces_collate_on_host():
    """The (base, n, start, length) table addresses exactly collate_fn's batch
    (checked with a host gather, no GPU)."""
    xs, us = make_sequences(1)
    ds = RandomChunkDataset(xs, us, min_len=20, max_len=200)
    ld = DeviceChunkLoader.__new__(DeviceChunkLoader)
    ld.ds, ld.n = ds, [x.shape[1] for x in xs]
    ld.xbase, ld.ubase = _bases(xs), _bases(us)
    xsrc = torch.cat([x.reshape(-1) for x in xs]).numpy()
    usrc = torch.cat([u.reshape(-1) for u in us]).numpy()
    ref = reference_batches(ds, 64, seed=3)[0]
    random.seed(3)
    meta, lengths = ld.plan(64)
    assert torch.equal(lengths, ref[2])
    tmax = int(lengths.max())
    for src, rows, want, C in ((xsrc, meta[:64], ref[0], 5), (usrc, meta[64:], ref[1], 4)):
        got = np.zeros((64, C, tmax), np.float32)
        for i, (base, n, s, L) in enumerate(rows.tolist()):
            for c in range(C):
                got[i, c, :L] = src[base + c * n + s: base + c * n + s + L]
        assert np.array_equal(got, want.numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("batch_size,drop_last", [(64, False), (128, True), (1000, False)])
def test_device_loader_bit_identical(batch_size, drop_last):
    xs, us = make_sequences(2)
    ds = RandomChunkDataset(xs, us, min_len=20, max_len=200)
    ref = reference_batches(ds, batch_size, seed=5)
    if drop_last and len(ds) % batch_size:
        ref = ref[:-1]
    random.seed(5)
    ld = DeviceChunkLoader(ds, batch_size, drop_last=drop_last, device="cuda")
    got = list(ld)
    assert len(got) == len(ld) == len(ref)
    for (x, u, L), (xr, ur, Lr) in zip(got, ref):
        assert x.is_cuda and u.is_cuda and not L.is_cuda and L.dtype == torch.int64
        assert torch.equal(L, Lr)
        assert torch.equal(x.cpu(), xr) and torch.equal(u.cpu(), ur)


def golden_collate_dataset():
    """The sequences tests/golden/make_golden.py:make_collate_case fed the REFERENCE's
    RandomChunkDataset (torch generator seed 99; lengths 230 / 180 / 260)."""
    g = torch.Generator().manual_seed(99)
    xs = [torch.randn(5, n, generator=g) for n in (230, 180, 260)]
    us = [torch.randn(4, n, generator=g) for n in (230, 180, 260)]
    return RandomChunkDataset(xs, us, min_len=20, max_len=200)


def test_dataset_and_collate_match_reference_fixture():
    """vqhmm.RandomChunkDataset items under random.seed(7) and vqhmm.collate_fn reproduce
    the reference's (VQ_VAE_HMM_fixed.py:10-29, 164-179) captured in collate.npz bit for bit."""
    from conftest import load_golden
    gold = load_golden("collate")
    ds = golden_collate_dataset()
    assert len(ds) == int(gold["len_ds"])
    random.seed(7)
    items = [ds[i] for i in range(6)]
    for i, (xi, ui, L) in enumerate(items):
        assert L == int(gold[f"item{i}/L"])
        assert np.array_equal(xi.numpy(), gold[f"item{i}/x"]) and np.array_equal(ui.numpy(), gold[f"item{i}/u"])
    x, u, lengths = collate_fn(items, device="cpu")
    assert lengths.dtype == torch.int64 and np.array_equal(lengths.numpy(), gold["lengths"])
    assert np.array_equal(x.numpy(), gold["x"]) and np.array_equal(u.numpy(), gold["u"])


@pytest.mark.gpu
def test_device_loader_matches_reference_fixture():
    """DeviceChunkLoader's first batch (batch_size 6, random.seed(7)) equals the reference's
    collate_fn output in collate.npz bit for bit."""
    from conftest import load_golden
    gold = load_golden("collate")
    ds = golden_collate_dataset()
    ld = DeviceChunkLoader(ds, 6, device="cuda")
    random.seed(7)
    x, u, lengths = next(iter(ld))
    assert x.is_cuda and u.is_cuda and not lengths.is_cuda
    assert np.array_equal(lengths.numpy(), gold["lengths"])
    assert np.array_equal(x.cpu().numpy(), gold["x"]) and np.array_equal(u.cpu().numpy(), gold["u"])
