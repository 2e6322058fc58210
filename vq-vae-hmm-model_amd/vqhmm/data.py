"""Batch producer of the training path (VQ_VAE_HMM_fixed.py:10-29, 164-179).

RandomChunkDataset keeps the reference's semantics exactly: __len__ is 1000,
__getitem__ ignores idx and draws (sequence, chunk length, start) from
Python's global `random` in the same order.  collate_fn zero-pads to the
batch maximum and returns (x, u, lengths) with lengths int64 on the CPU like
the reference; it pads on the host and moves each batch to the device with
one copy per tensor instead of the reference's B small device writes.

DeviceChunkLoader is the data step on the GPU: the same
batches as DataLoader(dataset, batch_size, collate_fn=collate_fn), with the
sequences uploaded once and each batch cut and zero-padded by one HIP gather
per tensor (vqhmm_gather_chunks_f32) instead of the per-sample host loop.
"""
import random

import torch

from . import _ext


class RandomChunkDataset:
    def __init__(self, x_sequences, u_sequences, min_len=20, max_len=200):
        self.x_seqs = x_sequences
        self.u_seqs = u_sequences
        self.min_len = min_len
        self.max_len = max_len

    def __len__(self):
        return 1000

    def draw(self):
        """One __getitem__ draw (:26-28): (sequence k, start s, length L) from the
        global `random`, same calls in the same order."""
        k = random.randint(0, len(self.x_seqs) - 1)
        n = self.x_seqs[k].shape[1]
        L = random.randint(self.min_len, min(self.max_len, n))
        s = random.randint(0, n - L)
        return k, s, L

    def __getitem__(self, idx):
        k, s, L = self.draw()
        return self.x_seqs[k][:, s:s + L], self.u_seqs[k][:, s:s + L], L


def default_device():
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


def collate_fn(batch, device=None):
    """[(x (C,L), u (U,L), L)] -> x (B,C,Lmax), u (B,U,Lmax) on `device`, lengths (B,) int64 (CPU)."""
    lengths = torch.tensor([it[2] for it in batch], dtype=torch.long)
    tmax = int(lengths.max().item())
    C, U = batch[0][0].shape[0], batch[0][1].shape[0]
    xb = torch.zeros(len(batch), C, tmax)
    ub = torch.zeros(len(batch), U, tmax)
    for i, (xs, us, L) in enumerate(batch):
        xb[i, :, :L] = xs
        ub[i, :, :L] = us
    dev = default_device() if device is None else torch.device(device)
    if dev.type != "cpu":
        xb = xb.pin_memory().to(dev, non_blocking=True)
        ub = ub.pin_memory().to(dev, non_blocking=True)
    return xb, ub, lengths


def _bases(seqs):
    out, off = [], 0
    for t in seqs:
        out.append(off)
        off += t.numel()
    return out


class DeviceChunkLoader:
    """DataLoader(dataset, batch_size, collate_fn=collate_fn) with the data step on the GPU.

    The dataset's sequences are uploaded once, concatenated.  Per batch, the
    (sequence, start, length) triples are drawn on the host exactly as
    __getitem__ draws them (RandomChunkDataset.draw: the same `random` calls in
    the same order — __getitem__ ignores its index, so a DataLoader's sampler
    order does not matter), a (B, 4) int64 table goes to the device, and
    vqhmm_gather_chunks_f32 writes x (B, C, Tmax) and u (B, U, Tmax)
    zero-padded, bit-identical to collate_fn's.  lengths stay int64 on the CPU
    like the reference's.  len() follows DataLoader: ceil(len(dataset) / B), or
    floor with drop_last."""

    def __init__(self, dataset, batch_size=1, drop_last=False, device=None):
        self.ds = dataset
        self.batch_size = int(batch_size)
        self.drop_last = bool(drop_last)
        self.device = torch.device(device) if device is not None else default_device()
        if self.device.type != "cuda":
            raise RuntimeError("DeviceChunkLoader runs on MI355X (HIP) only: pass a 'cuda' (ROCm) device")
        xs = [torch.as_tensor(x).to(torch.float32) for x in dataset.x_seqs]
        us = [torch.as_tensor(u).to(torch.float32) for u in dataset.u_seqs]
        self.C, self.U = int(xs[0].shape[0]), int(us[0].shape[0])
        self.n = [int(x.shape[1]) for x in xs]
        self.xbase, self.ubase = _bases(xs), _bases(us)
        self.xsrc = torch.cat([x.reshape(-1) for x in xs]).to(self.device)
        self.usrc = torch.cat([u.reshape(-1) for u in us]).to(self.device)

    def __len__(self):
        n = len(self.ds)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def plan(self, nb):
        """Host side of one batch of nb samples: (meta (2*nb, 4) int64 — x rows then
        u rows of {base, n, start, length} — and lengths (nb,) int64)."""
        draws = [self.ds.draw() for _ in range(nb)]
        rows = [(self.xbase[k], self.n[k], s, L) for k, s, L in draws]
        rows += [(self.ubase[k], self.n[k], s, L) for k, s, L in draws]
        meta = torch.tensor(rows, dtype=torch.int64)
        return meta, meta[:nb, 3].clone()

    def gather(self, meta, lengths):
        nb = lengths.numel()
        tmax = int(lengths.max())
        lib = _ext.load()
        dmeta = meta.pin_memory().to(self.device, non_blocking=True)
        x = torch.empty((nb, self.C, tmax), device=self.device)
        u = torch.empty((nb, self.U, tmax), device=self.device)
        st = _ext.stream_ptr(self.device)
        _ext.check(lib.vqhmm_gather_chunks_f32(_ext.ptr(self.xsrc), _ext.ptr(dmeta), nb, self.C, tmax, _ext.ptr(x),
                                               st), "gather_chunks")
        _ext.check(lib.vqhmm_gather_chunks_f32(_ext.ptr(self.usrc), _ext.ptr(dmeta[nb:]), nb, self.U, tmax,
                                               _ext.ptr(u), st), "gather_chunks")
        return x, u, lengths

    def __iter__(self):
        n = len(self.ds)
        for b0 in range(0, n, self.batch_size):
            nb = min(self.batch_size, n - b0)
            if nb < self.batch_size and self.drop_last:
                return
            yield self.gather(*self.plan(nb))
