"""Batch producer of the training path (VQ_VAE_HMM_fixed.py:10-29, 164-179).

RandomChunkDataset keeps the reference's semantics exactly: __len__ is 1000,
__getitem__ ignores idx and draws (sequence, chunk length, start) from
Python's global `random` in the same order.  collate_fn zero-pads to the
batch maximum and returns (x, u, lengths) with lengths int64 on the CPU like
the reference; it pads on the host and moves each batch to the device with
one copy per tensor instead of the reference's B small device writes.
"""
import random

import torch


class RandomChunkDataset:
    def __init__(self, x_sequences, u_sequences, min_len=20, max_len=200):
        self.x_seqs = x_sequences
        self.u_seqs = u_sequences
        self.min_len = min_len
        self.max_len = max_len

    def __len__(self):
        return 1000

    def __getitem__(self, idx):
        k = random.randint(0, len(self.x_seqs) - 1)
        xs, us = self.x_seqs[k], self.u_seqs[k]
        n = xs.shape[1]
        L = random.randint(self.min_len, min(self.max_len, n))
        s = random.randint(0, n - L)
        return xs[:, s:s + L], us[:, s:s + L], L


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
