"""Data parallelism for the training step.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
ROCm; "gloo" for CPU tests).  Each rank runs the whole step on its own batch
shard; the only exchange is ONE all-reduce (SUM) of the flat fp32 gradient
(138,596 B at cfg2), whose 1/world scale is folded into the fused Adam kernel.
Adam state is replicated, so every rank applies the same update.

Exactness: the reference normalises recon by the batch's valid count and the
prior/entropy terms by B (VQ_VAE_HMM_fixed.py:120,131,135).  Two modes:
  * local normalisers (default, the bench): each shard is normalised by its own
    count and B and Adam averages the summed gradient (1/world).  That equals the
    global-batch gradient when every shard has the same size and valid count
    (full-length synthetic chunks).
  * global normalisers (`global_norm`, ragged batches): each shard is normalised
    by the GLOBAL valid count and B ({count, B}, a device int64[2] handed to the
    kernels), so the shards' losses and gradients SUM to exactly the global
    batch's and Adam takes the sum (scale 1).  Shards must also share the global
    batch's padded length T: the reference's convs see the zero padding past a
    sequence's end (x = 0 but relu(bias) != 0 after the first conv), so a shard
    padded to a shorter T would differ at the longest sequence's last steps.
    `shard_batch` of a collated global batch keeps T; independently sampled
    per-rank batches are padded to the max T over ranks (`pad_to_common_T`).

RandomChunkDataset.__getitem__ ignores idx and draws from Python's global
`random` (:20-27), so index partitioning is meaningless; ranks instead sample
with a rank-specific seed (`seed_rank_sampling`).
"""
import os
import random

import torch


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env (MASTER_ADDR defaults to 127.0.0.1)."""
    if torch.distributed.is_initialized():
        return torch.distributed.get_rank(), torch.distributed.get_world_size()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
    torch.distributed.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world


def seed_rank_sampling(base_seed, rank):
    """Per-rank stream of RandomChunkDataset draws (the dataset ignores indices)."""
    random.seed(base_seed + 1000003 * rank)


def allreduce_sum_(flat, group=None):
    """In-place SUM all-reduce of one flat gradient buffer (a single collective per step)."""
    if torch.distributed.is_initialized() and torch.distributed.get_world_size(group) > 1:
        torch.distributed.all_reduce(flat, op=torch.distributed.ReduceOp.SUM, group=group)
    return flat


def shard_batch(x, u, lengths, rank, world):
    """Contiguous per-rank slice [r*B/n, (r+1)*B/n) of a global batch (equal shards)."""
    B = x.shape[0]
    if B % world:
        raise ValueError(f"global batch {B} is not divisible by world size {world}")
    s = slice(rank * (B // world), (rank + 1) * (B // world))
    return x[s], u[s], lengths[s]


def global_norm(lengths, T, group=None, reduce=True):
    """Loss normalisers {valid_count, batch} (device int64[2]) of the global batch.

    lengths: this rank's lengths (reduce=True: summed over ranks with one tiny
    all-reduce, no host sync) or the whole global batch's (reduce=False, e.g.
    every rank holds the collated global batch and trains on `shard_batch` of it).
    valid_count = sum_b min(max(L_b, 0), T) = mask.sum() (VQ_VAE_HMM_fixed.py:113,120)."""
    L = torch.as_tensor(lengths).to(torch.int64)
    n = torch.stack([L.clamp(0, int(T)).sum(), torch.tensor(L.numel(), dtype=torch.int64, device=L.device)])
    if reduce and torch.distributed.is_initialized() and torch.distributed.get_world_size(group) > 1:
        torch.distributed.all_reduce(n, op=torch.distributed.ReduceOp.SUM, group=group)
    return n


def pad_to_common_T(x, u, group=None):
    """Zero-pad (B, C, T) x and u on the time axis to the max T over ranks (collate_fn's padding, :171-177)."""
    T = torch.tensor([x.shape[-1]], dtype=torch.int64, device=x.device)
    if torch.distributed.is_initialized() and torch.distributed.get_world_size(group) > 1:
        torch.distributed.all_reduce(T, op=torch.distributed.ReduceOp.MAX, group=group)
    Tg = int(T.item())
    if Tg != x.shape[-1]:
        x = torch.nn.functional.pad(x, (0, Tg - x.shape[-1]))
    if Tg != u.shape[-1]:
        u = torch.nn.functional.pad(u, (0, Tg - u.shape[-1]))
    return x, u, Tg


def train_model_dp(model, dataloader, num_epochs=10, lr=1e-3, group=None, exact=True):
    """train_model (:145-162) with one RCCL gradient all-reduce per step.

    Every rank iterates its own loader.  exact=True (default): the ranks' batches
    form one global batch (padded to a common T, normalised by its global count
    and size), so each update is the reference's update on that union batch and
    the printed loss (rank 0) is the union batch's loss averaged over the epoch.
    exact=False: local normalisers, mean of the per-rank losses.  One scalar
    all-reduce per epoch for the print.
    """
    from .train import TrainState
    state = TrainState(model, lr=lr, process_group=group, distributed=True)
    world = state.world
    rank = torch.distributed.get_rank(group)
    model.train()
    for ep in range(num_epochs):
        state.epoch_acc.zero_()
        beta = min(1.0, 2.0 * (ep + 1) / num_epochs)
        for x, u, lengths in dataloader:
            norm = None
            if exact:
                x, u, lengths = state.prepare(x, u, lengths)
                x, u, T = pad_to_common_T(x, u, group)
                norm = global_norm(lengths, T, group)
            state.step(x, u, lengths, beta, norm)
        tot = state.epoch_acc / len(dataloader)
        torch.distributed.all_reduce(tot, group=group)
        if rank == 0:
            print(f"Epoch {ep+1}/{num_epochs}, Loss: {tot.item() / (1 if exact else world):.4f}")
    state.publish_grads()
    return model
