"""Data parallelism for the training step.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
ROCm; "gloo" for CPU tests).  Each rank runs the whole step on its own batch
shard; the only exchange is ONE all-reduce (SUM) of the flat fp32 gradient
(138,596 B at cfg2), whose 1/world scale is folded into the fused Adam kernel.
Adam state is replicated, so every rank applies the same update.

Exactness: the reference normalises recon by the batch's valid count and the
prior/entropy terms by B (VQ_VAE_HMM_fixed.py:120,131,135).  The mean of the
shard gradients equals the global-batch gradient when every shard has the
same size and the same valid count (full-length synthetic chunks: the bench).

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


def train_model_dp(model, dataloader, num_epochs=10, lr=1e-3, group=None):
    """train_model (:145-162) with one RCCL gradient all-reduce per step.

    Every rank iterates its own loader; the printed loss (rank 0) is the mean
    over ranks of the per-rank epoch averages (one scalar all-reduce per epoch).
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
            state.step(x, u, lengths, beta)
        tot = state.epoch_acc / len(dataloader)
        torch.distributed.all_reduce(tot, group=group)
        if rank == 0:
            print(f"Epoch {ep+1}/{num_epochs}, Loss: {tot.item() / world:.4f}")
    state.publish_grads()
    return model
