"""Data step timing at cfg2's batch (B=1024, chunks U[20, 200]): the reference's
per-sample loop (RandomChunkDataset.__getitem__ x B + collate_fn + device copy) vs
DeviceChunkLoader (host draws + one HIP gather per tensor).  One JSON line."""
import json
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vq-vae-hmm-model_amd"))
from vqhmm.data import DeviceChunkLoader, RandomChunkDataset, collate_fn  # noqa: E402


def main(B=1024, nb=20):
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(5, 4000, generator=g) for _ in range(16)]
    us = [torch.randn(4, 4000, generator=g) for _ in range(16)]
    ds = RandomChunkDataset(xs, us, 20, 200)
    ld = DeviceChunkLoader(ds, B, device="cuda")
    random.seed(0)
    for _ in range(2):
        ld.gather(*ld.plan(B))
        x, u, L = collate_fn([ds[i] for i in range(B)], device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(nb):
        x, u, L = collate_fn([ds[i] for i in range(B)], device="cuda")
    torch.cuda.synchronize()
    host = (time.perf_counter() - t0) / nb
    t0 = time.perf_counter()
    for _ in range(nb):
        x, u, L = ld.gather(*ld.plan(B))
    torch.cuda.synchronize()
    dev = (time.perf_counter() - t0) / nb
    t0 = time.perf_counter()
    for _ in range(nb):
        ld.plan(B)
    draws = (time.perf_counter() - t0) / nb
    print(json.dumps({"batch": B, "host_collate_ms": round(host * 1e3, 3), "device_loader_ms": round(dev * 1e3, 3),
                      "of_which_host_draws_ms": round(draws * 1e3, 3), "speedup": round(host / dev, 1)}))


if __name__ == "__main__":
    main()
