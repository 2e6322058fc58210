"""Generate the golden fixtures for the VAE_HMM hot path from the REFERENCE.

Run ONLY in the build container (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports /root/reference/VQ_VAE_HMM_fixed.py read-only, runs the reference
modules on CPU on seeded inputs and writes small .npz files next to this
script.  The fixtures are data only (inputs, weights, outputs); no reference
source is copied.  Captured per case:
  inputs x, u, lengths; the 18 weights; logits, q, mu, logvar, log_pi, log_A;
  loss at beta in {0.02, 0.5, 1.0} and the recon/prior/entropy pieces;
  the 18 gradients at beta=1; parameters after 1 and 3 Adam steps (lr=1e-3);
  and the printed lines of train_model on a fixed 2-batch loader.
"""
import contextlib
import io
import math
import os
import random
import sys

import numpy as np
import torch
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
import VQ_VAE_HMM_fixed as R  # noqa: E402  (reference, read-only, this container only)

BETAS = (0.02, 0.5, 1.0)


def pieces(model, x, u, lengths):
    """Recompute the three named loss pieces with the reference modules."""
    B, C, T = x.shape
    mask = torch.arange(T)[None, :] < lengths[:, None]
    log_pi, log_A = model.prior(u)
    logits = model.encoder(x)
    q = F.softmax(logits, dim=1)
    mu, logvar = model.decoder(q)
    var = logvar.exp().clamp(min=1e-8)
    nll = 0.5 * (torch.log(2 * math.pi * var) + (mu - x) ** 2 / var)
    recon = (nll * mask.unsqueeze(1).float()).sum() / (mask.sum() * C).clamp(min=1.0)
    init = (q[:, :, 0] * log_pi.unsqueeze(0)).sum(dim=1)
    qp = q[:, :, :-1].permute(0, 2, 1).unsqueeze(-1)
    qn = q[:, :, 1:].permute(0, 2, 1).unsqueeze(-2)
    tl = (qp * qn * log_A[:, 1:]).sum(dim=(2, 3))
    tl = (tl * (mask[:, 1:] & mask[:, :-1]).float()).sum(dim=1)
    prior = -(init + tl).mean()
    ent = -(q * F.log_softmax(logits, dim=1)).sum(dim=1)
    ent = (ent * mask.float()).sum() / B
    return dict(logits=logits, q=q, mu=mu, logvar=logvar, log_pi=log_pi, log_A=log_A,
                recon=recon, prior=prior, entropy=ent)


def make_case(name, dims, B, T, lengths, seed, weights=None, adam=True, train_lines=True):
    D, H, K, H2, U, TH = dims
    torch.manual_seed(0)
    model = R.VAE_HMM(D, H, K, H2, u_dim=U, trans_hidden=TH)
    if weights is not None:
        model.load_state_dict(torch.load(weights, weights_only=True, map_location="cpu"))
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, D, T, generator=g)
    u = torch.randn(B, U, T, generator=g)
    lengths = torch.tensor(lengths, dtype=torch.long)
    # zero the padded tail like collate_fn does (VQ_VAE_HMM_fixed.py:172-177)
    tmask = (torch.arange(T)[None, :] < lengths[:, None]).float()
    x = x * tmask[:, None, :]
    u = u * tmask[:, None, :]

    out = {"dims": np.array(dims, dtype=np.int64), "x": x.numpy(), "u": u.numpy(),
           "lengths": lengths.numpy(), "torch_version": np.array(torch.__version__)}
    for k, v in model.state_dict().items():
        out["w/" + k] = v.numpy().copy()
    with torch.no_grad():
        pc = pieces(model, x, u, lengths)
        for k in ("logits", "q", "mu", "logvar", "log_pi", "log_A"):
            out["fwd/" + k] = pc[k].numpy()
        for k in ("recon", "prior", "entropy"):
            out["piece/" + k] = np.array(pc[k].item(), dtype=np.float32)
        for b in BETAS:
            out[f"loss/{b}"] = model.compute_loss(x, u, lengths, b).numpy()
        (mu, logvar), qf = model(x)
        out["forward/mu"], out["forward/logvar"], out["forward/q"] = mu.numpy(), logvar.numpy(), qf.numpy()

    model.zero_grad()
    loss = model.compute_loss(x, u, lengths, 1.0)
    loss.backward()
    for k, p in model.named_parameters():
        out["grad/" + k] = p.grad.numpy().copy()

    if adam:
        # Adam steps as train_model does them (VQ_VAE_HMM_fixed.py:146-157), beta=1
        m2 = R.VAE_HMM(D, H, K, H2, u_dim=U, trans_hidden=TH)
        m2.load_state_dict(model.state_dict())
        opt = torch.optim.Adam(m2.parameters(), lr=1e-3)
        losses = []
        for step in range(3):
            opt.zero_grad()
            l = m2.compute_loss(x, u, lengths, 1.0)
            l.backward()
            opt.step()
            losses.append(l.item())
            if step in (0, 2):
                for k, v in m2.state_dict().items():
                    out[f"adam{step+1}/" + k] = v.numpy().copy()
        out["adam/losses"] = np.array(losses, dtype=np.float64)

    if train_lines:
        # train_model on a fixed loader of two half-batches, 3 epochs
        m3 = R.VAE_HMM(D, H, K, H2, u_dim=U, trans_hidden=TH)
        m3.load_state_dict(model.state_dict())
        h = B // 2
        loader = [(x[:h], u[:h], lengths[:h]), (x[h:], u[h:], lengths[h:])]
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            R.train_model(m3, loader, num_epochs=3, lr=1e-3)
        out["train/lines"] = np.array(buf.getvalue().strip().splitlines())
        for k, v in m3.state_dict().items():
            out["train/" + k] = v.numpy().copy()

    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path)/1e3:.1f} kB)")


def make_collate_case():
    """RandomChunkDataset + collate_fn (VQ_VAE_HMM_fixed.py:10-29,164-179) on fixed sequences."""
    g = torch.Generator().manual_seed(99)
    xs = [torch.randn(5, n, generator=g) for n in (230, 180, 260)]
    us = [torch.randn(4, n, generator=g) for n in (230, 180, 260)]
    ds = R.RandomChunkDataset(xs, us, min_len=20, max_len=200)
    random.seed(7)
    items = [ds[i] for i in range(6)]
    x, u, lengths = R.collate_fn(items)
    out = {"lengths": lengths.numpy(), "x": x.numpy(), "u": u.numpy(), "len_ds": np.array(len(ds))}
    for i, (xi, ui, L) in enumerate(items):
        out[f"item{i}/x"], out[f"item{i}/u"], out[f"item{i}/L"] = xi.numpy(), ui.numpy(), np.array(L)
    path = os.path.join(HERE, "collate.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}")


def main():
    torch.set_num_threads(1)
    cfg = (5, 64, 3, 32, 4, 128)
    make_case("cfg1_seeded", cfg, 8, 50, [50, 50, 37, 20, 44, 50, 23, 31], seed=1234)
    make_case("cfg1_trained", cfg, 8, 50, [50, 41, 20, 50, 33, 50, 27, 48], seed=4321,
              weights=os.path.join(REF, "models/vae_hmm.pt"))
    lens = [200] * 8 + [20, 57, 101, 150, 199, 180, 77, 133]
    make_case("cfg2_slice_seeded", cfg, 16, 200, lens, seed=1234, train_lines=False)
    make_case("cfg2_slice_trained", cfg, 16, 200, lens, seed=1234, adam=False, train_lines=False,
              weights=os.path.join(REF, "models/vae_hmm.pt"))
    make_case("k8_d16", (16, 64, 8, 32, 4, 128), 8, 64, [64, 64, 20, 40, 63, 1, 64, 33], seed=77)
    make_case("smoke_tiny", (5, 8, 3, 4, 2, 8), 2, 16, [16, 9], seed=5)
    # large codebook (K=32, K^2 = 1024 transition logits) with channel counts past 64
    make_case("k32_wide", (64, 80, 32, 72, 4, 16), 4, 24, [24, 24, 13, 7], seed=32, train_lines=False)
    make_collate_case()


if __name__ == "__main__":
    main()
