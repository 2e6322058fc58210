"""Functional torch-CPU restatement of the reference VAE_HMM training path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the product never imports it.

Every function takes an explicit parameter dict keyed by the reference's
state_dict names, runs on CPU in fp32 with the same ATen primitives the
reference's nn.Modules dispatch to, and so reproduces the reference values
bit-for-bit (pinned by tests/test_oracle_golden.py against fixtures captured
from /root/reference in this container).

Reference citations (VQ_VAE_HMM_fixed.py):
  encoder_logits   Encoder.forward             :38-41
  prior_tables     Prior.forward               :59-71
  decoder_params   Decoder.forward             :81-90
  elbo             VAE_HMM.compute_loss        :106-137
  train            train_model                 :145-162
  pad_batch        collate_fn                  :164-179
"""
import math

import torch
import torch.nn.functional as F

# Registration order of nn.Module.parameters() in the reference
# (VQ_VAE_HMM_fixed.py:92-98 builds encoder, prior, decoder in that order).
PARAM_ORDER = (
    "encoder.conv1.weight", "encoder.conv1.bias",
    "encoder.conv2.weight", "encoder.conv2.bias",
    "encoder.to_logits.weight", "encoder.to_logits.bias",
    "prior.log_prior",
    "prior.transition_net.0.weight", "prior.transition_net.0.bias",
    "prior.transition_net.2.weight", "prior.transition_net.2.bias",
    "decoder.embeddings.weight",
    "decoder.conv1.weight", "decoder.conv1.bias",
    "decoder.conv2.weight", "decoder.conv2.bias",
    "decoder.to_params.weight", "decoder.to_params.bias",
)


def param_shapes(input_dim, hidden_dim, K, hidden_dim2, u_dim, trans_hidden=128):
    """Shapes of the 18 tensors, as the reference constructors create them."""
    D, H, H2, U, TH = input_dim, hidden_dim, hidden_dim2, u_dim, trans_hidden
    return {
        "encoder.conv1.weight": (H, D, 3), "encoder.conv1.bias": (H,),
        "encoder.conv2.weight": (H2, H, 3), "encoder.conv2.bias": (H2,),
        "encoder.to_logits.weight": (K, H2, 1), "encoder.to_logits.bias": (K,),
        "prior.log_prior": (K,),
        "prior.transition_net.0.weight": (TH, U), "prior.transition_net.0.bias": (TH,),
        "prior.transition_net.2.weight": (K * K, TH), "prior.transition_net.2.bias": (K * K,),
        "decoder.embeddings.weight": (K, H),
        "decoder.conv1.weight": (H, H, 3), "decoder.conv1.bias": (H,),
        "decoder.conv2.weight": (H, H, 3), "decoder.conv2.bias": (H,),
        "decoder.to_params.weight": (2 * D, H, 1), "decoder.to_params.bias": (2 * D,),
    }


def _relu(z, mask=None):
    """F.relu, or — with `mask` — the same piecewise-linear branch fixed by a given
    pattern (z * mask): the gradient of a forward whose ReLU decisions are `mask`."""
    return F.relu(z) if mask is None else z * mask.to(z.dtype)


def encoder_logits(p, x, masks=None):
    """(B,D,T) -> logits (B,K,T).  Reference: Encoder.forward :38-41.
    masks: None, or the ReLU patterns (h1, h2, ...) to use (see _relu)."""
    m = masks or (None, None)
    a = _relu(F.conv1d(x, p["encoder.conv1.weight"], p["encoder.conv1.bias"], padding=1), m[0])
    a = _relu(F.conv1d(a, p["encoder.conv2.weight"], p["encoder.conv2.bias"], padding=1), m[1])
    return F.conv1d(a, p["encoder.to_logits.weight"], p["encoder.to_logits.bias"])


def prior_tables(p, u, K, u_dim):
    """u -> (log_pi (K,), log_A (B,T,K,K)).  Reference: Prior.forward :59-71.

    The reference treats a 3-D u whose dim 1 equals u_dim as channels-first
    (B,U,T) and permutes it (:64-65); any other 3-D u is taken as (B,T,U).
    """
    if u is None:
        raise ValueError("u required for non-stationary transitions")
    if u.dim() == 3 and u.shape[1] == u_dim:
        u = u.transpose(1, 2)
    nb, nt, _ = u.shape
    hid = F.relu(F.linear(u.reshape(nb * nt, -1),
                          p["prior.transition_net.0.weight"], p["prior.transition_net.0.bias"]))
    trans_logits = F.linear(hid, p["prior.transition_net.2.weight"], p["prior.transition_net.2.bias"])
    log_A = F.log_softmax(trans_logits.view(nb, nt, K, K), dim=-1)
    return F.log_softmax(p["prior.log_prior"], dim=-1), log_A


def decoder_params(p, q, masks=None):
    """q (B,K,T) -> (mu, logvar) each (B,D,T).  Reference: Decoder.forward :81-90.
    masks: None, or the ReLU patterns (g1, g2) to use (see _relu)."""
    m = masks or (None, None)
    emb = torch.matmul(q.transpose(1, 2), p["decoder.embeddings.weight"]).transpose(1, 2)
    a = _relu(F.conv1d(emb, p["decoder.conv1.weight"], p["decoder.conv1.bias"], padding=1), m[0])
    a = _relu(F.conv1d(a, p["decoder.conv2.weight"], p["decoder.conv2.bias"], padding=1), m[1])
    out = F.conv1d(a, p["decoder.to_params.weight"], p["decoder.to_params.bias"])
    half = out.shape[1] // 2
    return out[:, :half, :], out[:, half:, :]


def preactivations(p, x):
    """The four conv pre-activations whose sign is a ReLU decision, on this oracle's own
    branch: encoder conv1 / conv2 (:39-40) and decoder conv1 / conv2 (:85-86), each (B, C, T).
    Test infrastructure: bounds how far a device forward's ReLU patterns may differ from the
    oracle's (tests/test_gpu_configs.py)."""
    with torch.no_grad():
        z1 = F.conv1d(x, p["encoder.conv1.weight"], p["encoder.conv1.bias"], padding=1)
        z2 = F.conv1d(F.relu(z1), p["encoder.conv2.weight"], p["encoder.conv2.bias"], padding=1)
        logits = F.conv1d(F.relu(z2), p["encoder.to_logits.weight"], p["encoder.to_logits.bias"])
        q = F.softmax(logits, dim=1)
        emb = torch.matmul(q.transpose(1, 2), p["decoder.embeddings.weight"]).transpose(1, 2)
        y1 = F.conv1d(emb, p["decoder.conv1.weight"], p["decoder.conv1.bias"], padding=1)
        y2 = F.conv1d(F.relu(y1), p["decoder.conv2.weight"], p["decoder.conv2.bias"], padding=1)
    return z1, z2, y1, y2


def elbo_terms(p, x, u, lengths, K, u_dim, norm=None, relu_masks=None):
    """Returns the named pieces of the mean-field ELBO (reference :106-135).

    norm=(valid_count, batch) replaces the batch's own normalisers mask.sum()
    (:120) and B (:131 .mean(), :135) by a global batch's (data-parallel shard
    of it; the product's `norm` argument, include/vqhmm.h).  None = reference.
    relu_masks=(h1, h2, g1, g2) fixes the four conv ReLU decisions (see _relu):
    run in fp64 with a device forward's own patterns, this is the exact gradient of
    the branch that forward took, free of the fp32 ReLU-boundary flips that make two
    correct fp32 computations differ by ~1e-5 (tests/test_gpu_configs.py)."""
    nb, nc, nt = x.shape
    if lengths is None:
        raise ValueError("lengths required")
    valid = torch.arange(nt, device=x.device)[None, :] < lengths[:, None].to(x.device)
    log_pi, log_A = prior_tables(p, u, K, u_dim)
    rm = relu_masks or (None, None, None, None)
    logits = encoder_logits(p, x, rm[0:2])
    q = F.softmax(logits, dim=1)
    mu, logvar = decoder_params(p, q, rm[2:4])

    var = logvar.exp().clamp(min=1e-8)
    nll = 0.5 * (torch.log(2 * math.pi * var) + (mu - x) ** 2 / var)
    if norm is None:
        recon = (nll * valid.unsqueeze(1).float()).sum() / (valid.sum() * nc).clamp(min=1.0)
    else:
        recon = (nll * valid.unsqueeze(1).float()).sum() / max(float(norm[0]) * nc, 1.0)

    first = (q[:, :, 0] * log_pi.unsqueeze(0)).sum(dim=1)
    q_from = q[:, :, :-1].permute(0, 2, 1).unsqueeze(-1)
    q_to = q[:, :, 1:].permute(0, 2, 1).unsqueeze(-2)
    step = (q_from * q_to * log_A[:, 1:]).sum(dim=(2, 3))
    pair_valid = (valid[:, 1:] & valid[:, :-1]).float()
    chain = (step * pair_valid).sum(dim=1)
    prior_loss = -(first + chain).mean() if norm is None else -(first + chain).sum() / float(norm[1])

    ent = -(q * F.log_softmax(logits, dim=1)).sum(dim=1)
    ent = (ent * valid.float()).sum() / (nb if norm is None else float(norm[1]))
    return dict(recon=recon, prior=prior_loss, entropy=ent, logits=logits, q=q,
                mu=mu, logvar=logvar, log_pi=log_pi, log_A=log_A)


def elbo(p, x, u, lengths, beta, K, u_dim, norm=None, relu_masks=None):
    """Scalar loss = recon + beta*(prior - entropy).  Reference :137."""
    t = elbo_terms(p, x, u, lengths, K, u_dim, norm, relu_masks)
    return t["recon"] + beta * (t["prior"] - t["entropy"])


def pad_batch(items, device="cpu"):
    """List of (x (C,L), u (U,L), L) -> zero-padded (x, u, lengths).  Reference :164-179."""
    lens = torch.tensor([it[2] for it in items], dtype=torch.long)
    tmax = int(lens.max().item())
    nb, nc, nu = len(items), items[0][0].shape[0], items[0][1].shape[0]
    xb = torch.zeros(nb, nc, tmax, device=device)
    ub = torch.zeros(nb, nu, tmax, device=device)
    for i, (xs, us, n) in enumerate(items):
        xb[i, :, :n] = xs
        ub[i, :, :n] = us
    return xb, ub, lens


def train(p, batches, num_epochs, lr, K, u_dim, log=print):
    """Adam loop of train_model (reference :145-162) over a list of batches.

    `p` is updated in place (tensors must be leaf tensors with requires_grad).
    Returns the list of printed epoch lines.
    """
    params = [p[n] for n in PARAM_ORDER]
    opt = torch.optim.Adam(params, lr=lr)
    lines = []
    for ep in range(num_epochs):
        total = 0
        beta = min(1.0, 2.0 * (ep + 1) / num_epochs)
        for xb, ub, lb in batches:
            opt.zero_grad()
            loss = elbo(p, xb, ub, lb, beta, K, u_dim)
            loss.backward()
            opt.step()
            total += loss.item()
        line = f"Epoch {ep+1}/{num_epochs}, Loss: {total/len(batches):.4f}"
        log(line)
        lines.append(line)
    return lines
