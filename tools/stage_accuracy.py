"""Diagnostic: per-buffer error of the HIP training step's activations and data gradients
against an fp64 torch autograd of the same math (relative to each tensor's norm), to locate
where gradient error enters.  Buffers from vqhmm_elbo_debug_buffers."""
import argparse
import ctypes
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vq-vae-hmm-model_amd")]
import vqhmm  # noqa: E402
from vqhmm import _ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dims", default="16,64,8,32,4,128")
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--T", type=int, default=512)
ap.add_argument("--seed", type=int, default=4096)
a = ap.parse_args()
D, H, K, H2, U, TH = (int(v) for v in a.dims.split(","))
B, T = a.B, a.T
torch.manual_seed(0)
m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=U, trans_hidden=TH)
sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
gen = torch.Generator().manual_seed(a.seed)
x = torch.randn(B, D, T, generator=gen)
u = torch.randn(B, U, T, generator=gen)
L = torch.randint(20, T + 1, (B,), generator=gen)
L[: B // 2] = T


def reference(masks=None, dt=torch.float64):
  """fp64 (or dt) autograd of the step; masks = ReLU patterns to use instead of z > 0."""
  global p, z1, h1, z2, h2, logits, q, y1, g1, y2, g2, par
  relu = (lambda z, i: F.relu(z)) if masks is None else (lambda z, i: z * masks[i].to(z.dtype))
  p = {k: v.detach().cpu().to(dt).requires_grad_(True) for k, v in sd0.items()}
  xd, ud = x.to(dt), u.to(dt)
  z1 = F.conv1d(xd, p["encoder.conv1.weight"], p["encoder.conv1.bias"], padding=1); z1.retain_grad()
  h1 = relu(z1, 0)
  z2 = F.conv1d(h1, p["encoder.conv2.weight"], p["encoder.conv2.bias"], padding=1); z2.retain_grad()
  h2 = relu(z2, 1)
  logits = F.conv1d(h2, p["encoder.to_logits.weight"], p["encoder.to_logits.bias"]); logits.retain_grad()
  q = F.softmax(logits, 1); q.retain_grad()
  emb = torch.matmul(q.transpose(1, 2), p["decoder.embeddings.weight"]).transpose(1, 2)
  y1 = F.conv1d(emb, p["decoder.conv1.weight"], p["decoder.conv1.bias"], padding=1); y1.retain_grad()
  g1 = relu(y1, 2)
  y2 = F.conv1d(g1, p["decoder.conv2.weight"], p["decoder.conv2.bias"], padding=1); y2.retain_grad()
  g2 = relu(y2, 3)
  par = F.conv1d(g2, p["decoder.to_params.weight"], p["decoder.to_params.bias"]); par.retain_grad()
  mu, logvar = par[:, :D], par[:, D:]
  valid = torch.arange(T)[None, :] < L[:, None]
  var = logvar.exp().clamp(min=1e-8)
  nll = 0.5 * (torch.log(2 * math.pi * var) + (mu - xd) ** 2 / var)
  recon = (nll * valid.unsqueeze(1)).sum() / (valid.sum() * D).clamp(min=1.0)
  ut = ud.transpose(1, 2)
  hid = F.relu(F.linear(ut.reshape(B * T, -1), p["prior.transition_net.0.weight"], p["prior.transition_net.0.bias"]))
  log_A = F.log_softmax(F.linear(hid, p["prior.transition_net.2.weight"], p["prior.transition_net.2.bias"]).view(B, T, K, K), -1)
  log_pi = F.log_softmax(p["prior.log_prior"], -1)
  first = (q[:, :, 0] * log_pi[None]).sum(1)
  stp = (q[:, :, :-1].permute(0, 2, 1).unsqueeze(-1) * q[:, :, 1:].permute(0, 2, 1).unsqueeze(-2) * log_A[:, 1:]).sum((2, 3))
  chain = (stp * (valid[:, 1:] & valid[:, :-1])).sum(1)
  prior = -(first + chain).mean()
  ent = (-(q * F.log_softmax(logits, 1)).sum(1) * valid).sum() / B
  loss = recon + (prior - ent)
  loss.backward()

  return {k: v.grad.double().numpy() for k, v in p.items()}, (z1 > 0, z2 > 0, y1 > 0, y2 > 0)


cpu_g, cpu_masks = reference(dt=torch.float32)
ref_g, ref_masks = reference()  # last: the globals hold the fp64 intermediates
mg = m.cuda()
st = vqhmm.TrainState(mg, lr=1e-3)
xs, us, Ls = st.prepare(x, u, L)
st.forward_backward(xs, us, Ls, 1.0)
torch.cuda.synchronize()
ws = st.workspace(B, T)
ptrs = (ctypes.c_void_p * 16)()
_ext.check(_ext.load().vqhmm_elbo_debug_buffers(ctypes.byref(st.dims), B, T, _ext.ptr(ws), ptrs), "debug")
names = ["x", "h1", "h2", "logits", "q", "g1", "g2", "par", "dpar", "dg2", "dg1", "dq_dec", "dlogits", "dh2", "dh1",
         "dq_prior"]
chans = [D, H, H2, K, K, H, H, 2 * D, 2 * D, H, H, K, K, H2, H, K]
base = ws.data_ptr()


def pcl(i):
    c = chans[i]
    ld = (c + 3) // 4 * 4
    off = (ptrs[i] - base)
    t = ws[off: off + B * (T + 2) * ld * 4].view(torch.float32).view(B, T + 2, ld)[:, 1:T + 1, :c]
    return t.permute(0, 2, 1).double().cpu()


ref = {"x": x.double(), "h1": h1, "h2": h2, "logits": logits, "q": q, "g1": g1, "g2": g2, "par": par, "dpar": par.grad,
       "dg2": y2.grad, "dg1": y1.grad, "dlogits": logits.grad, "dh2": z2.grad, "dh1": z1.grad}
for i, n in enumerate(names):
    if n not in ref:
        continue
    r = ref[n].detach()
    g = pcl(i)
    rel = (g - r).norm() / max(r.norm(), 1e-300)
    mx = (g - r).abs().max() / max(r.abs().max(), 1e-300)
    print(f"{n:10s} norm-rel {rel:.2e}  max-rel {mx:.2e}")

# ReLU mask flips vs fp64 (GPU and CPU fp32), then the GPU's gradients against the fp64
# gradient of the GPU forward's own branch (its masks)
gm = [pcl(i) > 0 for i in (1, 2, 5, 6)]
for nm, gmask, cmask, rmask in zip(("h1", "h2", "g1", "g2"), gm, cpu_masks, ref_masks):
    print(f"mask flips {nm}: gpu {int((gmask != rmask).sum())}  cpu-f32 {int((cmask != rmask).sum())}")
br_g, _ = reference(masks=gm)
for i, n in enumerate(vqhmm.PARAM_ORDER):
    gg = st.grad[st.off[i]:st.off[i + 1]].double().cpu().numpy()
    r, rb, c = ref_g[n].reshape(-1), br_g[n].reshape(-1), cpu_g[n].reshape(-1)
    nn_ = max(np.linalg.norm(r), 1e-300)
    print(f"{n:32s} gpu-vs-f64 {np.linalg.norm(gg - r)/nn_:.2e}  gpu-vs-f64(gpu masks) "
          f"{np.linalg.norm(gg - rb)/max(np.linalg.norm(rb),1e-300):.2e}  cpu32-vs-f64 {np.linalg.norm(c - r)/nn_:.2e}")
