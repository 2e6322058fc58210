"""Diagnostic: gradient error of the HIP training step and of the fp32 CPU oracle, both
against the oracle run in fp64, at a given config (normwise relative, per tensor)."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vq-vae-hmm-model_amd")]
from oracle import ref_model as RM  # noqa: E402
import vqhmm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dims", default="16,64,8,32,4,128")
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--T", type=int, default=512)
ap.add_argument("--seed", type=int, default=4096)
a = ap.parse_args()
D, H, K, H2, U, TH = (int(v) for v in a.dims.split(","))
torch.manual_seed(0)
m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=U, trans_hidden=TH)
gen = torch.Generator().manual_seed(a.seed)
x = torch.randn(a.B, D, a.T, generator=gen)
u = torch.randn(a.B, U, a.T, generator=gen)
L = torch.randint(20, a.T + 1, (a.B,), generator=gen)
L[: a.B // 2] = a.T
res = {}
for name, dt in (("f32", torch.float32), ("f64", torch.float64)):
    p = {k: v.detach().clone().to(dt).requires_grad_(True) for k, v in m.state_dict().items()}
    loss = RM.elbo(p, x.to(dt), u.to(dt), L, 1.0, K, U)
    loss.backward()
    res[name] = (loss.item(), {k: v.grad.double().numpy() for k, v in p.items()})
mg = m.cuda()
loss = mg.compute_loss(x.cuda(), u.cuda(), L, 1.0)
loss.backward()
gpu = (loss.item(), {k: v.grad.double().cpu().numpy() for k, v in mg.named_parameters()})
ref = res["f64"]
print(f"loss rel err: gpu {abs(gpu[0]-ref[0])/abs(ref[0]):.2e}  cpu-f32 {abs(res['f32'][0]-ref[0])/abs(ref[0]):.2e}")
for k in RM.PARAM_ORDER:
    r = ref[1][k]
    n = max(np.linalg.norm(r), 1e-300)
    eg = np.linalg.norm(gpu[1][k] - r) / n
    ec = np.linalg.norm(res["f32"][1][k] - r) / n
    print(f"{k:34s} gpu {eg:.2e}  cpu-f32 {ec:.2e}  gpu-vs-cpu32 {np.linalg.norm(gpu[1][k]-res['f32'][1][k])/n:.2e}")
