"""Pin the CPU oracle (oracle/ref_model.py) to the reference's own outputs.

The fixtures in tests/golden/ were produced by importing the reference in the
build container (tests/golden/make_golden.py).  Forward values and the loss
must be bit-identical; gradients and Adam-updated parameters are compared
with a tight tolerance (the CPU reduction order of conv backward depends on
the thread count; SURVEY.md §0.5 measured 1.9e-6).
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN_CASES, golden_dims, load_golden
from oracle import ref_model as RM


def params_from(g, prefix="w/", grad=False):
    return {k: torch.tensor(g[prefix + k], requires_grad=grad) for k in RM.PARAM_ORDER}


@pytest.fixture(autouse=True)
def _one_thread():
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    yield
    torch.set_num_threads(n)


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_forward_bit_exact(case):
    g = load_golden(case)
    d = golden_dims(g)
    # requires_grad=True like nn.Parameters: torch.matmul picks its kernel
    # (fold-to-mm vs bmm) by requires_grad, which changes fp32 rounding.
    p = params_from(g, grad=True)
    x, u, L = (torch.tensor(g[k]) for k in ("x", "u", "lengths"))
    with torch.no_grad():
        t = RM.elbo_terms(p, x, u, L, d["K"], d["u_dim"])
        for k in ("logits", "q", "mu", "logvar", "log_pi", "log_A"):
            assert np.array_equal(t[k].numpy(), g["fwd/" + k]), k
        for k in ("recon", "prior", "entropy"):
            assert t[k].item() == float(g["piece/" + k]), k
        for beta in (0.02, 0.5, 1.0):
            got = RM.elbo(p, x, u, L, beta, d["K"], d["u_dim"]).numpy()
            assert np.array_equal(got, g[f"loss/{beta}"]), beta


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_grads(case):
    g = load_golden(case)
    d = golden_dims(g)
    p = params_from(g, grad=True)
    x, u, L = (torch.tensor(g[k]) for k in ("x", "u", "lengths"))
    RM.elbo(p, x, u, L, 1.0, d["K"], d["u_dim"]).backward()
    for k in RM.PARAM_ORDER:
        ref = g["grad/" + k]
        got = p[k].grad.numpy()
        scale = max(np.abs(ref).max(), 1e-30)
        assert np.abs(got - ref).max() <= 1e-5 * scale, k


@pytest.mark.parametrize("case", [c for c in GOLDEN_CASES if c != "cfg2_slice_trained"])
def test_adam_steps(case):
    g = load_golden(case)
    d = golden_dims(g)
    p = params_from(g, grad=True)
    x, u, L = (torch.tensor(g[k]) for k in ("x", "u", "lengths"))
    opt = torch.optim.Adam([p[k] for k in RM.PARAM_ORDER], lr=1e-3)
    for step in range(3):
        opt.zero_grad()
        RM.elbo(p, x, u, L, 1.0, d["K"], d["u_dim"]).backward()
        opt.step()
        if step in (0, 2):
            for k in RM.PARAM_ORDER:
                ref = g[f"adam{step+1}/" + k]
                assert np.abs(p[k].detach().numpy() - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max()), k


@pytest.mark.parametrize("case", ["cfg1_seeded", "cfg1_trained", "k8_d16", "smoke_tiny"])
def test_train_lines(case):
    g = load_golden(case)
    d = golden_dims(g)
    p = params_from(g, grad=True)
    x, u, L = (torch.tensor(g[k]) for k in ("x", "u", "lengths"))
    h = x.shape[0] // 2
    batches = [(x[:h], u[:h], L[:h]), (x[h:], u[h:], L[h:])]
    lines = RM.train(p, batches, 3, 1e-3, d["K"], d["u_dim"], log=lambda s: None)
    assert lines == list(g["train/lines"])


def test_pad_batch_matches_collate():
    g = load_golden("collate")
    items = [(torch.tensor(g[f"item{i}/x"]), torch.tensor(g[f"item{i}/u"]), int(g[f"item{i}/L"]))
             for i in range(6)]
    x, u, L = RM.pad_batch(items)
    assert np.array_equal(L.numpy(), g["lengths"])
    assert np.array_equal(x.numpy(), g["x"]) and np.array_equal(u.numpy(), g["u"])
