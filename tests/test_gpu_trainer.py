"""GPU parity of the clip-norm training loop (the reference's Trainer,
src/training/trainer.py:9-47): the native clip_grad_norm_ kernel against
torch.nn.utils.clip_grad_norm_, and vqhmm.Trainer against the CPU oracle running
compute_loss + backward + clip_grad_norm_(1.0) + Adam on the same batches.

Tolerances: clipped gradient and total norm 1e-6 relative (double-accumulated
norm vs torch's fp32 one); trained parameters as test_gpu_model's train_model
check (1e-4 of the tensor scale + 1e-6), epoch loss 1e-4.
"""
import contextlib
import io

import numpy as np
import pytest
import torch

from conftest import golden_dims, load_golden
from oracle import ref_model as RM

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scale, pre", [(1.0, 1.0), (1e-3, 1.0), (3.0, 0.5)])
def test_clip_grad_norm_matches_torch(scale, pre):
    import vqhmm
    from vqhmm import _ext
    m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128)
    shapes = [p.shape for p in m.ordered_parameters()]
    n = sum(int(np.prod(s)) for s in shapes)
    gen = torch.Generator().manual_seed(7)
    flat = torch.randn(n, generator=gen) * scale * 0.01
    ref = [t.clone().reshape(s) for t, s in zip(torch.split(flat * pre, [int(np.prod(s)) for s in shapes]), shapes)]
    params = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
    for p, r in zip(params, ref):
        p.grad = r
    tn_ref = torch.nn.utils.clip_grad_norm_(params, 1.0)
    ref_flat = torch.cat([p.grad.reshape(-1) for p in params])
    g = flat.cuda()
    tn = torch.zeros((), device="cuda")
    lib = _ext.load()
    _ext.check(lib.vqhmm_clip_grad_norm_f32(_ext.ptr(g), n, pre, 1.0, _ext.ptr(tn), _ext.stream_ptr()), "clip")
    torch.cuda.synchronize()
    assert abs(tn.item() - tn_ref.item()) <= 1e-6 * tn_ref.item()
    err = (g.cpu() - ref_flat).abs().max().item()
    assert err <= 1e-6 * ref_flat.abs().max().item()


def test_trainer_matches_oracle_clip_loop():
    import vqhmm
    g = load_golden("cfg1_seeded")
    d = golden_dims(g)
    w0 = {k[2:]: torch.tensor(v) for k, v in g.items() if k.startswith("w/")}
    x, u, L = torch.tensor(g["x"]), torch.tensor(g["u"]), torch.tensor(g["lengths"])
    h = x.shape[0] // 2
    loader = [(x[:h], u[:h], L[:h]), (x[h:], u[h:], L[h:])]
    epochs = 3

    # oracle: Trainer.train with compute_loss -> backward -> clip_grad_norm_(1.0) -> Adam.step
    p = {k: w0[k].clone().requires_grad_(True) for k in RM.PARAM_ORDER}
    plist = [p[k] for k in RM.PARAM_ORDER]
    opt = torch.optim.Adam(plist, lr=1e-3)
    ref_lines = []
    for ep in range(epochs):
        beta = min(1.0, 2.0 * (ep + 1) / epochs)
        tot = 0.0
        for xb, ub, Lb in loader:
            opt.zero_grad()
            loss = RM.elbo(p, xb, ub, Lb, beta, d["K"], d["u_dim"])
            loss.backward()
            torch.nn.utils.clip_grad_norm_(plist, 1.0)
            opt.step()
            tot += loss.item()
        ref_lines.append((ep, tot / len(loader), beta))

    m = vqhmm.VAE_HMM(d["input_dim"], d["hidden_dim"], d["K"], d["hidden_dim2"], u_dim=d["u_dim"],
                      trans_hidden=d["trans_hidden"])
    m.load_state_dict(w0)
    tr = vqhmm.Trainer(m, lr=1e-3, device="cuda")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(io.StringIO()):
        tr.train(loader, num_epochs=epochs)
    lines = [ln for ln in buf.getvalue().strip().splitlines() if ln.startswith("Epoch")]
    assert len(lines) == epochs
    for ln, (ep, ref_loss, beta) in zip(lines, ref_lines):
        assert ln.startswith(f"Epoch {ep+1}/{epochs}, Loss: ") and ln.endswith(f", Beta: {beta:.2f}"), ln
        got = float(ln.split("Loss:")[1].split(",")[0])
        assert abs(got - ref_loss) <= 1e-4 * max(1.0, abs(ref_loss)) + 1e-4, (ln, ref_loss)
    sd = m.state_dict()
    for k in RM.PARAM_ORDER:
        ref = p[k].detach().numpy().astype(np.float64)
        got = sd[k].cpu().numpy().astype(np.float64)
        assert np.abs(got - ref).max() <= 1e-4 * max(np.abs(ref).max(), 1e-30) + 1e-6, k


def test_trainer_custom_loss_fn_matches_default():
    """Trainer.train_epoch(loss_fn=...) (autograd path, native clip + Adam) equals the default path."""
    import vqhmm
    g = load_golden("cfg1_seeded")
    d = golden_dims(g)
    w0 = {k[2:]: torch.tensor(v) for k, v in g.items() if k.startswith("w/")}
    x, u, L = torch.tensor(g["x"]), torch.tensor(g["u"]), torch.tensor(g["lengths"])
    loader = [(x, u, L)] * 2
    out = []
    for fn in (None, lambda mod, xb, ub, Lb: mod.compute_loss(xb, ub, Lb, 0.5)):
        m = vqhmm.VAE_HMM(d["input_dim"], d["hidden_dim"], d["K"], d["hidden_dim2"], u_dim=d["u_dim"],
                          trans_hidden=d["trans_hidden"])
        m.load_state_dict(w0)
        tr = vqhmm.Trainer(m, lr=1e-3, device="cuda")
        with contextlib.redirect_stderr(io.StringIO()):
            loss = tr.train_epoch(loader, loss_fn=fn, beta=0.5)
        out.append((loss, {k: v.cpu().clone() for k, v in m.state_dict().items()}))
    assert abs(out[0][0] - out[1][0]) <= 1e-5 * abs(out[0][0])
    for k in RM.PARAM_ORDER:
        a, b = out[0][1][k], out[1][1][k]
        assert (a - b).abs().max().item() <= 1e-4 * max(b.abs().max().item(), 1e-30) + 1e-6, k


@pytest.mark.parametrize("B,K,D,H,H2,T", [(128, 3, 5, 64, 32, 200), (1024, 3, 5, 64, 32, 200),
                                          (64, 8, 16, 64, 32, 96), (40, 32, 64, 80, 72, 50),
                                          (24, 32, 64, 256, 128, 60)])  # cfg3 dims: thousands of tail blocks
def test_fused_tail_adam_bit_identical(B, K, D, H, H2, T):
    """The single-process step's backward tail in one launch (tail_adam_kernel: slab reduction +
    composed dW / dE + Adam, with the in-launch wait for the dWc segment) against the split path
    (grad_tail, compose_bwd, adam_kernel): identical gradients, moments and parameters, 4 steps."""
    import vqhmm
    gen = torch.Generator().manual_seed(B + K)
    x = torch.randn(B, D, T, generator=gen).cuda()
    u = torch.randn(B, 4, T, generator=gen).cuda()
    L = torch.randint(max(1, T // 4), T + 1, (B,), generator=gen)
    st = []
    for _ in range(2):
        torch.manual_seed(3)
        m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=4, trans_hidden=64).cuda()
        st.append(vqhmm.TrainState(m, lr=1e-3))
    fused, split = st
    xs, us, Ls = fused.prepare(x, u, L)
    for _ in range(4):
        fused.forward_backward_adam(xs, us, Ls, 0.7)
        split.forward_backward(xs, us, Ls, 0.7)
        split.apply_adam()
    torch.cuda.synchronize()
    assert torch.equal(fused.grad, split.grad)
    assert torch.equal(fused.exp_avg, split.exp_avg) and torch.equal(fused.exp_avg_sq, split.exp_avg_sq)
    assert torch.equal(fused.flat, split.flat)
    assert int(fused.step_dev.item()) == int(split.step_dev.item()) == 4


_SPLIT_RUN = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
import vqhmm
D, H, K, H2 = (int(v) for v in sys.argv[3].split(","))
B, T = (int(v) for v in sys.argv[4].split(",")) if len(sys.argv) > 4 else (96, 150)
gen = torch.Generator().manual_seed(5)
x = torch.randn(B, D, T, generator=gen).cuda()
u = torch.randn(B, 4, T, generator=gen).cuda()
L = torch.randint(30, T + 1, (B,), generator=gen)
torch.manual_seed(3)
m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=4, trans_hidden=128).cuda()
st = vqhmm.TrainState(m, lr=1e-3)
xs, us, Ls = st.prepare(x, u, L)
for _ in range(2):
    st.forward_backward(xs, us, Ls, 0.5)
    st.apply_adam()
for _ in range(2):
    st.forward_backward_adam(xs, us, Ls, 0.5)
torch.cuda.synchronize()
torch.save({"grad": st.grad.cpu(), "flat": st.flat.cpu(), "m": st.exp_avg.cpu(), "v": st.exp_avg_sq.cpu(),
            "loss": st.loss.cpu()}, sys.argv[2])
"""


def _run_both(tmp_path, env, dims, bt=(96, 150), extra=None):
    """The same 4 steps in two fresh processes, env=1 and env=0 (the switches are read once per
    process); loss, gradient, moments and parameters must agree bit for bit."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    pkg = os.path.join(ROOT, "vq-vae-hmm-model_amd")
    out = {}
    for flag in ("1", "0"):
        f = str(tmp_path / f"{env}{flag}.pt")
        subprocess.run([sys.executable, "-c", _SPLIT_RUN, pkg, f, ",".join(map(str, dims)), ",".join(map(str, bt))],
                       check=True,
                       timeout=300, env=dict(os.environ, **{env: flag}, **(extra or {})))
        out[flag] = torch.load(f, weights_only=True)
    for k in ("grad", "flat", "m", "v", "loss"):
        assert torch.equal(out["1"][k], out["0"][k]), k


def test_fused_tail_matches_separate_launches(tmp_path):
    """The one-launch backward tail (tail_kernel, both the DP form and the Adam-fused form) gives
    the same bits as grad_tail + compose_bwd / compose_adam as separate launches (VQHMM_TAIL_FUSED=0)."""
    _run_both(tmp_path, "VQHMM_TAIL_FUSED", (5, 64, 3, 32))


@pytest.mark.parametrize("dims", [(5, 64, 3, 32), (16, 64, 8, 32), (5, 48, 4, 40)])
def test_fused_conv_pairs_match_separate_launches(tmp_path, dims):
    """enc_conv1 -> enc_conv2 and dec_conv1 -> dec_conv2 fused into one launch each (conv2f_kernel:
    14-row tiles, the front rows computed in-tile) against the two-launch path (VQHMM_CONV_FUSE=0)."""
    _run_both(tmp_path, "VQHMM_CONV_FUSE", dims)


@pytest.mark.parametrize("dims,bt", [((5, 64, 3, 32), (96, 150)), ((4, 64, 4, 16), (40, 77)), ((3, 64, 2, 32), (8, 50)),
                                     ((5, 64, 3, 32), (256, 150))])  # 319 strips: workgroups run 2
def test_strip_forward_matches_pair_launches(tmp_path, dims, bt):
    """The four forward convolutions as ONE strip launch (strip.hip: 128-row windows, 3 recomputed
    halo rows a side, activations in LDS) against the pair launches (VQHMM_STRIP=0): same bits (the head
    as its own launch in both: fused, its slab sums run in another order, test_strip_head_*)."""
    _run_both(tmp_path, "VQHMM_STRIP", dims, bt, {"VQHMM_STRIP_HEAD": "0"})


@pytest.mark.parametrize("dims,bt", [((5, 64, 3, 32), (96, 150)), ((8, 64, 2, 30), (40, 77)), ((5, 64, 4, 31), (8, 50)),
                                     ((5, 64, 3, 32), (256, 150))])
def test_strip_backward_matches_pair_launches(tmp_path, dims, bt):
    """The backward's data-gradient convolutions (to_params -> dec_conv2 -> dec_conv1 + softmax backward
    + to_logits -> enc_conv2) as ONE strip launch against the pair launches (VQHMM_STRIP_BWD=0): same bits
    (the weight gradients as the grouped launch in both: folded into the strip they sum in another order,
    test_strip_wgrad_fold_*)."""
    _run_both(tmp_path, "VQHMM_STRIP_BWD", dims, bt, {"VQHMM_STRIP_WGRAD": "0"})


_HEAD_RUN = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
import vqhmm
D, H, K, H2, TH = (int(v) for v in sys.argv[3].split(","))
B, T = (int(v) for v in sys.argv[4].split(","))
gen = torch.Generator().manual_seed(7)
x = torch.randn(B, D, T, generator=gen).cuda()
u = torch.randn(B, 4, T, generator=gen).cuda()
L = torch.randint(max(1, T // 3), T + 1, (B,), generator=gen)
torch.manual_seed(3)
m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=4, trans_hidden=TH).cuda()
st = vqhmm.TrainState(m, lr=1e-3)
xs, us, Ls = st.prepare(x, u, L)
out = {}
for i in range(2):
    st.forward_backward(xs, us, Ls, 0.5)
    torch.cuda.synchronize()
    out["loss%d" % i] = st.loss.detach().cpu().clone()
    out["grad%d" % i] = st.grad.detach().cpu().clone()
    st.apply_adam()
loss = m.compute_loss(x, u, L, 0.5)  # the module path: forward with need_grad = 1 and backward
loss.backward()
out["mloss"] = loss.detach().cpu()
out["mgrad"] = torch.cat([p.grad.detach().flatten() for p in m.parameters()]).cpu()
torch.save(out, sys.argv[2])
"""


def _run_both_tol(tmp_path, env, dims, bt):
    """_HEAD_RUN in two fresh processes, env=1 and env=0: losses within 1e-6 relative, gradients within
    1e-6 normwise (the two forms differ only in a summation order)."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    pkg = os.path.join(ROOT, "vq-vae-hmm-model_amd")
    out = {}
    for flag in ("1", "0"):
        f = str(tmp_path / f"h{flag}.pt")
        subprocess.run([sys.executable, "-c", _HEAD_RUN, pkg, f, ",".join(map(str, dims)), ",".join(map(str, bt))],
                       check=True, timeout=300, env=dict(os.environ, **{env: flag}))
        out[flag] = torch.load(f, weights_only=True)
    for k in ("loss0", "loss1", "mloss"):
        a, b = out["1"][k].double(), out["0"][k].double()
        assert torch.allclose(a, b, rtol=1e-6, atol=0), (k, a, b)
    for k in ("grad0", "grad1", "mgrad"):
        a, b = out["1"][k].double(), out["0"][k].double()
        assert (a - b).norm() <= 1e-6 * b.norm(), (k, ((a - b).norm() / b.norm()).item())
    return out


@pytest.mark.parametrize("dims,bt", [((5, 64, 3, 32, 128), (96, 150)), ((4, 64, 2, 16, 64), (40, 77)),
                                     ((5, 64, 4, 32, 128), (256, 150))])
def test_strip_head_matches_head_launch(tmp_path, dims, bt):
    """The ELBO head fused into the forward strip launch (VQHMM_STRIP_HEAD=1, an A/B switch; its slabs / loss
    partials per strip workgroup) against the head's own launch: per-row outputs feed the same backward, the
    loss and the gradient differ only in the slab / partial summation order (1e-6 relative)."""
    _run_both_tol(tmp_path, "VQHMM_STRIP_HEAD", dims, bt)


@pytest.mark.parametrize("dims,bt", [((5, 64, 3, 32, 128), (96, 150)), ((3, 64, 2, 32, 64), (40, 77)),
                                     ((5, 64, 4, 31, 128), (8, 50)), ((4, 64, 3, 29, 128), (30, 200)),
                                     ((5, 64, 3, 32, 128), (128, 200)),   # the cfg2 N = 8 shard: 249 strips of 104
                                     ((5, 64, 3, 32, 128), (256, 150)),   # 512 strips: two per workgroup
                                     ((5, 64, 3, 32, 128), (1024, 200))])  # cfg2: 206k rows, 7 rounds
def test_strip_wgrad_fold_matches_grouped(tmp_path, dims, bt):
    """The six weight gradients folded into the backward strip launch (strip_bwdw.hip, the default) against the
    grouped weight-gradient launch (VQHMM_STRIP_WGRAD=0; above 2^17 rows with the backward pair too): the data-gradient chain is the
    same code, the weight / bias gradients sum per strip workgroup instead of per row chunk, so loss and
    gradients agree within 1e-6 (and every step's gradient against the oracle: test_strong_scaling_shards_*)."""
    out = _run_both_tol(tmp_path, "VQHMM_STRIP_WGRAD", dims, bt)
    assert torch.equal(out["1"]["loss0"], out["0"]["loss0"])  # the forward is untouched


def test_tail_rerun_after_one_forward_is_identical():
    """The backward (its one-launch tail included) run twice after ONE forward gives the same bits:
    the tail re-arms its own dWc counters, so the second launch waits for its own reduction
    (the counters used to be zeroed only by the forward's prologue)."""
    import vqhmm
    gen = torch.Generator().manual_seed(11)
    B, D, T = 64, 5, 120
    x = torch.randn(B, D, T, generator=gen).cuda()
    u = torch.randn(B, 4, T, generator=gen).cuda()
    L = torch.randint(20, T + 1, (B,), generator=gen)
    torch.manual_seed(4)
    m = vqhmm.VAE_HMM(D, 64, 3, 32, u_dim=4, trans_hidden=128).cuda()
    st = vqhmm.TrainState(m, lr=1e-3)
    xs, us, Ls = st.prepare(x, u, L)
    st.forward_backward(xs, us, Ls, 0.5)
    g1 = st.grad.clone()
    ws = st.workspace(B, T)
    d = __import__("ctypes").byref(st.dims)
    from vqhmm import _ext
    for _ in range(2):  # the backward alone, twice more, on the same forward
        _ext.check(st.lib.vqhmm_elbo_bwd_f32(d, st.ptrs, _ext.ptr(xs), None, B, T, 0.5, None, _ext.ptr(ws),
                                             ws.numel(), _ext.ptr(st.grad), _ext.stream_ptr()), "bwd")
        torch.cuda.synchronize()
        assert torch.equal(st.grad, g1)
    st.check_status()
