"""The fused ELBO heads across the shapes that select them (csrc/api.hip plan_elbo):

  head_coop.hip  elbo_head_pipe_kernel: K <= 4, U <= 4, TH = 128, D <= 16   (cfg1 / cfg2; the default there)
                 elbo_head_coop_kernel: K <= 8, U <= 4, TH in {64, 128, 256}, D <= 16 otherwise (cfg4)
  head_mfma.hip  K <= 4, U in 5..7, TH in {64, 128}
  staged         everything else (cfg3: K = 32); head_l1 by K: pow2 (16, 32), wide (other K <= 32), lane per row

Both head_coop kernels keep a wave's window-invariant phase-A operands in registers where their
workgroup runs two or more windows (coop: more than 512 windows of 63 rows at K <= 4, 31 at K <= 8;
pipe: more than 256 windows), so the cases marked "loops" run both forms in one launch; the pipelined
kernel's software pipeline (phase A one window ahead, the terms one behind) is exercised by every case
with more than one window per workgroup.

Each case is one training step's loss (1e-5 relative vs the fp32 CPU oracle) and all 18
gradients (normwise vs the fp64 oracle on the device forward's ReLU branch), through
check_step_vs_oracle; U < 4 covers the bias column of u' = [u, 1] (VQ_VAE_HMM_fixed.py:53-57)."""
import pytest
import torch

from test_gpu_configs import check_step_vs_oracle

pytestmark = pytest.mark.gpu

CASES = [
    # (D, H, K, H2, U, TH), B, T
    ((16, 32, 8, 16, 4, 128), 24, 70),
    ((16, 32, 8, 16, 4, 128), 96, 200),    # > 512 windows: workgroups loop over windows
    ((5, 32, 3, 16, 4, 128), 256, 200),    # pipe, loops (register-resident phase-A operands)
    ((5, 32, 2, 16, 1, 128), 300, 150),    # pipe, loops, K = 2, U = 1
    ((5, 32, 4, 16, 4, 128), 64, 200),     # pipe, one window per workgroup (operands from LDS)
    ((16, 32, 1, 16, 4, 128), 40, 90),     # pipe, K = 1, D = 16
    ((5, 32, 5, 16, 4, 64), 96, 200),      # loops, K = 5
    ((5, 32, 3, 16, 2, 64), 200, 180),     # loops, U < 4
    ((5, 32, 5, 16, 4, 64), 24, 70),
    ((7, 32, 6, 16, 3, 256), 16, 60),
    ((16, 32, 7, 16, 2, 128), 20, 45),
    ((16, 32, 8, 16, 1, 64), 12, 33),
    ((5, 32, 3, 16, 2, 64), 24, 70),       # coop, U < 4
    ((5, 32, 3, 16, 3, 128), 24, 70),
    ((5, 32, 4, 16, 5, 64), 24, 70),       # head_mfma, U = 5..7
    ((5, 32, 2, 16, 6, 128), 24, 70),
    ((5, 32, 3, 16, 7, 64), 24, 70),
    ((8, 32, 16, 16, 4, 64), 24, 70),      # staged, head_l1_pow2 K = 16
    ((8, 32, 32, 16, 3, 128), 40, 90),     # staged, head_l1_pow2 K = 32
    ((8, 32, 12, 16, 4, 64), 24, 70),      # staged, head_l1_wide (float4 rows)
    ((8, 32, 10, 16, 2, 64), 20, 45),      # staged, head_l1_wide (scalar rows)
    ((8, 32, 40, 16, 4, 64), 12, 33),      # staged, head_l1 lane per row (K > 32)
]


@pytest.mark.parametrize("dims,B,T", CASES)
def test_head_shapes_vs_oracle(dims, B, T):
    check_step_vs_oracle(dims, B, T, seed=B * 100 + T, rtol_norm=1e-5)


@pytest.mark.parametrize("dims", [(16, 64, 8, 32, 4, 128), (5, 64, 3, 32, 4, 128)])
def test_head_forward_only_matches_training_loss(dims):
    """compute_loss without autograd (need_grad = 0: no gradient buffers or slabs written) gives
    the same loss bits as the training forward."""
    import vqhmm
    D, H, K, H2, U, TH = dims
    torch.manual_seed(1)
    m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=U, trans_hidden=TH).cuda()
    gen = torch.Generator().manual_seed(3)
    B, T = 40, 90
    x = torch.randn(B, D, T, generator=gen).cuda()
    u = torch.randn(B, U, T, generator=gen).cuda()
    L = torch.randint(10, T + 1, (B,), generator=gen)
    with torch.no_grad():
        l0 = m.compute_loss(x, u, L, 0.8).item()
    l1 = m.compute_loss(x, u, L, 0.8)
    l1.backward()
    assert l0 == l1.item()


@pytest.mark.parametrize("dims", [(5, 64, 3, 32, 4, 128), (16, 64, 8, 32, 4, 128)])
@pytest.mark.parametrize("where", ["u", "logvar_bias", "transition_w2"])
def test_head_propagates_nan_like_the_reference(dims, where):
    """A NaN input or parameter gives a NaN loss, as the reference's torch arithmetic does
    (relu(NaN) = NaN, exp(NaN) = NaN): the head's ReLU / max / clamp must not swallow it
    (head kernels built with -fno-honor-nans)."""
    import vqhmm
    from oracle import ref_model as RM
    D, H, K, H2, U, TH = dims
    torch.manual_seed(2)
    m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=U, trans_hidden=TH)
    gen = torch.Generator().manual_seed(7)
    B, T = 8, 40
    x = torch.randn(B, D, T, generator=gen)
    u = torch.randn(B, U, T, generator=gen)
    L = torch.full((B,), T)
    with torch.no_grad():
        if where == "u":
            u[3, 1, 17] = float("nan")
        elif where == "logvar_bias":
            m.decoder.to_params.bias[D] = float("nan")
        else:
            m.prior.transition_net[2].weight[0, 5] = float("nan")
    p = {k: v.detach().clone() for k, v in m.state_dict().items()}
    ref = RM.elbo(p, x, u, L, 1.0, K, U).item()
    assert ref != ref  # the reference's arithmetic: NaN
    mg = m.cuda()
    with torch.no_grad():
        got = mg.compute_loss(x.cuda(), u.cuda(), L, 1.0).item()
    assert got != got, got
    st = vqhmm.TrainState(mg, lr=1e-3)
    xs, us, Ls = st.prepare(x, u, L)
    st.forward_backward(xs, us, Ls, 1.0)
    assert st.loss.item() != st.loss.item()
