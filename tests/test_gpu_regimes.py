"""Hard regimes and Viterbi regimes on the model's own outputs:

  hard_regimes(model, x)     softmax(encode(x)).argmax(dim=1)  (backtesting.py:154-155,
                             VQ_VAE+HMM.ipynb:830, visualize.ipynb:74) — one fused pass,
                             bit-exact vs torch's argmax on the q it returns, at every
                             position (no near-tie filtering), K = 3, 8 and 32.
  regime_argmax(q)           the same argmax rule on given probabilities: exact ties,
                             1-ulp gaps, NaN, -inf.
  viterbi_regimes(model,...) bit-exact vs the C oracle fed the model's own tables.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import c_oracle
from test_gpu_model import make_model

pytestmark = pytest.mark.gpu


def torch_argmax(q):
    return q.detach().cpu().argmax(dim=1)


@pytest.mark.parametrize("case", ["cfg1_trained", "cfg2_slice_seeded", "k8_d16", "k32_wide", "smoke_tiny"])
def test_hard_regimes_match_torch_argmax_everywhere(case):
    import vqhmm
    g = load_golden(case)
    m = make_model(g)
    x = torch.tensor(g["x"]).cuda()
    reg, q = vqhmm.hard_regimes(m, x)
    assert reg.dtype == torch.int64 and reg.shape == (x.shape[0], x.shape[2])
    assert torch.equal(reg.cpu(), torch_argmax(q))
    # q is the model's softmax(encode(x)) (1e-6 of the reference's)
    qref = g["fwd/q"]
    assert np.abs(q.cpu().numpy() - qref).max() <= 1e-6
    # vs the REFERENCE's argmax: wherever the product's q column equals the reference's
    # bit for bit, and wherever the reference's top-2 gap exceeds twice the measured q
    # difference (there no perturbation of that size can move the argmax), the regimes
    # must be the reference's
    qn = q.cpu().numpy()
    same = np.all(qn == qref, axis=1)
    srt = np.sort(qref, axis=1)
    decided = (srt[:, -1] - srt[:, -2]) > 2 * np.abs(qn - qref).max()
    ref_reg = torch.tensor(qref).argmax(dim=1).numpy()
    if qref.shape[1] <= 8:
        assert same.any()
    chk = same | decided
    assert chk.mean() > 0.9
    assert np.array_equal(reg.cpu().numpy()[chk], ref_reg[chk])


@pytest.mark.parametrize("K,D,H,H2", [(3, 5, 64, 32), (8, 16, 64, 32), (32, 64, 80, 72)])
def test_hard_regimes_exact_ties(K, D, H, H2):
    """to_logits rows made identical in pairs: those logits, hence q, tie exactly; the
    lowest index must win, as in torch.argmax."""
    import vqhmm
    torch.manual_seed(K)
    m = vqhmm.VAE_HMM(D, H, K, H2, u_dim=4, trans_hidden=16)
    with torch.no_grad():
        W, bb = m.encoder.to_logits.weight, m.encoder.to_logits.bias
        for k in range(1, K, 2):
            W[k] = W[k - 1]
            bb[k] = bb[k - 1]
        W[K - 1] = W[0]
        bb[K - 1] = bb[0]
    m = m.cuda()
    x = torch.randn(6, D, 70, device="cuda")
    reg, q = vqhmm.hard_regimes(m, x)
    assert torch.equal(reg.cpu(), torch_argmax(q))
    assert (reg.cpu() % 2 == 0).all()  # a tied pair never reports its odd member


@pytest.mark.parametrize("K", [3, 8, 32])
def test_regime_argmax_ulp_gaps_ties_nan(K):
    import vqhmm
    rng = np.random.default_rng(K)
    B, T = 5, 333
    q = rng.random((B, K, T)).astype(np.float32)
    top = q.max(axis=1, keepdims=True)
    # exact ties with the max at random channels, 1-ulp gaps below / above it
    for b in range(B):
        for t in range(0, T, 3):
            k1, k2 = rng.choice(K, 2, replace=False)
            v = np.float32(top[b, 0, t])
            q[b, k1, t] = v
            q[b, k2, t] = v if t % 2 == 0 else np.nextafter(v, np.float32(2.0))
            if t % 9 == 0:
                q[b, k2, t] = np.nextafter(v, np.float32(0.0))
    q[0, K - 1, 7] = np.nan
    q[1, :, 8] = np.nan
    q[2, :, 9] = -np.inf
    q[3, 1, 10] = np.inf
    got = vqhmm.regime_argmax(torch.from_numpy(q).cuda())
    assert torch.equal(got.cpu(), torch.from_numpy(q).argmax(dim=1))


@pytest.mark.parametrize("case", ["cfg1_trained", "cfg2_slice_seeded", "k8_d16", "k32_wide"])
def test_viterbi_regimes_vs_c_oracle(case):
    """The MAP path over the model's own (log_pi, log_A, em), identical tensors fed to the
    C oracle (never compare Viterbi on independently recomputed tables)."""
    import vqhmm
    g = load_golden(case)
    m = make_model(g)
    x, u = torch.tensor(g["x"]).cuda(), torch.tensor(g["u"]).cuda()
    L = torch.tensor(g["lengths"])
    path, score = vqhmm.viterbi_regimes(m, x, u, L)
    with torch.no_grad():
        em = torch.log_softmax(m.encode(x), dim=1).transpose(1, 2).contiguous()
        log_pi, log_A = m.prior(u)
    rp, rs = c_oracle.viterbi(log_pi.cpu().numpy(), log_A.cpu().numpy(), em.cpu().numpy(), L.numpy())
    assert np.array_equal(path.cpu().numpy(), rp)
    assert np.array_equal(score.cpu().numpy().view(np.uint32), rs.view(np.uint32))


@pytest.mark.parametrize("K,U,TH,B,T,lay", [
    (1, 4, 64, 37, 45, 0), (2, 3, 64, 20, 100, 0), (3, 4, 128, 70, 333, 0), (3, 2, 64, 9, 17, 1),
    (4, 4, 64, 33, 129, 1), (5, 4, 128, 9, 200, 0), (6, 1, 256, 11, 77, 0), (7, 4, 64, 13, 300, 1),
    (8, 4, 128, 37, 250, 0), (8, 4, 256, 5, 64, 0), (8, 4, 128, 6, 1000, 0)])
def test_prior_viterbi_fused_bit_exact(K, U, TH, B, T, lay):
    """Fused Prior-MLP -> Viterbi: the same path and score bits as
    Prior.forward's log_A fed to the Viterbi kernel, and as the C oracle on that log_A;
    ragged lengths (0, 1, 2, T, random), T not a multiple of the chunk, B not a multiple of
    the workgroup's sequences."""
    import vqhmm
    torch.manual_seed(1000 * K + TH + U)
    prior = vqhmm.Prior(K, u_dim=U, trans_hidden=TH)
    with torch.no_grad():  # sharper tables than the default init: paths that actually switch
        prior.transition_net[2].weight.mul_(4.0)
        prior.log_prior.normal_()
    prior = prior.cuda()
    u = 2.0 * torch.randn(B, U, T)
    if lay == 1:
        u = u.transpose(1, 2).contiguous()
    u = u.cuda()
    em = torch.log_softmax(3.0 * torch.randn(B, T, K), dim=2).cuda()
    L = torch.randint(1, T + 1, (B,))
    L[0] = T
    if B > 3:
        L[1], L[2], L[3] = 0, 1, 2
    got = vqhmm.prior_viterbi(prior, u, em, L)
    assert got is not None
    with torch.no_grad():
        log_pi, log_A = prior(u)
    ref = vqhmm.viterbi(log_pi, log_A, em, L)
    assert torch.equal(got[0].cpu(), ref[0].cpu())
    assert np.array_equal(got[1].cpu().numpy().view(np.uint32), ref[1].cpu().numpy().view(np.uint32))
    rp, rs = c_oracle.viterbi(log_pi.cpu().numpy(), log_A.cpu().numpy(), em.cpu().numpy(), L.numpy())
    assert np.array_equal(got[0].cpu().numpy(), rp)
    assert np.array_equal(got[1].cpu().numpy().view(np.uint32), rs.view(np.uint32))
    if K > 1:
        assert len(np.unique(rp[rp >= 0])) > 1


def test_prior_viterbi_outside_fused_range_falls_back():
    """K > 8 (or TH outside {64, 128, 256}): prior_viterbi reports None and viterbi_regimes
    runs Prior.forward + Viterbi (both native) with the same contract."""
    import vqhmm
    prior = vqhmm.Prior(9, u_dim=4, trans_hidden=64).cuda()
    u = torch.randn(3, 4, 40, device="cuda")
    em = torch.log_softmax(torch.randn(3, 40, 9, device="cuda"), dim=2)
    assert vqhmm.prior_viterbi(prior, u, em) is None
    prior = vqhmm.Prior(3, u_dim=4, trans_hidden=32).cuda()
    em = torch.log_softmax(torch.randn(3, 40, 3, device="cuda"), dim=2)
    assert vqhmm.prior_viterbi(prior, u, em) is None


def test_prior_viterbi_fused_cfg5_length():
    """cfg5's sequence length (T = 4096, K = 8, trans_hidden 128) on a 192-sequence slice of a shard:
    fused path and score bit-identical to Prior.forward + Viterbi, and the C oracle on that log_A."""
    import vqhmm
    torch.manual_seed(5)
    B, T, K = 192, 4096, 8
    prior = vqhmm.Prior(K, u_dim=4, trans_hidden=128)
    with torch.no_grad():
        prior.transition_net[2].weight.mul_(3.0)
    prior = prior.cuda()
    g = torch.Generator(device="cuda").manual_seed(11)
    u = torch.randn(B, 4, T, device="cuda", generator=g)
    em = torch.log_softmax(2.0 * torch.randn(B, T, K, device="cuda", generator=g), dim=2)
    L = torch.randint(T // 2, T + 1, (B,), generator=torch.Generator().manual_seed(3))
    L[0] = T
    got = vqhmm.prior_viterbi(prior, u, em, L)
    with torch.no_grad():
        log_pi, log_A = prior(u)
    ref = vqhmm.viterbi(log_pi, log_A, em, L)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    sl = slice(0, 24)  # the C oracle on a slice (same tables)
    rp, rs = c_oracle.viterbi(log_pi.cpu().numpy(), log_A[sl].cpu().numpy(), em[sl].cpu().numpy(), L[sl].numpy())
    assert np.array_equal(got[0][sl].cpu().numpy(), rp)
    assert np.array_equal(got[1][sl].cpu().numpy().view(np.uint32), rs.view(np.uint32))
