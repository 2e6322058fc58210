"""Autograd through the module surface alone (VQ_VAE_HMM_fixed.py:100-104 encode / decode, :139-143 forward):
examples/backtest_example.py:30 calls vae_hmm.encode(data) with grad enabled.  The backward runs on the HIP
kernels (vqhmm_encode_bwd_f32 / vqhmm_decode_bwd_f32 / vqhmm_forward_bwd_f32); every parameter gradient and
the input gradient are checked against the fp64 oracle's autograd (oracle/ref_model.py) within 1e-5 normwise.
"""
import pytest
import torch

from oracle import ref_model as RM

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _model(D=5, H=64, K=3, H2=32, seed=0):
    import vqhmm
    torch.manual_seed(seed)
    return vqhmm.VAE_HMM(D, H, K, H2, u_dim=4, trans_hidden=128).cuda()


def _p64(m):
    return {k: v.detach().cpu().double().requires_grad_(True) for k, v in m.state_dict().items()}


def _close(got, ref, name):
    got, ref = got.detach().cpu().double(), ref.detach().double()
    err = (got - ref).norm() / max(ref.norm().item(), 1e-30)
    assert err <= RTOL, f"{name}: {err:.2e}"


@pytest.mark.parametrize("B,T", [(16, 50), (8, 200)])
def test_encode_autograd_vs_oracle(B, T):
    m = _model()
    g = torch.Generator().manual_seed(B + T)
    x = torch.randn(B, 5, T, generator=g)
    G = torch.randn(B, 3, T, generator=g)
    xg = x.cuda().requires_grad_(True)
    logits = m.encode(xg)
    (logits * G.cuda()).sum().backward()
    p = _p64(m)
    x64 = x.double().requires_grad_(True)
    ref = RM.encoder_logits(p, x64)
    _close(logits, ref, "logits")
    (ref * G.double()).sum().backward()
    for k in ("encoder.conv1.weight", "encoder.conv1.bias", "encoder.conv2.weight", "encoder.conv2.bias",
              "encoder.to_logits.weight", "encoder.to_logits.bias"):
        _close(dict(m.named_parameters())[k].grad, p[k].grad, k)
    _close(xg.grad, x64.grad, "dx")
    for n, prm in m.named_parameters():  # encode touches nothing else
        if not n.startswith("encoder."):
            assert prm.grad is None, n


def test_encode_params_only_and_no_grad_path():
    """Parameters alone require grad (the usual case: x is data); under no_grad the inference path runs."""
    m = _model(seed=1)
    x = torch.randn(4, 5, 30).cuda()
    logits = m.encode(x)
    assert logits.requires_grad
    logits.square().sum().backward()
    assert m.encoder.conv1.weight.grad is not None and torch.isfinite(m.encoder.conv1.weight.grad).all()
    with torch.no_grad():
        l2 = m.encode(x)
    assert not l2.requires_grad and torch.equal(l2, logits.detach())


@pytest.mark.parametrize("B,T,K", [(16, 50, 3), (6, 120, 4)])
def test_decode_autograd_vs_oracle(B, T, K):
    m = _model(K=K, seed=2)
    g = torch.Generator().manual_seed(7 * B + T)
    q = torch.softmax(torch.randn(B, K, T, generator=g), 1)
    G1, G2 = torch.randn(B, 5, T, generator=g), torch.randn(B, 5, T, generator=g)
    qg = q.cuda().requires_grad_(True)
    mu, logvar = m.decode(qg)
    ((mu * G1.cuda()).sum() + (logvar * G2.cuda()).sum()).backward()
    p = _p64(m)
    q64 = q.double().requires_grad_(True)
    rmu, rlv = RM.decoder_params(p, q64)
    _close(mu, rmu, "mu")
    _close(logvar, rlv, "logvar")
    ((rmu * G1.double()).sum() + (rlv * G2.double()).sum()).backward()
    for k in ("decoder.embeddings.weight", "decoder.conv1.weight", "decoder.conv1.bias", "decoder.conv2.weight",
              "decoder.conv2.bias", "decoder.to_params.weight", "decoder.to_params.bias"):
        _close(dict(m.named_parameters())[k].grad, p[k].grad, k)
    _close(qg.grad, q64.grad, "dq")


@pytest.mark.parametrize("use_q", [False, True])
def test_forward_autograd_vs_oracle(use_q):
    """VAE_HMM.forward -> ((mu, logvar), q): a loss on mu / logvar (and on q) back through decode, the softmax
    and encode."""
    m = _model(seed=3)
    B, T = 12, 64
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, 5, T, generator=g)
    G1, G2, G3 = (torch.randn(B, c, T, generator=g) for c in (5, 5, 3))
    xg = x.cuda().requires_grad_(True)
    (mu, logvar), q = m(xg)
    loss = (mu * G1.cuda()).sum() + (logvar * G2.cuda()).sum() + ((q * G3.cuda()).sum() if use_q else 0.0)
    loss.backward()
    p = _p64(m)
    x64 = x.double().requires_grad_(True)
    rq = torch.softmax(RM.encoder_logits(p, x64), 1)
    rmu, rlv = RM.decoder_params(p, rq)
    _close(q, rq, "q")
    _close(mu, rmu, "mu")
    rl = (rmu * G1.double()).sum() + (rlv * G2.double()).sum() + ((rq * G3.double()).sum() if use_q else 0.0)
    rl.backward()
    for k, prm in m.named_parameters():
        if k.startswith("prior."):
            assert prm.grad is None, k
            continue
        _close(prm.grad, p[k].grad, k)
    _close(xg.grad, x64.grad, "dx")


@pytest.mark.parametrize("B,T,K,lay,with_pi", [(16, 50, 3, 0, True), (8, 200, 4, 1, True), (5, 33, 8, 0, False)])
def test_prior_autograd_vs_oracle(B, T, K, lay, with_pi):
    """Prior.forward alone (:59-71) in either u layout: log_prior / transition_net gradients and du."""
    m = _model(K=K, seed=4)
    g = torch.Generator().manual_seed(13 * B + T)
    u = torch.randn(B, 4, T, generator=g)
    if lay == 1:
        u = u.transpose(1, 2).contiguous()
    Gpi, GA = torch.randn(K, generator=g), torch.randn(B, T, K, K, generator=g)
    ug = u.cuda().requires_grad_(True)
    log_pi, log_A = m.prior(ug)
    loss = (log_A * GA.cuda()).sum() + ((log_pi * Gpi.cuda()).sum() if with_pi else 0.0)
    loss.backward()
    p = _p64(m)
    u64 = u.double().requires_grad_(True)
    rpi, rA = RM.prior_tables(p, u64, K, 4)
    _close(log_A, rA, "log_A")
    rl = (rA * GA.double()).sum() + ((rpi * Gpi.double()).sum() if with_pi else 0.0)
    rl.backward()
    for k, prm in m.named_parameters():
        if not k.startswith("prior."):
            assert prm.grad is None, k
            continue
        if k == "prior.log_prior" and not with_pi:
            assert prm.grad is None or prm.grad.abs().max() == 0, k
            continue
        _close(prm.grad, p[k].grad, k)
    _close(ug.grad, u64.grad, "du")


@pytest.mark.parametrize("D,H,K,H2", [(16, 64, 8, 32), (64, 256, 32, 128)])
def test_forward_autograd_wide_dims(D, H, K, H2):
    """the module backward at cfg4 dims (D = 16, K = 8) and cfg3 dims (D = 64, H = 256, K = 32),
    where other kernels run than at cfg2 (convbig / wgradbig past 64 channels, the channels-first dgrad
    outputs): every encoder / decoder gradient, dx and dq against the fp64 oracle, small B and T."""
    m = _model(D=D, H=H, K=K, H2=H2, seed=5)
    B, T = 4, 40
    g = torch.Generator().manual_seed(D + K)
    x = torch.randn(B, D, T, generator=g)
    G1, G2, G3 = (torch.randn(B, c, T, generator=g) for c in (D, D, K))
    xg = x.cuda().requires_grad_(True)
    (mu, logvar), q = m(xg)
    ((mu * G1.cuda()).sum() + (logvar * G2.cuda()).sum() + (q * G3.cuda()).sum()).backward()
    p = _p64(m)
    x64 = x.double().requires_grad_(True)
    rq = torch.softmax(RM.encoder_logits(p, x64), 1)
    rmu, rlv = RM.decoder_params(p, rq)
    _close(q, rq, "q")
    _close(mu, rmu, "mu")
    _close(logvar, rlv, "logvar")
    ((rmu * G1.double()).sum() + (rlv * G2.double()).sum() + (rq * G3.double()).sum()).backward()
    for k, prm in m.named_parameters():
        if k.startswith("prior."):
            assert prm.grad is None, k
            continue
        _close(prm.grad, p[k].grad, k)
    _close(xg.grad, x64.grad, "dx")


@pytest.mark.parametrize("D,H,K,H2", [(16, 64, 8, 32), (64, 256, 32, 128)])
def test_decode_autograd_wide_dims(D, H, K, H2):
    """decode alone at cfg4 / cfg3 dims: the decoder gradients and dq against the fp64 oracle."""
    m = _model(D=D, H=H, K=K, H2=H2, seed=6)
    B, T = 3, 33
    g = torch.Generator().manual_seed(3 * D + K)
    q = torch.softmax(torch.randn(B, K, T, generator=g), 1)
    G1, G2 = torch.randn(B, D, T, generator=g), torch.randn(B, D, T, generator=g)
    qg = q.cuda().requires_grad_(True)
    mu, logvar = m.decode(qg)
    ((mu * G1.cuda()).sum() + (logvar * G2.cuda()).sum()).backward()
    p = _p64(m)
    q64 = q.double().requires_grad_(True)
    rmu, rlv = RM.decoder_params(p, q64)
    ((rmu * G1.double()).sum() + (rlv * G2.double()).sum()).backward()
    for k in ("decoder.embeddings.weight", "decoder.conv1.weight", "decoder.conv1.bias", "decoder.conv2.weight",
              "decoder.conv2.bias", "decoder.to_params.weight", "decoder.to_params.bias"):
        _close(dict(m.named_parameters())[k].grad, p[k].grad, k)
    _close(qg.grad, q64.grad, "dq")
