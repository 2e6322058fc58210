"""Checkpoints: the reference's save_checkpoint/load_checkpoint
format (src/utils/data.py:47-60), with TrainState's Adam state exported as
torch.optim.Adam's own state_dict."""
import types

import pytest
import torch

import vqhmm
from vqhmm.checkpoint import adam_state_dict, load_adam_state_dict
from vqhmm.model import param_offsets


def fake_state(m, seed, step):
    off = param_offsets(m._dims())
    g = torch.Generator().manual_seed(seed)
    n = off[-1]
    return types.SimpleNamespace(model=m, off=off, exp_avg=torch.randn(n, generator=g),
                                 exp_avg_sq=torch.rand(n, generator=g), step_dev=torch.tensor(step),
                                 lr=2e-3, betas=(0.8, 0.99), eps=1e-7)


def test_adam_state_dict_is_torch_adam_format():
    m = vqhmm.VAE_HMM(5, 16, 3, 8, u_dim=4, trans_hidden=16)
    st = fake_state(m, 0, 7)
    sd = adam_state_dict(st)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    opt.load_state_dict(sd)
    assert opt.param_groups[0]["lr"] == 2e-3 and tuple(opt.param_groups[0]["betas"]) == (0.8, 0.99)
    for i, name in enumerate(vqhmm.PARAM_ORDER):
        p = dict(m.named_parameters())[name]
        a, b = st.off[i], st.off[i + 1]
        assert int(opt.state[p]["step"]) == 7
        assert torch.equal(opt.state[p]["exp_avg"].reshape(-1), st.exp_avg[a:b])
        assert torch.equal(opt.state[p]["exp_avg_sq"].reshape(-1), st.exp_avg_sq[a:b])
    st2 = fake_state(m, 1, 0)
    load_adam_state_dict(st2, sd)
    assert torch.equal(st2.exp_avg, st.exp_avg) and torch.equal(st2.exp_avg_sq, st.exp_avg_sq)
    assert int(st2.step_dev) == 7 and st2.lr == 2e-3 and st2.betas == (0.8, 0.99) and st2.eps == 1e-7


def test_reference_format_roundtrip_with_torch_adam(tmp_path):
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(5, 16, 3, 8, u_dim=4, trans_hidden=16)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    opt.step()
    path = tmp_path / "ck.pt"
    vqhmm.save_checkpoint(m, opt, 4, 123.5, str(path))
    ck = torch.load(str(path), weights_only=True)
    assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "loss"}
    m2 = vqhmm.VAE_HMM(5, 16, 3, 8, u_dim=4, trans_hidden=16)
    opt2 = torch.optim.Adam(m2.parameters(), lr=1e-3)
    assert vqhmm.load_checkpoint(m2, opt2, str(path)) == (4, 123.5)
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k


@pytest.mark.gpu
def test_train_state_resume_bit_identical(tmp_path):
    """3 steps straight == 2 steps, save, load into a fresh model + TrainState, 1 step."""
    B, T = 64, 120
    gen = torch.Generator().manual_seed(9)
    x = torch.randn(B, 5, T, generator=gen).cuda()
    u = torch.randn(B, 4, T, generator=gen).cuda()
    L = torch.randint(20, T + 1, (B,), generator=gen)

    def fresh(seed):
        torch.manual_seed(seed)
        m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128).cuda()
        return m, vqhmm.TrainState(m, lr=1e-3)

    ma, sa = fresh(0)
    for _ in range(3):
        sa.step(x, u, L, 1.0)
    mb, sb = fresh(0)
    for _ in range(2):
        sb.step(x, u, L, 1.0)
    path = str(tmp_path / "resume.pt")
    vqhmm.save_checkpoint(mb, sb, 2, float(sb.loss), path)
    mc, sc = fresh(123)
    assert vqhmm.load_checkpoint(mc, sc, path)[0] == 2
    sc.step(x, u, L, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(sa.flat, sc.flat)
    assert torch.equal(sa.exp_avg, sc.exp_avg) and torch.equal(sa.exp_avg_sq, sc.exp_avg_sq)
    assert int(sa.step_dev) == int(sc.step_dev) == 3
    # the same checkpoint resumes the reference's torch.optim.Adam on the CPU
    mr = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128)
    opt = torch.optim.Adam(mr.parameters(), lr=1e-3)
    vqhmm.load_checkpoint(mr, opt, path)
    for name, p in mr.named_parameters():
        assert int(opt.state[p]["step"]) == 2, name


def test_encoder_only_checkpoint_format(tmp_path):
    """VQ_VAE+HMM.ipynb:774 writes {'model_state_dict': trained.encoder.state_dict(),
    'config': {input_dim, hidden_dim, hidden_dim2, K}} and :818 / visualize.ipynb:62 rebuild
    Encoder(input_dim, hidden_dim, hidden_dim2, K) from it."""
    torch.manual_seed(3)
    m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128)
    path = tmp_path / "encoder_saved.pth"
    vqhmm.save_encoder(m, path)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert set(ck) == {"model_state_dict", "config"}
    assert ck["config"] == {"input_dim": 5, "hidden_dim": 64, "hidden_dim2": 32, "K": 3}
    assert list(ck["model_state_dict"]) == list(m.encoder.state_dict())
    # the notebook's own reading code, on the file we wrote
    cfg = ck.get("config", {})
    enc = vqhmm.Encoder(cfg.get("input_dim"), cfg.get("hidden_dim", 32), cfg.get("hidden_dim2", cfg["hidden_dim"]),
                        cfg.get("K"))
    enc.load_state_dict(ck["model_state_dict"])
    enc2 = vqhmm.load_encoder(path)
    for (k, a), (k2, b) in zip(m.encoder.state_dict().items(), enc2.state_dict().items()):
        assert k == k2 and torch.equal(a, b)
    # a file without hidden_dim2 falls back to hidden_dim (the notebook's .get default)
    torch.save({"model_state_dict": vqhmm.Encoder(5, 16, 16, 4).state_dict(),
                "config": {"input_dim": 5, "hidden_dim": 16, "K": 4}}, tmp_path / "e2.pth")
    e3 = vqhmm.load_encoder(tmp_path / "e2.pth")
    assert e3.conv2.weight.shape == (16, 16, 3) and e3.to_logits.weight.shape == (4, 16, 1)


@pytest.mark.gpu
def test_encoder_only_checkpoint_round_trip_on_device(tmp_path):
    """A reloaded encoder gives bit-identical logits and hard regimes to the trained model's."""
    torch.manual_seed(4)
    m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128).cuda()
    vqhmm.save_encoder(m, tmp_path / "enc.pth")
    enc = vqhmm.load_encoder(tmp_path / "enc.pth").cuda().eval()
    x = torch.randn(3, 5, 100, device="cuda")
    with torch.no_grad():
        assert torch.equal(enc(x), m.encode(x))
    r1, q1 = vqhmm.hard_regimes(m, x)
    r2, q2 = vqhmm.hard_regimes(enc, x)
    assert torch.equal(r1, r2) and torch.equal(q1, q2)
