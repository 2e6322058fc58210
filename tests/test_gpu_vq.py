"""GPU parity of the VQ argmin kernel vs the C oracle (bit-exact indices and
distances), through the C-ABI (vqhmm.vq_argmin -> vqhmm_vq_argmin_f32)."""
import numpy as np
import pytest
import torch

from oracle import c_oracle

pytestmark = pytest.mark.gpu


def run(z, cb):
    import vqhmm
    zt = torch.from_numpy(z).cuda()
    ct = torch.from_numpy(cb).cuda()
    idx, d = vqhmm.vq_argmin(zt, ct, return_dist=True)
    torch.cuda.synchronize()
    return idx.cpu().numpy(), d.cpu().numpy()


# T % 4 == 0 -> row-load MFMA kernel; otherwise the 32-position MFMA kernel; K > 32 -> VALU kernel
@pytest.mark.parametrize("B,Dv,T,K", [(3, 5, 200, 3), (2, 64, 100, 32), (2, 64, 96, 17), (3, 30, 64, 32),
                                      (1, 3, 4, 2), (4, 16, 77, 8), (1, 1, 1, 1), (2, 33, 129, 5),
                                      (3, 64, 50, 70), (5, 7, 3, 17)])
def test_vq_bit_exact(B, Dv, T, K):
    rng = np.random.default_rng(B * 1000 + Dv * 10 + K)
    z = rng.standard_normal((B, Dv, T)).astype(np.float32)
    cb = rng.standard_normal((K, Dv)).astype(np.float32)
    idx, d = run(z, cb)
    ridx, rd = c_oracle.vq_argmin(z, cb)
    assert np.array_equal(idx, ridx)
    assert np.array_equal(d.view(np.uint32), rd.view(np.uint32))


def test_vq_ties_and_duplicates():
    rng = np.random.default_rng(5)
    cb = rng.standard_normal((6, 8)).astype(np.float32)
    cb[3] = cb[1]  # exact duplicate codeword -> lowest index must win
    z = np.repeat(cb[[1, 3, 5]].T[None], 2, axis=0).astype(np.float32)  # z exactly on codewords
    idx, d = run(z, cb)
    assert np.all(idx[:, 0] == 1) and np.all(idx[:, 1] == 1) and np.all(idx[:, 2] == 5)
    ridx, rd = c_oracle.vq_argmin(z, cb)
    assert np.array_equal(d.view(np.uint32), rd.view(np.uint32))
    # expansion form: the distance of an exact hit is zero up to rounding of ||c||^2
    assert np.abs(d).max() <= 1e-5 * (cb ** 2).sum(1).max()


def test_vq_one_hot_equals_argmax():
    rng = np.random.default_rng(9)
    logits = torch.from_numpy(rng.standard_normal((8, 3, 200)).astype(np.float32)).cuda()
    q = torch.softmax(logits, dim=1)
    import vqhmm
    idx = vqhmm.vq_argmin(q, torch.eye(3, device="cuda"))
    assert torch.equal(idx.long(), q.argmax(dim=1))


def test_vq_cfg3_size_property():
    """cfg3 shape (B=2048, Dv=64, T=200, K=32): codeword-exact points map to themselves
    and a sampled slice matches the oracle bit-for-bit."""
    import vqhmm
    g = torch.Generator(device="cuda").manual_seed(1234)
    B, Dv, T, K = 2048, 64, 200, 32
    z = torch.randn(B, Dv, T, device="cuda", generator=g)
    cb = torch.randn(K, Dv, device="cuda", generator=g)
    lab = torch.randint(0, K, (B, T), device="cuda", generator=g)
    z[:, :, ::7] = cb[lab[:, ::7]].permute(0, 2, 1)
    idx = vqhmm.vq_argmin(z, cb)
    assert torch.equal(idx[:, ::7].long(), lab[:, ::7])
    sl = z[:64].cpu().numpy()
    assert np.array_equal(idx[:64].cpu().numpy(), c_oracle.vq_argmin(sl, cb.cpu().numpy(), want_dmin=False))


@pytest.mark.parametrize("B,Dv,T,K,beta", [(3, 5, 200, 3, 0.25), (2, 64, 50, 32, 1.0), (4, 16, 77, 8, 0.5),
                                           # the argmin kernel's fused epilogue (Dv % 4 == 0, T % 4 == 0)
                                           (8, 64, 200, 32, 0.25), (16, 16, 100, 8, 1.0), (5, 4, 64, 3, 0.5),
                                           (7, 32, 36, 17, 0.25), (1, 8, 4, 2, 2.0)])
def test_quantize_vs_pseudocode(B, Dv, T, K, beta):
    """vqhmm.quantize (pseudocode.txt:11-18): z_q, straight-through value, commit and
    codebook losses (fused quantize kernel: direct-difference squared errors in fp64), and their
    autograd gradients vs the restatement oracle/hmm_ref.quantize_f32 on the C oracle's indices."""
    import vqhmm
    from oracle import hmm_ref
    rng = np.random.default_rng(K * 31 + Dv)
    z = rng.standard_normal((B, Dv, T)).astype(np.float32)
    cb = rng.standard_normal((K, Dv)).astype(np.float32)
    w = rng.standard_normal((B, Dv, T)).astype(np.float32)
    zt = torch.from_numpy(z).cuda().requires_grad_(True)
    ct = torch.from_numpy(cb).cuda().requires_grad_(True)
    zq_st, idx, commit, cb_loss = vqhmm.quantize(zt, ct, beta=beta)
    ridx = c_oracle.vq_argmin(z, cb, want_dmin=False)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    ref = hmm_ref.quantize_f32(z, cb, ridx, beta)
    assert np.array_equal(zq_st.detach().cpu().numpy(), ref["z_q_st"])
    assert abs(commit.item() - ref["commit"]) <= 1e-6 * ref["commit"]
    assert abs(cb_loss.item() - ref["codebook"]) <= 1e-6 * ref["codebook"]
    (zq_st * torch.from_numpy(w).cuda()).sum().add(commit).add(cb_loss).backward()
    dz = zt.grad.cpu().numpy().astype(np.float64)
    assert np.abs(dz - (w + ref["dz_extra"])).max() <= 1e-6 * np.abs(w).max()
    dc = ct.grad.cpu().numpy().astype(np.float64)
    assert np.abs(dc - ref["dcodebook"]).max() <= 1e-5 * max(np.abs(ref["dcodebook"]).max(), 1e-12)
