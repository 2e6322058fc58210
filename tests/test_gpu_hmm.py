"""GPU parity of the Viterbi (bit-exact path + score) and forward-backward
(gamma: <= 1e-5 absolute per element AND <= 1e-5 normwise relative per sequence;
logZ rel <= 1e-5 vs the fp64 oracle) kernels, through the C-ABI.  Inputs are fed identically to both sides (never
compare Viterbi on independently recomputed log_A)."""
import numpy as np
import pytest
import torch

from oracle import c_oracle, hmm_ref

pytestmark = pytest.mark.gpu


def log_softmax(a, axis=-1):
    m = a.max(axis=axis, keepdims=True)
    return a - m - np.log(np.exp(a - m).sum(axis=axis, keepdims=True))


def random_hmm(seed, B, T, K, scale=1.5):
    rng = np.random.default_rng(seed)
    log_pi = log_softmax(rng.standard_normal(K)).astype(np.float32)
    log_A = log_softmax(rng.standard_normal((B, T, K, K)) * scale).astype(np.float32)
    em = log_softmax(rng.standard_normal((B, T, K)) * 2.0).astype(np.float32)
    return log_pi, log_A, em


def check_gamma(g, rg, tol=1e-5):
    """The gamma contract: every element within `tol` of the fp64 oracle, and
    per sequence ||g_b - ref_b|| <= tol ||ref_b|| (the north star's "within 1e-5 relative";
    sequences of length 0 have gamma = 0 on both sides)."""
    g = np.asarray(g, np.float64)
    assert np.abs(g - rg).max() <= tol
    d = np.linalg.norm((g - rg).reshape(len(g), -1), axis=1)
    n = np.linalg.norm(np.asarray(rg, np.float64).reshape(len(g), -1), axis=1)
    live = n > 0
    assert np.all(d[live] <= tol * n[live]), (d[live] / n[live]).max()
    assert np.all(d[~live] == 0)


def gpu(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


CASES = [(2, 3, 50), (3, 7, 41), (4, 5, 200), (5, 9, 64), (8, 6, 300), (8, 3, 1), (1, 4, 17), (3, 70, 33),
         # K > 8: one sequence per wave (hmm_wide.hip), both half widths
         (9, 5, 77), (12, 4, 130), (16, 6, 64), (17, 3, 45), (24, 5, 99), (32, 6, 200), (32, 3, 1), (32, 2, 1500)]


@pytest.mark.parametrize("K,B,T", CASES)
def test_viterbi_bit_exact(K, B, T):
    import vqhmm
    log_pi, log_A, em = random_hmm(K * 7 + B, B, T, K)
    rng = np.random.default_rng(K)
    L = rng.integers(0, T + 1, B).astype(np.int64)
    L[0] = T
    path, score = vqhmm.viterbi(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    rp, rs = c_oracle.viterbi(log_pi, log_A, em, L)
    assert np.array_equal(path.cpu().numpy(), rp)
    assert np.array_equal(score.cpu().numpy().view(np.uint32), rs.view(np.uint32))


def test_viterbi_ties():
    import vqhmm
    K, B, T = 4, 3, 30
    log_pi = np.zeros(K, np.float32)
    log_A = np.zeros((B, T, K, K), np.float32)
    em = np.zeros((B, T, K), np.float32)
    em[1, ::3, 2] = 1.0  # some structure, many exact ties elsewhere
    path, score = vqhmm.viterbi(*gpu(log_pi, log_A, em), torch.tensor([T, T, 5]))
    rp, rs = c_oracle.viterbi(log_pi, log_A, em, np.array([T, T, 5]))
    assert np.array_equal(path.cpu().numpy(), rp)


def test_viterbi_cfg5_long_sequence():
    """cfg5 sequence length (T=4096, K=8): bit-exact vs the C oracle on a slice of the batch."""
    import vqhmm
    B, T, K = 16, 4096, 8
    log_pi, log_A, em = random_hmm(55, B, T, K)
    L = np.full(B, T, np.int64)
    L[3] = 1000
    path, score = vqhmm.viterbi(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    rp, rs = c_oracle.viterbi(log_pi, log_A, em, L)
    assert np.array_equal(path.cpu().numpy(), rp)
    assert np.array_equal(score.cpu().numpy(), rs)


# K <= 8 forward-backward has three kernels: the parallel-in-time one (hmm_seg.hip: one wave per 64-step
# segment; by default for 5 <= K <= 8 and 128 <= T <= 1024, VQHMM_FB_SEG=1 forces it for every K <= 8 and
# T <= 1024, =0 turns it off), the LDS-resident one (whenever its table fits and one round of workgroups
# covers the batch) and the streaming one (VQHMM_FB_RES=0, read per call).  The streaming one forms gamma
# inside its chains where its LDS histories fit (T up to ~1000), else through the workspace and a gamma
# pass (VQHMM_FB_FUSE=0 forces that form; both switches read per call).  The fused form runs two sequence
# groups per 8-wave workgroup (VQHMM_FB_PAIR=0: one per 4-wave workgroup).
FB_KERNELS = ["segmented", "resident", "streaming", "streaming-single", "streaming-unfused"]


def use_fb_kernel(monkeypatch, kernel):
    monkeypatch.setenv("VQHMM_FB_SEG", "1" if kernel == "segmented" else "0")
    if kernel.startswith("streaming"):
        monkeypatch.setenv("VQHMM_FB_RES", "0")
    else:
        monkeypatch.delenv("VQHMM_FB_RES", raising=False)
    if kernel == "streaming-unfused":
        monkeypatch.setenv("VQHMM_FB_FUSE", "0")
    else:
        monkeypatch.delenv("VQHMM_FB_FUSE", raising=False)
    if kernel == "streaming-single":
        monkeypatch.setenv("VQHMM_FB_PAIR", "0")
    else:
        monkeypatch.delenv("VQHMM_FB_PAIR", raising=False)


@pytest.mark.parametrize("K,B,T", [(8, 7, 300), (8, 64, 512), (4, 33, 200), (3, 9, 130)])
def test_forward_backward_pair_matches_single(K, B, T, monkeypatch):
    """The 8-wave two-group fused kernel equals the 4-wave one bit for bit: ragged lengths so the two
    groups of a workgroup run different chunk counts of their own (the workgroup runs the longer), an
    odd group count so the last workgroup's second group is past the batch."""
    import vqhmm
    log_pi, log_A, em = random_hmm(K * 7 + B, B, T, K)
    rng = np.random.default_rng(B + T)
    L = rng.integers(0, T + 1, B).astype(np.int64)
    L[0], L[1] = T, 1
    args = (*gpu(log_pi, log_A, em), torch.from_numpy(L))
    monkeypatch.setenv("VQHMM_FB_RES", "0")
    monkeypatch.setenv("VQHMM_FB_SEG", "0")
    out = {}
    for pair in ("1", "0"):
        monkeypatch.setenv("VQHMM_FB_PAIR", pair)
        g, z = vqhmm.forward_backward(*args)
        out[pair] = (g.cpu().numpy(), z.cpu().numpy())
    assert np.array_equal(out["1"][0].view(np.uint32), out["0"][0].view(np.uint32))
    assert np.array_equal(out["1"][1].view(np.uint32), out["0"][1].view(np.uint32))
    rg, _ = hmm_ref.forward_backward_f64(log_pi, log_A, em, L)
    check_gamma(out["1"][0], rg)


@pytest.mark.parametrize("kernel", FB_KERNELS)
@pytest.mark.parametrize("K,B,T", CASES)
def test_forward_backward_vs_fp64(K, B, T, kernel, monkeypatch):
    import vqhmm
    use_fb_kernel(monkeypatch, kernel)
    log_pi, log_A, em = random_hmm(K * 11 + B, B, T, K)
    rng = np.random.default_rng(K + 1)
    L = rng.integers(0, T + 1, B).astype(np.int64)
    L[0] = T
    gamma, logZ = vqhmm.forward_backward(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A, em, L)
    g = gamma.cpu().numpy()
    check_gamma(g, rg)
    z = logZ.cpu().numpy()
    live = L > 0
    assert np.all(np.abs(z[live] - rz[live]) <= 1e-5 * np.maximum(1.0, np.abs(rz[live])))
    assert np.all(np.isnan(z[~live]))


def test_viterbi_cfg5_full_shard():
    """The unfused Viterbi on one GPU's full cfg5 shard (8192 sequences / 8 GPUs = 1024 x T=4096,
    K=8; log_A 1.07 GB built on the device as log_softmax(N(0,1))), with ragged
    lengths: path and score bit-exact vs the C oracle on a strided slice of 16 sequences, and
    every path entry past a sequence's length is -1."""
    import vqhmm
    B, T, K = 1024, 4096, 8
    g = torch.Generator(device="cuda").manual_seed(5)
    log_pi = torch.log_softmax(torch.randn(K, device="cuda", generator=g), -1)
    log_A = torch.log_softmax(torch.randn(B, T, K, K, device="cuda", generator=g), -1)
    em = torch.log_softmax(torch.randn(B, T, K, device="cuda", generator=g), -1)
    L = torch.full((B,), T, dtype=torch.int64)
    L[5::64] = torch.randint(1, T, (16,), generator=torch.Generator().manual_seed(6))
    path, score = vqhmm.viterbi(log_pi, log_A, em, L)
    sl = slice(5, B, 64)
    rp, rs = c_oracle.viterbi(log_pi.cpu().numpy(), log_A[sl].cpu().numpy(), em[sl].cpu().numpy(), L[sl].numpy())
    assert np.array_equal(path[sl].cpu().numpy(), rp)
    assert np.array_equal(score[sl].cpu().numpy().view(np.uint32), rs.view(np.uint32))
    sl2 = slice(0, B, 64)  # full-length rows of the same launch
    rp2, rs2 = c_oracle.viterbi(log_pi.cpu().numpy(), log_A[sl2].cpu().numpy(), em[sl2].cpu().numpy(), L[sl2].numpy())
    assert np.array_equal(path[sl2].cpu().numpy(), rp2)
    assert np.array_equal(score[sl2].cpu().numpy().view(np.uint32), rs2.view(np.uint32))
    p = path.cpu().numpy()
    past = np.arange(T)[None, :] >= L.numpy()[:, None]
    assert np.all(p[past] == -1) and np.all((p[~past] >= 0) & (p[~past] < K))


def test_forward_backward_long_T_precision():
    """T=4096: per-step normalisation keeps gamma within 1e-5 (a naive fp32 log-space
    recursion drifts to ~1e-3 here)."""
    import vqhmm
    B, T, K = 4, 4096, 8
    log_pi, log_A, em = random_hmm(99, B, T, K)
    gamma, logZ = vqhmm.forward_backward(*gpu(log_pi, log_A, em))
    rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A, em, np.full(B, T))
    check_gamma(gamma.cpu().numpy(), rg)
    assert np.all(np.abs(logZ.cpu().numpy() - rz) <= 1e-5 * np.abs(rz))


@pytest.mark.parametrize("kernel", FB_KERNELS)
@pytest.mark.parametrize("K", [3, 8, 13, 32])
def test_forward_backward_extreme_tables(K, kernel, monkeypatch):
    """Tables that push the fast base-2 step out of range, so chunks take the exact
    max-shifted recomputation: left-to-right transitions (log 0 = -inf), emissions of
    about -1e3 nats, a window with hundreds of nats of emission spread, and
    near-deterministic transitions.  Same 1e-5 contract vs the fp64 oracle."""
    import vqhmm
    use_fb_kernel(monkeypatch, kernel)
    B, T = 6, 150
    rng = np.random.default_rng(K + 100)
    log_pi, log_A, em = random_hmm(K + 200, B, T, K)
    log_A = log_A.astype(np.float64)
    em = em.astype(np.float64)
    tri = np.triu(np.ones((K, K), bool))
    la = np.where(tri, log_A[0], -np.inf)
    log_A[0] = la - np.logaddexp.reduce(la, axis=-1, keepdims=True)   # b0: left-to-right
    em[1] = em[1] * 50.0 - 1000.0                                      # b1: huge negative emissions
    em[2, 40:60] *= 150.0                                              # b2: 300+ nat spread
    log_A[3] = log_softmax(rng.standard_normal((T, K, K)) * 80.0)      # b3: near-deterministic
    L = np.array([T, T, T, T, 77, 1], np.int64)
    log_A = log_A.astype(np.float32)
    em = em.astype(np.float32)
    gamma, logZ = vqhmm.forward_backward(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    with np.errstate(divide="ignore", invalid="ignore"):
        rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A, em, L)
    check_gamma(gamma.cpu().numpy(), rg)
    z = logZ.cpu().numpy()
    assert np.all(np.abs(z - rz) <= 1e-5 * np.maximum(1.0, np.abs(rz)))


@pytest.mark.parametrize("kernel", FB_KERNELS)
@pytest.mark.parametrize("K,spread", [(8, 10.0), (8, 35.0), (8, 90.0), (4, 35.0), (3, 90.0)])
def test_forward_backward_tier_fallbacks(K, spread, kernel, monkeypatch):
    """Emission spreads that keep the linear tier in range (10), push some states below
    2^-96 so chunks fall back to the base-2 log tier (35), or beyond its range too (90),
    mixed per sequence and per window, at T = 512 (16 chunks per wave)."""
    import vqhmm
    use_fb_kernel(monkeypatch, kernel)
    B, T = 5, 512
    log_pi, log_A, em = random_hmm(K * 3 + int(spread), B, T, K)
    em = em.astype(np.float64)
    em[1] *= spread
    em[2, 100:140] *= spread
    em[3, 300:] *= spread
    em = em.astype(np.float32)
    L = np.array([T, T, T, 400, 1], np.int64)
    gamma, logZ = vqhmm.forward_backward(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A, em, L)
    check_gamma(gamma.cpu().numpy(), rg)
    assert np.all(np.abs(logZ.cpu().numpy() - rz) <= 1e-5 * np.maximum(1.0, np.abs(rz)))


@pytest.mark.parametrize("K,B,T,L", [(8, 512, 512, "full"), (8, 300, 512, "ragged"), (5, 40, 1024, "ragged"),
                                     (8, 17, 1000, "ragged"), (7, 9, 130, "ragged"), (8, 5, 65, "ragged"),
                                     (6, 3, 64, "full"), (3, 33, 200, "ragged"), (1, 4, 300, "ragged")])
def test_forward_backward_segmented(K, B, T, L, monkeypatch):
    """The parallel-in-time kernel (hmm_seg.hip) against the fp64 oracle: the cfg4 shard shape (512 x 512,
    K = 8), ragged lengths that end inside, at and before segment boundaries (incl. 0 and 1), T not a
    multiple of 64, 16 segments (T = 1024), one segment (T = 64), K < 8 (padded lanes)."""
    import vqhmm
    monkeypatch.setenv("VQHMM_FB_SEG", "1")
    log_pi, log_A, em = random_hmm(K * 31 + B + T, B, T, K)
    if L == "full":
        Ls = np.full(B, T, np.int64)
    else:
        Ls = np.random.default_rng(T + B).integers(0, T + 1, B).astype(np.int64)
        Ls[0] = T
        Ls[1 % B] = 1
        for k, v in enumerate((64, 65, 63, 128, 0, 2)):
            if 2 + k < B:
                Ls[2 + k] = min(v, T)
    gamma, logZ = vqhmm.forward_backward(*gpu(log_pi, log_A, em), torch.from_numpy(Ls))
    sl = slice(0, B, max(1, B // 24))  # the fp64 oracle on a strided slice of the batch
    rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A[sl], em[sl], Ls[sl])
    check_gamma(gamma.cpu().numpy()[sl], rg)
    z = logZ.cpu().numpy()[sl]
    live = Ls[sl] > 0
    assert np.all(np.abs(z[live] - rz[live]) <= 1e-5 * np.maximum(1.0, np.abs(rz[live])))
    assert np.all(np.isnan(z[~live]))
    g = gamma.cpu().numpy()
    past = np.arange(T)[None, :] >= Ls[:, None]
    assert np.all(g[past] == 0)


@pytest.mark.parametrize("K,B,T", [(8, 300, 64), (4, 1100, 40), (8, 2, 560), (2, 3, 1000)])
def test_forward_backward_resident_boundaries(K, B, T, monkeypatch):
    """Shapes at the resident kernel's limits: several workgroups per CU (small T), batches
    near one round, and T past the LDS table (streaming kernel)."""
    import vqhmm
    monkeypatch.setenv("VQHMM_FB_SEG", "0")
    log_pi, log_A, em = random_hmm(K * 13 + B + T, B, T, K)
    L = np.random.default_rng(T).integers(0, T + 1, B).astype(np.int64)
    L[0] = T
    gamma, logZ = vqhmm.forward_backward(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A, em, L)
    check_gamma(gamma.cpu().numpy(), rg)
    live = L > 0
    z = logZ.cpu().numpy()
    assert np.all(np.abs(z[live] - rz[live]) <= 1e-5 * np.maximum(1.0, np.abs(rz[live])))


def test_gamma_sums_to_one_and_viterbi_on_model_tables():
    """Use the model's own Prior tables and encoder posteriors as inputs."""
    import vqhmm
    torch.manual_seed(0)
    m = vqhmm.VAE_HMM(5, 64, 3, 32, u_dim=4, trans_hidden=128).cuda()
    x = torch.randn(8, 5, 200, device="cuda")
    u = torch.randn(8, 4, 200, device="cuda")
    with torch.no_grad():
        log_pi, log_A = m.prior(u)
        em = torch.log_softmax(m.encode(x), dim=1).transpose(1, 2).contiguous()
    gamma, logZ = vqhmm.forward_backward(log_pi, log_A, em)
    assert torch.allclose(gamma.sum(-1), torch.ones(8, 200, device="cuda"), atol=1e-5)
    path, score = vqhmm.viterbi(log_pi, log_A, em)
    rp, rs = c_oracle.viterbi(log_pi.cpu().numpy(), log_A.cpu().numpy(), em.cpu().numpy(), np.full(8, 200))
    assert np.array_equal(path.cpu().numpy(), rp)


def test_viterbi_wide_ties():
    """K = 32 with all-equal tables: every step ties across all i; lowest index wins."""
    import vqhmm
    K, B, T = 32, 3, 40
    log_pi = np.zeros(K, np.float32)
    log_A = np.zeros((B, T, K, K), np.float32)
    em = np.zeros((B, T, K), np.float32)
    em[1, ::3, 20] = 1.0
    em[2, :, 17:] = 0.5  # ties inside the upper half only
    L = np.array([T, T, 7])
    path, score = vqhmm.viterbi(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    rp, rs = c_oracle.viterbi(log_pi, log_A, em, L)
    assert np.array_equal(path.cpu().numpy(), rp)
    assert np.array_equal(score.cpu().numpy(), rs)


@pytest.mark.parametrize("K,B,T", [(33, 4, 60), (48, 3, 41), (64, 5, 130), (100, 2, 33), (256, 2, 20)])
def test_hmm_generic_k_over_32(K, B, T):
    """32 < K <= 256 (hmm_generic.hip: one workgroup per sequence, thread = state): Viterbi path and
    score bit-exact vs the C oracle, gamma / logZ vs the fp64 oracle, ragged lengths incl. 0 and 1."""
    import vqhmm
    log_pi, log_A, em = random_hmm(K + B + T, B, T, K)
    L = np.random.default_rng(K).integers(1, T + 1, B).astype(np.int64)
    L[0] = T
    if B > 2:
        L[1] = 0
    path, score = vqhmm.viterbi(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    rp, rs = c_oracle.viterbi(log_pi, log_A, em, L)
    assert np.array_equal(path.cpu().numpy(), rp)
    assert np.array_equal(score.cpu().numpy().view(np.uint32), rs.view(np.uint32))
    gamma, logZ = vqhmm.forward_backward(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A, em, L)
    check_gamma(gamma.cpu().numpy(), rg)
    z = logZ.cpu().numpy()
    live = L > 0
    assert np.all(np.abs(z[live] - rz[live]) <= 1e-5 * np.maximum(1.0, np.abs(rz[live])))
    assert np.all(np.isnan(z[~live]))


def test_hmm_generic_left_to_right():
    """K = 40 with left-to-right transitions (log 0 = -inf below the diagonal) and T = 300."""
    import vqhmm
    K, B, T = 40, 2, 300
    log_pi, log_A, em = random_hmm(3, B, T, K)
    tri = np.triu(np.ones((K, K), bool))
    la = np.where(tri, log_A.astype(np.float64), -np.inf)
    log_A = (la - np.logaddexp.reduce(la, axis=-1, keepdims=True)).astype(np.float32)
    path, score = vqhmm.viterbi(*gpu(log_pi, log_A, em))
    rp, rs = c_oracle.viterbi(log_pi, log_A, em, np.full(B, T))
    assert np.array_equal(path.cpu().numpy(), rp)
    gamma, logZ = vqhmm.forward_backward(*gpu(log_pi, log_A, em))
    with np.errstate(divide="ignore", invalid="ignore"):
        rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A, em, np.full(B, T))
    check_gamma(gamma.cpu().numpy(), rg)
    assert np.all(np.abs(logZ.cpu().numpy() - rz) <= 1e-5 * np.abs(rz))


@pytest.mark.parametrize("K,B,T", [(257, 2, 9), (300, 3, 12), (600, 2, 7), (1100, 2, 4)])
def test_hmm_generic_k_over_256(K, B, T):
    """K > 256 (hmm_generic.hip with several states per thread, 16-bit backpointers): Viterbi bit-exact vs the
    C oracle, gamma / logZ vs the fp64 oracle, ragged lengths (the API takes any (B, T, K))."""
    import vqhmm
    log_pi, log_A, em = random_hmm(K + B + T, B, T, K)
    L = np.full(B, T, np.int64)
    L[-1] = T - 2
    path, score = vqhmm.viterbi(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    rp, rs = c_oracle.viterbi(log_pi, log_A, em, L)
    assert np.array_equal(path.cpu().numpy(), rp)
    assert np.array_equal(score.cpu().numpy().view(np.uint32), rs.view(np.uint32))
    gamma, logZ = vqhmm.forward_backward(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A, em, L)
    check_gamma(gamma.cpu().numpy(), rg)
    assert np.all(np.abs(logZ.cpu().numpy() - rz) <= 1e-5 * np.maximum(1.0, np.abs(rz)))


def test_hmm_k_over_4096_rejected():
    import vqhmm
    K, B, T = 4097, 1, 1
    log_pi, log_A, em = random_hmm(1, B, T, K)
    with pytest.raises(RuntimeError, match="unsupported"):
        vqhmm.viterbi(*gpu(log_pi, log_A, em))


@pytest.mark.parametrize("kernel", FB_KERNELS)
@pytest.mark.parametrize("K,T", [(4, 60), (8, 90), (16, 70), (48, 40)])
def test_forward_backward_impossible_sequence(K, T, kernel, monkeypatch):
    """A sequence with zero probability (every emission -inf at one step): logZ = -inf for it, as the
    fp64 oracle gives, and the batch's other sequences are unaffected (the K > 32 kernel used to
    turn -inf - -inf into a NaN logZ).  Its gamma (0 / 0: NaN in the oracle) is not a contract: the K <= 8
    and K > 32 kernels give NaN, the 8 < K <= 32 one does not."""
    import vqhmm
    use_fb_kernel(monkeypatch, kernel)
    B = 3
    log_pi, log_A, em = random_hmm(K * 5 + T, B, T, K)
    em[1, T // 3, :] = -np.inf
    L = np.array([T, T, T - 7], np.int64)
    gamma, logZ = vqhmm.forward_backward(*gpu(log_pi, log_A, em), torch.from_numpy(L))
    with np.errstate(divide="ignore", invalid="ignore"):
        rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A, em, L)
    g, z = gamma.cpu().numpy(), logZ.cpu().numpy()
    assert z[1] == -np.inf and rz[1] == -np.inf
    ok = [0, 2]
    check_gamma(g[ok], rg[ok])
    assert np.all(np.abs(z[ok] - rz[ok]) <= 1e-5 * np.maximum(1.0, np.abs(rz[ok])))


def test_forward_backward_segmented_tiers(monkeypatch):
    """Which path the parallel-in-time kernel takes per sequence: the linear fast path leaves the workspace
    untouched (it keeps both histories in LDS), the exact path writes the sequence's alpha / beta there.
    Model-like tables (log_softmax of N(0,1)) must take the fast path; the extreme ones (left-to-right
    -inf transitions, -1e3-nat emissions, 300-nat spreads, near-deterministic transitions) the exact path,
    and both give gamma / logZ within the contract."""
    import vqhmm
    from vqhmm import _ext
    monkeypatch.setenv("VQHMM_FB_SEG", "1")
    B, T, K = 6, 300, 8
    rng = np.random.default_rng(77)
    log_pi, log_A, em = random_hmm(78, B, T, K, scale=1.0)
    log_A = log_A.astype(np.float64)
    em = em.astype(np.float64)
    tri = np.triu(np.ones((K, K), bool))
    la = np.where(tri, log_A[1], -np.inf)
    log_A[1] = la - np.logaddexp.reduce(la, axis=-1, keepdims=True)   # b1: left-to-right
    em[2] = em[2] * 50.0 - 1000.0                                      # b2: huge negative emissions
    em[3, 100:120] *= 150.0                                            # b3: 300+ nat spread
    log_A[4] = log_softmax(rng.standard_normal((T, K, K)) * 80.0)      # b4: near-deterministic
    log_A, em = log_A.astype(np.float32), em.astype(np.float32)
    L = np.array([T, T, T, T, T, 200], np.int64)
    lp, lA, e, Lt = (*gpu(log_pi, log_A, em), torch.from_numpy(L).cuda())
    gamma = torch.empty(B, T, K, device="cuda")
    logZ = torch.empty(B, device="cuda")
    lib = _ext.load()
    nb = lib.vqhmm_fwdbwd_workspace_size(B, T, K)
    ws = torch.full((nb // 4,), float("nan"), device="cuda")
    _ext.check(lib.vqhmm_fwdbwd_f32(_ext.ptr(lp), _ext.ptr(lA), _ext.ptr(e), _ext.ptr(Lt), B, T, K, _ext.ptr(gamma),
                                    _ext.ptr(logZ), _ext.ptr(ws), nb, _ext.stream_ptr()), "forward_backward")
    al = ws[: B * T * K].view(B, T, K).cpu().numpy()
    touched = ~np.isnan(al).all(axis=(1, 2))
    assert list(touched) == [False, True, True, True, True, False], touched
    with np.errstate(divide="ignore", invalid="ignore"):
        rg, rz = hmm_ref.forward_backward_f64(log_pi, log_A, em, L)
    check_gamma(gamma.cpu().numpy(), rg)
    z = logZ.cpu().numpy()
    assert np.all(np.abs(z - rz) <= 1e-5 * np.maximum(1.0, np.abs(rz)))
