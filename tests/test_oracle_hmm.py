"""Pin the VQ / forward-backward / Viterbi oracles (no reference code exists for
them) with known-answer tests:
  * brute-force enumeration of all K^L state paths (K <= 4, L <= 7) for logZ,
    gamma and the MAP path;
  * the numpy fp32 Viterbi and the C fp32 Viterbi agree bit-for-bit;
  * the one-hot-codebook identity argmin_k ||q - e_k||^2 == argmax_k q used by
    the reference's hard regimes (backtesting.py:154-155);
  * C fmaf-chain VQ argmin agrees with a float64 argmin away from near-ties.
"""
import numpy as np
import pytest

from oracle import c_oracle, hmm_ref


def log_softmax(a, axis=-1):
    m = a.max(axis=axis, keepdims=True)
    return a - m - np.log(np.exp(a - m).sum(axis=axis, keepdims=True))


def random_hmm(rng, B, T, K, dtype=np.float32):
    log_pi = log_softmax(rng.standard_normal(K)).astype(dtype)
    log_A = log_softmax(rng.standard_normal((B, T, K, K)) * 1.5).astype(dtype)
    em = log_softmax(rng.standard_normal((B, T, K)) * 2.0).astype(dtype)
    return log_pi, log_A, em


@pytest.mark.parametrize("K,T", [(2, 7), (3, 6), (4, 5)])
def test_brute_force_kat(K, T):
    rng = np.random.default_rng(K * 100 + T)
    B = 5
    log_pi, log_A, em = random_hmm(rng, B, T, K)
    lengths = np.array([T, T - 1, 1, 3, T], np.int64)
    gamma, logZ = hmm_ref.forward_backward_f64(log_pi, log_A, em, lengths)
    path_np, score_np = hmm_ref.viterbi_f32(log_pi, log_A, em, lengths)
    path_c, score_c = c_oracle.viterbi(log_pi, log_A, em, lengths)
    assert np.array_equal(path_np, path_c)
    assert np.array_equal(score_np, score_c)
    for b in range(B):
        n = int(lengths[b])
        bz, bg, bpath, bscore = hmm_ref.brute_force(log_pi, log_A[b], em[b], n)
        assert abs(logZ[b] - bz) <= 1e-12 * max(1.0, abs(bz))
        assert np.abs(gamma[b, :n] - bg).max() <= 1e-12
        assert np.all(gamma[b, n:] == 0)
        assert tuple(path_c[b, :n]) == bpath
        assert np.all(path_c[b, n:] == -1)
        assert abs(float(score_c[b]) - bscore) <= 1e-5 * max(1.0, abs(bscore))


def test_gamma_identities():
    rng = np.random.default_rng(3)
    log_pi, log_A, em = random_hmm(rng, 4, 40, 5)
    lengths = np.array([40, 17, 1, 39])
    gamma, logZ = hmm_ref.forward_backward_f64(log_pi, log_A, em, lengths)
    for b, n in enumerate(lengths):
        assert np.allclose(gamma[b, :n].sum(-1), 1.0, atol=1e-12)


def test_viterbi_ties_lowest_index():
    K, T = 3, 6
    log_pi = np.zeros(K, np.float32)
    log_A = np.zeros((1, T, K, K), np.float32)
    em = np.zeros((1, T, K), np.float32)
    path, score = c_oracle.viterbi(log_pi, log_A, em, np.array([T]))
    assert np.all(path == 0) and score[0] == 0.0
    p2, s2 = hmm_ref.viterbi_f32(log_pi, log_A, em, np.array([T]))
    assert np.array_equal(path, p2)


def test_viterbi_zero_length():
    rng = np.random.default_rng(0)
    log_pi, log_A, em = random_hmm(rng, 2, 5, 3)
    path, score = c_oracle.viterbi(log_pi, log_A, em, np.array([0, 5]))
    assert np.all(path[0] == -1) and np.isneginf(score[0])


def test_vq_one_hot_identity():
    rng = np.random.default_rng(1)
    B, K, T = 4, 6, 50
    logits = rng.standard_normal((B, K, T)).astype(np.float32)
    q = np.exp(log_softmax(logits, axis=1)).astype(np.float32)
    idx = c_oracle.vq_argmin(q, np.eye(K, dtype=np.float32), want_dmin=False)
    assert np.array_equal(idx, q.argmax(axis=1))


def test_vq_matches_float64_away_from_ties():
    rng = np.random.default_rng(2)
    B, Dv, T, K = 3, 16, 70, 12
    z = rng.standard_normal((B, Dv, T)).astype(np.float32)
    cb = rng.standard_normal((K, Dv)).astype(np.float32)
    idx, dmin = c_oracle.vq_argmin(z, cb)
    idx64, d64 = hmm_ref.vq_argmin_np(z, cb)
    assert np.abs(dmin - d64).max() <= 1e-5 * d64.max()
    # disagreements only where the best two float64 distances nearly tie
    d_all = ((z[:, None].astype(np.float64) - cb[None, :, :, None]) ** 2).sum(2)
    srt = np.sort(d_all, axis=1)
    gap = srt[:, 1] - srt[:, 0]
    assert np.all((idx == idx64) | (gap < 1e-4))


def test_vq_ties_lowest_index():
    z = np.zeros((1, 2, 3), np.float32)
    cb = np.array([[1, 0], [0, 1], [-1, 0]], np.float32)  # all at distance 1
    idx = c_oracle.vq_argmin(z, cb, want_dmin=False)
    assert np.all(idx == 0)
