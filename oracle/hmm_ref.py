"""numpy restatement of the three hot-path kernels the reference specifies only
in prose — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Semantic sources (no reference code exists for these):
  VQ argmin        pseudocode.txt:11-18 (quantize / straight-through / commit
                   + codebook MSE); hard-regime argmax backtesting.py:154-155.
  forward-backward math.md:23-67 (pi, row-stochastic A_t conditioned on u_t);
                   tables from Prior.forward VQ_VAE_HMM_fixed.py:59-71 with
                   log_A[:, t] = transition t-1 -> t (:125-127; t=0 unused).
  Viterbi          same tables, max-plus instead of log-sum-exp.

Exact contracts (the HIP kernels follow them operation for operation):
  vq_argmin  expansion form ||z||^2 + ||c_k||^2 - 2 z.c_k, evaluated as
             cn[k]   = fmaf chain over d = 0..Dv-1 of c[k,d]^2 from +0.0f,
             s[n,k]  = fmaf chain over d = 0..Dv-1 of z[n,d]*(-2 c[k,d])
                       starting from cn[k]  (what a f32 MFMA computes),
             idx     = first k with the smallest s (ties -> lowest k),
             dmin    = s[n,idx] + ((q0 + q1) + (q2 + q3)), q_r = fmaf chain
                       of z^2 over the d = r (mod 4).
             (fmaf is exact in the C oracle, oracle/c/hmm_oracle.c; the
             pure-numpy `vq_argmin_np` uses float64 and is only used for KATs.)
  viterbi    d0[j] = log_pi[j] + e[0,j];
             d_t[j] = (max_i (d_{t-1}[i] + log_A[t,i,j])) + e[t,j]   (fp32,
             i ascending, strict '>' so ties keep the lowest i);
             last = first argmax_j d_{L-1}[j]; path[t >= L] = -1;
             score = d_{L-1}[last]; L = 0 -> path all -1, score = -inf.
  fwd-bwd    log-space alpha/beta; gamma_t = softmax(alpha_t + beta_t) for
             t < L, 0 beyond; logZ = LSE_j alpha_{L-1}[j]  (fp64 reference).
"""
import itertools

import numpy as np


# ----------------------------------------------------------------- VQ argmin
def vq_argmin_np(z, codebook):
    """z (B,Dv,T), codebook (K,Dv) -> idx (B,T) int32 (float64 distances; KAT use)."""
    z = np.asarray(z, np.float64)
    c = np.asarray(codebook, np.float64)
    d = ((z[:, None, :, :] - c[None, :, :, None]) ** 2).sum(axis=2)  # (B,K,T)
    return d.argmin(axis=1).astype(np.int32), d.min(axis=1)


def quantize_f32(z, codebook, idx, beta=0.25):
    """pseudocode.txt:11-18 in fp32 numpy on channels-first z (B, Dv, T), given the
    argmin indices idx (B, T) (c_oracle.vq_argmin: the kernel contract):
      z_q      = codebook[idx]                         (quantize, :12)
      z_q_st   = z + (z_q - z)   [value of z_e + (z_q - z_e).detach(), :13]
      commit   = beta * mean((z - z_q)^2)               (:17)
      cb_loss  = mean((z_q - z)^2)                      (:18)
    and the gradients autograd gives them for a loss sum(w * z_q_st) + commit + cb_loss:
      dz        = w + beta * 2 (z - z_q) / N            (ST passes w straight through)
      dcodebook = sum over positions n with idx = k of 2 (z_q - z)_n / N
    with N = z.size.  Returns a dict of float32 / float64 arrays."""
    z = np.asarray(z, np.float32)
    c = np.asarray(codebook, np.float32)
    idx = np.asarray(idx, np.int64)
    zq = np.transpose(c[idx], (0, 2, 1)).astype(np.float32)      # (B, Dv, T)
    zq_st = (z + (zq - z)).astype(np.float32)
    d = (z.astype(np.float64) - zq.astype(np.float64))
    n = z.size
    commit = beta * (d ** 2).mean()
    cb_loss = (d ** 2).mean()
    return {"z_q": zq, "z_q_st": zq_st, "commit": commit, "codebook": cb_loss,
            "dz_extra": beta * 2.0 * d / n,
            "dcodebook": np.stack([(-2.0 * d / n).transpose(1, 0, 2)[:, idx == k].sum(axis=1)
                                   for k in range(c.shape[0])])}


# ------------------------------------------------------------------- Viterbi
def viterbi_f32(log_pi, log_A, em, lengths):
    """fp32 max-plus Viterbi with the exact op order of the contract above.

    log_pi (K,), log_A (B,T,K,K), em (B,T,K), lengths (B,) -> path (B,T) int32, score (B,) f32
    """
    log_pi = np.asarray(log_pi, np.float32)
    log_A = np.asarray(log_A, np.float32)
    em = np.asarray(em, np.float32)
    B, T, K = em.shape
    L = np.minimum(np.asarray(lengths, np.int64), T)
    path = np.full((B, T), -1, np.int32)
    score = np.full(B, -np.inf, np.float32)
    if T == 0:
        return path, score
    bp = np.zeros((B, T, K), np.int8)
    delta = (log_pi[None, :] + em[:, 0, :]).astype(np.float32)
    hist = [delta.copy()]
    for t in range(1, T):
        best = delta[:, 0, None] + log_A[:, t, 0, :]         # (B,K) fp32
        arg = np.zeros((B, K), np.int8)
        for i in range(1, K):
            v = delta[:, i, None] + log_A[:, t, i, :]
            gt = v > best
            best = np.where(gt, v, best)
            arg = np.where(gt, np.int8(i), arg)
        nd = (best + em[:, t, :]).astype(np.float32)
        live = (t < L)[:, None]
        delta = np.where(live, nd, delta)
        bp[:, t] = arg
        hist.append(delta.copy())
    for b in range(B):
        n = int(L[b])
        if n <= 0:
            continue
        dl = hist[n - 1][b]
        s = int(np.argmax(dl))  # first maximum
        score[b] = dl[s]
        path[b, n - 1] = s
        for t in range(n - 1, 0, -1):
            s = int(bp[b, t, s])
            path[b, t - 1] = s
    return path, score


# ---------------------------------------------------------- forward-backward
def _lse(a, axis):
    m = np.max(a, axis=axis, keepdims=True)
    m = np.where(np.isfinite(m), m, 0.0)
    return (m + np.log(np.sum(np.exp(a - m), axis=axis, keepdims=True))).squeeze(axis)


def forward_backward_f64(log_pi, log_A, em, lengths):
    """fp64 log-space alpha/beta.  Returns gamma (B,T,K) f64, logZ (B,) f64."""
    log_pi = np.asarray(log_pi, np.float64)
    log_A = np.asarray(log_A, np.float64)
    em = np.asarray(em, np.float64)
    B, T, K = em.shape
    L = np.minimum(np.asarray(lengths, np.int64), T)
    alpha = np.zeros((B, T, K))
    beta = np.zeros((B, T, K))
    alpha[:, 0] = log_pi[None] + em[:, 0]
    for t in range(1, T):
        alpha[:, t] = _lse(alpha[:, t - 1, :, None] + log_A[:, t], axis=1) + em[:, t]
    for t in range(T - 2, -1, -1):
        nxt = beta[:, t + 1] + em[:, t + 1]                       # (B,K) over j
        cand = _lse(log_A[:, t + 1] + nxt[:, None, :], axis=2)     # (B,K) over i
        live = (t + 1 < L)[:, None]
        beta[:, t] = np.where(live, cand, 0.0)
    logZ = np.full(B, np.nan)
    gamma = np.zeros((B, T, K))
    for b in range(B):
        n = int(L[b])
        if n <= 0:
            continue
        logZ[b] = _lse(alpha[b, n - 1], axis=0)
        g = alpha[b, :n] + beta[b, :n] - logZ[b]
        gamma[b, :n] = np.exp(g)
    return gamma, logZ


# ------------------------------------------------------ brute-force pinning
def brute_force(log_pi, log_A, em, length):
    """Enumerate all K^L paths of ONE sequence (small K, L only).

    Returns (logZ, gamma (L,K), best_path tuple, best_score) in float64.
    The MAP path is the lexicographically-first among exact-score ties.
    """
    log_pi = np.asarray(log_pi, np.float64)
    log_A = np.asarray(log_A, np.float64)
    em = np.asarray(em, np.float64)
    K = em.shape[-1]
    L = int(length)
    scores, paths = [], []
    for z in itertools.product(range(K), repeat=L):
        s = log_pi[z[0]] + em[0, z[0]]
        for t in range(1, L):
            s += log_A[t, z[t - 1], z[t]] + em[t, z[t]]
        scores.append(s)
        paths.append(z)
    scores = np.array(scores)
    m = scores.max()
    logZ = m + np.log(np.exp(scores - m).sum())
    w = np.exp(scores - logZ)
    gamma = np.zeros((L, K))
    for wi, z in zip(w, paths):
        for t in range(L):
            gamma[t, z[t]] += wi
    bi = int(np.argmax(scores))
    return logZ, gamma, paths[bi], scores[bi]
