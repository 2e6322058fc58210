"""Hard-regime kernels: VQ nearest-codeword argmin, HMM forward-backward and
Viterbi over the Prior's tables.  HIP only (libvqhmm.so).

The reference defines these only in prose:
  VQ         pseudocode.txt:11-18 (`quantize`), hard regimes backtesting.py:154-155
  fwd-bwd    math.md:23-67 with Prior.forward tables (VQ_VAE_HMM_fixed.py:59-71)
  Viterbi    same tables, max-plus
The exact numerical contracts are documented in include/vqhmm.h.
"""
import torch

from . import _ext


def vq_argmin(z, codebook, return_dist=False):
    """z (B, Dv, T) channels-first, codebook (K, Dv) -> idx (B, T) int32 [, dmin (B, T)].

    idx[b, t] = argmin_k sum_d (z[b, d, t] - codebook[k, d])^2, ties -> lowest k.
    """
    _ext.require_device(z, codebook)
    if z.dim() != 3 or codebook.dim() != 2 or z.shape[1] != codebook.shape[1]:
        raise ValueError(f"vq_argmin: expected z (B,Dv,T) and codebook (K,Dv), got {tuple(z.shape)} {tuple(codebook.shape)}")
    z = z.contiguous().float()
    codebook = codebook.contiguous().float()
    B, Dv, T = z.shape
    K = codebook.shape[0]
    idx = torch.empty((B, T), dtype=torch.int32, device=z.device)
    dmin = torch.empty((B, T), dtype=torch.float32, device=z.device) if return_dist else None
    lib = _ext.load()
    _ext.check(lib.vqhmm_vq_argmin_f32(_ext.ptr(z), B, Dv, T, _ext.ptr(codebook), K, _ext.ptr(idx),
                                       _ext.ptr(dmin), _ext.stream_ptr(z.device)), "vq_argmin")
    return (idx, dmin) if return_dist else idx


def regime_argmax(q):
    """q (B, K, T) -> (B, T) int64: q.argmax(dim=1) by torch.argmax's rule (first index on
    ties, NaN is the maximum), the hard regimes of backtesting.py:154-155 on given probabilities."""
    _ext.require_device(q)
    if q.dim() != 3:
        raise ValueError(f"regime_argmax: expected q (B, K, T), got {tuple(q.shape)}")
    q = q.contiguous().float()
    B, K, T = q.shape
    idx = torch.empty((B, T), dtype=torch.int32, device=q.device)
    _ext.check(_ext.load().vqhmm_argmax_f32(_ext.ptr(q), B, K, T, _ext.ptr(idx), _ext.stream_ptr(q.device)),
               "regime_argmax")
    return idx.long()


def quantize(z, codebook, beta=0.25):
    """VQ-VAE quantizer of pseudocode.txt:11-18 on channels-first z (B, Dv, T).

    Returns (z_q_st, idx, commit_loss, codebook_loss):
      z_q = codebook[idx] (B, Dv, T); z_q_st = z + (z_q - z).detach() (straight-through, :12);
      commit = beta * MSE(z, sg(z_q)) (:16); codebook = MSE(z_q, sg(z)) (:17).
    The argmin is the HIP kernel; the gather/MSE are small elementwise ops on
    its output.
    """
    idx = vq_argmin(z.detach(), codebook.detach())
    z_q = codebook[idx.long()].permute(0, 2, 1)
    z_q_st = z + (z_q - z).detach()
    commit = beta * torch.mean((z - z_q.detach()) ** 2)
    cb_loss = torch.mean((z_q - z.detach()) ** 2)
    return z_q_st, idx, commit, cb_loss


def _hmm_inputs(log_pi, log_A, em, lengths):
    _ext.require_device(log_pi, log_A, em)
    if log_A.dim() != 4 or em.dim() != 3 or log_A.shape[:2] != em.shape[:2] or log_A.shape[2:] != (em.shape[2],) * 2:
        raise ValueError(f"expected log_A (B,T,K,K) and em (B,T,K), got {tuple(log_A.shape)} {tuple(em.shape)}")
    B, T, K = em.shape
    if log_pi.shape != (K,):
        raise ValueError(f"log_pi must have shape ({K},)")
    if lengths is None:
        lengths = torch.full((B,), T, dtype=torch.int64, device=em.device)
    lengths = torch.as_tensor(lengths).to(em.device, torch.int64).contiguous()
    return (log_pi.contiguous().float(), log_A.contiguous().float(), em.contiguous().float(), lengths, B, T, K)


def viterbi(log_pi, log_A, em, lengths=None):
    """MAP state path under the Prior's tables.

    log_pi (K,), log_A (B,T,K,K) with log_A[:, t] the t-1 -> t transition
    (as Prior.forward returns it, VQ_VAE_HMM_fixed.py:69-71), em (B,T,K)
    emission log-potentials, lengths (B,) -> path (B,T) int32 (-1 past the
    length), score (B,) fp32.  Bit-exact vs the fp32 oracle contract.
    """
    log_pi, log_A, em, lengths, B, T, K = _hmm_inputs(log_pi, log_A, em, lengths)
    path = torch.empty((B, T), dtype=torch.int32, device=em.device)
    score = torch.empty((B,), dtype=torch.float32, device=em.device)
    lib = _ext.load()
    nb = lib.vqhmm_viterbi_workspace_size(B, T, K)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=em.device)
    _ext.check(lib.vqhmm_viterbi_f32(_ext.ptr(log_pi), _ext.ptr(log_A), _ext.ptr(em), _ext.ptr(lengths), B, T, K,
                                     _ext.ptr(path), _ext.ptr(score), _ext.ptr(ws), nb, _ext.stream_ptr(em.device)),
               "viterbi")
    return path, score


def forward_backward(log_pi, log_A, em, lengths=None):
    """Posterior state marginals gamma (B,T,K) and log-partition logZ (B,)."""
    log_pi, log_A, em, lengths, B, T, K = _hmm_inputs(log_pi, log_A, em, lengths)
    gamma = torch.empty((B, T, K), dtype=torch.float32, device=em.device)
    logZ = torch.empty((B,), dtype=torch.float32, device=em.device)
    lib = _ext.load()
    nb = lib.vqhmm_fwdbwd_workspace_size(B, T, K)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=em.device)
    _ext.check(lib.vqhmm_fwdbwd_f32(_ext.ptr(log_pi), _ext.ptr(log_A), _ext.ptr(em), _ext.ptr(lengths), B, T, K,
                                    _ext.ptr(gamma), _ext.ptr(logZ), _ext.ptr(ws), nb, _ext.stream_ptr(em.device)),
               "forward_backward")
    return gamma, logZ
