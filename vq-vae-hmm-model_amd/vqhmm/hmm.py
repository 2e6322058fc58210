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


class _Quantize(torch.autograd.Function):
    """Forward: ONE fused kernel pass (vqhmm_vq_quantize_f32: argmin, z_q gather, straight-through
    value, sum (z - z_q)^2 in fp64) + a fixed-order partial sum.  Backward (autograd of
    pseudocode.txt:13,17-18): the straight-through output passes its gradient to z unchanged;
    commit = beta * sse / n adds beta * 2 (z - z_q) / n to dz; the codebook loss sse / n gives
    dcodebook[k] = sum over positions with idx = k of 2 (z_q - z) / n."""

    @staticmethod
    def forward(ctx, z, codebook, beta):
        B, Dv, T = z.shape
        K = codebook.shape[0]
        idx = torch.empty((B, T), dtype=torch.int32, device=z.device)
        zq_st = torch.empty_like(z)
        sse = torch.zeros((), dtype=torch.float64, device=z.device)
        lib = _ext.load()
        nb = lib.vqhmm_vq_quantize_workspace_size(B, Dv, T, K)
        ws = torch.empty(max(nb, 8), dtype=torch.uint8, device=z.device)
        _ext.check(lib.vqhmm_vq_quantize_f32(_ext.ptr(z), B, Dv, T, _ext.ptr(codebook), K, _ext.ptr(idx),
                                             _ext.ptr(zq_st), _ext.ptr(sse), _ext.ptr(ws), ws.numel(),
                                             _ext.stream_ptr(z.device)), "quantize")
        n = float(max(z.numel(), 1))
        mse = (sse / n).float()
        ctx.save_for_backward(z, codebook, idx)
        ctx.beta, ctx.n = float(beta), n
        ctx.mark_non_differentiable(idx)
        return zq_st, idx, beta * mse, mse

    @staticmethod
    def backward(ctx, g_zq, g_idx, g_commit, g_cb):
        z, codebook, idx = ctx.saved_tensors
        dz = dcb = None
        zq = codebook[idx.long()].permute(0, 2, 1)  # (B, Dv, T)
        diff = z - zq
        if ctx.needs_input_grad[0]:
            dz = g_zq if g_zq is not None else torch.zeros_like(z)
            if g_commit is not None:
                dz = dz + g_commit * (ctx.beta * 2.0 / ctx.n) * diff
        if ctx.needs_input_grad[1] and g_cb is not None:
            w = (g_cb * (-2.0 / ctx.n)) * diff  # d cb_loss / d z_q
            dcb = torch.zeros_like(codebook).index_add_(0, idx.long().reshape(-1),
                                                        w.permute(0, 2, 1).reshape(-1, codebook.shape[1]))
        return dz, dcb, None


def quantize(z, codebook, beta=0.25):
    """VQ-VAE quantizer of pseudocode.txt:11-18 on channels-first z (B, Dv, T).

    Returns (z_q_st, idx, commit_loss, codebook_loss):
      idx = argmin_k ||z - c_k||^2 (the vq_argmin contract); z_q = codebook[idx];
      z_q_st = z + (z_q - z).detach() (straight-through, :13); commit = beta * MSE(z, sg(z_q)) (:17);
      codebook = MSE(z_q, sg(z)) (:18).
    The forward is one HIP pass (argmin + gather + straight-through value + the squared-error
    partial sums in the kernel's epilogue); the gradients follow the reference's autograd.
    """
    _ext.require_device(z, codebook)
    if z.dim() != 3 or codebook.dim() != 2 or z.shape[1] != codebook.shape[1]:
        raise ValueError(f"quantize: expected z (B,Dv,T) and codebook (K,Dv), got {tuple(z.shape)} "
                         f"{tuple(codebook.shape)}")
    return _Quantize.apply(z.contiguous().float(), codebook.contiguous().float(), float(beta))


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
