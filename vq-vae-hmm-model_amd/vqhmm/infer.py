"""Eval path on the fused kernels.

  infer(model, x)           POST /infer of inference_api/app.py:56-73 without the
                            web server: x [C][T] -> {'mu', 'logvar', 'regime_probs'}
                            lists, through the fused forward (vqhmm_forward_f32:
                            encode -> softmax -> decode, one call).
  hard_regimes(model, x)    backtesting.py:154-155: softmax(encode(x)).argmax(dim=1),
                            one fused pass (vqhmm_regimes_f32: the to_logits epilogue
                            computes q and its first argmax, torch.argmax's rule).
  viterbi_regimes(...)      MAP state path under the Prior's tables with the encoder
                            posterior as emission (log_softmax(logits)).
  prior_viterbi(...)        Viterbi over Prior.forward's tables computed on the chip from u
                            (vqhmm_prior_viterbi_f32): log_A never touches HBM;
                            bit-identical to viterbi(*model.prior(u), em).
"""
import ctypes

import torch

from . import _ext
from .hmm import viterbi


def _device(model):
    return next(model.parameters()).device


def infer(model, x):
    """x: [C][T] nested list (or (C, T) tensor) -> dict of lists, as app.py returns."""
    xt = torch.as_tensor(x, dtype=torch.float32).unsqueeze(0).to(_device(model))
    with torch.no_grad():
        (mu, logvar), q = model(xt)
    return {"mu": mu.squeeze(0).cpu().tolist(), "logvar": logvar.squeeze(0).cpu().tolist(),
            "regime_probs": q.squeeze(0).cpu().tolist()}


def hard_regimes(model, x):
    """x (B, C, T) on the device -> (regimes (B, T) int64, q (B, K, T)).

    regimes == q.argmax(dim=1) bit for bit (first index on ties, NaN counts as the
    maximum), computed in the same epilogue that produces q."""
    _ext.require_device(x)
    enc = model.encoder if hasattr(model, "encoder") else model
    if x.dim() != 3 or x.shape[1] != enc.conv1.weight.shape[1]:
        raise RuntimeError(f"hard_regimes: expected x (B, {enc.conv1.weight.shape[1]}, T), got {tuple(x.shape)}")
    x = x.contiguous().float()
    B, _, T = x.shape
    d = enc._dims()
    q = torch.empty((B, d.K, T), device=x.device)
    reg = torch.empty((B, T), dtype=torch.int32, device=x.device)
    if B * T:
        from .model import _ptr_array
        lib = _ext.load()
        nb = ctypes.c_size_t()
        _ext.check(lib.vqhmm_infer_workspace_size(ctypes.byref(d), B, T, ctypes.byref(nb)), "workspace")
        ws = torch.empty(nb.value, dtype=torch.uint8, device=x.device)
        w = [None] * _ext.NPARAMS
        w[0:6] = [enc.conv1.weight, enc.conv1.bias, enc.conv2.weight, enc.conv2.bias, enc.to_logits.weight,
                  enc.to_logits.bias]
        with torch.no_grad():
            _ext.check(lib.vqhmm_regimes_f32(ctypes.byref(d), _ptr_array([t.detach() if t is not None else None
                                                                           for t in w]),
                                             _ext.ptr(x), B, T, _ext.ptr(q), _ext.ptr(reg), _ext.ptr(ws), nb.value,
                                             _ext.stream_ptr(x.device)), "hard_regimes")
    return reg.long(), q


def prior_viterbi(prior, u, em, lengths=None):
    """viterbi(*prior(u), em, lengths) without materialising log_A: the fused
    Prior-MLP -> Viterbi kernel (K <= 8, u_dim <= 4, trans_hidden in {64, 128, 256}).
    Returns None when the dims are outside the fused kernel's range (the caller then
    runs prior + viterbi, both native)."""
    _ext.require_device(u, em)
    lay = prior.u_layout(u)
    u = u.contiguous().float()
    B = u.shape[0]
    T = u.shape[2] if lay == 0 else u.shape[1]
    K = prior.K
    if em.shape != (B, T, K):
        raise ValueError(f"expected em (B,T,K) = ({B},{T},{K}), got {tuple(em.shape)}")
    em = em.contiguous().float()
    if lengths is None:
        lengths = torch.full((B,), T, dtype=torch.int64, device=em.device)
    lengths = torch.as_tensor(lengths).to(em.device, torch.int64).contiguous()
    lin0, lin2 = prior.transition_net[0], prior.transition_net[2]
    d = _ext.Dims(1, 1, K, 1, prior.u_dim, lin0.weight.shape[0])
    path = torch.empty((B, T), dtype=torch.int32, device=em.device)
    score = torch.empty((B,), dtype=torch.float32, device=em.device)
    lib = _ext.load()
    nb = lib.vqhmm_prior_viterbi_workspace_size(ctypes.byref(d), B, T)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=em.device)
    from .model import _ptr_array
    w = [None] * _ext.NPARAMS
    w[6:11] = [prior.log_prior, lin0.weight, lin0.bias, lin2.weight, lin2.bias]
    with torch.no_grad():
        rc = lib.vqhmm_prior_viterbi_f32(ctypes.byref(d), _ptr_array([t.detach() if t is not None else None
                                                                      for t in w]),
                                         _ext.ptr(u), lay, _ext.ptr(em), _ext.ptr(lengths), B, T, _ext.ptr(path),
                                         _ext.ptr(score), _ext.ptr(ws), nb, _ext.stream_ptr(em.device))
    if rc == _ext.EUNSUPPORTED:
        return None
    _ext.check(rc, "prior_viterbi")
    return path, score


def viterbi_regimes(model, x, u, lengths=None, fused=True):
    """MAP regime path (B, T) int32 (-1 past each length) and its score (B,).
    fused: Prior MLP inside the Viterbi kernel (prior_viterbi) where its dims allow;
    otherwise Prior.forward writes log_A and viterbi reads it (same bits either way)."""
    with torch.no_grad():
        em = torch.log_softmax(model.encode(x), dim=1).transpose(1, 2).contiguous()
        if fused:
            r = prior_viterbi(model.prior, u, em, lengths)
            if r is not None:
                return r
        log_pi, log_A = model.prior(u)
        return viterbi(log_pi, log_A, em, lengths)
