"""Eval path on the fused kernels.

  infer(model, x)           POST /infer of inference_api/app.py:56-73 without the
                            web server: x [C][T] -> {'mu', 'logvar', 'regime_probs'}
                            lists, through the fused forward (vqhmm_forward_f32:
                            encode -> softmax -> decode, one call).
  hard_regimes(model, x)    backtesting.py:154-155: argmax_k softmax(encode(x))_k,
                            as the VQ argmin kernel over the one-hot codebook
                            (argmin_k ||q - e_k||^2 = argmax_k q, first index on ties).
  viterbi_regimes(...)      MAP state path under the Prior's tables with the encoder
                            posterior as emission (log_softmax(logits)).
"""
import torch

from .hmm import viterbi, vq_argmin


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

    Exact for q_max >= 1/4 (1 - 2q is then exact in fp32); below that, two
    probabilities within one ulp of 1 - 2q can tie where torch.argmax would not."""
    with torch.no_grad():
        q = torch.softmax(model.encode(x), dim=1)
        eye = torch.eye(q.shape[1], device=q.device)
        return vq_argmin(q, eye).long(), q


def viterbi_regimes(model, x, u, lengths=None):
    """MAP regime path (B, T) int32 (-1 past each length) and its score (B,)."""
    with torch.no_grad():
        em = torch.log_softmax(model.encode(x), dim=1).transpose(1, 2).contiguous()
        log_pi, log_A = model.prior(u)
        return viterbi(log_pi, log_A, em, lengths)
