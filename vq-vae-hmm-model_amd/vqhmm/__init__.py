"""vqhmm — MI355X-native (gfx950) implementation of the VAE_HMM training hot path
of yashnaray/VQ-VAE-HMM-model.

Drop-in surface (VQ_VAE_HMM_fixed.py): VAE_HMM, Encoder, Prior, Decoder,
train_model, RandomChunkDataset, collate_fn — plus the hard-regime kernels
vq_argmin / forward_backward / viterbi.  All compute runs in hand-written HIP
kernels in libvqhmm.so; there is no CPU fallback.
"""
from . import _ext  # noqa: F401
from .checkpoint import load_checkpoint, load_encoder, save_checkpoint, save_encoder  # noqa: F401
from .data import DeviceChunkLoader, RandomChunkDataset, collate_fn  # noqa: F401
from .hmm import forward_backward, quantize, regime_argmax, viterbi, vq_argmin  # noqa: F401
from .infer import hard_regimes, infer, prior_viterbi, viterbi_regimes  # noqa: F401
from .model import PARAM_ORDER, VAE_HMM, Decoder, Encoder, Prior  # noqa: F401
from .train import Trainer, TrainState, train_model  # noqa: F401

__all__ = ["VAE_HMM", "Encoder", "Prior", "Decoder", "train_model", "Trainer", "TrainState", "RandomChunkDataset",
           "collate_fn", "DeviceChunkLoader", "vq_argmin", "quantize", "regime_argmax", "viterbi", "forward_backward", "PARAM_ORDER",
           "save_checkpoint", "load_checkpoint", "save_encoder", "load_encoder", "infer", "hard_regimes", "viterbi_regimes",
           "prior_viterbi"]
