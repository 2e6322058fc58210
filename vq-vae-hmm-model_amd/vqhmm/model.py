"""Drop-in nn.Module surface of VQ_VAE_HMM_fixed.py, executed by libvqhmm.so.

Same class names, constructor signatures, submodule names and parameter
shapes as the reference, so `state_dict()` keys are identical and reference
checkpoints (e.g. models/vae_hmm.pt) load unchanged:

    Encoder(input_dim, hidden_dim, hidden_dim2, K)          VQ_VAE_HMM_fixed.py:31-41
    Prior(K, u_dim=None, trans_hidden=128)                  :43-71
    Decoder(K, latent_dim, hidden_dim, output_dim)          :73-90
    VAE_HMM(input_dim, hidden_dim, K, hidden_dim2, u_dim=None, trans_hidden=128)   :92-143

The parameters are ordinary nn.Parameters (nn.Conv1d / nn.Linear /
nn.Embedding); only the compute is replaced: every forward/backward FLOP runs
in the hand-written HIP kernels behind the C-ABI.  CPU tensors are refused
(no fallback).  Error conventions of the reference are kept (ValueError for a
missing u_dim / u / lengths).
"""
import ctypes

import torch
import torch.nn as nn

from . import _ext

PARAM_ORDER = (
    "encoder.conv1.weight", "encoder.conv1.bias",
    "encoder.conv2.weight", "encoder.conv2.bias",
    "encoder.to_logits.weight", "encoder.to_logits.bias",
    "prior.log_prior",
    "prior.transition_net.0.weight", "prior.transition_net.0.bias",
    "prior.transition_net.2.weight", "prior.transition_net.2.bias",
    "decoder.embeddings.weight",
    "decoder.conv1.weight", "decoder.conv1.bias",
    "decoder.conv2.weight", "decoder.conv2.bias",
    "decoder.to_params.weight", "decoder.to_params.bias",
)

_PtrArray = ctypes.c_void_p * _ext.NPARAMS


def _tracks_grad(*tensors):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


def _module_ws(d, B, T, device):
    nb = ctypes.c_size_t()
    _ext.check(_ext.load().vqhmm_module_bwd_workspace_size(ctypes.byref(d), B, T, ctypes.byref(nb)), "workspace")
    return _workspace(device, nb.value), nb.value


class _EncodeFn(torch.autograd.Function):
    """Encoder.forward as one autograd node (VQ_VAE_HMM_fixed.py:38-41): forward vqhmm_encode_f32, backward
    vqhmm_encode_bwd_f32 (the encoder's data and weight gradients on the HIP kernels)."""

    @staticmethod
    def forward(ctx, enc, x, *params):
        ctx.dims = enc._dims()
        ctx.save_for_backward(x, *params)
        return enc._infer(x)

    @staticmethod
    def backward(ctx, glogits):
        x, *params = ctx.saved_tensors
        d = ctx.dims
        B, _, T = x.shape
        off = param_offsets(d)
        grad = torch.zeros(off[-1], device=x.device)
        dx = torch.empty_like(x) if ctx.needs_input_grad[1] else None
        ws, nb = _module_ws(d, B, T, x.device)
        w = [None] * _ext.NPARAMS
        w[0:6] = params
        _ext.check(_ext.load().vqhmm_encode_bwd_f32(ctypes.byref(d), _ptr_array(w), _ext.ptr(x),
                                                    _ext.ptr(glogits.contiguous().float()), B, T, _ext.ptr(ws), nb,
                                                    _ext.ptr(grad), _ext.ptr(dx), _ext.stream_ptr(x.device)),
                   "encode backward")
        return (None, dx, *[grad[off[i]:off[i + 1]].view_as(p) for i, p in enumerate(params)])


class _DecodeFn(torch.autograd.Function):
    """Decoder.forward as one autograd node (VQ_VAE_HMM_fixed.py:81-90): forward vqhmm_decode_f32, backward
    vqhmm_decode_bwd_f32 (dq, and the embedding / conv / to_params gradients; the embedding's through the
    composed conv1, dE = sum_{o,tap} dW'[o][k][tap] W[o][h][tap])."""

    @staticmethod
    def forward(ctx, dec, q, *params):
        ctx.dims = dec._dims()
        ctx.save_for_backward(q, *params)
        return dec._infer(q)

    @staticmethod
    def backward(ctx, gmu, glogvar):
        q, *params = ctx.saved_tensors
        d = ctx.dims
        B, _, T = q.shape
        off = param_offsets(d)
        grad = torch.zeros(off[-1], device=q.device)
        dq = torch.empty_like(q) if ctx.needs_input_grad[1] else None
        dpar = torch.cat([gmu, glogvar], 1).contiguous().float()  # [dmu | dlogvar]: to_params' output channels
        ws, nb = _module_ws(d, B, T, q.device)
        w = [None] * _ext.NPARAMS
        w[11:18] = params
        _ext.check(_ext.load().vqhmm_decode_bwd_f32(ctypes.byref(d), _ptr_array(w), _ext.ptr(q), _ext.ptr(dpar), B, T,
                                                    _ext.ptr(ws), nb, _ext.ptr(grad), _ext.ptr(dq),
                                                    _ext.stream_ptr(q.device)), "decode backward")
        return (None, dq, *[grad[off[11 + i]:off[12 + i]].view_as(p) for i, p in enumerate(params)])


class _ForwardFn(torch.autograd.Function):
    """VAE_HMM.forward as one autograd node (VQ_VAE_HMM_fixed.py:139-143): (mu, logvar, q) by vqhmm_forward_f32;
    backward vqhmm_forward_bwd_f32 through decode, the softmax of q and encode."""

    @staticmethod
    def forward(ctx, model, x, *params):
        ctx.dims = model._dims()
        ctx.save_for_backward(x, *params)
        (mu, logvar), q = model._infer(x)
        return mu, logvar, q

    @staticmethod
    def backward(ctx, gmu, glogvar, gq):
        x, *params = ctx.saved_tensors
        d = ctx.dims
        B, _, T = x.shape
        off = param_offsets(d)
        grad = torch.zeros(off[-1], device=x.device)
        dx = torch.empty_like(x) if ctx.needs_input_grad[1] else None
        dpar = torch.cat([gmu, glogvar], 1).contiguous().float()
        ws, nb = _module_ws(d, B, T, x.device)
        w = [None] * _ext.NPARAMS
        w[0:6] = params[0:6]
        w[11:18] = params[6:13]
        _ext.check(_ext.load().vqhmm_forward_bwd_f32(ctypes.byref(d), _ptr_array(w), _ext.ptr(x), _ext.ptr(dpar),
                                                     _ext.ptr(gq.contiguous().float()), B, T, _ext.ptr(ws), nb,
                                                     _ext.ptr(grad), _ext.ptr(dx), _ext.stream_ptr(x.device)),
                   "forward backward")
        idx = list(range(0, 6)) + list(range(11, 18))
        return (None, dx, *[grad[off[i]:off[i + 1]].view_as(p) for i, p in zip(idx, params)])


class _PriorFn(torch.autograd.Function):
    """Prior.forward as one autograd node (VQ_VAE_HMM_fixed.py:59-71): forward vqhmm_prior_f32, backward
    vqhmm_prior_bwd_f32 (the two log_softmax backwards, the MLP's data and weight gradients, du)."""

    @staticmethod
    def forward(ctx, prior, u, lay, *params):
        ctx.dims, ctx.lay = prior._dims(), lay
        ctx.save_for_backward(u, *params)
        return prior._infer(u, lay)

    @staticmethod
    def backward(ctx, gpi, gA):
        u, *params = ctx.saved_tensors
        d, lay = ctx.dims, ctx.lay
        B = u.shape[0]
        T = u.shape[2] if lay == 0 else u.shape[1]
        off = param_offsets(d)
        grad = torch.zeros(off[-1], device=u.device)
        du = torch.empty((B, d.u_dim, T), device=u.device) if ctx.needs_input_grad[1] else None
        lib = _ext.load()
        nb = ctypes.c_size_t()
        _ext.check(lib.vqhmm_prior_bwd_workspace_size(ctypes.byref(d), B, T, ctypes.byref(nb)), "workspace")
        ws = _workspace(u.device, nb.value)
        w = [None] * _ext.NPARAMS
        w[6:11] = params
        gpi = None if gpi is None else gpi.contiguous().float()
        gA = torch.zeros((B, T, d.K, d.K), device=u.device) if gA is None else gA.contiguous().float()
        _ext.check(lib.vqhmm_prior_bwd_f32(ctypes.byref(d), _ptr_array(w), _ext.ptr(u), lay, _ext.ptr(gpi),
                                           _ext.ptr(gA), B, T, _ext.ptr(ws), nb.value, _ext.ptr(grad), _ext.ptr(du),
                                           _ext.stream_ptr(u.device)), "prior backward")
        if du is not None and lay == 1:
            du = du.transpose(1, 2)
        return (None, du, None, *[grad[off[6 + i]:off[7 + i]].view_as(p) for i, p in enumerate(params)])


def _ptr_array(tensors):
    arr = _PtrArray()
    for i, t in enumerate(tensors):
        if t is not None:
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError("vqhmm: parameters must be contiguous float32")
            arr[i] = t.data_ptr()
    return arr


def _workspace(device, nbytes):
    return torch.empty(int(nbytes), dtype=torch.uint8, device=device)


class Encoder(nn.Module):
    """Conv1d(D->H,k3) ReLU Conv1d(H->H2,k3) ReLU Conv1d(H2->K,1)  (:31-41)."""

    def __init__(self, input_dim, hidden_dim, hidden_dim2, K):
        super().__init__()
        self.conv1 = nn.Conv1d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv1d(hidden_dim, hidden_dim2, 3, padding=1)
        self.to_logits = nn.Conv1d(hidden_dim2, K, 1)

    def _dims(self):
        H, D, _ = self.conv1.weight.shape
        H2 = self.conv2.weight.shape[0]
        K = self.to_logits.weight.shape[0]
        return _ext.Dims(D, H, K, H2, 1, 1)

    def _params(self):
        return [self.conv1.weight, self.conv1.bias, self.conv2.weight, self.conv2.bias, self.to_logits.weight,
                self.to_logits.bias]

    def forward(self, x):
        _ext.require_device(x)
        if x.dim() != 3 or x.shape[1] != self.conv1.weight.shape[1]:
            raise RuntimeError(f"Encoder: expected input (B, {self.conv1.weight.shape[1]}, T), got {tuple(x.shape)}")
        x = x.contiguous().float()
        if _tracks_grad(x, *self._params()):  # differentiable: the backward runs on the HIP kernels too
            return _EncodeFn.apply(self, x, *self._params())
        return self._infer(x)

    def _infer(self, x):
        B, _, T = x.shape
        d = self._dims()
        lib = _ext.load()
        logits = torch.empty((B, d.K, T), device=x.device)
        if B * T == 0:
            return logits
        nb = ctypes.c_size_t()
        _ext.check(lib.vqhmm_infer_workspace_size(ctypes.byref(d), B, T, ctypes.byref(nb)), "workspace")
        ws = _workspace(x.device, nb.value)
        w = [None] * _ext.NPARAMS
        w[0:6] = self._params()
        _ext.check(lib.vqhmm_encode_f32(ctypes.byref(d), _ptr_array(w), _ext.ptr(x), B, T, _ext.ptr(logits),
                                        _ext.ptr(ws), nb.value, _ext.stream_ptr(x.device)), "encode")
        return logits


class Prior(nn.Module):
    """Input-conditioned HMM prior: log_pi (K,), log_A (B,T,K,K)  (:43-71)."""

    def __init__(self, K, u_dim=None, trans_hidden=128):
        super().__init__()
        self.K = K
        self.u_dim = u_dim
        self.log_prior = nn.Parameter(torch.zeros(K))
        if u_dim is None:
            raise ValueError('Stationary transitions not implemented')
        self.transition_net = nn.Sequential(
            nn.Linear(u_dim, trans_hidden),
            nn.ReLU(),
            nn.Linear(trans_hidden, K * K),
        )

    def u_layout(self, u):
        """0 = (B, U, T) channels-first, 1 = (B, T, U) — the reference's rule (:64-65)."""
        if u.dim() == 3 and u.shape[1] == self.u_dim:
            return 0
        if u.dim() == 3 and u.shape[2] == self.u_dim:
            return 1
        raise RuntimeError(f"Prior: expected u of shape (B, {self.u_dim}, T) or (B, T, {self.u_dim}), got {tuple(u.shape)}")

    def _dims(self):
        lin0 = self.transition_net[0]
        return _ext.Dims(1, 1, self.K, 1, self.u_dim, lin0.weight.shape[0])

    def _params(self):
        lin0, lin2 = self.transition_net[0], self.transition_net[2]
        return [self.log_prior, lin0.weight, lin0.bias, lin2.weight, lin2.bias]

    def forward(self, u=None):
        if u is None:
            raise ValueError('u required for non-stationary transitions')
        _ext.require_device(u)
        lay = self.u_layout(u)
        u = u.contiguous().float()
        if _tracks_grad(u, *self._params()):  # differentiable: the backward runs on the HIP kernels too
            return _PriorFn.apply(self, u, lay, *self._params())
        return self._infer(u, lay)

    def _infer(self, u, lay):
        B = u.shape[0]
        T = u.shape[2] if lay == 0 else u.shape[1]
        K = self.K
        d = self._dims()
        log_pi = torch.empty(K, device=u.device)
        log_A = torch.empty((B, T, K, K), device=u.device)
        w = [None] * _ext.NPARAMS
        w[6:11] = self._params()
        _ext.check(_ext.load().vqhmm_prior_f32(ctypes.byref(d), _ptr_array(w), _ext.ptr(u), lay, B, T,
                                               _ext.ptr(log_pi), _ext.ptr(log_A), _ext.stream_ptr(u.device)), "prior")
        return log_pi, log_A


class Decoder(nn.Module):
    """Soft codebook embedding q^T E, then Conv1d x2 + 1x1 -> (mu, logvar)  (:73-90)."""

    def __init__(self, K, latent_dim, hidden_dim, output_dim):
        super().__init__()
        self.embeddings = nn.Embedding(K, latent_dim)
        self.conv1 = nn.Conv1d(latent_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv1d(hidden_dim, hidden_dim, 3, padding=1)
        self.to_params = nn.Conv1d(hidden_dim, output_dim * 2, 1)

    def _dims(self):
        K, Hl = self.embeddings.weight.shape
        H = self.conv1.weight.shape[0]
        if Hl != H or self.conv2.weight.shape[0] != H:
            raise RuntimeError("vqhmm: Decoder with latent_dim != hidden_dim is not supported "
                               "(VAE_HMM always builds Decoder(K, H, H, D), :98)")
        D = self.to_params.weight.shape[0] // 2
        return _ext.Dims(D, H, K, 1, 1, 1)

    def _ptrs(self):
        w = [None] * _ext.NPARAMS
        w[11:18] = [self.embeddings.weight, self.conv1.weight, self.conv1.bias, self.conv2.weight,
                    self.conv2.bias, self.to_params.weight, self.to_params.bias]
        return w

    def forward(self, q):
        _ext.require_device(q)
        d = self._dims()
        if q.dim() != 3 or q.shape[1] != d.K:
            raise RuntimeError(f"Decoder: expected q of shape (B, {d.K}, T), got {tuple(q.shape)}")
        q = q.contiguous().float()
        params = self._ptrs()[11:18]
        if _tracks_grad(q, *params):  # differentiable: the backward runs on the HIP kernels too
            return _DecodeFn.apply(self, q, *params)
        return self._infer(q)

    def _infer(self, q):
        d = self._dims()
        B, _, T = q.shape
        mu = torch.empty((B, d.input_dim, T), device=q.device)
        logvar = torch.empty((B, d.input_dim, T), device=q.device)
        if B * T == 0:
            return mu, logvar
        lib = _ext.load()
        nb = ctypes.c_size_t()
        _ext.check(lib.vqhmm_infer_workspace_size(ctypes.byref(d), B, T, ctypes.byref(nb)), "workspace")
        ws = _workspace(q.device, nb.value)
        _ext.check(lib.vqhmm_decode_f32(ctypes.byref(d), _ptr_array(self._ptrs()), _ext.ptr(q), B, T, _ext.ptr(mu),
                                        _ext.ptr(logvar), _ext.ptr(ws), nb.value, _ext.stream_ptr(q.device)),
                   "decode")
        return mu, logvar


class _ElboLoss(torch.autograd.Function):
    """compute_loss as one autograd node: forward + backward are native executors."""

    @staticmethod
    def forward(ctx, model, x, u, lengths, beta, *params):
        d = model._dims()
        B, _, T = x.shape
        lay = model.prior.u_layout(u)
        lib = _ext.load()
        nb = ctypes.c_size_t()
        _ext.check(lib.vqhmm_elbo_workspace_size(ctypes.byref(d), B, T, ctypes.byref(nb)), "workspace")
        ws = _workspace(x.device, nb.value)
        loss = torch.empty((), device=x.device)
        need_grad = any(ctx.needs_input_grad[5:])
        ptrs = _ptr_array(params)
        _ext.check(lib.vqhmm_elbo_fwd_f32(ctypes.byref(d), ptrs, _ext.ptr(x), _ext.ptr(u), lay, _ext.ptr(lengths),
                                          None, B, T, float(beta), int(need_grad), _ext.ptr(ws), nb.value,
                                          _ext.ptr(loss), None, _ext.stream_ptr(x.device)), "compute_loss forward")
        ctx.state = (d, ws, nb.value, B, T, float(beta))
        ctx.save_for_backward(x, *params)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        d, ws, nbytes, B, T, beta = ctx.state
        x, *params = ctx.saved_tensors
        lib = _ext.load()
        off = param_offsets(d)
        grad = torch.empty(off[-1], device=x.device)
        gl = gloss.contiguous().float()
        _ext.check(lib.vqhmm_elbo_bwd_f32(ctypes.byref(d), _ptr_array(params), _ext.ptr(x), None, B, T,
                                          beta, _ext.ptr(gl), _ext.ptr(ws), nbytes, _ext.ptr(grad),
                                          _ext.stream_ptr(x.device)), "compute_loss backward")
        grads = [grad[off[i]:off[i + 1]].view_as(p) for i, p in enumerate(params)]
        return (None, None, None, None, None, *grads)


def param_offsets(d):
    off = (ctypes.c_int64 * (_ext.NPARAMS + 1))()
    _ext.check(_ext.load().vqhmm_param_layout(ctypes.byref(d), off), "param_layout")
    return list(off)


class VAE_HMM(nn.Module):
    """Mean-field VAE with an input-conditioned HMM prior (:92-143)."""

    def __init__(self, input_dim, hidden_dim, K, hidden_dim2, u_dim=None, trans_hidden=128):
        super().__init__()
        self.K = K
        self.encoder = Encoder(input_dim, hidden_dim, hidden_dim2, K)
        self.prior = Prior(K, u_dim, trans_hidden)
        self.decoder = Decoder(K, hidden_dim, hidden_dim, input_dim)

    def _dims(self):
        H, D, _ = self.encoder.conv1.weight.shape
        return _ext.Dims(D, H, self.K, self.encoder.conv2.weight.shape[0], self.prior.u_dim,
                         self.prior.transition_net[0].weight.shape[0])

    def ordered_parameters(self):
        named = dict(self.named_parameters())
        return [named[n] for n in PARAM_ORDER]

    def encode(self, x):
        return self.encoder(x)

    def decode(self, q):
        return self.decoder(q)

    def compute_loss(self, x, u=None, lengths=None, beta=1.0):
        B, C, T = x.shape
        if lengths is None:
            raise ValueError('lengths required')
        if u is None:
            raise ValueError('u required for non-stationary transitions')
        _ext.require_device(x, u)
        if C != self.encoder.conv1.weight.shape[1]:
            raise RuntimeError(f"compute_loss: x has {C} channels, model expects {self.encoder.conv1.weight.shape[1]}")
        lay = self.prior.u_layout(u)
        if u.shape[0] != B or (u.shape[2] if lay == 0 else u.shape[1]) != T:
            raise RuntimeError(f"compute_loss: u {tuple(u.shape)} does not match x {tuple(x.shape)}")
        x = x.contiguous().float()
        u = u.contiguous().float()
        lengths = torch.as_tensor(lengths).to(device=x.device, dtype=torch.int64, non_blocking=True).contiguous()
        if lengths.shape != (B,):
            raise RuntimeError(f"compute_loss: lengths must have shape ({B},)")
        return _ElboLoss.apply(self, x, u, lengths, float(beta), *self.ordered_parameters())

    def forward(self, x):
        _ext.require_device(x)
        x = x.contiguous().float()
        params = self.encoder._params() + self.decoder._ptrs()[11:18]
        if _tracks_grad(x, *params):  # differentiable: the backward runs on the HIP kernels too
            mu, logvar, q = _ForwardFn.apply(self, x, *params)
            return (mu, logvar), q
        return self._infer(x)

    def _infer(self, x):
        B, _, T = x.shape
        d = self._dims()
        mu = torch.empty((B, d.input_dim, T), device=x.device)
        logvar = torch.empty_like(mu)
        q = torch.empty((B, self.K, T), device=x.device)
        if B * T == 0:
            return (mu, logvar), q
        lib = _ext.load()
        nb = ctypes.c_size_t()
        _ext.check(lib.vqhmm_infer_workspace_size(ctypes.byref(d), B, T, ctypes.byref(nb)), "workspace")
        ws = _workspace(x.device, nb.value)
        _ext.check(lib.vqhmm_forward_f32(ctypes.byref(d), _ptr_array(self.ordered_parameters()), _ext.ptr(x), B, T,
                                         _ext.ptr(mu), _ext.ptr(logvar), _ext.ptr(q), _ext.ptr(ws), nb.value,
                                         _ext.stream_ptr(x.device)), "forward")
        return (mu, logvar), q
