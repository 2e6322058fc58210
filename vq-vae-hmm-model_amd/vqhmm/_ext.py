"""ctypes binding of libvqhmm.so (the C-ABI declared in include/vqhmm.h).

There is no fallback: if the library or a HIP device is missing, every op
raises.  The library is built in-tree by `make -C vq-vae-hmm-model_amd`
(or `__graft_entry__.build()`).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# VQHMM_LIB_PATH: load another build of the same library (kernel A/B experiments only)
LIB_PATH = os.environ.get("VQHMM_LIB_PATH") or os.path.join(_HERE, "libvqhmm.so")
NPARAMS = 18
ABI_VERSION = 6

EUNSUPPORTED = -4
_ERRORS = {-1: "invalid argument", -2: "kernel launch failed", -3: "workspace too small",
           -4: "unsupported shape"}

_lib = None

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p
c_sz = ctypes.c_size_t


class Dims(ctypes.Structure):
    """Mirror of vqhmm_dims_t."""
    _fields_ = [("input_dim", c_i32), ("hidden_dim", c_i32), ("K", c_i32),
                ("hidden_dim2", c_i32), ("u_dim", c_i32), ("trans_hidden", c_i32)]


# name -> (restype, argtypes)
_SIGS = {
    "vqhmm_abi_version": (c_i32, []),
    "vqhmm_param_layout": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_i64)]),
    "vqhmm_vq_argmin_f32": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "vqhmm_vq_quantize_workspace_size": (c_sz, [c_i64, c_i64, c_i64, c_i64]),
    "vqhmm_vq_quantize_f32": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_sz,
                                             c_vp]),
    "vqhmm_viterbi_workspace_size": (c_sz, [c_i64, c_i64, c_i64]),
    "vqhmm_viterbi_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "vqhmm_fwdbwd_workspace_size": (c_sz, [c_i64, c_i64, c_i64]),
    "vqhmm_fwdbwd_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "vqhmm_elbo_workspace_size": (ctypes.c_int, [ctypes.POINTER(Dims), c_i64, c_i64, ctypes.POINTER(c_sz)]),
    "vqhmm_elbo_fwd_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_vp, ctypes.c_int,
                                          c_vp, c_vp, c_i64, c_i64, c_f32, ctypes.c_int, c_vp, c_sz, c_vp, c_vp,
                                          c_vp]),
    "vqhmm_elbo_bwd_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_vp, c_i64, c_i64, c_f32,
                                          c_vp, c_vp, c_sz, c_vp, c_vp]),
    "vqhmm_elbo_bwd_loss_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_vp, c_i64, c_i64,
                                               c_f32, c_vp, c_vp, c_sz, c_vp, c_vp, c_vp, c_vp]),
    "vqhmm_elbo_bwd_adam_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_vp, c_i64, c_i64,
                                               c_f32, c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, ctypes.c_double,
                                               ctypes.c_double, ctypes.c_double, ctypes.c_double, c_vp, c_f32, c_vp,
                                               c_vp, c_vp]),
    "vqhmm_elbo_pieces": (ctypes.c_int, [ctypes.POINTER(Dims), c_i64, c_i64, c_vp, ctypes.POINTER(c_vp),
                                         ctypes.POINTER(c_vp)]),
    "vqhmm_adam_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_double, ctypes.c_double, c_vp, c_f32, c_vp]),
    "vqhmm_elbo_num_stages": (ctypes.c_int, []),
    "vqhmm_elbo_stage_info": (ctypes.c_int, [ctypes.POINTER(Dims), c_i64, c_i64, ctypes.c_int, ctypes.c_char_p, c_sz,
                                             ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_int)]),
    "vqhmm_elbo_stage_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_vp, ctypes.c_int,
                                            c_vp, c_vp, c_i64, c_i64, c_f32, c_vp, c_sz, c_vp, ctypes.c_int, c_vp]),
    "vqhmm_clip_grad_norm_f32": (ctypes.c_int, [c_vp, c_i64, c_f32, c_f32, c_vp, c_vp]),
    "vqhmm_gather_chunks_f32": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "vqhmm_infer_workspace_size": (ctypes.c_int, [ctypes.POINTER(Dims), c_i64, c_i64, ctypes.POINTER(c_sz)]),
    "vqhmm_encode_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_i64, c_i64, c_vp,
                                        c_vp, c_sz, c_vp]),
    "vqhmm_decode_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_i64, c_i64, c_vp,
                                        c_vp, c_vp, c_sz, c_vp]),
    "vqhmm_forward_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_i64, c_i64, c_vp,
                                         c_vp, c_vp, c_vp, c_sz, c_vp]),
    "vqhmm_module_bwd_workspace_size": (ctypes.c_int, [ctypes.POINTER(Dims), c_i64, c_i64, ctypes.POINTER(c_sz)]),
    "vqhmm_prior_bwd_workspace_size": (ctypes.c_int, [ctypes.POINTER(Dims), c_i64, c_i64, ctypes.POINTER(ctypes.c_size_t)]),
    "vqhmm_prior_bwd_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, ctypes.c_int, c_vp, c_vp,
                                           c_i64, c_i64, c_vp, ctypes.c_size_t, c_vp, c_vp, c_vp]),
    "vqhmm_encode_bwd_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_vp, c_i64, c_i64,
                                            c_vp, c_sz, c_vp, c_vp, c_vp]),
    "vqhmm_decode_bwd_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_vp, c_i64, c_i64,
                                            c_vp, c_sz, c_vp, c_vp, c_vp]),
    "vqhmm_forward_bwd_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_vp, c_vp, c_i64,
                                             c_i64, c_vp, c_sz, c_vp, c_vp, c_vp]),
    "vqhmm_prior_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, ctypes.c_int, c_i64,
                                       c_i64, c_vp, c_vp, c_vp]),
    "vqhmm_prior_viterbi_workspace_size": (c_sz, [ctypes.POINTER(Dims), c_i64, c_i64]),
    "vqhmm_prior_viterbi_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, ctypes.c_int, c_vp,
                                               c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "vqhmm_regimes_f32": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(c_vp), c_vp, c_i64, c_i64, c_vp,
                                         c_vp, c_vp, c_sz, c_vp]),
    "vqhmm_argmax_f32": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "vqhmm_elbo_debug_buffers": (ctypes.c_int, [ctypes.POINTER(Dims), c_i64, c_i64, c_vp, ctypes.POINTER(c_vp)]),
    "vqhmm_elbo_status_offset": (ctypes.c_int, [ctypes.POINTER(Dims), c_i64, c_i64, ctypes.POINTER(c_sz)]),
    "vqhmm_debug_prof": (ctypes.c_int, [ctypes.c_int, c_vp, c_i64]),
}

# bits of the step's device status word (include/vqhmm.h VQHMM_STATUS_*): bit 1 is reserved and no kernel
# sets it since the backward tail lost its in-launch wait (round 4)
STATUS_BITS = {1: "reserved (no kernel sets it)"}


def load():
    """Load and type the library (no GPU needed).  Raises if missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"vqhmm: native library not built ({LIB_PATH}); run `make -C {os.path.dirname(_HERE)}`")
        lib = ctypes.CDLL(LIB_PATH)
        # the version first: a stale library lacks newer symbols and would fail below with a bare
        # "undefined symbol" instead
        ver = getattr(lib, "vqhmm_abi_version", None)
        if ver is None:
            raise RuntimeError(f"vqhmm: {LIB_PATH} exports no vqhmm_abi_version; rebuild the library")
        ver.restype, ver.argtypes = c_i32, []
        if ver() != ABI_VERSION:
            raise RuntimeError(f"vqhmm: ABI version mismatch (library {ver()}, package {ABI_VERSION}); rebuild the library")
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def exported_symbols():
    return list(_SIGS)


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"vqhmm: {what} failed: {_ERRORS.get(rc, rc)}")


def require_device(*tensors):
    """The product path is HIP-only: refuse CPU tensors loudly (no fallback)."""
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("vqhmm runs on MI355X (HIP) only: move tensors to a 'cuda' (ROCm) device")


def stream_ptr(device=None):
    return c_vp(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return c_vp(t.data_ptr()) if t is not None else c_vp(0)
