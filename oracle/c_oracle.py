"""ctypes loader for oracle/_build/liboracle.so — TEST INFRASTRUCTURE ONLY."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = ctypes.CDLL(_LIB)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def vq_argmin(z, codebook, want_dmin=True):
    """z (B,Dv,T) f32, codebook (K,Dv) f32 -> idx (B,T) int32[, dmin (B,T) f32]."""
    z = np.ascontiguousarray(z, np.float32)
    c = np.ascontiguousarray(codebook, np.float32)
    B, Dv, T = z.shape
    K = c.shape[0]
    idx = np.empty((B, T), np.int32)
    dmin = np.empty((B, T), np.float32)
    i64 = ctypes.c_int64
    lib().oracle_vq_argmin_f32(_p(z), i64(B), i64(Dv), i64(T), _p(c), i64(K), _p(idx), _p(dmin))
    return (idx, dmin) if want_dmin else idx


def viterbi(log_pi, log_A, em, lengths):
    """fp32 Viterbi (contract in hmm_ref.py) -> path (B,T) int32, score (B,) f32."""
    log_pi = np.ascontiguousarray(log_pi, np.float32)
    log_A = np.ascontiguousarray(log_A, np.float32)
    em = np.ascontiguousarray(em, np.float32)
    lengths = np.ascontiguousarray(lengths, np.int64)
    B, T, K = em.shape
    path = np.empty((B, T), np.int32)
    score = np.empty(B, np.float32)
    i64 = ctypes.c_int64
    lib().oracle_viterbi_f32(_p(log_pi), _p(log_A), _p(em), _p(lengths), i64(B), i64(T), i64(K),
                             _p(path), _p(score))
    return path, score
