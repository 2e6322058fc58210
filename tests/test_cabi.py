"""CPU checks of the C-ABI boundary: libvqhmm.so loads without a GPU and
exports every function include/vqhmm.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "vqhmm.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vqhmm_\w+)\s*\(", src)))


def test_header_declares_functions():
    names = declared_functions()
    assert "vqhmm_vq_argmin_f32" in names and len(names) >= 3


def test_library_exports_every_declared_symbol():
    from vqhmm import _ext
    lib = _ext.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes signature table covers the header exactly
    assert sorted(_ext.exported_symbols()) == declared_functions()


def test_param_layout_matches_reference_shapes():
    from oracle import ref_model as RM
    from vqhmm import _ext
    lib = _ext.load()
    d = _ext.Dims(5, 64, 3, 32, 4, 128)
    off = (ctypes.c_int64 * 19)()
    assert lib.vqhmm_param_layout(ctypes.byref(d), off) == 0
    shapes = RM.param_shapes(5, 64, 3, 32, 4, 128)
    import math
    sizes = [math.prod(shapes[n]) for n in RM.PARAM_ORDER]
    assert [off[i + 1] - off[i] for i in range(18)] == sizes
    assert off[18] == 34649  # 34,649 params at cfg2


def test_invalid_args_rejected_without_gpu():
    from vqhmm import _ext
    lib = _ext.load()
    # null pointers with a non-empty problem are rejected before any launch
    rc = lib.vqhmm_vq_argmin_f32(None, 2, 4, 8, None, 3, None, None, None)
    assert rc == -1


def test_cpu_tensors_fail_loudly():
    import torch
    import vqhmm
    with pytest.raises(RuntimeError, match="HIP"):
        vqhmm.vq_argmin(torch.zeros(1, 2, 3), torch.zeros(4, 2))


@pytest.mark.parametrize("dims,B,T", [((5, 64, 3, 32, 4, 128), 1024, 200), ((16, 64, 8, 32, 4, 128), 512, 512),
                                      ((64, 256, 32, 128, 4, 128), 8, 50)])
def test_status_word_inside_workspace(dims, B, T):
    """The step's device status word (vqhmm_elbo_status_offset) lies inside the workspace, 8-byte
    aligned, for the configs' shapes (host-only query)."""
    from vqhmm import _ext
    lib = _ext.load()
    d = _ext.Dims(*dims)
    nb, off = ctypes.c_size_t(), ctypes.c_size_t()
    assert lib.vqhmm_elbo_workspace_size(ctypes.byref(d), B, T, ctypes.byref(nb)) == 0
    assert lib.vqhmm_elbo_status_offset(ctypes.byref(d), B, T, ctypes.byref(off)) == 0
    assert off.value % 8 == 0 and off.value + 8 <= nb.value
    assert lib.vqhmm_elbo_status_offset(ctypes.byref(d), 0, T, ctypes.byref(off)) == -1


# the A/B switches the release library may read (common.h VQHMM_ENV): each selects between launch paths the
# GPU tests prove bit-identical (VQHMM_STRIP_HEAD / VQHMM_HEAD: equal within their stated tolerance)
RELEASE_SWITCHES = {"VQHMM_CONV_FUSE", "VQHMM_TAIL_FUSED", "VQHMM_STRIP", "VQHMM_STRIP_BWD", "VQHMM_STRIP_WGRAD", "VQHMM_STRIP_HEAD",
                    "VQHMM_FB_RES", "VQHMM_FB_FUSE", "VQHMM_FB_PAIR", "VQHMM_FB_SEG", "VQHMM_HEAD"}


def test_release_library_reads_no_profiling_knobs():
    """result-changing timing / tuning knobs (VQHMM_WGRAD_JOBMASK, VQHMM_STRIP_DBG,
    VQHMM_HEAD_DBG, VQHMM_PV_MODE, the chunk-count overrides, ...) exist only in the profiling build
    (make prof): the release library's strings name no environment variable but the A/B switches."""
    from vqhmm import _ext
    data = open(_ext.LIB_PATH if "prof" not in _ext.LIB_PATH else _ext.LIB_PATH.replace("_prof", ""), "rb").read()
    names = set(m.decode() for m in re.findall(rb"VQHMM_[A-Z0-9_]+", data))
    names = {n for n in names if not n.startswith("VQHMM_STATUS")}
    assert names <= RELEASE_SWITCHES, sorted(names - RELEASE_SWITCHES)
    assert "VQHMM_WGRAD_JOBMASK" not in names and "VQHMM_STRIP_DBG" not in names
