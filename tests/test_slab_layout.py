"""The backward strip stores its two 64-wide layers' weight-gradient rows output-fastest and the tail maps each
slab column back to the parameter (kernels.h::seg_out_index, SlabSeg::trO).  Checked on the host (no GPU):
seg_out_index, compiled by hipcc into a host-only program, is the inverse of the strip's store formula
(strip_bwdw.hip store_d2 / store_e2: column (c * 3 + tap) * O + o holds dW[o][c][tap]) and a bijection onto the
parameter's (O, C, 3) layout, for the cfg2 shapes and an O that is not a multiple of 4 (the scalar-store path)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CSRC = os.path.join(ROOT, "vq-vae-hmm-model_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

PROG = r"""
#include "kernels.h"
#include <cstdio>
int main() {
  const int shapes[][2] = {{64, 64}, {32, 64}, {31, 64}};
  for (auto& s : shapes) {
    vqhmm::SlabSeg sg{};
    sg.trO = s[0];
    sg.trC = s[1];
    const long n = (long)s[0] * s[1] * 3;
    for (long col = 0; col < n; ++col) printf("%ld\n", (long)vqhmm::seg_out_index(sg, col));
  }
  return 0;
}
"""


@pytest.fixture(scope="module")
def mapped(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("slab")
    src, exe = d / "seg.hip", d / "seg"
    src.write_text(PROG)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-std=c++17", "-I", CSRC,
                    "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True,
                   capture_output=True, timeout=300)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=60).stdout.split()
    return np.array(out, dtype=np.int64)


def test_seg_out_index_inverts_the_strip_store(mapped):
    pos = 0
    for O, C in ((64, 64), (32, 64), (31, 64)):
        n = O * C * 3
        got = mapped[pos:pos + n]
        pos += n
        o, c, tap = np.meshgrid(np.arange(O), np.arange(C), np.arange(3), indexing="ij")
        col = (c * 3 + tap) * O + o                      # where the strip stores dW[o][c][tap]
        want = (o * C + c) * 3 + tap                      # its index in the parameter
        np.testing.assert_array_equal(got[col.ravel()], want.ravel())
        assert np.array_equal(np.sort(got), np.arange(n))  # a bijection onto the parameter
    assert pos == mapped.size
