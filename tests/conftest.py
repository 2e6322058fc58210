import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "vq-vae-hmm-model_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_CASES = ("cfg1_seeded", "cfg1_trained", "cfg2_slice_seeded", "cfg2_slice_trained", "k32_wide",
                "k8_d16", "smoke_tiny")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def golden_dims(g):
    D, H, K, H2, U, TH = (int(v) for v in g["dims"])
    return dict(input_dim=D, hidden_dim=H, K=K, hidden_dim2=H2, u_dim=U, trans_hidden=TH)


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
