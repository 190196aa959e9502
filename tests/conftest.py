import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libpdd.so")


@pytest.fixture(scope="session")
def golden():
    return np.load(os.path.join(GOLDEN, "golden.npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def golden_meta():
    with open(os.path.join(GOLDEN, "golden_meta.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import __graft_entry__ as g
    g.build()
    return torch.device("cuda")


def band(C, descending=True, lo=1250.0, hi=1550.0):
    """Frequencies built like filterbank.py:85 (same helper as make_golden)."""
    foff = (hi - lo) / C
    if descending:
        fch1, foff = hi - foff / 2.0, -foff
    else:
        fch1 = lo + foff / 2.0
    return fch1 + foff * np.arange(C)


def u8_data(C, N, seed):
    rng = np.random.default_rng(seed)
    return np.clip(np.round(rng.normal(128, 16, size=(C, N))), 0, 255).astype(np.uint8)


PADS = [0, 3.5, "mean", "median", "rotate"]


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.max(np.abs(b)) if b.size else 0.0, 1e-30)
    return float(np.max(np.abs(a - b)) / scale) if a.size else 0.0
