import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm (MI355X) device and libpertrender.so")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def assert_close(actual, expected, rtol=1e-5, atol_rel=1e-6, name=""):
    """|a - e| <= rtol*|e| + atol_rel*max|e| elementwise (the 1e-5 relative fp32 bar)."""
    a = np.asarray(actual.detach().cpu() if torch.is_tensor(actual) else actual, np.float64)
    e = np.asarray(expected.detach().cpu() if torch.is_tensor(expected) else expected, np.float64)
    assert a.shape == e.shape, f"{name}: shape {a.shape} != {e.shape}"
    scale = np.abs(e).max() if e.size else 0.0
    tol = rtol * np.abs(e) + atol_rel * scale + 1e-30
    bad = np.abs(a - e) > tol
    if bad.any():
        i = np.unravel_index(np.argmax(np.abs(a - e) - tol), a.shape)
        raise AssertionError(f"{name}: {bad.sum()} / {a.size} elements out of tolerance; worst at {i}: "
                             f"{a[i]!r} vs {e[i]!r} (tol {tol[i]:.3e})")


@pytest.fixture(scope="session")
def device():
    return torch.device("cuda:0")
