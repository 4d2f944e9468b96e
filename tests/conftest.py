"""pytest configuration: the ``gpu`` marker and shared helpers.

``-m "not gpu"`` runs here (no GPU): oracle vs golden vectors / KATs, host
logic, C-ABI load + symbol checks, gloo world_size-2 decomposition tests.
``-m gpu`` runs on the MI355X box and calls the HIP path through the C-ABI;
there it must never silently skip -- a missing GPU or library is a failure.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def lib():
    from spim_registration_amd import _lib
    from spim_registration_amd.build import build
    build(verbose=False)
    return _lib.load()


@pytest.fixture(scope="session")
def gpu(lib):
    from spim_registration_amd import _lib
    n = _lib.num_devices()
    assert n >= 1, "gpu test without a visible GPU (no CPU fallback exists)"
    return 0


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
