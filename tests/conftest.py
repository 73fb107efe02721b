import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
PKG = os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP (MI355X) device")
    config.addinivalue_line("markers", "slow: long-running (full-size configs)")


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def kat():
    return load_golden("quant_kat.npz")


@pytest.fixture(scope="session")
def cfg1():
    return load_golden("e2e_cfg1.npz")


@pytest.fixture(scope="session")
def trace():
    return load_golden("trace_s.npz")


@pytest.fixture(scope="session")
def nb():
    return load_golden("e2e_nb.npz")


@pytest.fixture(scope="session")
def large():
    return load_golden("sum_large.npz")
