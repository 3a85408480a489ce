"""pytest configuration: registers the `gpu` marker and puts the repo root and
the product source root (distributed-training-ina_amd/) on sys.path."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "distributed-training-ina_amd")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")


@pytest.fixture(autouse=True)
def _store_contract_checked(request):
    """Under a checked build (INA_LIBRARY=libina_storecheck.so, csrc/ina_device.h
    INA_STORE_CHECK) every GPU test ends with zero stream_store contract violations."""
    yield
    if request.node.get_closest_marker("gpu") is None or not os.environ.get("INA_LIBRARY"):
        return
    import ctypes
    from ina_amd import _lib
    lib = _lib.load()
    if not hasattr(lib, "ina_store_check_violations"):
        assert "storecheck" not in os.environ["INA_LIBRARY"], "the checked build exports its counter"
        return
    n = ctypes.c_ulonglong(0)
    assert lib.ina_store_check_violations(ctypes.byref(n)) == 0
    assert n.value == 0, f"{n.value} stream_store contract violations"
