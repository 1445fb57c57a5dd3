import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# MCC_PKG_ROOT=build/checked: import the package built by `make checked`
# (device bounds checks compiled in) instead of the in-tree one
if os.environ.get("MCC_PKG_ROOT"):
    sys.path.insert(0, os.path.join(ROOT, os.environ["MCC_PKG_ROOT"]))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture
def cuda():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch

    return torch.device("cuda", 0)
