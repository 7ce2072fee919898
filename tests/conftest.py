import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); skipped on CPU-only hosts")
    config.addinivalue_line("markers", "slow: long-running")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def data_dir():
    return DATA


@pytest.fixture(scope="session")
def ctx():
    from cylon_amd import CylonContext
    return CylonContext(config=None, distributed=False, device="cpu")


@pytest.fixture(scope="session")
def gpu_ctx():
    from cylon_amd import CylonContext
    return CylonContext(config=None, distributed=False, device="cuda:0")
