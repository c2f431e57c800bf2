import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(autouse=True)
def _test_seed():
    from oryx_amd.utils import rng
    rng.use_test_seed()
    yield


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oryx_amd import native
    native.require_kernels()
    return torch.device("cuda", 0)
