import os
import sys

import pytest

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_ROOT, "bigdl-1_amd"))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(autouse=True)
def _seed():
    import torch
    from bigdl.utils.random import RNG
    RNG.setSeed(1)
    torch.manual_seed(1)
    yield


def gpu_available():
    import torch
    return torch.cuda.is_available()
