import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def _make(path):
    subprocess.run(["make", "-s", "-C", path], check=True)


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle and libmibminet.so in-tree (no-ops when up to date)."""
    _make(os.path.join(ROOT, "oracle"))
    _make(os.path.join(ROOT, "mi-bminet_amd"))
    yield


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return torch.device("cuda:0")
