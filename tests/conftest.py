import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "blockchain-simulator_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")
    config.addinivalue_line("markers", "slow: long-running")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def engine_lib():
    import bcsim
    if not os.path.exists(bcsim.LIB_PATH):
        bcsim.build()
    return bcsim.lib()
