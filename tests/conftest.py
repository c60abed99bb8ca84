import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "noise-robust-speech-embedding_amd")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device and libnrse_hip.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def nrse_device():
    """Initialise libnrse_hip on cuda:0 (fails loudly if the library or a gfx950 is missing)."""
    import torch
    from nrse_amd import _lib
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    _lib.init_device(0)
    torch.manual_seed(0)
    return torch.device("cuda:0")
