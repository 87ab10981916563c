import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm MI355X GPU and the native _C extension")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def native():
    """The native HIP module; fails loudly (no fallback) when a GPU is present but _C is not."""
    if not gpu_available():
        pytest.skip("no GPU")
    from pytorch_ddp_mnist_amd.ops.native import require_gpu
    return require_gpu()


@pytest.fixture(scope="session")
def small_mnist():
    from pytorch_ddp_mnist_amd.data.synthetic import make_split
    x, y = make_split(4096, seed=7)
    xt, yt = make_split(1024, seed=8)
    return x, y, xt, yt
