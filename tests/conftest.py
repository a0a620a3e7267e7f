import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libsw kernels)")
    config.addinivalue_line("markers", "slow: larger sizes")


def gpu_available():
    try:
        import torch  # noqa: F401  (device probe only)

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def libsw():
    """The loaded HIP library.  On a GPU box a missing library is an error, not a skip."""
    from juliaraytracingsw_amd import _lib

    return _lib.load()
