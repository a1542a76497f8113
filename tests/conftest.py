import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "analytics-zoo_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(autouse=True)
def _seed():
    import torch
    torch.manual_seed(1337)
    yield


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zoo.ops import native
    native()
    return torch.device("cuda")
