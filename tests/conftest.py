import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librandblas_hip.so on the device)")


@pytest.fixture(scope="session")
def cuda():
    """The device under test. GPU tests fail (not skip) without one: they are selected with -m gpu."""
    import torch

    assert torch.cuda.is_available(), "gpu tests need a visible MI355X"
    return torch.device("cuda:0")
