"""Shared test setup.  `-m gpu` tests need an MI355X and the built HIP library;
everything else runs on CPU (oracle, host logic, C-ABI symbol checks, gloo)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return True
