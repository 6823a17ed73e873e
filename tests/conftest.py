"""Shared pytest setup.

Markers: ``gpu`` = needs an MI355X (run with ``-m gpu`` on the GPU box); everything else runs on
CPU here.  GPU tests call the HIP library through its C-ABI and check it against the CPU oracle
(oracle/, test infrastructure only).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP library parity / perf checks)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def qg():
    """The package (built if needed)."""
    import _pkg
    return _pkg.package(build=True)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible (run -m gpu on the MI355X box)")
    return torch.device("cuda:0")
