import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# Preloaded successors (TPI_PRELOAD, on by default) import PyTorch in a parked process next to
# every Python rank; the tests that are about them turn them on in their tasks' variables,
# the rest run without the extra processes.
os.environ.setdefault("TPI_PRELOAD", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def native():
    from terraform_provider_iterative_amd.ops import native as _native

    return _native()
