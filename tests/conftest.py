import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build what is stale, once (build_hip serialises concurrent callers on a file lock: the
    first xdist worker compiles, the others find the library fresh)."""
    import __graft_entry__ as g
    g.build_hip()
    from oracle import oracle as orc
    orc.build()
    yield
