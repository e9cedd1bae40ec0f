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
    """Build what is stale, once: xdist workers take a file lock, so only the first one compiles
    and the others find the libraries fresh."""
    import fcntl
    import __graft_entry__ as g
    from oracle import oracle as orc
    os.makedirs(g.LIBDIR, exist_ok=True)
    with open(os.path.join(g.LIBDIR, ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        try:
            g.build_hip()
            orc.build()
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)
    yield
