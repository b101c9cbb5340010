import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (runs through libbsaccel.so)')
    config.addinivalue_line('markers', 'slow: larger sizes (still seconds on the GPU box)')


@pytest.fixture(scope='session')
def ctx():
    """One HIP context for the whole GPU session (single process on the card)."""
    from bluesky_amd import _lib
    c = _lib.default_context(0)
    yield c
