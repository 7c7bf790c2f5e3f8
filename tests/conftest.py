import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "vision-transformer_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP path through the C-ABI")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture
def libopt():
    """Set libvit_hip launch options (vit_set_option) for one test; every option is restored at teardown."""
    from VisionTransformer import _lib
    saved = {}

    def set_(name, value):
        prev = _lib.set_option(name, value)
        saved.setdefault(name, prev)

    yield set_
    for name, value in saved.items():
        _lib.set_option(name, value)
