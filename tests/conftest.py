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
    # The tests pin the forward paths they name (two-chain split, query-0 pruned block, SDPA host attention), which a
    # probability-storing forward replaces; store_attention_probs=None (auto) would turn that on for their small
    # batches.  So auto stores nothing here, and the auto rule has tests of its own (test_attention_probs_auto_*),
    # which restore the shipped budget.  Through the environment as well, so spawned worker processes (the
    # multi-rank tests) run the same paths as the single-process runs they are compared with.
    os.environ["VIT_ATTENTION_PROBS_AUTO_BYTES"] = "0"
    from VisionTransformer import vit
    vit.ATTENTION_PROBS_AUTO_BYTES = 0


@pytest.fixture
def probs_auto_budget(monkeypatch):
    """The shipped store_attention_probs=None budget (pinned to 0 for every other test, pytest_configure)."""
    from VisionTransformer import vit
    monkeypatch.setattr(vit, "ATTENTION_PROBS_AUTO_BYTES", 256 << 20)
    return vit.ATTENTION_PROBS_AUTO_BYTES


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
