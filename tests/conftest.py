import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(autouse=True)
def _reset_engine_tuning(request):
    """After EVERY GPU test: every ptyx_set_tuning key back to its measured default, so a variant
    one test selects can never leak into the next (a leaked gather variant failed a
    later test's split-invariance check)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    from ptyrad_amd import _lib
    if _lib._lib is None:
        return
    for k in _lib.TUNING_KEYS:
        _lib.set_tuning(k, -1)
