import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ofdm-sync-math_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture
def variant():
    """Setter of the library's debug / A-B variants (include/ofdmsync.h ofs_debug_set_variant):
    ``variant("EXACT", 0)`` forces one, ``variant("EXACT", None)`` clears it; all are cleared
    after the test.  The library reads no environment, so this is the only way to select one."""
    from ofdm_sync_amd import _lib
    _lib.reset_variants()
    yield _lib.set_variant
    _lib.reset_variants()
