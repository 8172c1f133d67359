import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "whisper-diarize-rs_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# Contexts size their KV pool for WDR_DECODE_CHAINS chains at creation (library default 40: 62 GB
# for large-v3).  Several contexts can be alive at once in one test process (module fixtures beside
# a test's own), so the suite pins the pool at 24 chains unless a test sets its own; results are
# identical for every chain count (tests/test_gpu_chains.py).
os.environ.setdefault("WDR_DECODE_CHAINS", "24")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libwdr's HIP path)")
    config.addinivalue_line("markers", "slow: longer CPU cases")


@pytest.fixture(scope="session")
def lib():
    """libwdr loaded through the wdr ctypes mirror (builds nothing; __graft_entry__.build() does)."""
    from wdr import _lib
    return _lib.load()
