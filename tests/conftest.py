import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

# Every scan in the test session verifies the frame-table invariant the
# unmask tile index stands on (non-decreasing frame ends; include/hvws.h
# hvws_set_table_checks) and fails loudly if a producer breaks it.
os.environ.setdefault("HVWS_CHECK_TABLES", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE.json) configurations")


@pytest.fixture(scope="session")
def eng():
    import libhv_amd

    e = libhv_amd.Engine(0)
    yield e
    e.close()
