"""Shared fixtures.  Markers: `gpu` = needs an MI355X (HIP device)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "unpaper-gpu_amd", "python"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE_FIXTURES = os.path.join(GOLDEN, "reference")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a HIP device (MI355X)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def oracle():
    from oracle_py import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def hip():
    """The product backend; GPU tests FAIL (not skip) if it cannot load."""
    from unpaper_hip.device import Backend
    return Backend()


@pytest.fixture(scope="session")
def ref_path():
    def f(name):
        return os.path.join(REFERENCE_FIXTURES, name)
    return f
