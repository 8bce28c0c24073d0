import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "moeva2-ijcai22-replication_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
RES = os.path.join(PKG, "resources")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via the C-ABI library)")
    config.addinivalue_line("markers", "slow: CPU test of more than ~10 s (still in the default run)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)

    return load


@pytest.fixture(autouse=True)
def _device_index_checks(request):
    """In a device-index-checks build (MOEVA_MI355X_LIB=...libmoeva_mi355x_checks.so, built
    with -DMV_CHECKS: csrc/check.h), every GPU test also asserts that no kernel computed an
    out-of-range row / slot / gene index."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    if "checks" not in os.environ.get("MOEVA_MI355X_LIB", "") and \
            not os.environ.get("MV_ASSERT_CHECKS"):
        return
    from moeva2_amd import _native

    on, rec = _native.debug_checks()
    assert on, "MOEVA_MI355X_LIB is not a checks build"
    assert rec[0] == 0, f"device index check failed: {rec}"
