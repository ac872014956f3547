import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "akarirender-1_amd", ROOT / "oracle", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"
CORNELL_MESH = GOLDEN / "CornellBox-Original.obj.mesh"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libakr_hip.so on device 0)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    import __graft_entry__
    __graft_entry__.build()


@pytest.fixture(scope="session")
def hip_ctx_factory():
    from akari_amd import capi
    if capi.device_count() == 0:
        pytest.fail("gpu test selected but no HIP device is visible")
    return capi.HipContext
