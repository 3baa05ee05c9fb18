import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")

# MIOpen find results kept in-tree (as bench.py uses them): the conv tests skip the exhaustive search
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "tuning", "miopen", "db"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(REPO, "tuning", "miopen", "cache"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def gpu_available() -> bool:
    import torch
    return torch.cuda.is_available()


@pytest.fixture(autouse=True)
def _lss_debug_checks(request):
    """LSS_DEBUG=1 (liblss_hip_debug.so): after every GPU test, no device-side index check may have
    failed (include/lss_hip.h, lss_debug_status)."""
    yield
    if os.environ.get("LSS_DEBUG", "0") != "1" or request.node.get_closest_marker("gpu") is None:
        return
    import torch
    if not torch.cuda.is_available():
        return
    from lss_carla_amd import _lib
    torch.cuda.synchronize()
    st = _lib.debug_status(clear=True)
    assert _lib.load().lss_debug_checks() == 1, "LSS_DEBUG=1 but the product library was loaded"
    assert st[0] == 0, f"device index check failed: {st[0]} failures, first: code {st[1]} value {st[2]} bound {st[3]}"
