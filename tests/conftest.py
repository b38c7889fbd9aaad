import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def pytest_report_header(config):
    lib = os.environ.get("DQ_GPU_LIB")
    return f"DQ_GPU_LIB={lib}" if lib else None


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


@pytest.fixture(autouse=True)
def _device_checks(request):
    """Under the device bounds-checked build (DQ_GPU_LIB=.../libdisq_gpu_checked.so), a test whose
    kernels failed a device check fails."""
    yield
    lib_path = os.environ.get("DQ_GPU_LIB", "")
    if "checked" not in os.path.basename(lib_path) or request.node.get_closest_marker("gpu") is None:
        return
    from disq_amd import _lib
    checked, fails = _lib.checked_report()
    assert checked, f"{lib_path} is not a DQ_CHECKED build"
    if fails:
        print(f"\n[DQ_CHECKED] {request.node.nodeid}: failed device checks {fails}")
    assert not fails, fails
