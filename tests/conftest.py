import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    from tests.oracle_lib import Oracle
    return Oracle()


@pytest.fixture(autouse=True)
def _gpu_fault_guard(request):
    """After every GPU test: collect the test's garbage (engine contexts destroyed here, not at some
    later test's GC point), then drain the device.  A fault of work a test queued asynchronously
    is then reported against that test, not at the next unrelated torch call."""
    from paritypartyfs_amd import _native

    before = _native.debug_faults() if request.node.get_closest_marker("gpu") is not None else None
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import gc

    gc.collect()
    import torch

    if torch.cuda.is_available():
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:  # sticky asynchronous error: name the test that queued it
            pytest.fail(f"asynchronous GPU fault after {request.node.nodeid}: {e}", pytrace=False)
    # PPFS_ECC_DEBUG builds (PPFS_ECC_LIB=.../libppfs_ecc_debug.so): kernels count the global
    # accesses outside the extents their launch implies (csrc/dbg.hpp)
    after = _native.debug_faults()
    if after is not None and after != (before or 0):
        pytest.fail(f"{after - (before or 0)} out-of-bounds kernel accesses in {request.node.nodeid} "
                    "(PPFS_ECC_DEBUG; details on stdout)", pytrace=False)
