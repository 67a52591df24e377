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

    gpu = request.node.get_closest_marker("gpu") is not None
    before = _native.debug_faults() if gpu else None
    reg_before = _native.host_registered() if gpu else None
    dma_before = _native.debug_dma_rejects() if gpu else None
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
    # PPFS_ECC_DEBUG builds refuse every engine copy with an end that is not page-locked / device
    # memory over its whole range (api.cpp dma_async): none may have been refused
    dma_after = _native.debug_dma_rejects()
    if dma_after is not None and dma_after != (dma_before or 0):
        pytest.fail(f"{dma_after - (dma_before or 0)} engine copies refused in {request.node.nodeid}: an end was not "
                    "page-locked / device memory over its range (PPFS_ECC_DEBUG; details on stderr)", pytrace=False)
    # no range registered through ppfs_ecc_host_register outlives the test that registered it (a stale
    # registration would make a later buffer at the same address look page-locked to the engine)
    reg_after = _native.host_registered()
    if reg_after is not None and reg_after[0] > (reg_before[0] if reg_before else 0):
        pytest.fail(f"{reg_after[0] - (reg_before[0] if reg_before else 0)} host range(s) registered through "
                    f"ppfs_ecc_host_register outlived {request.node.nodeid} ({reg_after[1]} B registered)", pytrace=False)
