"""The C++ IBlockDevice adapter (include/ppfs_gpu/block_device.hpp) and its test program.

CPU: the adapter header and tests/cpp/test_block_devices.cpp compile and link against the
engine library and the oracle.  GPU: the program runs the reference's block-device unit tests
(restated) and differential operation sequences against the oracle's device model.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "_build", "test_block_devices")


def _build():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return BIN


def test_cpp_adapter_builds():
    if not os.path.exists(os.path.join(ROOT, "paritypartyfs_amd", "_lib", "libppfs_ecc.so")):
        pytest.skip("engine library not built (run __graft_entry__.build())")
    assert os.path.exists(_build())


@pytest.mark.gpu
def test_cpp_adapter_reference_tests_and_differential():
    exe = _build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout[-4000:] + r.stderr[-4000:]
