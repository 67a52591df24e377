"""CPU tests of the C-ABI library: it loads, exports every symbol include/*.h declares, and
validates parameters without touching the GPU.  No compute calls (no GPU here)."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "paritypartyfs_amd", "_lib", "libppfs_ecc.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-j8", "-C", os.path.join(ROOT, "paritypartyfs_amd", "csrc")], check=True,
                       capture_output=True)
    from paritypartyfs_amd import _native
    return _native.lib()


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(ppfs_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_header_declares_the_abi():
    names = declared_functions()
    from paritypartyfs_amd._native import EXPORTED_SYMBOLS
    assert names == set(EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(rf"\bT {name}$", out, flags=re.M), name


def test_library_has_gfx950_code_object():
    data = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    secs = subprocess.run(["readelf", "-S", LIB], capture_output=True, text=True).stdout
    assert ".hip_fatbin" in secs


def test_param_validation_without_gpu(lib):
    from paritypartyfs_amd._native import EccParams
    h = ctypes.c_void_p()
    bad = [EccParams(4, 0, 3, 0, 0), EccParams(4, 8192, 3, 0, 0), EccParams(9, 512, 3, 0, 0),
           EccParams(1, 512, 0, 0, 1), EccParams(1, 4, 0, 0, 0x1EDC6F41 | (1 << 32)),
           EccParams(1, 1, 0, 0, 0x107)]  # CRC degree 32 on 4 B / degree 8 on 1 B: no payload byte
    for p in bad:
        assert lib.ppfs_ecc_create(ctypes.byref(p), 0, ctypes.byref(h)) == -22
        assert lib.ppfs_ecc_last_error()


def test_crc_implicit_to_explicit(lib):
    assert lib.ppfs_ecc_crc_implicit_to_explicit(0xad0424f3) == 0x15a0849e7


def test_normal_build_has_no_debug_checks(lib):
    # PPFS_ECC_DEBUG instrumentation (csrc/dbg.hpp) is compiled out of the product library
    assert lib.ppfs_ecc_debug_faults() == -1
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    assert "ppfs_dbg_faults_" not in out


def test_debug_build_exports_its_counters():
    dbg = os.path.join(ROOT, "paritypartyfs_amd", "_lib", "alt", "libppfs_ecc_debug.so")
    if not os.path.exists(dbg):
        pytest.skip("no PPFS_ECC_DEBUG build (tools/build_alt.sh --product debug -DPPFS_ECC_DEBUG=1)")
    out = subprocess.run(["nm", "-D", "--defined-only", dbg], capture_output=True, text=True).stdout
    units = re.findall(r"\bT (ppfs_dbg_faults_\w+)$", out, flags=re.M)
    assert len(units) == 11, units  # 7 RS instantiations, generic RS, bit, bit-fast, vote


def test_inject_rejects_bad_buffers_without_gpu(lib):
    """bench.py's fault injection validates its buffers in the Python mirror (CPU tensors, short
    position / value arrays) and the C ABI rejects null pointers and bad modes before any launch."""
    import torch

    from paritypartyfs_amd import inject_bytes

    raw = torch.zeros(10 * 255, dtype=torch.uint8)
    pos = torch.zeros(10, dtype=torch.uint8)
    with pytest.raises(ValueError):
        inject_bytes(raw, 255, pos, pos)  # host tensors
    assert lib.ppfs_inject_device(None, 255, 4, None, None, 0, None) < 0
    buf = ctypes.create_string_buffer(64)
    assert lib.ppfs_inject_device(buf, 0, 4, buf, buf, 0, None) < 0  # zero stride
    assert lib.ppfs_inject_device(buf, 16, 4, buf, buf, 2, None) < 0  # unknown mode
    assert lib.ppfs_inject_device(None, 255, 0, None, None, 0, None) == 0  # nothing to do


def test_time_next_launch_arguments_without_gpu(lib):
    """The timing hook (bench.py's dispatch-packet kernel times) needs both events or neither."""
    assert lib.ppfs_ecc_time_next_launch(ctypes.c_void_p(1), None) == -22  # -EINVAL
    assert lib.ppfs_ecc_time_next_launch(None, ctypes.c_void_p(1)) == -22
    assert lib.ppfs_ecc_time_next_launch(None, None) == 0
