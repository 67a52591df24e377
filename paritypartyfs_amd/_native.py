"""ctypes binding of the C ABI in include/ppfs_ecc.h (libppfs_ecc.so, built in-tree).

The library is the product path: it holds the HIP kernels for gfx950.  Loading fails loudly
when it is missing -- there is no CPU fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_longlong, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# PPFS_ECC_LIB: an alternative build of the same library (ablation runs, tools/)
LIB_PATH = os.environ.get("PPFS_ECC_LIB") or os.path.join(_HERE, "_lib", "libppfs_ecc.so")

# ECCType (lib/blockdevice/include/ppfs/blockdevice/ecc_type.hpp:8-14)
ECC_NONE, ECC_CRC, ECC_HAMMING, ECC_PARITY, ECC_REED_SOLOMON = 0, 1, 2, 3, 4

STATUS_OK, STATUS_CORRECTED, STATUS_CORRECTION_ERROR = 0, 1, 5

# every symbol include/ppfs_ecc.h declares
EXPORTED_SYMBOLS = (
    "ppfs_ecc_crc_implicit_to_explicit",
    "ppfs_ecc_create",
    "ppfs_ecc_destroy",
    "ppfs_ecc_raw_block_size",
    "ppfs_ecc_data_size",
    "ppfs_ecc_kernel_name",
    "ppfs_ecc_stream_kernel_name",
    "ppfs_ecc_time_next_launch",
    "ppfs_ecc_encode_device",
    "ppfs_ecc_decode_device",
    "ppfs_ecc_write_device",
    "ppfs_ecc_encode_host",
    "ppfs_ecc_decode_host",
    "ppfs_ecc_write_host",
    "ppfs_ecc_host_chunk_blocks",
    "ppfs_ecc_scrub_host",
    "ppfs_ecc_scrub_device",
    "ppfs_vote3_device",
    "ppfs_vote3_host",
    "ppfs_copy_device",
    "ppfs_inject_device",
    "ppfs_ecc_host_register",
    "ppfs_ecc_host_unregister",
    "ppfs_ecc_host_registered",
    "ppfs_ecc_group_create",
    "ppfs_ecc_group_destroy",
    "ppfs_ecc_group_size",
    "ppfs_ecc_group_ctx",
    "ppfs_ecc_group_encode_host",
    "ppfs_ecc_group_decode_host",
    "ppfs_ecc_group_write_host",
    "ppfs_ecc_last_error",
    "ppfs_ecc_debug_faults",
    "ppfs_ecc_debug_selftest",
    "ppfs_ecc_debug_dma_rejects",
    "ppfs_ecc_debug_dma_selftest",
)


class EccParams(ctypes.Structure):
    _fields_ = [
        ("ecc_type", c_uint32),
        ("block_size", c_uint32),
        ("rs_correctable_bytes", c_uint32),
        ("reserved", c_uint32),
        ("crc_polynomial", c_uint64),
    ]


class NativeLibraryMissing(RuntimeError):
    pass


_lib = None


def lib() -> ctypes.CDLL:
    """Load libppfs_ecc.so (raises NativeLibraryMissing if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} not found: build it with `make -C paritypartyfs_amd/csrc` "
            "(or __graft_entry__.build()); the HIP engine has no CPU fallback")
    # torch bundles its own libamdhip64; with both runtimes in one process torch's has to
    # initialise first (measured: the other order leaves torch with "No HIP GPUs are available")
    try:
        import torch

        torch.cuda.is_available()
    except Exception:
        pass
    L = ctypes.CDLL(LIB_PATH)
    u8p = POINTER(c_uint8)
    L.ppfs_ecc_debug_faults.restype = c_longlong
    L.ppfs_ecc_debug_faults.argtypes = []
    L.ppfs_ecc_debug_selftest.restype = c_longlong
    L.ppfs_ecc_debug_selftest.argtypes = []
    L.ppfs_ecc_debug_dma_rejects.restype = c_longlong
    L.ppfs_ecc_debug_dma_rejects.argtypes = []
    L.ppfs_ecc_debug_dma_selftest.restype = c_longlong
    L.ppfs_ecc_debug_dma_selftest.argtypes = []
    L.ppfs_ecc_host_registered.restype = c_longlong
    L.ppfs_ecc_host_registered.argtypes = [POINTER(c_size_t)]
    L.ppfs_ecc_time_next_launch.restype = c_int
    L.ppfs_ecc_time_next_launch.argtypes = [c_void_p, c_void_p]
    L.ppfs_ecc_stream_kernel_name.restype = c_char_p
    L.ppfs_ecc_stream_kernel_name.argtypes = [c_void_p, c_void_p]
    L.ppfs_ecc_crc_implicit_to_explicit.restype = c_uint64
    L.ppfs_ecc_crc_implicit_to_explicit.argtypes = [c_uint64]
    L.ppfs_ecc_create.restype = c_int
    L.ppfs_ecc_create.argtypes = [POINTER(EccParams), c_int, POINTER(c_void_p)]
    L.ppfs_ecc_destroy.restype = None
    L.ppfs_ecc_destroy.argtypes = [c_void_p]
    L.ppfs_ecc_raw_block_size.restype = c_size_t
    L.ppfs_ecc_raw_block_size.argtypes = [c_void_p]
    L.ppfs_ecc_data_size.restype = c_size_t
    L.ppfs_ecc_data_size.argtypes = [c_void_p]
    L.ppfs_ecc_kernel_name.restype = c_char_p
    L.ppfs_ecc_kernel_name.argtypes = [c_void_p]
    L.ppfs_ecc_encode_device.restype = c_int
    L.ppfs_ecc_encode_device.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    L.ppfs_ecc_decode_device.restype = c_int
    L.ppfs_ecc_decode_device.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_void_p,
                                         c_void_p]
    L.ppfs_ecc_write_device.restype = c_int
    L.ppfs_ecc_write_device.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    L.ppfs_ecc_host_chunk_blocks.restype = c_size_t
    L.ppfs_ecc_host_chunk_blocks.argtypes = [c_void_p]
    L.ppfs_ecc_encode_host.restype = c_int
    L.ppfs_ecc_encode_host.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t]
    L.ppfs_ecc_decode_host.restype = c_int
    L.ppfs_ecc_decode_host.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_void_p]
    L.ppfs_ecc_write_host.restype = c_int
    L.ppfs_ecc_write_host.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]
    L.ppfs_ecc_scrub_host.restype = c_int
    L.ppfs_ecc_scrub_host.argtypes = [c_void_p, c_void_p, c_size_t, c_size_t, c_void_p, POINTER(c_size_t)]
    L.ppfs_ecc_scrub_device.restype = c_int
    L.ppfs_ecc_scrub_device.argtypes = [c_void_p, c_void_p, c_size_t, c_size_t, c_void_p, c_void_p]
    L.ppfs_vote3_device.restype = c_int
    L.ppfs_vote3_device.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_size_t, c_void_p, c_void_p]
    L.ppfs_copy_device.restype = c_int
    L.ppfs_copy_device.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p]
    L.ppfs_inject_device.restype = c_int
    L.ppfs_inject_device.argtypes = [c_void_p, c_size_t, c_size_t, c_void_p, c_void_p, c_int, c_void_p]
    L.ppfs_vote3_host.restype = c_int
    L.ppfs_vote3_host.argtypes = [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_size_t, c_void_p]
    L.ppfs_ecc_host_register.restype = c_int
    L.ppfs_ecc_host_register.argtypes = [c_void_p, c_size_t]
    L.ppfs_ecc_host_unregister.restype = c_int
    L.ppfs_ecc_host_unregister.argtypes = [c_void_p]
    L.ppfs_ecc_group_create.restype = c_int
    L.ppfs_ecc_group_create.argtypes = [POINTER(EccParams), POINTER(c_int), c_int, POINTER(c_void_p)]
    L.ppfs_ecc_group_destroy.restype = None
    L.ppfs_ecc_group_destroy.argtypes = [c_void_p]
    L.ppfs_ecc_group_size.restype = c_int
    L.ppfs_ecc_group_size.argtypes = [c_void_p]
    L.ppfs_ecc_group_ctx.restype = c_void_p
    L.ppfs_ecc_group_ctx.argtypes = [c_void_p, c_int]
    L.ppfs_ecc_group_encode_host.restype = c_int
    L.ppfs_ecc_group_encode_host.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t]
    L.ppfs_ecc_group_decode_host.restype = c_int
    L.ppfs_ecc_group_decode_host.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_void_p]
    L.ppfs_ecc_group_write_host.restype = c_int
    L.ppfs_ecc_group_write_host.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]
    L.ppfs_ecc_last_error.restype = c_char_p
    L.ppfs_ecc_last_error.argtypes = []
    _ = u8p
    _lib = L
    return L


class EccError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"ppfs_ecc error {code}: {what}")
        self.code = code


def check(rc: int) -> None:
    if rc != 0:
        raise EccError(rc, lib().ppfs_ecc_last_error().decode(errors="replace"))


def host_registered() -> tuple[int, int] | None:
    """(ranges, bytes) still registered through ppfs_ecc_host_register; None if the library is not
    loaded yet (nothing can have been registered through it then)."""
    if _lib is None:
        return None
    b = c_size_t(0)
    n = int(_lib.ppfs_ecc_host_registered(ctypes.byref(b)))
    return n, int(b.value)


def debug_dma_rejects() -> int | None:
    """Copies a PPFS_ECC_DEBUG build refused (an end not page-locked / device memory over its whole
    range); None for a normal build or when the library is not loaded yet."""
    if _lib is None:
        return None
    v = int(_lib.ppfs_ecc_debug_dma_rejects())
    return None if v < 0 else v


def debug_faults() -> int | None:
    """Out-of-bounds global accesses detected so far by a PPFS_ECC_DEBUG build of the library
    (csrc/dbg.hpp); None when the loaded library is a normal build or is not loaded yet."""
    if _lib is None:
        return None
    v = int(_lib.ppfs_ecc_debug_faults())
    if v == -1:
        return None
    if v < 0:
        raise RuntimeError(f"ppfs_ecc_debug_faults failed ({v})")
    return v
