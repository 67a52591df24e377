"""paritypartyfs_amd -- MI355X-native per-block ECC engine behind PPFS's block-device layer.

Product path: paritypartyfs_amd/csrc (HIP kernels for gfx950 + the C ABI of include/ppfs_ecc.h),
loaded from the in-tree libppfs_ecc.so.  Python pieces:
  - ecc.EccEngine            batch encode/decode/write/scrub on HBM tensors or host arrays
  - ecc.EccGroup             the host calls sharded over several GPUs (one thread per device)
  - ecc.vote3 / vote3_host   2-of-3 bitwise voting of replicated records (superblock copies)
  - block_device.*           IBlockDevice mirror (ReedSolomon/Crc/Hamming/Parity/Raw devices)
"""
from ._native import (ECC_CRC, ECC_HAMMING, ECC_NONE, ECC_PARITY, ECC_REED_SOLOMON, STATUS_CORRECTED,
                      STATUS_CORRECTION_ERROR, STATUS_OK, NativeLibraryMissing)
from .ecc import EccEngine, EccGroup, crc_implicit_to_explicit, device_copy, inject_bytes, pinned, vote3, vote3_host

__all__ = [
    "EccEngine", "EccGroup", "crc_implicit_to_explicit", "device_copy", "inject_bytes", "pinned", "vote3", "vote3_host", "NativeLibraryMissing",
    "ECC_NONE", "ECC_CRC", "ECC_HAMMING", "ECC_PARITY", "ECC_REED_SOLOMON",
    "STATUS_OK", "STATUS_CORRECTED", "STATUS_CORRECTION_ERROR",
]
