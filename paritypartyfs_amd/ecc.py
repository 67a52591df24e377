"""EccEngine: one codec context on one GPU (wraps ppfs_ecc_ctx from include/ppfs_ecc.h).

Device-resident calls take torch uint8 CUDA tensors (HBM buffers, packed blocks) and enqueue
the HIP kernels on the current torch stream; host calls take numpy uint8 arrays and go through
the library's pinned, double-buffered staging.  torch is used only as the HBM allocator and
stream provider.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_void_p
from typing import Optional

import numpy as np

from . import _native
from ._native import EccParams, check, lib


def _ptr(x) -> Optional[int]:
    """Device/host address of a torch tensor or numpy array (None passes NULL)."""
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        if not x.flags["C_CONTIGUOUS"] or x.dtype != np.uint8:
            raise ValueError("numpy buffers must be C-contiguous uint8")
        return x.ctypes.data
    # torch tensor
    if not x.is_contiguous() or x.element_size() != 1:
        raise ValueError("tensors must be contiguous uint8")
    return x.data_ptr()


def _size(x) -> int:
    """Bytes of a uint8 buffer (numpy array or torch tensor)."""
    return int(x.size) if isinstance(x, np.ndarray) else int(x.numel())


def _need(name: str, x, nbytes: int, kind: str) -> None:
    """Reject a buffer shorter than the call will touch (the library trusts its sizes: a short
    host array would overflow the heap, a short tensor would be written out of bounds in HBM),
    and a buffer of the wrong memory kind for the entry point."""
    if x is None:
        return
    if kind == "device":
        if isinstance(x, np.ndarray) or not getattr(x, "is_cuda", False):
            raise ValueError(f"{name}: device entry points take CUDA tensors")
    elif not isinstance(x, np.ndarray):
        raise ValueError(f"{name}: host entry points take numpy arrays")
    if _size(x) < nbytes:
        raise ValueError(f"{name}: {_size(x)} bytes < {nbytes} needed")


def _host_blocks(x, per_block: int, name: str) -> int:
    """Blocks a host array holds (the block count the *_host calls take from it)."""
    if not isinstance(x, np.ndarray):
        raise ValueError(f"{name}: host entry points take numpy arrays")
    return x.size // per_block


def _stream_handle(stream) -> Optional[int]:
    if stream is not None:
        return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
    import torch

    return torch.cuda.current_stream().cuda_stream


class EccEngine:
    """Codec context: params follow PpFS::_createAppropriateBlockDevice (ppfs.cpp:35-70)."""

    def __init__(self, ecc_type: int, block_size: int, rs_correctable_bytes: int = 3,
                 crc_polynomial_explicit: int = 0, device: int = 0):
        p = EccParams(int(ecc_type), int(block_size), int(rs_correctable_bytes), 0, int(crc_polynomial_explicit))
        h = c_void_p()
        check(lib().ppfs_ecc_create(byref(p), int(device), byref(h)))
        self._h = h
        self.ecc_type = int(ecc_type)
        self.block_size = int(block_size)
        self.device = int(device)
        self.raw_block_size = int(lib().ppfs_ecc_raw_block_size(h))
        self.data_size = int(lib().ppfs_ecc_data_size(h))
        self.kernel_name = lib().ppfs_ecc_kernel_name(h).decode()

    def stream_kernel_name(self, stream=None) -> str:
        """The kernel path a device call on `stream` (default: torch's current stream) takes
        (ppfs_ecc_stream_kernel_name): kernel_name, except that RS 2t <= 8 runs its static-walk
        kernels on a 17th distinct stream and on a stream capturing a graph."""
        return lib().ppfs_ecc_stream_kernel_name(self._h, _stream_handle(stream)).decode()

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().ppfs_ecc_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------- device-resident batches (torch CUDA uint8 tensors) ----------------
    def _check(self, kind, n, data=None, raw=None, status=None, spill=None) -> None:
        if n < 0:
            raise ValueError("nblocks must be >= 0")
        _need("data", data, n * self.data_size, kind)
        _need("raw", raw, n * self.raw_block_size, kind)
        _need("status", status, n, kind)
        _need("spill", spill, n * self.spill_bytes_per_block(), kind)

    def _nblocks(self, data, raw) -> int:
        """Blocks a call covers when nblocks is not given: from the payloads, or from the raw
        blocks for codecs without payload bytes (Hamming power 0, 1-byte parity blocks)."""
        return _size(data) // self.data_size if self.data_size else _size(raw) // self.raw_block_size

    def encode(self, data, raw, nblocks: Optional[int] = None, stream=None) -> None:
        n = nblocks if nblocks is not None else self._nblocks(data, raw)
        self._check("device", n, data, raw)
        check(lib().ppfs_ecc_encode_device(self._h, _ptr(data), _ptr(raw), n, _stream_handle(stream)))

    def decode(self, raw, data=None, status=None, write_back: bool = True, spill=None,
               nblocks: Optional[int] = None, stream=None) -> None:
        n = nblocks if nblocks is not None else raw.numel() // self.raw_block_size
        self._check("device", n, data, raw, status, spill)
        check(lib().ppfs_ecc_decode_device(self._h, _ptr(raw), _ptr(data), _ptr(status), n, int(bool(write_back)),
                                           _ptr(spill), _stream_handle(stream)))

    def write(self, data, raw, status=None, nblocks: Optional[int] = None, stream=None) -> None:
        n = nblocks if nblocks is not None else self._nblocks(data, raw)
        self._check("device", n, data, raw, status)
        check(lib().ppfs_ecc_write_device(self._h, _ptr(data), _ptr(raw), _ptr(status), n,
                                          _stream_handle(stream)))

    # ---------------- host-memory batches (numpy uint8) ----------------
    def encode_host(self, data: np.ndarray, raw: np.ndarray) -> None:
        n = _host_blocks(data, self.data_size, "data") if self.data_size else _host_blocks(raw, self.raw_block_size, "raw")
        self._check("host", n, data, raw)
        check(lib().ppfs_ecc_encode_host(self._h, _ptr(data), _ptr(raw), n))

    def decode_host(self, raw: np.ndarray, data: Optional[np.ndarray] = None, status: Optional[np.ndarray] = None,
                    write_back: bool = True, spill: Optional[np.ndarray] = None) -> None:
        n = _host_blocks(raw, self.raw_block_size, "raw")
        self._check("host", n, data, raw, status, spill)
        check(lib().ppfs_ecc_decode_host(self._h, _ptr(raw), _ptr(data), _ptr(status), n, int(bool(write_back)),
                                         _ptr(spill)))

    def write_host(self, data: np.ndarray, raw: np.ndarray, status: Optional[np.ndarray] = None) -> None:
        n = _host_blocks(data, self.data_size, "data") if self.data_size else _host_blocks(raw, self.raw_block_size, "raw")
        self._check("host", n, data, raw, status)
        check(lib().ppfs_ecc_write_host(self._h, _ptr(data), _ptr(raw), _ptr(status), n))

    def host_chunk_blocks(self) -> int:
        """Blocks per staging chunk of the *_host calls (ppfs_ecc_host_chunk_blocks)."""
        return int(lib().ppfs_ecc_host_chunk_blocks(self._h))

    def spill_bytes_per_block(self) -> int:
        return 256 - min(self.raw_block_size, 255)

    # ---------------- whole-image scrub ----------------
    def scrub_host(self, image: np.ndarray, nblocks: Optional[int] = None, status: Optional[np.ndarray] = None):
        """readBlock(i) for every block of a host image, in order, for its write-back effect only
        (include/ppfs_ecc.h ppfs_ecc_scrub_host).  Returns (ok, corrected, failed) block counts."""
        n = nblocks if nblocks is not None else _host_blocks(image, self.raw_block_size, "image")
        self._check("host", n, raw=image, status=status)
        counts = (ctypes.c_size_t * 3)()
        check(lib().ppfs_ecc_scrub_host(self._h, _ptr(image), image.size, n, _ptr(status), counts))
        return int(counts[0]), int(counts[1]), int(counts[2])

    def scrub(self, image, status=None, nblocks: Optional[int] = None, stream=None) -> None:
        """Device-resident scrub of a torch uint8 image (ppfs_ecc_scrub_device)."""
        n = nblocks if nblocks is not None else image.numel() // self.raw_block_size
        self._check("device", n, raw=image, status=status)
        check(lib().ppfs_ecc_scrub_device(self._h, _ptr(image), image.numel(), n, _ptr(status),
                                          _stream_handle(stream)))


class EccGroup:
    """Multi-GPU host path (include/ppfs_ecc.h ppfs_ecc_group_*): one context per
    listed device (a device may repeat); the *_host calls shard a batch into contiguous block
    ranges, one host thread per context, with no data exchanged between devices."""

    def __init__(self, ecc_type: int, block_size: int, rs_correctable_bytes: int = 3,
                 crc_polynomial_explicit: int = 0, devices=(0,)):
        p = EccParams(int(ecc_type), int(block_size), int(rs_correctable_bytes), 0, int(crc_polynomial_explicit))
        devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        h = c_void_p()
        check(lib().ppfs_ecc_group_create(byref(p), devs, len(devices), byref(h)))
        self._h = h
        self.devices = tuple(int(d) for d in devices)
        c0 = lib().ppfs_ecc_group_ctx(h, 0)
        self.raw_block_size = int(lib().ppfs_ecc_raw_block_size(c0))
        self.data_size = int(lib().ppfs_ecc_data_size(c0))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().ppfs_ecc_group_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, n, data=None, raw=None, status=None, spill=None) -> None:
        _need("data", data, n * self.data_size, "host")
        _need("raw", raw, n * self.raw_block_size, "host")
        _need("status", status, n, "host")
        _need("spill", spill, n * (256 - min(self.raw_block_size, 255)), "host")

    def encode_host(self, data: np.ndarray, raw: np.ndarray) -> None:
        n = _host_blocks(data, self.data_size, "data")
        self._check(n, data, raw)
        check(lib().ppfs_ecc_group_encode_host(self._h, _ptr(data), _ptr(raw), n))

    def decode_host(self, raw: np.ndarray, data: Optional[np.ndarray] = None, status: Optional[np.ndarray] = None,
                    write_back: bool = True, spill: Optional[np.ndarray] = None) -> None:
        n = _host_blocks(raw, self.raw_block_size, "raw")
        self._check(n, data, raw, status, spill)
        check(lib().ppfs_ecc_group_decode_host(self._h, _ptr(raw), _ptr(data), _ptr(status), n,
                                               int(bool(write_back)), _ptr(spill)))

    def write_host(self, data: np.ndarray, raw: np.ndarray, status: Optional[np.ndarray] = None) -> None:
        n = _host_blocks(data, self.data_size, "data")
        self._check(n, data, raw, status)
        check(lib().ppfs_ecc_group_write_host(self._h, _ptr(data), _ptr(raw), _ptr(status), n))


class pinned:
    """Page-lock numpy arrays for the duration of a `with` block (ppfs_ecc_host_register): the
    *_host calls then DMA them directly instead of copying through staging buffers."""

    def __init__(self, *arrays: np.ndarray):
        self._arrays = [a for a in arrays if a is not None and a.nbytes]

    def __enter__(self):
        done = []
        try:
            for a in self._arrays:
                check(lib().ppfs_ecc_host_register(_ptr(a), a.nbytes))
                done.append(a)
        except Exception:
            for a in done:
                lib().ppfs_ecc_host_unregister(_ptr(a))
            raise
        return self

    def __exit__(self, *exc):
        # every array is released even when one release fails; the first failure is raised after
        rcs = [lib().ppfs_ecc_host_unregister(_ptr(a)) for a in self._arrays]
        for rc in rcs:
            check(rc)
        return False


def vote3_host(a: np.ndarray, b: np.ndarray, c: np.ndarray, rec_bytes: Optional[int] = None, device: int = 0):
    """2-of-3 bitwise majority of replicated records (SuperBlockManager::_performBitVoting,
    super_block_manager.cpp:133-165) on the GPU.  Returns (voted bytes, per-record damage bits:
    bit k = copy k+1 differs from the majority)."""
    a, b, c = (np.ascontiguousarray(x, dtype=np.uint8).reshape(-1) for x in (a, b, c))
    if not (a.size == b.size == c.size):
        raise ValueError("vote3: copies differ in size")
    rb = int(rec_bytes) if rec_bytes is not None else a.size
    if rb < 0 or (rb == 0 and a.size) or (rb and a.size % rb):
        raise ValueError("vote3: the copies must hold a whole number of records")
    nrec = a.size // rb if rb else 0
    out = np.empty_like(a)
    dmg = np.zeros(nrec, dtype=np.uint32)
    check(lib().ppfs_vote3_host(int(device), _ptr(a), _ptr(b), _ptr(c), _ptr(out), rb, nrec, dmg.ctypes.data))
    return out, dmg


def vote3(a, b, c, out, rec_bytes: int, damaged=None, stream=None) -> None:
    """Device-resident vote3 over torch uint8 tensors; damaged: int32 tensor of nrec (or None)."""
    if rec_bytes <= 0:
        raise ValueError("vote3: rec_bytes must be > 0")
    nrec = a.numel() // rec_bytes
    nbytes = nrec * rec_bytes
    for name, x in (("b", b), ("c", c), ("out", out)):
        _need(name, x, nbytes, "device")
    _need("a", a, nbytes, "device")
    if damaged is not None:
        if damaged.element_size() != 4 or not damaged.is_contiguous() or damaged.numel() < nrec:
            raise ValueError("vote3: damaged must be a contiguous 4-byte tensor of >= nrec elements")
        if not damaged.is_cuda:
            raise ValueError("vote3: damaged must be a CUDA tensor")
    dptr = None if damaged is None else damaged.data_ptr()
    check(lib().ppfs_vote3_device(_ptr(a), _ptr(b), _ptr(c), _ptr(out), rec_bytes, nrec, dptr,
                                  _stream_handle(stream)))


def device_copy(dst, src, nbytes: Optional[int] = None, stream=None) -> None:
    """dst[:nbytes] = src[:nbytes] on the device (torch uint8 tensors): the full-grid copy kernel
    bench.py times as the HBM ceiling next to the roofline (not part of the reference interface)."""
    n = int(src.numel() if nbytes is None else nbytes)
    if n > dst.numel() or n > src.numel():
        raise ValueError("device_copy: nbytes exceeds a buffer")
    check(lib().ppfs_copy_device(_ptr(dst), _ptr(src), n, _stream_handle(stream)))


def inject_bytes(raw, stride: int, pos, val, nblocks: Optional[int] = None, xor: bool = False, stream=None) -> None:
    """Corrupt one byte per block of a device raw image (torch uint8 tensors): block b's byte
    pos[b] becomes val[b] (or byte ^ val[b] with xor=True); pos[b] >= stride skips the block.
    bench.py's fault injection (not part of the reference interface; the reference's bit flipper,
    usage_simulator/simulation/src/bit_flipper.cpp, is a simulator and out of scope)."""
    nb = int(pos.numel() if nblocks is None else nblocks)
    for name, t in (("raw", raw), ("pos", pos), ("val", val)):
        if not t.is_cuda or t.element_size() != 1 or not t.is_contiguous():
            raise ValueError(f"inject_bytes: {name} must be a contiguous CUDA uint8 tensor")
    if stride <= 0 or nb > pos.numel() or nb > val.numel() or nb * stride > raw.numel():
        raise ValueError("inject_bytes: a buffer is shorter than nblocks implies")
    check(lib().ppfs_inject_device(_ptr(raw), stride, nb, _ptr(pos), _ptr(val), 1 if xor else 0,
                                   _stream_handle(stream)))


def crc_implicit_to_explicit(p: int) -> int:
    """CrcPolynomial::MsgImplicit (crc_polynomial.cpp:41-54) -> explicit form."""
    return int(lib().ppfs_ecc_crc_implicit_to_explicit(ctypes.c_uint64(p)))


__all__ = ["EccEngine", "crc_implicit_to_explicit", "device_copy", "inject_bytes", "pinned", "vote3", "vote3_host", "_native"]
