"""Python mirror of PPFS's block-device layer, backed by the MI355X ECC engine.

Same class names, constructor arguments, return conventions and error behaviour as the
reference (lib/blockdevice/include/ppfs/blockdevice/*.hpp, iblock_device.hpp:34-97), so the
parity tests read like the reference's unit tests:

  - ``writeBlock(data, DataLocation(i, off)) -> Expected[int]`` (bytes written)
  - ``readBlock(DataLocation(i, off), n, capacity=None) -> Expected[bytes]``
  - ``rawBlockSize() / dataSize() / numOfBlocks() / formatBlock(i)``

All codec arithmetic runs in the HIP kernels (EccEngine host path); this layer only moves
bytes between the disk and the engine and reproduces the reference's read-modify-write,
write-back and logging order.  Batched ``readBlocks`` / ``writeBlocks`` run a contiguous
range of blocks through one engine call (the GPU-worthwhile form).
"""
from __future__ import annotations

import enum
import math
from dataclasses import dataclass
from typing import Generic, List, Optional, Tuple, TypeVar

import numpy as np

from ._native import (ECC_CRC, ECC_HAMMING, ECC_NONE, ECC_PARITY, ECC_REED_SOLOMON, STATUS_CORRECTED,
                      STATUS_CORRECTION_ERROR)
from .ecc import EccEngine

MAX_BLOCK_SIZE = 4096  # iblock_device.hpp:3
MAX_RS_BLOCK_SIZE = 255  # rs_block_device.hpp:7


class ECCType(enum.IntEnum):  # ecc_type.hpp:8-14
    None_ = ECC_NONE
    Crc = ECC_CRC
    Hamming = ECC_HAMMING
    Parity = ECC_PARITY
    ReedSolomon = ECC_REED_SOLOMON


class FsError(enum.IntEnum):  # lib/common/include/ppfs/common/types.hpp:11-80 (block-device subset)
    Bitmap_IndexOutOfRange = 0
    Bitmap_NotFound = 1
    BlockManager_AlreadyTaken = 2
    BlockManager_AlreadyFree = 3
    BlockManager_NoMoreFreeBlocks = 4
    BlockDevice_CorrectionError = 5
    DirectoryManager_NameTaken = 6
    DirectoryManager_NotFound = 7
    DirectoryManager_InvalidRequest = 8
    Disk_OutOfBounds = 9
    Disk_InvalidRequest = 10
    Disk_IOError = 11


T = TypeVar("T")


class Expected(Generic[T]):
    """std::expected<T, FsError> stand-in."""

    __slots__ = ("_v", "_e")

    def __init__(self, value: T = None, error: Optional[FsError] = None):
        self._v, self._e = value, error

    @staticmethod
    def unexpected(e: FsError) -> "Expected":
        return Expected(None, FsError(e))

    def has_value(self) -> bool:
        return self._e is None

    __bool__ = has_value

    def value(self) -> T:
        if self._e is not None:
            raise RuntimeError(f"bad expected access: {self._e.name}")
        return self._v

    def error(self) -> FsError:
        return self._e


@dataclass
class DataLocation:  # iblock_device.hpp:14-20
    block_index: int
    offset: int = 0


# ------------------------------------------------------------------------------------
# Disks (lib/disk): byte-addressed, out-of-range accesses fail whole (stack_disk.hpp:19-44)
# ------------------------------------------------------------------------------------
class IDisk:
    def read(self, address: int, size: int) -> Expected[bytes]:
        raise NotImplementedError

    def write(self, address: int, data) -> Expected[int]:
        raise NotImplementedError

    def size(self) -> int:
        raise NotImplementedError


class HeapDisk(IDisk):
    def __init__(self, size: int):
        self.buf = np.zeros(int(size), dtype=np.uint8)

    def size(self) -> int:
        return int(self.buf.size)

    def read(self, address: int, size: int) -> Expected[bytes]:
        if address + size > self.buf.size:
            return Expected.unexpected(FsError.Disk_OutOfBounds)
        return Expected(self.buf[address:address + size].tobytes())

    def write(self, address: int, data) -> Expected[int]:
        d = np.frombuffer(bytes(data), dtype=np.uint8)
        if address + d.size > self.buf.size:
            return Expected.unexpected(FsError.Disk_OutOfBounds)
        self.buf[address:address + d.size] = d
        return Expected(int(d.size))


class StackDisk(HeapDisk):
    """StackDisk<power> (default 2^22 bytes, zero-initialised)."""

    def __init__(self, power: int = 22):
        super().__init__(1 << power)


# ------------------------------------------------------------------------------------
# Logger (lib/data_collection): only ErrorCorrectionEvent is emitted by block devices
# ------------------------------------------------------------------------------------
class Logger:
    def __init__(self):
        self.corrections: List[Tuple[str, int]] = []

    def logEvent(self, kind: str, block_index: int) -> None:
        self.corrections.append((kind, int(block_index)))


# ------------------------------------------------------------------------------------
# CrcPolynomial (lib/ecc_helpers/src/crc_polynomial.cpp)
# ------------------------------------------------------------------------------------
class CrcPolynomial:
    def __init__(self, explicit_poly: int):
        self._p = int(explicit_poly)
        self._n = self._p.bit_length() - 1  # _findDegree :7-17

    @staticmethod
    def MsgExplicit(p: int) -> "CrcPolynomial":  # :27-39
        return CrcPolynomial(p)

    @staticmethod
    def MsgImplicit(p: int) -> "CrcPolynomial":  # :41-54
        return CrcPolynomial(((int(p) << 1) + 1) & 0xFFFFFFFFFFFFFFFF)

    def getDegree(self) -> int:
        return self._n

    def getExplicitPolynomial(self) -> int:
        return self._p

    def getCoefficients(self) -> List[bool]:  # MSB first, with the explicit +1
        return [bool((self._p >> (self._n - j)) & 1) for j in range(self._n + 1)]


# ------------------------------------------------------------------------------------
# Block devices
# ------------------------------------------------------------------------------------
class IBlockDevice:
    _engine: Optional[EccEngine] = None

    def rawBlockSize(self) -> int:
        raise NotImplementedError

    def dataSize(self) -> int:
        raise NotImplementedError

    def numOfBlocks(self) -> int:
        return self._disk.size() // self.rawBlockSize()

    # batch API: whole blocks [first, first+count); the per-block loop (codecs override it with
    # one engine call per range)
    def readBlocks(self, first: int, count: int) -> Tuple[np.ndarray, np.ndarray]:
        """Decode `count` whole blocks; returns (payloads [count, dataSize], FsError-or-0 per block)."""
        out = np.zeros((count, self.dataSize()), dtype=np.uint8)
        err = np.zeros(count, dtype=np.uint8)
        for i in range(count):
            r = self.readBlock(DataLocation(first + i, 0), self.dataSize())
            if r:
                out[i] = np.frombuffer(r.value(), dtype=np.uint8)
            else:
                err[i] = int(r.error())
        return out, err

    def scrub(self, first: int = 0, count: Optional[int] = None) -> Tuple[Tuple[int, int, int], np.ndarray]:
        """Whole-image scrub: the disk and log effect of readBlock(DataLocation(i, 0),
        dataSize()) for i in [first, first+count), in order, without the payloads.
        Returns ((ok, corrected, failed) block counts, FsError-or-0 per block)."""
        count = self.numOfBlocks() - first if count is None else count
        _, err = self.readBlocks(first, count)
        failed = int(np.count_nonzero(err))
        return (count - failed, 0, failed), err

    def writeBlocks(self, first: int, payloads: np.ndarray) -> np.ndarray:
        err = np.zeros(len(payloads), dtype=np.uint8)
        for i, p in enumerate(payloads):
            r = self.writeBlock(bytes(p), DataLocation(first + i, 0))
            if not r:
                err[i] = int(r.error())
        return err


class RawBlockDevice(IBlockDevice):  # raw_block_device.cpp
    def __init__(self, block_size: int, disk: IDisk):
        self._bs, self._disk = int(block_size), disk

    def rawBlockSize(self) -> int:
        return self._bs

    def dataSize(self) -> int:
        return self._bs

    def formatBlock(self, block_index: int) -> Expected[None]:
        return Expected(None)

    def writeBlock(self, data, loc: DataLocation) -> Expected[int]:
        data = bytes(data)
        to_write = min(len(data), self._bs - loc.offset)
        r = self._disk.write(loc.block_index * self._bs + loc.offset, data[:to_write])
        return Expected(to_write) if r else Expected.unexpected(r.error())

    def readBlock(self, loc: DataLocation, bytes_to_read: int, capacity: Optional[int] = None) -> Expected[bytes]:
        to_read = min(bytes_to_read, self._bs - loc.offset)
        addr = loc.block_index * self._bs + loc.offset
        if addr + to_read > self._disk.size():
            return Expected.unexpected(FsError.Disk_OutOfBounds)
        if capacity is not None and capacity < to_read:
            return Expected.unexpected(FsError.Disk_InvalidRequest)
        return self._disk.read(addr, to_read)


class _EngineDevice(IBlockDevice):
    """Shared read-modify-write plumbing for the ECC codecs."""

    _log_name = ""

    def __init__(self, engine: EccEngine, disk: IDisk, logger: Optional[Logger]):
        self._engine, self._disk, self._logger = engine, disk, logger
        self._raw, self._ds = engine.raw_block_size, engine.data_size

    def rawBlockSize(self) -> int:
        return self._raw

    def dataSize(self) -> int:
        return self._ds

    def _read_raw(self, block_index: int) -> Expected[np.ndarray]:
        r = self._disk.read(block_index * self._raw, self._raw)
        if not r:
            return Expected.unexpected(r.error())
        return Expected(np.frombuffer(r.value(), dtype=np.uint8).copy())

    def _log(self, block_index: int) -> None:
        if self._logger is not None and self._log_name:
            self._logger.logEvent(self._log_name, block_index)

    # decode one old block on the GPU; apply the reference's write-back; returns payload
    def _check_fix(self, block_index: int, raw: np.ndarray) -> Expected[np.ndarray]:
        raise NotImplementedError

    def formatBlock(self, block_index: int) -> Expected[None]:
        r = self._disk.write(block_index * self._raw, bytes(self._raw))
        return Expected(None) if r else Expected.unexpected(r.error())

    # ---- batched whole-block I/O: one engine call per contiguous range ----
    def _has_spill(self) -> bool:
        return self._engine.ecc_type == ECC_REED_SOLOMON and self._raw < 255

    def _write_back(self, block_index: int, old: np.ndarray, fixed: np.ndarray, spill) -> Optional[FsError]:
        raise NotImplementedError

    def readBlocks(self, first: int, count: int) -> Tuple[np.ndarray, np.ndarray]:
        """== readBlock(DataLocation(i, 0), dataSize()) for i in [first, first+count), in order:
        same payloads, per-block errors, disk contents and correction log."""
        out = np.zeros((count, self._ds), dtype=np.uint8)
        err = np.zeros(count, dtype=np.uint8)
        e = self._engine
        wb = e.ecc_type in (ECC_REED_SOLOMON, ECC_HAMMING)
        done = 0
        while done < count:
            nb = count - done
            r = self._disk.read((first + done) * self._raw, nb * self._raw)
            if not r:
                # range not on the disk: per-block calls report it block by block
                for i in range(done, count):
                    rr = self.readBlock(DataLocation(first + i, 0), self._ds)
                    if rr:
                        out[i] = np.frombuffer(rr.value(), dtype=np.uint8)
                    else:
                        err[i] = int(rr.error())
                break
            raw = np.frombuffer(r.value(), dtype=np.uint8).copy()
            fixed = raw.copy()
            status = np.zeros(nb, dtype=np.uint8)
            spill = np.zeros(nb * e.spill_bytes_per_block(), dtype=np.uint8) if self._has_spill() else None
            e.decode_host(fixed, out[done:].reshape(-1), status, write_back=wb, spill=spill)
            if spill is None:
                # no write-back leaves its block: the per-block write-backs together are the
                # changed bytes of the range, written once; the log keeps block order
                bad = np.nonzero(status == STATUS_CORRECTION_ERROR)[0]
                err[done + bad] = int(FsError.BlockDevice_CorrectionError)
                out[done + bad] = 0
                if wb:
                    for i in np.nonzero(status == STATUS_CORRECTED)[0]:
                        self._log(first + done + int(i))
                    changed = np.nonzero(fixed != raw)[0]
                    if changed.size:
                        lo, hi = int(changed[0]), int(changed[-1]) + 1
                        self._disk.write((first + done) * self._raw + lo, fixed[lo:hi].tobytes())
                done += nb
                continue
            i = 0
            while i < nb:
                st = int(status[i])
                if st == STATUS_CORRECTION_ERROR:
                    err[done + i] = int(FsError.BlockDevice_CorrectionError)
                    out[done + i] = 0
                elif st == STATUS_CORRECTED and wb:
                    sp = spill[i * e.spill_bytes_per_block():(i + 1) * e.spill_bytes_per_block()] \
                        if spill is not None else None
                    fe = self._write_back(first + done + i, raw[i * self._raw:(i + 1) * self._raw],
                                          fixed[i * self._raw:(i + 1) * self._raw], sp)
                    if fe is not None:
                        err[done + i] = int(fe)
                    if sp is not None and int(sp[0]) and i + 1 < nb:
                        i += 1  # the write-back ran into the next block: re-read from there
                        break
                i += 1
            done += i
        return out, err

    def scrub(self, first: int = 0, count: Optional[int] = None) -> Tuple[Tuple[int, int, int], np.ndarray]:
        """Whole-image scrub in one engine call (EccEngine.scrub_host): the disk
        image from block `first` to the disk end goes through ppfs_ecc_scrub_host, which applies
        the reference's read-path write-back block by block in index order (RS codeword incl.
        bytes past a shortened block, Hamming flipped byte); corrected blocks are logged in order.
        Returns ((ok, corrected, failed) block counts, FsError-or-0 per block)."""
        n_all = self.numOfBlocks()
        count = n_all - first if count is None else count
        base = first * self._raw
        r = self._disk.read(base, self._disk.size() - base) if 0 <= first and first + count <= n_all else None
        if not r:
            log0 = self._log_count()
            _, err = self.readBlocks(first, count)  # blocks off the disk: per-block semantics
            failed = int(np.count_nonzero(err))
            corrected = self._log_count() - log0
            return (count - failed - corrected, corrected, failed), err
        image = np.frombuffer(r.value(), dtype=np.uint8).copy()
        before = image.copy()
        status = np.zeros(count, dtype=np.uint8)
        counts = self._engine.scrub_host(image, nblocks=count, status=status)
        err = np.where(status == STATUS_CORRECTION_ERROR, int(FsError.BlockDevice_CorrectionError), 0).astype(np.uint8)
        for i in np.nonzero(status == STATUS_CORRECTED)[0]:
            self._log(first + int(i))
        changed = np.nonzero(image != before)[0]
        if changed.size:
            lo, hi = int(changed[0]), int(changed[-1]) + 1
            w = self._disk.write(base + lo, image[lo:hi].tobytes())
            if not w:
                err[:] = int(w.error())
        return counts, err

    def _log_count(self) -> int:
        return len(self._logger.corrections) if self._logger is not None else 0

    def writeBlocks(self, first: int, payloads: np.ndarray) -> np.ndarray:
        """== writeBlock(payload_i, DataLocation(first+i, 0)) in order (full-block writes)."""
        payloads = np.ascontiguousarray(payloads, dtype=np.uint8).reshape(-1, self._ds)
        count = payloads.shape[0]
        err = np.zeros(count, dtype=np.uint8)
        r = self._disk.read(first * self._raw, count * self._raw)
        if self._has_spill() or not r:
            return super().writeBlocks(first, payloads)  # per-block order (spill / out of range)
        raw = np.frombuffer(r.value(), dtype=np.uint8).copy()
        status = np.zeros(count, dtype=np.uint8)
        self._engine.write_host(payloads.reshape(-1), raw, status)
        for i in range(count):
            if status[i] == STATUS_CORRECTION_ERROR:
                err[i] = int(FsError.BlockDevice_CorrectionError)  # block left untouched
            elif status[i] == STATUS_CORRECTED:
                self._log(first + i)  # the old block's write-back is overwritten below
        w = self._disk.write(first * self._raw, raw.tobytes())
        if not w:
            err[:] = int(w.error())
        return err

    def readBlock(self, loc: DataLocation, bytes_to_read: int, capacity: Optional[int] = None) -> Expected[bytes]:
        if capacity is not None and capacity < bytes_to_read:
            return Expected.unexpected(FsError.Disk_InvalidRequest)
        to_read = min(self._ds - loc.offset, bytes_to_read)
        raw = self._read_raw(loc.block_index)
        if not raw:
            return Expected.unexpected(raw.error())
        dec = self._check_fix(loc.block_index, raw.value())
        if not dec:
            return Expected.unexpected(dec.error())
        return Expected(dec.value()[loc.offset:loc.offset + to_read].tobytes())

    def writeBlock(self, data, loc: DataLocation) -> Expected[int]:
        data = np.frombuffer(bytes(data), dtype=np.uint8)
        to_write = min(data.size, self._ds - loc.offset)
        raw = self._read_raw(loc.block_index)
        if not raw:
            return Expected.unexpected(raw.error())
        raw = raw.value()
        dec = self._check_fix(loc.block_index, raw)
        if not dec:
            return Expected.unexpected(dec.error())
        payload = dec.value().copy()
        payload[loc.offset:loc.offset + to_write] = data[:to_write]
        self._engine.encode_host(payload, raw)  # raw: fixed old block (tail bits / parity byte base)
        w = self._disk.write(loc.block_index * self._raw, raw.tobytes())
        if not w:
            return Expected.unexpected(w.error())
        return Expected(int(to_write))


class ReedSolomonBlockDevice(_EngineDevice):  # rs_block_device.cpp
    _log_name = "ReedSolomon"

    def __init__(self, disk: IDisk, raw_block_size: int, correctable_bytes: int, logger: Optional[Logger] = None,
                 device: int = 0):
        super().__init__(EccEngine(ECC_REED_SOLOMON, raw_block_size, correctable_bytes, device=device), disk, logger)

    def _check_fix(self, block_index: int, raw: np.ndarray) -> Expected[np.ndarray]:
        e = self._engine
        data = np.zeros(self._ds, dtype=np.uint8)
        status = np.zeros(1, dtype=np.uint8)
        spill = np.zeros(e.spill_bytes_per_block(), dtype=np.uint8)
        fixed = raw.copy()
        e.decode_host(fixed, data, status, write_back=True, spill=spill)
        if status[0] == STATUS_CORRECTED:
            self._write_back(block_index, raw, fixed, spill)
        return Expected(data)

    def _write_back(self, block_index, old, fixed, spill) -> Optional[FsError]:
        self._log(block_index)  # :171-173
        extra = int(spill[0]) if (spill is not None and self._raw < 255) else 0
        wb = fixed.tobytes() + (spill[1:1 + extra].tobytes() if extra else b"")
        self._disk.write(block_index * self._raw, wb)  # result ignored (:180)
        return None

    def writeBlock(self, data, loc: DataLocation) -> Expected[int]:
        # the new codeword depends only on the patched payload (:61-93)
        return super().writeBlock(data, loc)


class CrcBlockDevice(_EngineDevice):  # crc_block_device.cpp
    def __init__(self, polynomial: CrcPolynomial, disk: IDisk, block_size: int, logger: Optional[Logger] = None,
                 device: int = 0):
        self.polynomial = polynomial
        super().__init__(EccEngine(ECC_CRC, block_size, crc_polynomial_explicit=polynomial.getExplicitPolynomial(),
                                   device=device), disk, logger)

    def _check_fix(self, block_index: int, raw: np.ndarray) -> Expected[np.ndarray]:
        data = np.zeros(self._ds, dtype=np.uint8)
        status = np.zeros(1, dtype=np.uint8)
        self._engine.decode_host(raw.copy(), data, status, write_back=False)
        if status[0] == STATUS_CORRECTION_ERROR:
            return Expected.unexpected(FsError.BlockDevice_CorrectionError)
        return Expected(data)

    def formatBlock(self, block_index: int) -> Expected[None]:
        # _calculateAndWrite on an all-zero block (:124-134)
        raw = np.zeros(self._raw, dtype=np.uint8)
        self._engine.encode_host(np.zeros(self._ds, dtype=np.uint8), raw)
        r = self._disk.write(block_index * self._raw, raw.tobytes())
        return Expected(None) if r else Expected.unexpected(r.error())


class HammingBlockDevice(_EngineDevice):  # hamming_block_device.cpp
    _log_name = "Hamming"

    def __init__(self, block_size_power: int, disk: IDisk, logger: Optional[Logger] = None, device: int = 0):
        super().__init__(EccEngine(ECC_HAMMING, 1 << int(block_size_power), device=device), disk, logger)

    def _check_fix(self, block_index: int, raw: np.ndarray) -> Expected[np.ndarray]:
        data = np.zeros(self._ds, dtype=np.uint8)
        status = np.zeros(1, dtype=np.uint8)
        fixed = raw.copy()
        self._engine.decode_host(fixed, data, status, write_back=True)
        if status[0] == STATUS_CORRECTION_ERROR:
            return Expected.unexpected(FsError.BlockDevice_CorrectionError)
        if status[0] == STATUS_CORRECTED:
            fe = self._write_back(block_index, raw, fixed, None)
            if fe is not None:
                return Expected.unexpected(fe)
            raw[:] = fixed
        return Expected(data)

    def _write_back(self, block_index, old, fixed, spill) -> Optional[FsError]:
        diff = np.nonzero(fixed != old)[0]
        byte = int(diff[0]) if diff.size else 0
        w = self._disk.write(block_index * self._raw + byte, fixed[byte:byte + 1].tobytes())  # :41-51
        if not w:
            return w.error()
        self._log(block_index)  # :53-57
        return None


class ParityBlockDevice(_EngineDevice):  # parity_block_device.cpp
    def __init__(self, block_size: int, disk: IDisk, logger: Optional[Logger] = None, device: int = 0):
        super().__init__(EccEngine(ECC_PARITY, block_size, device=device), disk, logger)

    def _check_fix(self, block_index: int, raw: np.ndarray) -> Expected[np.ndarray]:
        data = np.zeros(self._ds, dtype=np.uint8)
        status = np.zeros(1, dtype=np.uint8)
        self._engine.decode_host(raw.copy(), data, status, write_back=False)
        if status[0] == STATUS_CORRECTION_ERROR:
            return Expected.unexpected(FsError.BlockDevice_CorrectionError)
        return Expected(data)


def create_block_device(disk: IDisk, block_size: int, ecc_type: ECCType, crc_polynomial_explicit: int = 0,
                        rs_correctable_bytes: int = 3, logger: Optional[Logger] = None,
                        device: int = 0) -> IBlockDevice:
    """PpFS::_createAppropriateBlockDevice (lib/filesystem/src/ppfs.cpp:35-70)."""
    t = ECCType(ecc_type)
    if t == ECCType.None_:
        return RawBlockDevice(block_size, disk)
    if t == ECCType.Parity:
        return ParityBlockDevice(block_size, disk, logger, device)
    if t == ECCType.Crc:
        return CrcBlockDevice(CrcPolynomial.MsgExplicit(crc_polynomial_explicit), disk, block_size, logger, device)
    if t == ECCType.Hamming:
        return HammingBlockDevice(int(math.log2(block_size)), disk, logger, device)
    return ReedSolomonBlockDevice(disk, block_size, rs_correctable_bytes, logger, device)
