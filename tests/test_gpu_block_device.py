"""Python block-device mirror (paritypartyfs_amd.block_device) on the GPU.

1. The reference's block-device unit tests restated (unit_tests/test_rs_block_device.cpp,
   test_crc_block_device.cpp:73-200, test_hamming_block_device.cpp, test_parity_block_device.cpp).
2. Differential sequences vs the oracle's device model (tests/oracle_lib.OracleDevice): random
   formatBlock / writeBlock (any offset, length) / readBlock (any capacity) / readBlocks /
   writeBlocks / scrub / raw corruption; every return value, payload, the log and the disk image
   must match.
"""
import zlib

import numpy as np
import pytest

from tests.oracle_lib import OracleDevice

pytestmark = pytest.mark.gpu

bd = pytest.importorskip("paritypartyfs_amd.block_device")
DL = bd.DataLocation


# ----------------------------------------------------------------- reference unit tests
@pytest.mark.parametrize("t,bad", [(2, []), (1, [(120, 0x00)]), (2, [(10, 0xEE), (200, 0x44)]),
                                   (3, [(10, 0xEE), (100, 0x61), (200, 0x44)])])
def test_rs_reference_unit_tests(t, bad):
    disk = bd.StackDisk()
    rs = bd.ReedSolomonBlockDevice(disk, 255, t)
    data = bytes([0xAB]) * rs.dataSize()
    assert rs.formatBlock(0).has_value()
    assert rs.writeBlock(data, DL(0, 0)).has_value()
    raw = bytearray(disk.read(0, rs.rawBlockSize()).value())
    for pos, v in bad:
        raw[pos] = v
    assert disk.write(0, bytes(raw)).has_value()
    r = rs.readBlock(DL(0, 0), rs.dataSize(), capacity=512)
    assert r.has_value() and r.value() == data


@pytest.mark.parametrize("imp,bs,flips", [(0xEA, 256, [(1, 0x01)]),
                                          (0xC1ACF, 512, [(1, 0x01), (111, 0x08), (200, 0x02)]),
                                          (0x9960034C, 512, [(1, 0x01), (111, 0x08), (200, 0x02), (11, 0x08),
                                                             (20, 0x02)])])
def test_crc_reference_unit_tests(imp, bs, flips):
    disk = bd.StackDisk()
    crc = bd.CrcBlockDevice(bd.CrcPolynomial.MsgImplicit(imp), disk, bs)
    assert crc.formatBlock(0).has_value()
    data = bytes(crc.dataSize())
    assert crc.writeBlock(data, DL(0, 0)).has_value()
    assert crc.readBlock(DL(0, 0), crc.dataSize()).value() == data
    for a, v in flips:
        assert disk.write(a, bytes([v])).has_value()
    r = crc.readBlock(DL(0, 0), crc.dataSize())
    assert not r.has_value() and r.error() == bd.FsError.BlockDevice_CorrectionError


def test_hamming_reference_unit_tests():
    rng = np.random.default_rng(5)
    for i in range(10):
        disk = bd.StackDisk()
        h = bd.HammingBlockDevice(4, disk)
        msg = f"Round{i}".encode()
        assert h.writeBlock(msg, DL(0, 0)).has_value()
        bit = int(rng.integers(0, h.dataSize() * 8))
        b = disk.read(bit // 8, 1).value()[0] ^ (1 << (bit % 8))
        disk.write(bit // 8, bytes([b]))
        assert h.readBlock(DL(0, 0), len(msg)).value() == msg
    disk = bd.StackDisk()
    h = bd.HammingBlockDevice(4, disk)
    assert h.writeBlock(b"slay", DL(0, 0)).has_value()
    for bit in (3, 17):
        b = disk.read(bit // 8, 1).value()[0] ^ (1 << (bit % 8))
        disk.write(bit // 8, bytes([b]))
    r = h.readBlock(DL(0, 0), 4)
    assert not r.has_value() and r.error() == bd.FsError.BlockDevice_CorrectionError


def test_parity_reference_unit_tests():
    disk = bd.StackDisk()
    p = bd.ParityBlockDevice(256, disk)
    data = bytes([0x55]) * p.dataSize()
    assert p.formatBlock(0).has_value() and p.writeBlock(data, DL(0, 0)).has_value()
    assert p.readBlock(DL(0, 0), p.dataSize()).value() == data
    raw = bytearray(disk.read(0, 256).value())
    raw[10] ^= 4
    disk.write(0, bytes(raw))
    assert not p.readBlock(DL(0, 0), p.dataSize()).has_value()


# ----------------------------------------------------------------- differential sequences
CFGS = [
    ("rs512_t3", bd.ECCType.ReedSolomon, 512, 3, 0),
    ("rs4096_t16", bd.ECCType.ReedSolomon, 4096, 16, 0),
    ("rs64_t3", bd.ECCType.ReedSolomon, 64, 3, 0),
    ("crc512", bd.ECCType.Crc, 512, 0, (0x9960034C << 1) + 1),
    ("crc100_deg3", bd.ECCType.Crc, 100, 0, 0xB),
    ("hamming512", bd.ECCType.Hamming, 512, 0, 0),
    ("hamming16", bd.ECCType.Hamming, 16, 0, 0),
    ("parity256", bd.ECCType.Parity, 256, 0, 0),
    ("raw512", bd.ECCType.None_, 512, 0, 0),
]


@pytest.mark.parametrize("name,typ,bs,t,poly", CFGS, ids=[c[0] for c in CFGS])
def test_block_device_differential(oracle, name, typ, bs, t, poly):
    NB, disk_size = 32, 1 << 20
    disk = bd.HeapDisk(disk_size)
    log = bd.Logger()
    dev = bd.create_block_device(disk, bs, typ, crc_polynomial_explicit=poly, rs_correctable_bytes=t, logger=log)
    od = OracleDevice(oracle, int(typ), bs, t, poly, disk_size)
    raw, ds = dev.rawBlockSize(), dev.dataSize()
    assert (raw, ds) == (od.raw_block_size(), od.data_size())
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    for b in range(NB):
        assert bool(dev.formatBlock(b)) == (od.format(b) == 0)

    def same():
        return np.array_equal(disk.buf, od.disk) and [x[1] for x in log.corrections] == od.log_entries()

    for op in range(70):
        kind = int(rng.integers(0, 9))
        b = int(rng.integers(0, NB + 1))
        if kind == 0:
            assert bool(dev.formatBlock(b)) == (od.format(b) == 0)
        elif kind <= 2:
            off = int(rng.integers(0, ds)) if rng.integers(0, 4) == 0 else 0
            ln = int(rng.integers(0, ds + 8)) if rng.integers(0, 3) == 0 else ds
            data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            r = dev.writeBlock(data, DL(b, off))
            rc, wr = od.write(b, off, data)
            assert bool(r) == (rc == 0)
            if r:
                assert r.value() == wr
            else:
                assert int(r.error()) == rc
        elif kind <= 4:
            off = int(rng.integers(0, ds)) if rng.integers(0, 4) == 0 else 0
            n = int(rng.integers(0, ds + 8)) if rng.integers(0, 3) == 0 else ds
            cap = max(n - 1, 0) if rng.integers(0, 8) == 0 else 4096
            r = dev.readBlock(DL(b, off), n, capacity=cap)
            rc, out = od.read(b, off, n, cap)
            assert bool(r) == (rc == 0)
            if r:
                assert r.value() == out
            else:
                assert int(r.error()) == rc
        elif kind == 5:
            for _ in range(int(rng.integers(1, 5))):
                blk = int(rng.integers(0, NB))
                for _ in range(int(rng.integers(0, (t + 3) if typ == bd.ECCType.ReedSolomon else 3))):
                    pos = blk * raw + int(rng.integers(0, raw))
                    m = int(rng.integers(1, 256)) if typ == bd.ECCType.ReedSolomon else 1 << int(rng.integers(0, 8))
                    disk.buf[pos] ^= m
                    od.disk[pos] ^= m
        elif kind == 6:
            first = int(rng.integers(0, NB))
            cnt = int(rng.integers(1, NB - first + 1))
            out, err = dev.readBlocks(first, cnt)
            for i in range(cnt):
                rc, o = od.read(first + i, 0, ds, 4096)
                assert int(err[i]) == rc
                if rc == 0:
                    assert out[i].tobytes() == o
        elif kind == 8:
            first = int(rng.integers(0, NB))
            cnt = int(rng.integers(1, NB - first + 1))
            _, err = dev.scrub(first, cnt)
            for i in range(cnt):
                rc, _ = od.read(first + i, 0, ds, 4096)
                assert int(err[i]) == rc
        else:
            first = int(rng.integers(0, NB))
            cnt = int(rng.integers(1, NB - first + 1))
            pl = rng.integers(0, 256, (cnt, ds), dtype=np.uint8)
            err = dev.writeBlocks(first, pl)
            for i in range(cnt):
                rc, _ = od.write(first + i, 0, pl[i].tobytes())
                assert int(err[i]) == rc
        assert same(), f"{name}: state diverged after op {op} (kind {kind}, block {b})"
