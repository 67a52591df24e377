"""SURVEY 8f-3 whole-image scrub and 8f-4 superblock 2-of-3 bit voting.

CPU: the oracle's bit-by-bit restatement of SuperBlockManager::_performBitVoting
(super_block_manager.cpp:133-165) against plain bitwise majority.
GPU: ppfs_vote3_{host,device} vs the oracle; ppfs_ecc_scrub_{host,device} vs the oracle's
sequential readBlock over the same disk image (every block in index order: statuses, disk bytes
and correction log), including shortened RS codes whose write-back runs past the block end.
"""
import zlib

import numpy as np
import pytest

from tests.oracle_lib import OracleDevice


def _flip_bits(rng, x, nflips):
    x = x.copy()
    for _ in range(nflips):
        i = int(rng.integers(0, x.size))
        x[i] ^= np.uint8(1 << int(rng.integers(0, 8)))
    return x


def _majority(a, b, c):
    return (a & b) | (a & c) | (b & c)


def test_oracle_vote3_is_bitwise_majority(oracle):
    rng = np.random.default_rng(11)
    rec = 49  # sizeof(SuperBlock) (super_block.hpp)
    a = rng.integers(0, 256, rec * 40, dtype=np.uint8)
    b = _flip_bits(rng, a, 30)
    c = _flip_bits(rng, a, 30)
    out, dmg = oracle.vote3(a, b, c, rec)
    assert np.array_equal(out, _majority(a, b, c))
    m = out.reshape(-1, rec)
    for k, x in enumerate((a, b, c)):
        want = (x.reshape(-1, rec) != m).any(axis=1)
        assert np.array_equal((dmg >> k) & 1, want.astype(np.uint32))


def test_oracle_vote3_signature_recovery(oracle):
    sb = np.frombuffer(b"PPFS" + bytes(range(45)), dtype=np.uint8).copy()
    bad = sb.copy()
    bad[0] ^= 0xFF  # one copy's signature destroyed
    out, dmg = oracle.vote3(sb, bad, sb, 49)
    assert out[:4].tobytes() == b"PPFS" and np.array_equal(out, sb)
    assert int(dmg[0]) == 0b010


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("rec,nrec", [(49, 1), (49, 1000), (1, 4096), (4096, 64), (7, 0)])
def test_vote3_host_matches_oracle(oracle, rec, nrec):
    from paritypartyfs_amd import vote3_host

    rng = np.random.default_rng(rec * 1000 + nrec)
    a = rng.integers(0, 256, rec * nrec, dtype=np.uint8)
    b = _flip_bits(rng, a, max(1, nrec // 2)) if nrec else a.copy()
    c = _flip_bits(rng, a, max(1, nrec // 2)) if nrec else a.copy()
    out, dmg = vote3_host(a, b, c, rec)
    o_out, o_dmg = oracle.vote3(a, b, c, rec)
    assert np.array_equal(out, o_out)
    assert np.array_equal(dmg, o_dmg)


@pytest.mark.gpu
def test_vote3_device_matches_oracle(oracle):
    import torch

    from paritypartyfs_amd import vote3

    rng = np.random.default_rng(3)
    rec, nrec = 49, 1 << 15
    a = rng.integers(0, 256, rec * nrec, dtype=np.uint8)
    b, c = _flip_bits(rng, a, 5000), _flip_bits(rng, a, 5000)
    ta, tb, tc = (torch.from_numpy(x).cuda() for x in (a, b, c))
    out = torch.empty_like(ta)
    dmg = torch.full((nrec,), 99, dtype=torch.int32, device="cuda")
    vote3(ta, tb, tc, out, rec, dmg)
    torch.cuda.synchronize()
    o_out, o_dmg = oracle.vote3(a, b, c, rec)
    assert np.array_equal(out.cpu().numpy(), o_out)
    assert np.array_equal(dmg.cpu().numpy().astype(np.uint32), o_dmg)


SCRUB_CFGS = [
    ("rs512_t3", 4, 512, 3, 0, 300),
    ("rs4096_t16", 4, 4096, 16, 0, 300),
    ("rs64_t3", 4, 64, 3, 0, 400),       # shortened: write-back may run into the next blocks
    ("rs32_t5", 4, 32, 5, 0, 400),       # spill longer than a block
    ("hamming512", 2, 512, 0, 0, 200),
    ("hamming4096", 2, 4096, 0, 0, 64),
    ("crc4096", 1, 4096, 0, (0x9960034C << 1) + 1, 64),
    ("crc100_deg3", 1, 100, 0, 0xB, 200),
    ("parity256", 3, 256, 0, 0, 200),
]


def _scrub_case(oracle, typ, bs, t, poly, nb, seed, tail):
    """An encoded image with errors, plus `tail` bytes after the last block (part of the disk)."""
    from paritypartyfs_amd import EccEngine

    eng = EccEngine(typ, bs, t, crc_polynomial_explicit=poly)
    raw, ds = eng.raw_block_size, eng.data_size
    rng = np.random.default_rng(seed)
    image = np.zeros(nb * raw + tail, np.uint8)
    eng.encode_host(rng.integers(0, 256, nb * ds, dtype=np.uint8), image[:nb * raw])
    image[nb * raw:] = rng.integers(0, 256, tail, dtype=np.uint8)
    for blk in range(nb):
        k = blk % ((t + 5) if typ == 4 else 4)  # 0 .. t+4 byte errors (RS), 0..3 bit flips
        for _ in range(k):
            pos = blk * raw + int(rng.integers(0, raw))
            image[pos] ^= np.uint8(int(rng.integers(1, 256)) if typ == 4 else 1 << int(rng.integers(0, 8)))
    od = OracleDevice(oracle, typ, bs, t, poly, image.size)
    od.disk[:] = image
    o_err = np.array([od.read(i, 0, ds, 4096)[0] for i in range(nb)], dtype=np.int64)
    return eng, image, od, o_err


@pytest.mark.gpu
@pytest.mark.parametrize("name,typ,bs,t,poly,nb", SCRUB_CFGS, ids=[c[0] for c in SCRUB_CFGS])
@pytest.mark.parametrize("tail", [0, 37])
def test_scrub_host_matches_sequential_reference(oracle, name, typ, bs, t, poly, nb, tail):
    eng, image, od, o_err = _scrub_case(oracle, typ, bs, t, poly, nb, zlib.crc32(name.encode()), tail)
    st = np.full(nb, 77, np.uint8)
    ok, corrected, failed = eng.scrub_host(image, nblocks=nb, status=st)
    assert np.array_equal(image, od.disk), f"{name}: scrubbed image differs from the sequential reference"
    assert np.array_equal(np.where(st == 5, 5, 0), o_err)
    assert sorted(np.nonzero(st == 1)[0].tolist()) == od.log_entries()
    assert (ok, corrected, failed) == (int((st == 0).sum()), int((st == 1).sum()), int((st == 5).sum()))
    if typ == 4 and bs < 255:
        assert corrected > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name,typ,bs,t,poly,nb", [c for c in SCRUB_CFGS if c[1] in (2, 4)],
                         ids=[c[0] for c in SCRUB_CFGS if c[1] in (2, 4)])
def test_scrub_device_matches_host(oracle, name, typ, bs, t, poly, nb):
    import torch

    eng, image, od, _ = _scrub_case(oracle, typ, bs, t, poly, nb, 99, 11)
    d_img = torch.from_numpy(image.copy()).cuda()
    d_st = torch.full((max(nb, 16),), 77, dtype=torch.uint8, device="cuda")
    eng.scrub(d_img, d_st, nblocks=nb)
    torch.cuda.synchronize()
    h_img = image.copy()
    h_st = np.zeros(nb, np.uint8)
    eng.scrub_host(h_img, nblocks=nb, status=h_st)
    assert np.array_equal(d_img.cpu().numpy(), h_img)
    assert np.array_equal(d_st.cpu().numpy()[:nb], h_st)
    assert np.array_equal(h_img, od.disk)


@pytest.mark.gpu
def test_block_device_scrub_matches_reads(oracle):
    """IBlockDevice.scrub() on the Python adapter == readBlock of every block in order."""
    bd = pytest.importorskip("paritypartyfs_amd.block_device")
    for typ, bs, t in ((bd.ECCType.ReedSolomon, 64, 3), (bd.ECCType.Hamming, 512, 0)):
        disk_size = 1 << 16
        disk = bd.HeapDisk(disk_size)
        log = bd.Logger()
        dev = bd.create_block_device(disk, bs, typ, rs_correctable_bytes=t, logger=log)
        od = OracleDevice(oracle, int(typ), bs, t, 0, disk_size)
        rng = np.random.default_rng(int(typ))
        nb = dev.numOfBlocks()
        pl = rng.integers(0, 256, (nb, dev.dataSize()), dtype=np.uint8)
        assert not dev.writeBlocks(0, pl).any()
        for i in range(nb):
            assert od.write(i, 0, pl[i].tobytes())[0] == 0
        for _ in range(nb * 2):
            pos = int(rng.integers(0, nb * dev.rawBlockSize()))
            m = int(rng.integers(1, 256)) if typ == bd.ECCType.ReedSolomon else 1 << int(rng.integers(0, 8))
            disk.buf[pos] ^= m
            od.disk[pos] ^= m
        (ok, corrected, failed), err = dev.scrub()
        o_err = [od.read(i, 0, dev.dataSize(), 4096)[0] for i in range(nb)]
        assert err.tolist() == o_err
        assert np.array_equal(disk.buf, od.disk)
        assert [x[1] for x in log.corrections] == od.log_entries()
        assert ok + corrected + failed == nb and corrected == len(log.corrections)


@pytest.mark.gpu
def test_device_copy_ragged():
    """ppfs_copy_device (bench.py's HBM-ceiling reference): every alignment of source and
    destination, sizes around the 16-byte body, bytes outside the range untouched."""
    import torch

    from paritypartyfs_amd import device_copy

    rng = np.random.default_rng(11)
    src = torch.from_numpy(rng.integers(0, 256, 1 << 16, dtype=np.uint8)).cuda()
    for so, do, n in [(0, 0, 0), (0, 0, 1), (0, 0, 16), (0, 0, 65536 - 64), (3, 3, 1000), (5, 1, 4099),
                      (15, 15, 17), (1, 0, 31), (7, 9, 60000), (0, 8, 48)]:
        dst = torch.full((1 << 16,), 0xA5, dtype=torch.uint8, device="cuda")
        device_copy(dst[do:], src[so:], n)
        torch.cuda.synchronize()
        d = dst.cpu().numpy()
        s = src.cpu().numpy()
        assert np.array_equal(d[do:do + n], s[so:so + n]), (so, do, n)
        assert (d[:do] == 0xA5).all() and (d[do + n:] == 0xA5).all(), (so, do, n)
