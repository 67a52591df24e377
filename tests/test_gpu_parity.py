"""GPU parity tests: HIP kernels (through the C ABI) vs the CPU oracle, bit-exact.

Every case compares the device results with oracle/ppfs_oracle.c on the same seeded inputs:
codewords / raw blocks, payloads, per-block status, write-back bytes (and RS spill for
shortened codes).  Edge cases follow the reference tests: 0..t+3 byte errors for RS
(miscorrection included), 0..3 bit flips for Hamming (parity, data and unused tail bits),
CRC flips including the undetected last payload bit, ragged batch sizes.
"""
import zlib

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

if gpu_available():
    import torch

from paritypartyfs_amd import (ECC_CRC, ECC_HAMMING, ECC_NONE, ECC_PARITY, ECC_REED_SOLOMON, EccEngine)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def rng_for(*k):
    return np.random.default_rng(zlib.crc32(repr(k).encode()))


# ------------------------------------------------------------------------------------
# Reed-Solomon
# ------------------------------------------------------------------------------------
RS_CASES = [(512, 3), (255, 1), (255, 2), (256, 4), (1024, 5), (4096, 8), (4096, 16),  # fast path
            (255, 6), (255, 7), (64, 3), (128, 10), (32, 1)]                           # generic path


@pytest.mark.parametrize("bs,t", RS_CASES, ids=lambda x: str(x))
@pytest.mark.parametrize("nblocks", [1, 300, 1024, 2333])
def test_rs_encode_matches_oracle(oracle, bs, t, nblocks):
    n, k, tt = oracle.rs_sizes(bs, t)
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    assert (eng.raw_block_size, eng.data_size) == (n, k)
    rng = rng_for("rse", bs, t, nblocks)
    data = rng.integers(0, 256, nblocks * k, dtype=np.uint8)
    if nblocks > 2:  # all-zero and all-0xFF payloads
        data[:k] = 0
        data[k:2 * k] = 0xFF
    raw = torch.zeros(nblocks * n, dtype=torch.uint8, device="cuda")
    eng.encode(dev(data), raw, nblocks=nblocks)
    assert np.array_equal(host(raw), oracle.rs_encode(bs, t, data))


def inject_rs(rng, cw, n, t, nblocks):
    bad = cw.copy().reshape(nblocks, n)
    for b in range(nblocks):
        ne = b % (t + 4)  # 0..t+3 errors
        pos = rng.choice(n, min(ne, n), replace=False)
        bad[b, pos] ^= rng.integers(1, 256, pos.size, dtype=np.uint8)
    return bad.reshape(-1)


@pytest.mark.parametrize("bs,t", RS_CASES, ids=lambda x: str(x))
@pytest.mark.parametrize("nblocks", [300, 1024])
def test_rs_decode_matches_oracle(oracle, bs, t, nblocks):
    n, k, _ = oracle.rs_sizes(bs, t)
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    rng = rng_for("rsd", bs, t, nblocks)
    data = rng.integers(0, 256, nblocks * k, dtype=np.uint8)
    cw = oracle.rs_encode(bs, t, data)
    bad = inject_rs(rng, cw, n, t, nblocks)
    o_data, o_st, o_fixed, o_wbl, rc = oracle.rs_decode(bs, t, bad)
    assert rc == 0
    raw_d = dev(bad)
    data_d = torch.zeros(nblocks * k, dtype=torch.uint8, device="cuda")
    st_d = torch.full((nblocks,), 77, dtype=torch.uint8, device="cuda")
    spill_d = torch.zeros(nblocks * eng.spill_bytes_per_block(), dtype=torch.uint8, device="cuda")
    eng.decode(raw_d, data_d, st_d, write_back=True, spill=spill_d, nblocks=nblocks)
    assert np.array_equal(host(st_d), o_st)
    assert np.array_equal(host(data_d), o_data)
    assert np.array_equal(host(raw_d), o_fixed)  # in-place write-back == reference's written bytes
    sp = host(spill_d).reshape(nblocks, -1)
    for b in range(nblocks):
        extra = max(0, int(o_wbl[b]) - n)
        assert sp[b, 0] == extra
    # <= t errors are always corrected to the original payload
    okb = np.array([b % (t + 4) <= t for b in range(nblocks)])
    assert np.array_equal(host(data_d).reshape(nblocks, k)[okb], data.reshape(nblocks, k)[okb])


@pytest.mark.parametrize("bs,t", [(512, 3), (4096, 16)])
def test_rs_decode_no_writeback_and_status_only(oracle, bs, t):
    """Status-only decode (no payload output), no write-back: statuses as the reference, the
    codewords untouched (t = 16: the byte-slice decode's emission-free path)."""
    nb = 777
    n, k, _ = oracle.rs_sizes(bs, t)
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    rng = rng_for("rsnw", bs, t)
    cw = oracle.rs_encode(bs, t, rng.integers(0, 256, nb * k, dtype=np.uint8))
    bad = inject_rs(rng, cw, n, t, nb)
    o_data, o_st, _, _, _ = oracle.rs_decode(bs, t, bad)
    raw_d = dev(bad)
    st_d = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    eng.decode(raw_d, None, st_d, write_back=False, nblocks=nb)
    assert np.array_equal(host(st_d), o_st)
    assert np.array_equal(host(raw_d), bad)


def inject_rs_fast(rng, cw, n, t, nblocks):
    """Vectorised inject_rs for large batches: block b gets b % (t + 4) distinct error bytes."""
    bad = cw.copy().reshape(nblocks, n)
    ne = np.arange(nblocks) % (t + 4)
    start = rng.integers(0, n, nblocks)
    for j in range(t + 3):
        rows = np.nonzero(ne > j)[0]
        pos = (start[rows] + 37 * j) % n  # 37 is a unit mod 255: distinct positions per block
        bad[rows, pos] ^= rng.integers(1, 256, rows.size, dtype=np.uint8)
    return bad.reshape(-1)


@pytest.mark.parametrize("bs,t", [(512, 3), (256, 4), (255, 1), (1024, 5), (4096, 8), (4096, 16)],
                         ids=lambda x: str(x))
def test_rs_many_tiles_per_workgroup(oracle, bs, t):
    """Batches past one resident grid (2-4 workgroups/CU x 256 CUs x 64 blocks): every workgroup
    walks several tiles, so the double-buffered prefetch of the next tile and the ragged last tile
    run (segment kernels for 2t <= 8, lane-per-block for 8 < 2t <= 16, pair kernels above)."""
    n, k, _ = oracle.rs_sizes(bs, t)
    nb = 3 * 768 * 64 + 37
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    rng = rng_for("rsbig", bs, t)
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    raw_d = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
    eng.encode(dev(data), raw_d, nblocks=nb)
    cw = oracle.rs_encode(bs, t, data)
    assert np.array_equal(host(raw_d), cw)
    bad = inject_rs_fast(rng, cw, n, t, nb)
    o_data, o_st, o_fixed, _, _ = oracle.rs_decode(bs, t, bad)
    raw_d = dev(bad)
    data_d = torch.zeros(nb * k, dtype=torch.uint8, device="cuda")
    st_d = torch.full((nb,), 77, dtype=torch.uint8, device="cuda")
    eng.decode(raw_d, data_d, st_d, write_back=True, nblocks=nb)
    assert np.array_equal(host(st_d), o_st)
    assert np.array_equal(host(data_d), o_data)
    assert np.array_equal(host(raw_d), o_fixed)


@pytest.mark.parametrize("bs,t", [(512, 3), (4096, 16)])
def test_rs_ragged_tiles(oracle, bs, t):
    """Batch sizes around the wave / workgroup tiles of the fast paths (64 blocks per tile for
    2t <= 8, 32 per wave tile for the byte-slice 2t = 32 kernels): every partial-tile size from 1
    to 33 blocks, exact multiples, and a grid whose last round covers only some waves (one resident
    grid of 256 workgroups x 12 waves x 32 blocks, plus 5).  Encode, then decode with 0..t+3
    errors per block and write-back, all vs the oracle."""
    n, k, _ = oracle.rs_sizes(bs, t)
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    for nb in list(range(1, 34)) + [63, 64, 65, 96, 127, 128, 129, 256 * 12 * 32 + 5]:
        rng = rng_for("rsrag", bs, t, nb)
        data = rng.integers(0, 256, nb * k, dtype=np.uint8)
        raw_d = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
        eng.encode(dev(data), raw_d, nblocks=nb)
        cw = oracle.rs_encode(bs, t, data)
        assert np.array_equal(host(raw_d), cw), nb
        bad = inject_rs_fast(rng, cw, n, t, nb)
        o_data, o_st, o_fixed, _, _ = oracle.rs_decode(bs, t, bad)
        raw_d = dev(bad)
        data_d = torch.zeros(nb * k, dtype=torch.uint8, device="cuda")
        st_d = torch.full((nb,), 77, dtype=torch.uint8, device="cuda")
        eng.decode(raw_d, data_d, st_d, write_back=True, nblocks=nb)
        assert np.array_equal(host(st_d), o_st), nb
        assert np.array_equal(host(data_d), o_data), nb
        assert np.array_equal(host(raw_d), o_fixed), nb


@pytest.mark.parametrize("bs,t", [(512, 3), (4096, 16)], ids=["t3", "t16"])
def test_rs_ticket_sets_after_a_small_launch(oracle, bs, t):
    """One engine, one stream: a large batch (8 XCD ticket counters), then batches of fewer than 8
    tiles (a grid of < 8 workgroups counts on fewer counters and used to zero only those of the
    set the large launch left dirty), then large again -- encode and decode, each vs the oracle.  A
    stale counter would start the second large launch's tickets past tiles nobody then encodes
    (rs_wg_tk.hpp tk_clear).  t = 16: the byte-slice kernels' per-wave tickets (round 5,
    rs_bs.hpp BsWalk) on the same counter sets."""
    n, k, _ = oracle.rs_sizes(bs, t)
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    for step, nb in enumerate([3 * 768 * 64 + 11, 448, 100, 7, 3 * 768 * 64 + 11, 1 << 16, 130, 1 << 16]):
        rng = rng_for("tkclear", step, nb)
        data = rng.integers(0, 256, nb * k, dtype=np.uint8)
        raw_d = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
        eng.encode(dev(data), raw_d, nblocks=nb)
        cw = oracle.rs_encode(bs, t, data)
        assert np.array_equal(host(raw_d), cw), (step, nb)
        bad = inject_rs_fast(rng, cw, n, t, nb)
        o_data, o_st, o_fixed, _, _ = oracle.rs_decode(bs, t, bad)
        raw_d = dev(bad)
        data_d = torch.zeros(nb * k, dtype=torch.uint8, device="cuda")
        st_d = torch.full((nb,), 77, dtype=torch.uint8, device="cuda")
        eng.decode(raw_d, data_d, st_d, write_back=True, nblocks=nb)
        assert np.array_equal(host(st_d), o_st), (step, nb)
        assert np.array_equal(host(data_d), o_data), (step, nb)
        assert np.array_equal(host(raw_d), o_fixed), (step, nb)


def test_rs_full_batch_roundtrip_properties():
    """BASELINE configs[1]/[2] at full size (2^20 RS(255,249) blocks): encode, one byte error per
    block, decode with write-back.  Size-independent properties: every payload restored, every
    status 'corrected', the write-back restores the exact codewords, and a clean re-decode reports
    nothing.  (Bit-exactness vs the oracle at this size: test_rs_many_tiles_per_workgroup.)"""
    bs, t, nb = 512, 3, 1 << 20
    n, k = 255, 249
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    g = torch.Generator(device="cuda").manual_seed(7)
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device="cuda", generator=g)
    raw = torch.empty(nb * n, dtype=torch.uint8, device="cuda")
    eng.encode(data, raw, nblocks=nb)
    clean = raw.clone()
    pos = torch.randint(0, n, (nb,), device="cuda", generator=g) + torch.arange(nb, device="cuda") * n
    val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device="cuda", generator=g)
    raw[pos] ^= val
    out = torch.empty(nb * k, dtype=torch.uint8, device="cuda")
    st = torch.full((nb,), 77, dtype=torch.uint8, device="cuda")
    eng.decode(raw, out, st, write_back=True, nblocks=nb)
    torch.cuda.synchronize()
    assert torch.equal(out, data)
    assert bool((st == 1).all())
    assert torch.equal(raw, clean)
    eng.decode(raw, out, st, write_back=True, nblocks=nb)
    torch.cuda.synchronize()
    assert bool((st == 0).all()) and torch.equal(out, data) and torch.equal(raw, clean)


FULL_CFGS = [  # BASELINE configs at their per-GPU sizes (2^20 blocks)
    ("cfg5_rs_t16", ECC_REED_SOLOMON, 4096, 16, 0),
    ("cfg4_hamming", ECC_HAMMING, 4096, 0, 0),
    ("cfg4_crc32", ECC_CRC, 4096, 0, (0x9960034C << 1) + 1),
    ("parity4096", ECC_PARITY, 4096, 0, 0),
]


@pytest.mark.parametrize("name,typ,bs,t,poly", FULL_CFGS, ids=[c[0] for c in FULL_CFGS])
def test_full_size_roundtrip_properties(name, typ, bs, t, poly):
    """2^20 blocks on the device, one fault per block, size-independent properties:
    RS t=16 -- one byte error: every block corrected, payloads and codewords restored, a clean
    re-decode reports nothing; Hamming -- one bit flip in the used bits: corrected, the single
    byte written back; CRC -- one flipped payload bit (not the undetectable last one): every block
    fails its check (status 5); parity -- one flipped bit: every block fails.  Bit-exactness vs
    the oracle is covered at smaller sizes by the tests above."""
    nb = 1 << 20
    eng = EccEngine(typ, bs, t, crc_polynomial_explicit=poly)
    n, k = eng.raw_block_size, eng.data_size
    g = torch.Generator(device="cuda").manual_seed(11)
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device="cuda", generator=g)
    raw = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
    eng.encode(data, raw, nblocks=nb)
    clean = raw.clone()
    base = torch.arange(nb, device="cuda", dtype=torch.int64) * n
    if typ == ECC_REED_SOLOMON:
        pos = base + torch.randint(0, n, (nb,), device="cuda", generator=g)
        raw[pos] ^= torch.randint(1, 256, (nb,), dtype=torch.uint8, device="cuda", generator=g)
    else:
        # a bit inside the payload bytes [0, k - 1) (CRC: not the undetectable last payload bit)
        byte = torch.randint(0, k - 1, (nb,), device="cuda", generator=g)
        bit = torch.randint(0, 8, (nb,), device="cuda", generator=g).to(torch.uint8)
        raw[base + byte] ^= torch.bitwise_left_shift(torch.ones_like(bit), bit)
    out = torch.empty(nb * k, dtype=torch.uint8, device="cuda")
    st = torch.full((nb,), 77, dtype=torch.uint8, device="cuda")
    eng.decode(raw, out, st, write_back=True, nblocks=nb)
    torch.cuda.synchronize()
    if typ in (ECC_REED_SOLOMON, ECC_HAMMING):
        assert bool((st == 1).all())
        assert torch.equal(out, data)
        assert torch.equal(raw, clean)
        eng.decode(raw, out, st, write_back=True, nblocks=nb)
        torch.cuda.synchronize()
        assert bool((st == 0).all()) and torch.equal(out, data)
    else:
        assert bool((st == 5).all())
        eng.decode(clean, out, st, write_back=False, nblocks=nb)
        torch.cuda.synchronize()
        assert bool((st == 0).all()) and torch.equal(out, data)


def test_rs_generic_spill_matches_oracle(oracle):
    """Shortened code (n = 64): miscorrections past the block are reported in the spill."""
    bs, t, nb = 64, 3, 600
    n, k, _ = oracle.rs_sizes(bs, t)
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    rng = rng_for("spill")
    cw = oracle.rs_encode(bs, t, rng.integers(0, 256, nb * k, dtype=np.uint8)).reshape(nb, n)
    for b in range(nb):
        pos = rng.choice(n, 5, replace=False)
        cw[b, pos] ^= rng.integers(1, 256, 5, dtype=np.uint8)
    bad = cw.reshape(-1)
    spill_d = torch.zeros(nb * eng.spill_bytes_per_block(), dtype=torch.uint8, device="cuda")
    eng.decode(dev(bad), None, None, write_back=False, spill=spill_d, nblocks=nb)
    sp = host(spill_d).reshape(nb, -1)
    nspill = 0
    for b in range(nb):
        st, _, fixed, wl, _ = oracle.rs_decode_one_full(bs, t, bad[b * n:(b + 1) * n])
        extra = max(0, wl - n)
        assert sp[b, 0] == extra
        assert sp[b, 1:1 + extra].tobytes() == fixed[n:n + extra].tobytes()
        nspill += extra > 0
    assert nspill > 0


# ------------------------------------------------------------------------------------
# CRC
# ------------------------------------------------------------------------------------
# bs 1024/2048/4096 with a degree <= 32 polynomial run the streaming kernels of bit_fast.hip
# (0xc1acf: degree 20, a partial last CRC byte whose low bits keep the old contents)
# Degrees 29 and 25 at bs >= 1024: a 4-byte field whose last byte keeps old low bits.
CRC_CASES = [(0xea, 256), (0xc1acf, 512), (0x9960034c, 512), (0x9960034c, 4096), (0x5, 64), (0x3, 256),
             (0x42F0E1EBA9EA3693 >> 1, 1024), (0x1021 >> 1, 4096), (0x9960034c, 1024), (0x9960034c, 2048),
             (0xea, 2048), (0xc1acf, 1024), (0xc1acf, 4096), (0x1EDC6F41, 1024), (0x1000003, 4096),
             (0x1EDC6F41, 2048)]


@pytest.mark.parametrize("imp,bs", CRC_CASES, ids=lambda x: hex(x) if x > 4096 else str(x))
def test_crc_encode_check_match_oracle(oracle, imp, bs):
    P = oracle.crc_explicit(imp)
    eng = EccEngine(ECC_CRC, bs, crc_polynomial_explicit=P)
    ds = oracle.crc_data_size(bs, P)
    assert (eng.raw_block_size, eng.data_size) == (bs, ds)
    nb = 257 if bs >= 1024 else 1001
    if (imp, bs) == (0x9960034c, 4096):
        nb = 5003  # workgroups walk 32 / 16 blocks (CRC_BPW = 8 encode, 4 check): ragged last workgroups
    rng = rng_for("crc", imp, bs)
    data = rng.integers(0, 256, nb * ds, dtype=np.uint8)
    old = rng.integers(0, 256, nb * bs, dtype=np.uint8)  # tail bits must survive
    exp = oracle.crc_encode(bs, P, data, raw_old=old)
    raw_d = dev(old)
    eng.encode(dev(data), raw_d, nblocks=nb)
    got = host(raw_d)
    assert np.array_equal(got, exp)
    # flips: none / random bit / last payload bit (undetected) / CRC field bit
    bad = got.reshape(nb, bs).copy()
    for b in range(nb):
        kind = b % 4
        if kind == 1:
            f = int(rng.integers(0, bs * 8))
        elif kind == 2:
            f = ds * 8 - 1
        elif kind == 3:
            f = ds * 8 + int(rng.integers(0, P.bit_length() - 1))
        else:
            continue
        bad[b, f // 8] ^= 0x80 >> (f % 8)
    bad = bad.reshape(-1)
    o_data, o_st = oracle.crc_check(bs, P, bad)
    data_d = torch.zeros(nb * ds, dtype=torch.uint8, device="cuda")
    st_d = torch.full((nb,), 77, dtype=torch.uint8, device="cuda")
    eng.decode(dev(bad), data_d, st_d, nblocks=nb)
    assert np.array_equal(host(st_d), o_st)
    assert np.array_equal(host(data_d), o_data)
    assert (o_st[2::4] == 0).all()  # last payload bit flips pass the check (reference quirk)


# ------------------------------------------------------------------------------------
# Hamming
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize("bs,nb", [(1, 999), (2, 1000), (4, 1000), (8, 1000), (16, 1000), (32, 1000), (64, 1000), (128, 1000),
                                   (256, 1000), (512, 1000), (1024, 1000),
                                   (2048, 700), (4096, 300), (4096, 5003)])
def test_hamming_matches_oracle(oracle, bs, nb):
    """bs >= 1024 runs the streaming kernels of bit_fast.hip; 5003 blocks of 4 KiB make every
    persistent wave walk several blocks (next-block prefetch) and end on a ragged last block.
    bs 1, 2, 4 (block_size_power 0-2, hamming_block_device.cpp:11-19) run the thread-per-block
    kernels: 0 / 8 / 24 payload bits, tail bits 13-15 / 30-31 kept from the old block, and at
    power 0 used bits {1, 2, 4} only."""
    eng = EccEngine(ECC_HAMMING, bs)
    ds = oracle.ham_data_size(bs)
    assert (eng.raw_block_size, eng.data_size) == (bs, ds)
    rng = rng_for("ham", bs, nb)
    data = rng.integers(0, 256, nb * ds, dtype=np.uint8)
    old = rng.integers(0, 256, nb * bs, dtype=np.uint8)
    exp = oracle.ham_encode(bs, data, raw_old=old)
    raw_d = dev(old)
    eng.encode(dev(data), raw_d, nblocks=nb)
    got = host(raw_d)
    assert np.array_equal(got, exp)
    bad = got.reshape(nb, bs).copy()
    for b in range(nb):
        nf = b % 4
        for f in rng.choice(bs * 8, nf, replace=False):
            bad[b, f // 8] ^= 0x80 >> (f % 8)
    bad = bad.reshape(-1)
    o_data, o_st, o_fixed, _ = oracle.ham_decode(bs, bad)
    raw_d = dev(bad)
    data_d = torch.zeros(nb * ds, dtype=torch.uint8, device="cuda")
    st_d = torch.full((nb,), 77, dtype=torch.uint8, device="cuda")
    eng.decode(raw_d, data_d, st_d, write_back=True, nblocks=nb)
    st = host(st_d)
    assert np.array_equal(st, o_st)
    assert np.array_equal(host(raw_d), o_fixed)
    ok = st != 5
    assert np.array_equal(host(data_d).reshape(nb, ds)[ok], o_data.reshape(nb, ds)[ok])


# ------------------------------------------------------------------------------------
# Parity and raw
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize("bs,nb", [(1, 999), (2, 999), (16, 999), (255, 999), (256, 999), (1024, 999), (2048, 999),
                                   (4096, 999), (4096, 5003)])
def test_parity_matches_oracle(oracle, bs, nb):
    eng = EccEngine(ECC_PARITY, bs)
    rng = rng_for("par", bs, nb)
    data = rng.integers(0, 256, nb * (bs - 1), dtype=np.uint8)
    old = rng.integers(0, 256, nb * bs, dtype=np.uint8)
    exp = oracle.parity_encode(bs, data, raw_old=old)
    raw_d = dev(old)
    eng.encode(dev(data), raw_d, nblocks=nb)
    got = host(raw_d)
    assert np.array_equal(got, exp)
    bad = got.reshape(nb, bs).copy()
    bad[1::3, 0] ^= 0x10
    bad = bad.reshape(-1)
    o_data, o_st = oracle.parity_check(bs, bad)
    data_d = torch.zeros(nb * (bs - 1), dtype=torch.uint8, device="cuda")
    st_d = torch.full((nb,), 77, dtype=torch.uint8, device="cuda")
    eng.decode(dev(bad), data_d, st_d, nblocks=nb)
    assert np.array_equal(host(st_d), o_st)
    assert np.array_equal(host(data_d), o_data)


def test_raw_copy():
    eng = EccEngine(ECC_NONE, 512)
    x = torch.randint(0, 256, (512 * 10,), dtype=torch.uint8, device="cuda")
    y = torch.zeros_like(x)
    eng.encode(x, y)
    assert torch.equal(x, y)


# ------------------------------------------------------------------------------------
# writeBlock (read-modify-write) batches
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize("codec", ["rs", "crc", "hamming", "parity"])
def test_write_rmw_matches_oracle(oracle, codec):
    rng = rng_for("rmw", codec)
    nb = 500
    if codec == "rs":
        bs, t = 512, 3
        n, k, _ = oracle.rs_sizes(bs, t)
        eng = EccEngine(ECC_REED_SOLOMON, bs, t)
        old = inject_rs(rng, oracle.rs_encode(bs, t, rng.integers(0, 256, nb * k, dtype=np.uint8)), n, t, nb)
        data = rng.integers(0, 256, nb * k, dtype=np.uint8)
        _, o_st, _, _, _ = oracle.rs_decode(bs, t, old)
        exp = oracle.rs_encode(bs, t, data)
    elif codec == "crc":
        bs, P = 512, oracle.crc_explicit(0xc1acf)  # degree 20: tail bits in play
        ds = oracle.crc_data_size(bs, P)
        eng = EccEngine(ECC_CRC, bs, crc_polynomial_explicit=P)
        old = oracle.crc_encode(bs, P, rng.integers(0, 256, nb * ds, dtype=np.uint8),
                                raw_old=rng.integers(0, 256, nb * bs, dtype=np.uint8)).reshape(nb, bs)
        old[::3, 7] ^= 1
        old = old.reshape(-1)
        data = rng.integers(0, 256, nb * ds, dtype=np.uint8)
        _, o_st = oracle.crc_check(bs, P, old)
        enc = oracle.crc_encode(bs, P, data, raw_old=old).reshape(nb, bs)
        exp = np.where((o_st == 5)[:, None], old.reshape(nb, bs), enc).reshape(-1)
    elif codec == "hamming":
        bs = 512
        ds = oracle.ham_data_size(bs)
        eng = EccEngine(ECC_HAMMING, bs)
        old = oracle.ham_encode(bs, rng.integers(0, 256, nb * ds, dtype=np.uint8),
                                raw_old=rng.integers(0, 256, nb * bs, dtype=np.uint8)).reshape(nb, bs)
        for b in range(nb):
            for f in rng.choice(bs * 8, b % 3, replace=False):
                old[b, f // 8] ^= 0x80 >> (f % 8)
        old = old.reshape(-1)
        data = rng.integers(0, 256, nb * ds, dtype=np.uint8)
        _, o_st, o_fixed, _ = oracle.ham_decode(bs, old)
        enc = oracle.ham_encode(bs, data, raw_old=o_fixed).reshape(nb, bs)
        exp = np.where((o_st == 5)[:, None], old.reshape(nb, bs), enc).reshape(-1)
    else:
        bs = 256
        eng = EccEngine(ECC_PARITY, bs)
        old = oracle.parity_encode(bs, rng.integers(0, 256, nb * (bs - 1), dtype=np.uint8)).reshape(nb, bs)
        old[::4, 3] ^= 2
        old = old.reshape(-1)
        data = rng.integers(0, 256, nb * (bs - 1), dtype=np.uint8)
        _, o_st = oracle.parity_check(bs, old)
        enc = oracle.parity_encode(bs, data, raw_old=old).reshape(nb, bs)
        exp = np.where((o_st == 5)[:, None], old.reshape(nb, bs), enc).reshape(-1)
    raw_d = dev(old)
    st_d = torch.full((nb,), 77, dtype=torch.uint8, device="cuda")
    eng.write(dev(data), raw_d, st_d, nblocks=nb)
    assert np.array_equal(host(st_d), o_st)
    assert np.array_equal(host(raw_d), exp)


# ------------------------------------------------------------------------------------
# host-memory path (pinned staging, several chunks)
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize("chunks", [4, 8], ids=["5chunks", "ramp"])
def test_host_path_multichunk(oracle, chunks):
    # 4 chunks of ppfs_ecc_host_chunk_blocks (64 Ki RS(255,249) blocks) and a ragged one: every
    # staging slot is reused at least once; 8+ chunks: the ramped chunk sizes (api.cpp ramp_chunk:
    # 8 Ki, 16 Ki, 32 Ki, 64 Ki ... halving tail).  The 1-error decode returns patch lists.
    bs, t = 512, 3
    n, k, _ = oracle.rs_sizes(bs, t)
    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    assert eng.host_chunk_blocks() == 1 << 16
    nb = chunks * eng.host_chunk_blocks() + (8001 if chunks == 4 else 12345)
    rng = rng_for("host")
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    raw = np.zeros(nb * n, np.uint8)
    eng.encode_host(data, raw)
    sample = rng.choice(nb, 2000, replace=False)
    ref = oracle.rs_encode(bs, t, data.reshape(nb, k)[sample].reshape(-1)).reshape(-1, n)
    assert np.array_equal(raw.reshape(nb, n)[sample], ref)
    bad = raw.reshape(nb, n).copy()
    bad[np.arange(nb), rng.integers(0, n, nb)] ^= rng.integers(1, 256, nb, dtype=np.uint8)
    bad = bad.reshape(-1)
    out = np.zeros(nb * k, np.uint8)
    st = np.zeros(nb, np.uint8)
    eng.decode_host(bad, out, st, write_back=True)
    assert (st == 1).all()
    assert np.array_equal(out, data)
    assert np.array_equal(bad, raw)


@pytest.mark.parametrize("typ,bs,t,poly", [(ECC_REED_SOLOMON, 512, 3, 0), (ECC_REED_SOLOMON, 64, 3, 0),
                                           (ECC_HAMMING, 4096, 0, 0), (ECC_CRC, 4096, 0, (0x9960034C << 1) + 1)],
                         ids=["rs512", "rs64", "ham4096", "crc4096"])
def test_host_path_pinned_equals_pageable(typ, bs, t, poly):
    """Page-locked caller buffers (ppfs_ecc_host_register) take the direct-DMA path of the host
    calls; results must be byte-identical to the staged (pageable) path, across chunks."""
    from paritypartyfs_amd import pinned

    eng = EccEngine(typ, bs, t, crc_polynomial_explicit=poly)
    n, k = eng.raw_block_size, eng.data_size
    nb = 70001 if bs <= 512 else 3001
    rng = rng_for("pin", bs)
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    outs = []
    for kind in ("pageable", "pinned"):
        raw = np.zeros(nb * n, np.uint8)
        d = data.copy()
        out = np.zeros(nb * k, np.uint8)
        st = np.full(nb, 77, np.uint8)
        sp = np.zeros(nb * eng.spill_bytes_per_block(), np.uint8)
        ctx = pinned(d, raw, out, st, sp) if kind == "pinned" else None
        if ctx:
            ctx.__enter__()
        try:
            eng.encode_host(d, raw)
            r2 = np.random.default_rng(5)
            pos = r2.integers(0, n, nb) + np.arange(nb) * n
            raw[pos] ^= r2.integers(1, 256, nb, dtype=np.uint8)
            eng.decode_host(raw, out, st, write_back=True, spill=sp if bs < 255 else None)
        finally:
            if ctx:
                ctx.__exit__(None, None, None)
        outs.append((raw, out, st))
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("prior", ["none", "eager"])
@pytest.mark.parametrize("kind", ["pageable", "pinned"])
@pytest.mark.parametrize("codec", ["rs512", "ham1024"])
def test_host_decode_returns_only_changed_codewords(oracle, kind, codec, prior):
    """decode_host with write-back fetches codewords back only where the decode changed them
    (status 1): not at all for a clean chunk, as a packed gather for a few, as the whole range for
    many (RS(255, k) and Hamming: as patch lists of the changed bytes).  One set per chunk
    (ppfs_ecc_host_chunk_blocks): clean / 100 errors / every block / 5,000 blocks / a short tail;
    every path must leave the caller's image equal to the oracle's write-back.  prior="eager": the
    context's previous call ended on a chunk where every block changed, so this call's first chunks
    (queued before any has landed: api.cpp host_run_chunks, three staging slots) fetch their
    codewords eagerly."""
    from paritypartyfs_amd import pinned

    rng = rng_for("lazyraw", codec, kind)
    if codec == "rs512":
        eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
    else:
        eng = EccEngine(ECC_HAMMING, 1024, 0)
    ch = eng.host_chunk_blocks()
    nb = 4 * ch + 777
    n, k = eng.raw_block_size, eng.data_size
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    raw = np.zeros(nb * n, np.uint8)
    eng.encode_host(data, raw)
    bad = raw.reshape(nb, n).copy()
    sets = [np.array([], np.int64), ch + rng.choice(ch, 100, replace=False), 2 * ch + np.arange(ch),
            3 * ch + rng.choice(ch, 5000, replace=False), 4 * ch + rng.choice(777, 9, replace=False)]
    hit = np.concatenate(sets)
    if codec.startswith("rs"):
        bad[hit, rng.integers(0, n, hit.size)] ^= rng.integers(1, 256, hit.size, dtype=np.uint8)
    else:  # single bit flips (corrected, 1 byte written back); a few double flips (status 5, no write)
        pos = rng.integers(0, 8 * n, hit.size)
        bad[hit, pos // 8] ^= (0x80 >> (pos % 8)).astype(np.uint8)
        dbl = hit[::7]
        bad[dbl, 3] ^= 0x01
    bad = bad.reshape(-1)
    if codec == "rs512":
        o_data, o_st, o_fixed, _, _ = oracle.rs_decode(512, 3, bad)
    else:
        o_data, o_st, o_fixed, _ = oracle.ham_decode(1024, bad)
    if prior == "eager":  # two chunks, every codeword corrupted: the predictor ends eager
        pre = raw[: 2 * ch * n].reshape(2 * ch, n).copy()
        if codec.startswith("rs"):
            pre[:, 7] ^= 0x5A
        else:
            pre[:, 9] ^= 0x10
        pre = pre.reshape(-1)
        eng.decode_host(pre, None, np.zeros(2 * ch, np.uint8), write_back=True)
        assert np.array_equal(pre, raw[: 2 * ch * n])
    img = bad.copy()
    out = np.zeros(nb * k, np.uint8)
    st = np.full(nb, 77, np.uint8)
    ctx = pinned(img, out, st) if kind == "pinned" else None
    if ctx:
        ctx.__enter__()
    try:
        eng.decode_host(img, out, st, write_back=True)
    finally:
        if ctx:
            ctx.__exit__(None, None, None)
    assert np.array_equal(st, o_st)
    assert np.array_equal(img, o_fixed)
    ok = o_st != 5
    assert np.array_equal(out.reshape(nb, k)[ok], o_data.reshape(nb, k)[ok])
    # status-only decode (the scrub's form): same image
    img2 = bad.copy()
    st2 = np.full(nb, 77, np.uint8)
    eng.decode_host(img2, None, st2, write_back=True)
    assert np.array_equal(st2, o_st) and np.array_equal(img2, o_fixed)


@pytest.mark.parametrize("devices", [(0, 0), (0, 0, 0)], ids=["g2", "g3"])
@pytest.mark.parametrize("codec", ["rs512", "rs4096t16", "crc4096", "ham1024"])
def test_group_host_path_matches_single_context(oracle, devices, codec):
    """ppfs_ecc_group_* (SURVEY 8e host path): contiguous shards, one host thread per context
    (here several contexts on GPU 0).  Every shard boundary must leave results byte-identical to
    one context's calls and to the oracle."""
    from paritypartyfs_amd import EccGroup

    if codec == "rs512":
        args = (ECC_REED_SOLOMON, 512, 3, 0)
    elif codec == "rs4096t16":  # BASELINE configs[4]'s RS(255,223), sharded over the group
        args = (ECC_REED_SOLOMON, 4096, 16, 0)
    elif codec == "crc4096":
        args = (ECC_CRC, 4096, 0, (0x9960034C << 1) + 1)
    else:
        args = (ECC_HAMMING, 1024, 0, 0)
    grp = EccGroup(*args, devices=devices)
    one = EccEngine(*args)
    n, k = one.raw_block_size, one.data_size
    assert (grp.raw_block_size, grp.data_size) == (n, k)
    nb = 40007 if n <= 512 else 3001
    rng = rng_for("group", codec, len(devices))
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    raw_g = np.zeros(nb * n, np.uint8)
    raw_1 = np.zeros(nb * n, np.uint8)
    grp.encode_host(data, raw_g)
    one.encode_host(data, raw_1)
    assert np.array_equal(raw_g, raw_1)
    bad = raw_g.reshape(nb, n).copy()
    hit = rng.choice(nb, nb // 3, replace=False)
    if codec.startswith("rs"):
        bad[hit, rng.integers(0, n, hit.size)] ^= rng.integers(1, 256, hit.size, dtype=np.uint8)
    else:
        pos = rng.integers(0, 8 * n, hit.size)
        bad[hit, pos // 8] ^= (0x80 >> (pos % 8)).astype(np.uint8)
    bad = bad.reshape(-1)
    outs = []
    for eng in (grp, one):
        img = bad.copy()
        out = np.zeros(nb * k, np.uint8)
        st = np.full(nb, 77, np.uint8)
        eng.decode_host(img, out, st, write_back=True)
        outs.append((img, out, st))
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    if codec.startswith("rs"):
        o_data, o_st, o_fixed, _, _ = oracle.rs_decode(args[1], args[2], bad)
        assert np.array_equal(outs[0][2], o_st) and np.array_equal(outs[0][0], o_fixed)
        assert np.array_equal(outs[0][1], o_data)
    # read-modify-write of new payloads over the corrupted image
    new = rng.integers(0, 256, nb * k, dtype=np.uint8)
    res = []
    for eng in (grp, one):
        img = bad.copy()
        st = np.full(nb, 77, np.uint8)
        eng.write_host(new, img, st)
        res.append((img, st))
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])
    grp.close()
    one.close()


@pytest.mark.parametrize("nb", [1, 3, 31, 33, 129])
def test_crc4096_small_batches_match_oracle(oracle, nb):
    """The CRC streaming kernels cover 32 blocks per workgroup: batches below, at and just past
    one workgroup's range (and across several) match the oracle, encode and check."""
    P = oracle.crc_explicit(0x9960034C)
    eng = EccEngine(ECC_CRC, 4096, crc_polynomial_explicit=P)
    ds = eng.data_size
    rng = rng_for("crc-small", nb)
    data = rng.integers(0, 256, nb * ds, dtype=np.uint8)
    old = rng.integers(0, 256, nb * 4096, dtype=np.uint8)
    raw_d = dev(old)
    eng.encode(dev(data), raw_d, nblocks=nb)
    got = host(raw_d)
    assert np.array_equal(got, oracle.crc_encode(4096, P, data, raw_old=old))
    bad = got.reshape(nb, 4096).copy()
    bad[::2, 100] ^= 0x10
    bad = bad.reshape(-1)
    o_data, o_st = oracle.crc_check(4096, P, bad)
    data_d = torch.zeros(nb * ds, dtype=torch.uint8, device="cuda")
    st_d = torch.full((nb,), 77, dtype=torch.uint8, device="cuda")
    eng.decode(dev(bad), data_d, st_d, nblocks=nb)
    assert np.array_equal(host(st_d), o_st)
    assert np.array_equal(host(data_d), o_data)


@pytest.mark.parametrize("bs,t", [(512, 3), (4096, 16)], ids=["t3", "t16"])
@pytest.mark.parametrize("kind", ["pageable", "pinned"])
def test_host_decode_patch_lists_many_errors(oracle, bs, t, kind):
    """decode_host with write-back over two chunks with 0 .. t + 3 byte errors per block: the patch
    lists carry every byte the write-back changed, miscorrections (more than t errors) included --
    the caller's image must equal the oracle's write-back exactly."""
    from paritypartyfs_amd import pinned

    eng = EccEngine(ECC_REED_SOLOMON, bs, t)
    n, k = eng.raw_block_size, eng.data_size
    nb = 2 * eng.host_chunk_blocks() + 333
    rng = rng_for("patch-many", bs, kind)
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    raw = np.zeros(nb * n, np.uint8)
    eng.encode_host(data, raw)
    bad = raw.reshape(nb, n).copy()
    ne = np.arange(nb) % (t + 4)
    for e in range(1, t + 4):
        rows = np.nonzero(ne == e)[0]
        cols = np.argsort(rng.random((rows.size, n)), axis=1)[:, :e]
        bad[rows[:, None], cols] ^= rng.integers(1, 256, (rows.size, e), dtype=np.uint8)
    bad = bad.reshape(-1)
    o_data, o_st, o_fixed, _, _ = oracle.rs_decode(bs, t, bad)
    img = bad.copy()
    out = np.zeros(nb * k, np.uint8)
    st = np.full(nb, 77, np.uint8)
    ctx = pinned(img, out, st) if kind == "pinned" else None
    if ctx:
        ctx.__enter__()
    try:
        eng.decode_host(img, out, st, write_back=True)
    finally:
        if ctx:
            ctx.__exit__(None, None, None)
    assert np.array_equal(st, o_st)
    assert np.array_equal(img, o_fixed)
    assert np.array_equal(out, o_data)
    eng.close()
