"""GPU tests of the resident small-batch server (api.cpp server_call, rs_wg.hpp rs_wg_server_kernel):
the per-block readBlock / writeBlock calls of every codec (batches of <= 64 blocks through
the host entry points) are served by one resident workgroup polling a mailbox in host-coherent
memory.  Every result is compared with the oracle (rs_block_device.cpp semantics: payload,
status, written-back codeword bytes) and with the launch path (PPFS_ECC_SERVER=0); the server is
exercised across its idle exit and relaunch, several contexts at once, and teardown with a
launch resident.
"""
import os
import time
import zlib

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine

# every RS table layout: 2t <= 8 segment path, 2t = 10 / 16 lane-per-block, 2t = 32 pair path,
# and the generic path (2t = 12 at n = 255; shortened codes n < 255)
SERVER_CASES = [(512, 3), (255, 1), (255, 2), (256, 4), (256, 16), (4096, 16), (1024, 5), (4096, 8), (255, 6),
                (64, 3), (128, 10), (32, 1)]


def rng_for(*k):
    return np.random.default_rng(zlib.crc32(repr(k).encode()))


def inject(rng, cw, n, t, nb):
    bad = cw.copy().reshape(nb, n)
    for b in range(nb):
        ne = b % (t + 4)  # 0..t+3 byte errors: corrected, detected, miscorrected
        pos = rng.choice(n, ne, replace=False)
        bad[b, pos] ^= rng.integers(1, 256, pos.size, dtype=np.uint8)
    return bad.reshape(-1)


def engine(bs, t, server=True):
    """A context whose first small call (where the choice is made) sees PPFS_ECC_SERVER."""
    old = os.environ.get("PPFS_ECC_SERVER")
    os.environ["PPFS_ECC_SERVER"] = "1" if server else "0"
    try:
        eng = EccEngine(ECC_REED_SOLOMON, bs, t)
        n, k = eng.raw_block_size, eng.data_size
        eng.encode_host(np.zeros(k, np.uint8), np.zeros(n, np.uint8))  # decides the path
    finally:
        if old is None:
            del os.environ["PPFS_ECC_SERVER"]
        else:
            os.environ["PPFS_ECC_SERVER"] = old
    return eng


@pytest.mark.parametrize("bs,t", SERVER_CASES, ids=lambda x: str(x))
@pytest.mark.parametrize("nb", [1, 2, 17, 63, 64])
def test_server_encode_decode_write_match_oracle(oracle, bs, t, nb):
    eng = engine(bs, t)
    n, k, _ = oracle.rs_sizes(bs, t)
    rng = rng_for("srv", bs, t, nb)
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    raw = np.zeros(nb * n, np.uint8)
    eng.encode_host(data, raw)
    assert np.array_equal(raw, oracle.rs_encode(bs, t, data))
    bad = inject(rng, raw, n, t, nb)
    o_data, o_st, o_fixed, _, rc = oracle.rs_decode(bs, t, bad)
    assert rc == 0
    img, out, st = bad.copy(), np.zeros(nb * k, np.uint8), np.full(nb, 77, np.uint8)
    eng.decode_host(img, out, st, write_back=True)
    assert np.array_equal(st, o_st)
    assert np.array_equal(out, o_data)
    assert np.array_equal(img, o_fixed)
    # no write-back, status only
    img2, st2 = bad.copy(), np.full(nb, 77, np.uint8)
    eng.decode_host(img2, None, st2, write_back=False)
    assert np.array_equal(st2, o_st) and np.array_equal(img2, bad)
    # writeBlock: old block checked for its status, new payload encoded over it
    new = rng.integers(0, 256, nb * k, dtype=np.uint8)
    img3, st3 = bad.copy(), np.full(nb, 77, np.uint8)
    eng.write_host(new, img3, st3)
    assert np.array_equal(st3, o_st)
    assert np.array_equal(img3, oracle.rs_encode(bs, t, new))
    eng.close()


@pytest.mark.parametrize("bs,t", [(512, 3), (256, 16)], ids=lambda x: str(x))
def test_server_equals_launch_path(oracle, bs, t):
    nb = 40
    a, b = engine(bs, t, server=True), engine(bs, t, server=False)
    n, k, _ = oracle.rs_sizes(bs, t)
    rng = rng_for("srv-vs-launch")
    for it in range(20):
        data = rng.integers(0, 256, nb * k, dtype=np.uint8)
        ra, rb = np.zeros(nb * n, np.uint8), np.zeros(nb * n, np.uint8)
        a.encode_host(data, ra)
        b.encode_host(data, rb)
        assert np.array_equal(ra, rb)
        bad = inject(rng, ra, n, t, nb)
        outs = []
        for e in (a, b):
            img, out, st = bad.copy(), np.zeros(nb * k, np.uint8), np.zeros(nb, np.uint8)
            e.decode_host(img, out, st, write_back=True)
            outs.append((img, out, st))
        for x, y in zip(*outs):
            assert np.array_equal(x, y)
    a.close()
    b.close()


def test_server_relaunch_after_idle_exit(oracle):
    """A launch leaves after 20 ms without a request; the next call relaunches it."""
    bs, t = 512, 3
    eng = engine(bs, t)
    n, k, _ = oracle.rs_sizes(bs, t)
    rng = rng_for("srv-idle")
    for it in range(6):
        data = rng.integers(0, 256, 3 * k, dtype=np.uint8)
        raw = np.zeros(3 * n, np.uint8)
        eng.encode_host(data, raw)
        assert np.array_equal(raw, oracle.rs_encode(bs, t, data))
        time.sleep(0.005 if it % 2 else 0.06)  # alternately inside and past the idle limit
    eng.close()


def test_server_many_contexts_interleaved_and_torn_down(oracle):
    bs, t = 512, 3
    n, k, _ = oracle.rs_sizes(bs, t)
    engs = [engine(bs, t) for _ in range(6)]
    rng = rng_for("srv-many")
    for it in range(10):
        for i, e in enumerate(engs):
            data = rng.integers(0, 256, (1 + i) * k, dtype=np.uint8)
            raw = np.zeros((1 + i) * n, np.uint8)
            e.encode_host(data, raw)
            assert np.array_equal(raw, oracle.rs_encode(bs, t, data))
    for e in engs:  # each with its launch still resident
        e.close()


def test_server_large_batches_take_the_chunked_path(oracle):
    """> 64 blocks go through the staged, chunked path; the same context keeps serving small calls."""
    bs, t = 512, 3
    eng = engine(bs, t)
    n, k, _ = oracle.rs_sizes(bs, t)
    rng = rng_for("srv-large")
    for nb in (1, 65, 3, 1000, 64):
        data = rng.integers(0, 256, nb * k, dtype=np.uint8)
        raw = np.zeros(nb * n, np.uint8)
        eng.encode_host(data, raw)
        assert np.array_equal(raw, oracle.rs_encode(bs, t, data))
    eng.close()


# ------------------------------------------------------------------------------------
# CRC / Hamming / parity (bit_server_kernel)
# ------------------------------------------------------------------------------------
from paritypartyfs_amd import ECC_CRC, ECC_HAMMING, ECC_PARITY  # noqa: E402

BIT_CASES = [("crc", 0xea, 256), ("crc", 0x9960034c, 4096), ("crc", 0xc1acf, 512), ("crc", 0x42F0E1EBA9EA3693 >> 1, 1024),
             ("ham", 0, 256), ("ham", 0, 4096), ("ham", 0, 64), ("ham", 0, 8), ("par", 0, 256),
             ("par", 0, 4096), ("par", 0, 2)]


def bit_engine(oracle, codec, imp, bs, server=True):
    old = os.environ.get("PPFS_ECC_SERVER")
    os.environ["PPFS_ECC_SERVER"] = "1" if server else "0"
    try:
        if codec == "crc":
            eng = EccEngine(ECC_CRC, bs, crc_polynomial_explicit=oracle.crc_explicit(imp))
        elif codec == "ham":
            eng = EccEngine(ECC_HAMMING, bs)
        else:
            eng = EccEngine(ECC_PARITY, bs)
        eng.encode_host(np.zeros(eng.data_size, np.uint8), np.zeros(eng.raw_block_size, np.uint8))
    finally:
        if old is None:
            del os.environ["PPFS_ECC_SERVER"]
        else:
            os.environ["PPFS_ECC_SERVER"] = old
    return eng


@pytest.mark.parametrize("codec,imp,bs", BIT_CASES, ids=[f"{c}-{bs}" + (f"-{i:x}" if i else "") for c, i, bs in BIT_CASES])
@pytest.mark.parametrize("nb", [1, 7, 64])
def test_bit_server_matches_oracle_and_launch_path(oracle, codec, imp, bs, nb):
    a = bit_engine(oracle, codec, imp, bs, server=True)
    b = bit_engine(oracle, codec, imp, bs, server=False)
    n, k = a.raw_block_size, a.data_size
    rng = rng_for("bitsrv", codec, imp, bs, nb)
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    old = rng.integers(0, 256, nb * n, dtype=np.uint8)  # old raw contents (tail bits the encode keeps)
    ra, rb = old.copy(), old.copy()
    a.encode_host(data, ra)
    b.encode_host(data, rb)
    assert np.array_equal(ra, rb)
    if codec == "crc":
        P = oracle.crc_explicit(imp)
        assert np.array_equal(ra, oracle.crc_encode(bs, P, data, raw_old=old))
    elif codec == "ham":
        assert np.array_equal(ra, oracle.ham_encode(bs, data, raw_old=old))
    else:
        assert np.array_equal(ra, oracle.parity_encode(bs, data, raw_old=old))
    # corrupt: 0..2 bit flips per block
    bad = ra.copy().reshape(nb, n)
    for blk in range(nb):
        for f in rng.choice(n * 8, blk % 3, replace=False):
            bad[blk, f // 8] ^= 0x80 >> (f % 8)
    bad = bad.reshape(-1)
    for wb in (True, False):
        outs = []
        for e in (a, b):
            img, out, st = bad.copy(), np.zeros(nb * k, np.uint8), np.full(nb, 77, np.uint8)
            e.decode_host(img, out, st, write_back=wb)
            outs.append((img, out, st))
        (ia, oa, sa), (ib, ob, sb) = outs
        assert np.array_equal(sa, sb) and np.array_equal(ia, ib)
        ok = sa != 5  # payloads are defined where the block was not rejected
        assert np.array_equal(oa.reshape(nb, k)[ok], ob.reshape(nb, k)[ok])
    new = rng.integers(0, 256, nb * k, dtype=np.uint8)
    wa, wb_ = bad.copy(), bad.copy()
    sa, sb = np.full(nb, 77, np.uint8), np.full(nb, 77, np.uint8)
    a.write_host(new, wa, sa)
    b.write_host(new, wb_, sb)
    assert np.array_equal(sa, sb) and np.array_equal(wa, wb_)
    a.close()
    b.close()
