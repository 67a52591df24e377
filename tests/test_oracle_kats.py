"""CPU tests: pin the oracle (oracle/ppfs_oracle.c) to the reference's own known answers, to
the SURVEY-recorded reference outputs, and to an independent literal restatement
(tests/ref_model.py).  These run without a GPU."""
import json
import os

import numpy as np
import pytest

from tests import ref_model as RM
from tests.oracle_lib import OracleDevice

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def aa_pattern(n):
    return ((0xAA + np.arange(n)) & 0xFF).astype(np.uint8)


# ---------------- reference unit-test known answers ----------------
def test_crc_division_reference_kats(oracle):
    for case in GOLD["reference_tests"]["crc_division"]:
        bits = [(case["ulong"] >> (63 - i)) & 1 for i in range(64)]  # BitHelpers::ulongToBits
        rem = oracle.crc_divide_bits(case["explicit_poly"], np.array(bits, np.uint8))
        assert list(rem) == case["remainder"], case["source"]
        assert RM.crc_divide(case["explicit_poly"], bits) == case["remainder"]


def test_crc_conversion_and_degree(oracle):
    c = GOLD["reference_tests"]["crc_conversion"]
    assert oracle.crc_explicit(c["implicit"]) == c["explicit"]
    assert c["explicit"].bit_length() - 1 == c["degree"]
    d = GOLD["reference_tests"]["crc_explicit_implicit_difference"]["poly"]
    assert (d.bit_length()) != (oracle.crc_explicit(d).bit_length())
    dev = GOLD["reference_tests"]["crc_device"]
    assert oracle.crc_data_size(dev["block_size"], oracle.crc_explicit(dev["implicit"])) == dev["data_size"]


def test_bits_msb_first():
    b = GOLD["reference_tests"]["bits_block_to_bits"]
    assert RM.bytes_to_bits(bytes(b["bytes"])) == b["bits"]
    u = GOLD["reference_tests"]["bits_ulong_to_bits"]
    bits = [(u["ulong"] >> (63 - i)) & 1 for i in range(64)]
    assert bits == [0] * u["zeros_then_ones"] + [1] * (64 - u["zeros_then_ones"])


# ---------------- the reference's GF256 binary (oracle/_ref) ----------------
GF_GOLD = os.path.join(os.path.dirname(__file__), "golden", "gf256_ref.npz")
REF_GF_LIB = os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle", "_ref", "libppfs_ref_gf256.so")


def test_gf256_matches_reference_binary_fixture(oracle):
    """Every product, quotient (a/0 = 0), inverse (inv 0 = 0), log and power of the oracle's
    GF(2^8) equals the reference's own GF256 (gf256.cpp:6-83, compiled unmodified into
    oracle/_ref by oracle/Makefile; fixture written by tests/golden/gen_gf256_ref.py)."""
    gold = np.load(GF_GOLD)  # plain arrays, allow_pickle=False
    mine = oracle.gf_dump()
    for k in ("mul", "div", "inv", "log", "pow"):
        assert np.array_equal(mine[k], gold[k]), k
    # spot facts of the reference field: alpha = 2 over 0x11D, EXP[255] = EXP[0] (gf256.cpp:16)
    assert gold["pow"][8] == 0x1D and gold["pow"][255] == 1 and gold["div"][7, 0] == 0


def test_gf256_matches_reference_binary_live(oracle):
    """Same check against the reference binary itself, where it was built (this container)."""
    if not os.path.exists(REF_GF_LIB):
        pytest.skip("oracle/_ref not built (no /root/reference here): the committed fixture pins it")
    from tests.golden.gen_gf256_ref import dump

    ref = dump(REF_GF_LIB)
    mine = oracle.gf_dump()
    for k in ref:
        assert np.array_equal(mine[k], ref[k]), k


def test_rs_generator_from_reference_field():
    """g(x) = prod_{i=1..2t} (x + alpha^i) (rs_block_device.cpp:195-208) multiplied out over the
    reference binary's own product table gives the SURVEY-recorded generators."""
    gold = np.load(GF_GOLD)
    mul, pw = gold["mul"], gold["pow"]
    for t, want in ((3, GOLD["survey_recorded"]["rs_generator"]["t3"]),
                    (16, GOLD["survey_recorded"]["rs_generator"]["t16"])):
        g = [1]
        for i in range(1, 2 * t + 1):
            ng = [0] * (len(g) + 1)
            for k, c in enumerate(g):
                ng[k] ^= int(mul[c, pw[i]])
                ng[k + 1] ^= c
            g = ng
        assert bytes(g).hex() == want


# ---------------- SURVEY-recorded reference outputs ----------------
def test_rs_generator_kats(oracle):
    g = GOLD["survey_recorded"]["rs_generator"]
    assert oracle.rs_generator(512, 3).tobytes().hex() == g["t3"]
    assert oracle.rs_generator(4096, 16).tobytes().hex() == g["t16"]
    assert bytes(RM.rs_generator(3).c[:7]).hex() == g["t3"]


def test_rs_parity_kat(oracle):
    k = GOLD["survey_recorded"]["rs_parity_aa"]
    n, kk, t = oracle.rs_sizes(k["block_size"], k["t"])
    assert (n, kk, t) == (255, 249, 3)
    cw = oracle.rs_encode(k["block_size"], k["t"], aa_pattern(kk))
    assert cw[:6].tobytes().hex() == k["parity"]
    assert (cw[6:] == aa_pattern(kk)).all()
    assert RM.rs_encode(512, 3, aa_pattern(kk).tobytes()) == cw.tobytes()


@pytest.mark.parametrize("case", GOLD["survey_recorded"]["crc_bytes_aa"], ids=lambda c: str(c["block_size"]))
def test_crc_kat(oracle, case):
    P = oracle.crc_explicit(case["implicit"])
    ds = oracle.crc_data_size(case["block_size"], P)
    for faithful in (False, True):
        raw = oracle.crc_encode(case["block_size"], P, aa_pattern(ds), faithful=faithful)
        assert raw[ds:].tobytes().hex() == case["crc"]


# ---------------- cross-checks of the oracle's fast paths ----------------
@pytest.mark.parametrize("implicit,bs", [(0xea, 256), (0xc1acf, 512), (0x9960034c, 512), (0x9960034c, 4096),
                                         (0x5, 64), (0x1021 >> 1, 128), (0x42F0E1EBA9EA3693 >> 1, 256)])
def test_crc_fast_equals_faithful(oracle, implicit, bs):
    rng = np.random.default_rng(bs ^ implicit & 0xFFFF)
    P = oracle.crc_explicit(implicit)
    ds = oracle.crc_data_size(bs, P)
    nb = 16 if bs <= 512 else 3
    data = rng.integers(0, 256, nb * ds, dtype=np.uint8)
    old = rng.integers(0, 256, nb * bs, dtype=np.uint8)
    a = oracle.crc_encode(bs, P, data, raw_old=old, faithful=False)
    b = oracle.crc_encode(bs, P, data, raw_old=old, faithful=True)
    assert (a == b).all()
    # python literal model of the early-stopping division
    for blk in range(min(nb, 2)):
        bits = RM.crc_stored_bits(P, data[blk * ds:(blk + 1) * ds].tobytes())
        got = [(a[blk * bs + ds + i // 8] >> (7 - i % 8)) & 1 for i in range(P.bit_length() - 1)]
        assert got == bits
    # single-bit flips: fast and faithful checks agree
    bad = a.copy()
    flips = rng.integers(0, bs * 8, nb)
    for blk, f in enumerate(flips):
        bad[blk * bs + f // 8] ^= 0x80 >> (f % 8)
    _, s1 = oracle.crc_check(bs, P, bad, faithful=False)
    _, s2 = oracle.crc_check(bs, P, bad, faithful=True)
    assert (s1 == s2).all()


def test_crc_last_data_bit_undetected(oracle):
    """SURVEY finding 4: with the early stop a flip of the last payload bit goes undetected."""
    P = oracle.crc_explicit(0x9960034c)
    ds = oracle.crc_data_size(512, P)
    raw = oracle.crc_encode(512, P, aa_pattern(ds))
    raw[ds - 1] ^= 0x01
    _, st = oracle.crc_check(512, P, raw, faithful=True)
    assert st[0] == 0


@pytest.mark.parametrize("t", [1, 2, 3, 5])
def test_rs_oracle_matches_literal_model(oracle, t):
    """Independent restatement check incl. >t errors (miscorrection) -- small sample."""
    rng = np.random.default_rng(100 + t)
    n, k, _ = oracle.rs_sizes(255, t)
    for trial in range(12):
        d = rng.integers(0, 256, k, dtype=np.uint8)
        cw = oracle.rs_encode(255, t, d)
        assert cw.tobytes() == RM.rs_encode(255, t, d.tobytes())
        nerr = trial % (t + 4)
        bad = cw.copy()
        pos = rng.choice(255, nerr, replace=False)
        bad[pos] ^= rng.integers(1, 256, nerr, dtype=np.uint8)
        data, st, fixed, wbl, rc = oracle.rs_decode(255, t, bad)
        s2, d2, wb2 = RM.rs_decode(255, t, bad.tobytes())
        assert rc == 0 and st[0] == s2 and data.tobytes() == d2
        if s2:
            assert wbl[0] == len(wb2) and fixed[:len(wb2)].tobytes() == wb2
        if nerr <= t:
            assert (data == d).all()


def test_rs_shortened_code_spill(oracle):
    """n < 255: a miscorrection may land past the block; write-back length > n."""
    rng = np.random.default_rng(7)
    seen = 0
    for trial in range(400):
        bs, t = 64, 3
        n, k, _ = oracle.rs_sizes(bs, t)
        cw = oracle.rs_encode(bs, t, rng.integers(0, 256, k, dtype=np.uint8))
        bad = cw.copy()
        pos = rng.choice(n, 5, replace=False)
        bad[pos] ^= rng.integers(1, 256, 5, dtype=np.uint8)
        st, data, fixed, wl, nr = oracle.rs_decode_one_full(bs, t, bad)
        s2, d2, wb2 = RM.rs_decode(bs, t, bad.tobytes())
        assert st == s2 and data.tobytes() == d2 and wl == len(wb2) and fixed[:wl].tobytes() == wb2
        seen += wl > n
    assert seen > 0


# ---------------- reference unit tests restated on the oracle device model ----------------
def test_oracle_rs_device_reference_tests(oracle):
    # test_rs_block_device.cpp:9-138
    cases = [(2, [], 0xAB), (1, [(120, 0x00)], 0x7E), (2, [(10, 0xEE), (200, 0x44)], 0xAB),
             (3, [(10, 0xEE), (100, 0x61), (200, 0x44)], 0xAB)]
    for t, corrupt, fill in cases:
        dev = OracleDevice(oracle, 4, 255, t=t)
        ds = dev.data_size()
        assert dev.format(0) == 0
        assert dev.write(0, 0, bytes([fill]) * ds) == (0, ds)
        for pos, val in corrupt:
            dev.disk[pos] = val
        rc, out = dev.read(0, 0, ds)
        assert rc == 0 and out == bytes([fill]) * ds


def test_oracle_crc_device_reference_tests(oracle):
    # test_crc_block_device.cpp:73-200
    P = oracle.crc_explicit(0xea)
    dev = OracleDevice(oracle, 1, 256, poly=P)
    assert dev.raw_block_size() == 256 and dev.data_size() == 255
    assert dev.format(0) == 0
    assert dev.write(0, 0, b"\x55" * 255)[0] == 0
    assert dev.read(0, 0, 255) == (0, b"\x55" * 255)
    dev = OracleDevice(oracle, 1, 256, poly=P)
    dev.format(0)
    dev.write(0, 0, bytes(255))
    dev.disk[1] = 0x01
    assert dev.read(0, 0, 255)[0] == 5
    for imp, flips in [(0xc1acf, [(1, 1), (111, 8), (200, 2)]),
                       (0x9960034c, [(1, 1), (111, 8), (200, 2), (11, 8), (20, 2)])]:
        dev = OracleDevice(oracle, 1, 512, poly=oracle.crc_explicit(imp))
        dev.format(0)
        dev.write(0, 0, bytes(dev.data_size()))
        for a, v in flips:
            dev.disk[a] = v
        assert dev.read(0, 0, dev.data_size())[0] == 5


def test_oracle_hamming_device_reference_tests(oracle):
    # test_hamming_block_device.cpp:34-143 (random bits made deterministic)
    rng = np.random.default_rng(3)
    dev = OracleDevice(oracle, 2, 16)
    assert dev.write(0, 0, b"hello") == (0, 5)
    assert dev.read(0, 0, 5) == (0, b"hello")
    for i in range(30):
        dev = OracleDevice(oracle, 2, 16)
        msg = f"Round{i}".encode()
        dev.write(0, 0, msg)
        bit = int(rng.integers(0, dev.data_size() * 8))
        dev.disk[bit // 8] ^= 1 << (bit % 8)
        assert dev.read(0, 0, len(msg)) == (0, msg)
        assert dev.log_entries() == [0]
        dev = OracleDevice(oracle, 2, 16)
        dev.write(0, 0, b"slay")
        b1, b2 = rng.choice(dev.data_size() * 8, 2, replace=False)
        for b in (b1, b2):
            dev.disk[b // 8] ^= 1 << (b % 8)
        assert dev.read(0, 0, 4)[0] == 5


def test_oracle_parity_device_reference_tests(oracle):
    # test_parity_block_device.cpp:8-59
    dev = OracleDevice(oracle, 3, 256)
    ds = dev.data_size()
    dev.format(0)
    dev.write(0, 0, b"\xaa" * ds)
    assert dev.read(0, 0, ds) == (0, b"\xaa" * ds)
    dev.write(0, 0, b"\x55" * ds)
    dev.disk[10] ^= 4
    assert dev.read(0, 0, ds)[0] == 5


def test_hamming_oracle_layout():
    # data bit i -> i-th integer >= 3 that is not a power of two
    bs, ds = RM.hamming_layout(12)
    assert (bs, ds) == (4096, 4091)
    idx = RM.hamming_data_indices(bs, ds)
    assert idx[:5] == [3, 5, 6, 7, 9] and idx[-1] == 32743


@pytest.mark.parametrize("bs,t", [(512, 3), (255, 1), (256, 4), (4096, 8), (4096, 16), (64, 3), (128, 10)])
def test_table_codec_equals_long_division(oracle, bs, t):
    """The CPU baseline's optimised column (LFSR encode, table syndromes) gives the restated
    long-division encode's codewords and its decode's payloads / statuses / write-backs."""
    n, k, tt = oracle.rs_sizes(bs, t)
    rng = np.random.default_rng(bs * 100 + t)
    nb = 400
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    cw = oracle.rs_encode(bs, t, data)
    assert np.array_equal(oracle.rs_encode_table(bs, t, data), cw)
    bad = cw.reshape(nb, n).copy()
    for b in range(nb):
        ne = b % (tt + 3)
        pos = rng.choice(n, ne, replace=False)
        bad[b, pos] ^= rng.integers(1, 256, ne, dtype=np.uint8)
    bad = bad.reshape(-1)
    d1, s1, f1, _, rc1 = oracle.rs_decode(bs, t, bad)
    d2, s2, f2, rc2 = oracle.rs_decode_table(bs, t, bad)
    assert rc1 == rc2
    if rc1 == 0:
        assert np.array_equal(d1, d2) and np.array_equal(s1, s2) and np.array_equal(f1, f2)
