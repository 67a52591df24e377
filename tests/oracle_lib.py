"""ctypes wrapper of the CPU oracle (oracle/ppfs_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, and only
as the checker.  The oracle is built from oracle/ppfs_oracle.c by oracle/Makefile.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_int, c_int32, c_size_t, c_uint8, c_uint64, c_void_p

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libppfs_oracle.so")


def _p(a):
    return None if a is None else a.ctypes.data_as(c_void_p)


def build_oracle() -> str:
    if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(
            os.path.join(ROOT, "oracle", "ppfs_oracle.c")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return ORACLE_SO


class Oracle:
    def __init__(self):
        L = ctypes.CDLL(build_oracle())
        self.L = L
        vp = c_void_p
        L.oracle_gf_mul.restype = c_uint8
        L.oracle_gf_mul.argtypes = [c_uint8, c_uint8]
        L.oracle_gf_div.restype = c_uint8
        L.oracle_gf_div.argtypes = [c_uint8, c_uint8]
        L.oracle_gf_inv.restype = c_uint8
        L.oracle_gf_inv.argtypes = [c_uint8]
        L.oracle_gf_dump.restype = None
        L.oracle_gf_dump.argtypes = [vp, vp, vp, vp, vp]
        L.oracle_rs_sizes.argtypes = [c_int, c_int, POINTER(c_int), POINTER(c_int)]
        L.oracle_rs_generator.argtypes = [c_int, c_int, vp]
        L.oracle_rs_encode.argtypes = [c_int, c_int, vp, vp, c_size_t]
        L.oracle_rs_decode.argtypes = [c_int, c_int, vp, vp, vp, vp, vp, c_size_t]
        L.oracle_rs_encode_table.argtypes = [c_int, c_int, vp, vp, c_size_t]
        L.oracle_rs_decode_table.argtypes = [c_int, c_int, vp, vp, vp, vp, c_size_t]
        L.oracle_rs_decode_one_full.argtypes = [c_int, c_int, vp, vp, vp, POINTER(c_int32), POINTER(c_int32)]
        L.oracle_crc_implicit_to_explicit.restype = c_uint64
        L.oracle_crc_implicit_to_explicit.argtypes = [c_uint64]
        L.oracle_crc_data_size.argtypes = [c_int, c_uint64]
        L.oracle_crc_divide_bits.argtypes = [c_uint64, vp, c_size_t, vp]
        L.oracle_crc_encode.argtypes = [c_int, c_uint64, vp, vp, c_size_t, c_int]
        L.oracle_crc_check.argtypes = [c_int, c_uint64, vp, vp, vp, c_size_t, c_int]
        L.oracle_hamming_data_size.argtypes = [c_int]
        L.oracle_hamming_encode.argtypes = [c_int, vp, vp, c_size_t]
        L.oracle_hamming_decode.argtypes = [c_int, vp, vp, vp, vp, vp, c_size_t]
        L.oracle_parity_encode.argtypes = [c_int, vp, vp, c_size_t]
        L.oracle_parity_check.argtypes = [c_int, vp, vp, vp, c_size_t]
        L.oracle_vote3.restype = None
        L.oracle_vote3.argtypes = [vp, vp, vp, vp, c_size_t, c_size_t, vp]
        L.oracle_dev_create.restype = vp
        L.oracle_dev_create.argtypes = [c_int, c_int, c_int, c_uint64, vp, c_size_t, vp, c_size_t]
        L.oracle_dev_destroy.argtypes = [vp]
        L.oracle_dev_log_len.restype = c_size_t
        L.oracle_dev_log_len.argtypes = [vp]
        L.oracle_dev_raw_block_size.restype = c_size_t
        L.oracle_dev_raw_block_size.argtypes = [vp]
        L.oracle_dev_data_size.restype = c_size_t
        L.oracle_dev_data_size.argtypes = [vp]
        L.oracle_dev_format.argtypes = [vp, ctypes.c_uint]
        L.oracle_dev_read.argtypes = [vp, c_int, c_size_t, c_size_t, c_size_t, vp, POINTER(c_size_t)]
        L.oracle_dev_write.argtypes = [vp, c_int, c_size_t, vp, c_size_t, POINTER(c_size_t)]

    # ---------------- GF / RS ----------------
    def gf_dump(self):
        """{mul, div (256 x 256), inv, log, pow} of the oracle's GF(2^8) (oracle_gf_dump)."""
        t = {k: np.zeros(n, np.uint8) for k, n in (("mul", 65536), ("div", 65536), ("inv", 256), ("log", 256),
                                                     ("pow", 256))}
        self.L.oracle_gf_dump(*[_p(t[k]) for k in ("mul", "div", "inv", "log", "pow")])
        t["mul"] = t["mul"].reshape(256, 256)
        t["div"] = t["div"].reshape(256, 256)
        return t

    def rs_sizes(self, block_size, t):
        n, k = c_int(), c_int()
        tt = self.L.oracle_rs_sizes(block_size, t, ctypes.byref(n), ctypes.byref(k))
        return n.value, k.value, tt

    def rs_generator(self, block_size, t):
        g = np.zeros(256, np.uint8)
        m = self.L.oracle_rs_generator(block_size, t, _p(g))
        return g[:m].copy()

    def rs_encode(self, block_size, t, data):
        n, k, _ = self.rs_sizes(block_size, t)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        nb = data.size // k
        raw = np.zeros(nb * n, np.uint8)
        rc = self.L.oracle_rs_encode(block_size, t, _p(data), _p(raw), nb)
        assert rc == 0, "reference-undefined behaviour hit"
        return raw

    def rs_decode(self, block_size, t, raw):
        n, k, _ = self.rs_sizes(block_size, t)
        raw = np.ascontiguousarray(raw, dtype=np.uint8)
        nb = raw.size // n
        data = np.zeros(nb * k, np.uint8)
        status = np.zeros(nb, np.uint8)
        fixed = np.zeros(nb * n, np.uint8)
        wbl = np.zeros(nb, np.int32)
        rc = self.L.oracle_rs_decode(block_size, t, _p(raw), _p(data), _p(status), _p(fixed), _p(wbl), nb)
        return data, status, fixed, wbl, rc

    def rs_encode_table(self, block_size, t, data):
        """The table-driven (LFSR) encode of the CPU baseline's optimised column."""
        n, k, _ = self.rs_sizes(block_size, t)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        nb = data.size // k
        raw = np.zeros(nb * n, np.uint8)
        assert self.L.oracle_rs_encode_table(block_size, t, _p(data), _p(raw), nb) == 0
        return raw

    def rs_decode_table(self, block_size, t, raw):
        """Table syndromes + the restated decode for non-zero ones: (data, status, fixed, rc)."""
        n, k, _ = self.rs_sizes(block_size, t)
        raw = np.ascontiguousarray(raw, dtype=np.uint8)
        nb = raw.size // n
        data = np.zeros(nb * k, np.uint8)
        status = np.zeros(nb, np.uint8)
        fixed = np.zeros(nb * n, np.uint8)
        rc = self.L.oracle_rs_decode_table(block_size, t, _p(raw), _p(data), _p(status), _p(fixed), nb)
        return data, status, fixed, rc

    def rs_decode_one_full(self, block_size, t, raw):
        n, k, _ = self.rs_sizes(block_size, t)
        data = np.zeros(k, np.uint8)
        fixed = np.zeros(256, np.uint8)
        wl, nr = c_int32(), c_int32()
        st = self.L.oracle_rs_decode_one_full(block_size, t, _p(np.ascontiguousarray(raw, np.uint8)), _p(data),
                                              _p(fixed), ctypes.byref(wl), ctypes.byref(nr))
        return st, data, fixed, wl.value, nr.value

    # ---------------- CRC ----------------
    def crc_explicit(self, implicit):
        return int(self.L.oracle_crc_implicit_to_explicit(implicit))

    def crc_data_size(self, bs, P):
        return self.L.oracle_crc_data_size(bs, P)

    def crc_divide_bits(self, P, bits):
        bits = np.ascontiguousarray(bits, np.uint8)
        n = P.bit_length() - 1
        rem = np.zeros(64, np.uint8)
        self.L.oracle_crc_divide_bits(P, _p(bits), bits.size, _p(rem))
        return rem[:n].copy()

    def crc_encode(self, bs, P, data, raw_old=None, faithful=False):
        ds = self.crc_data_size(bs, P)
        data = np.ascontiguousarray(data, np.uint8)
        nb = data.size // ds
        raw = np.zeros(nb * bs, np.uint8) if raw_old is None else np.array(raw_old, np.uint8, copy=True)
        assert self.L.oracle_crc_encode(bs, P, _p(data), _p(raw), nb, int(faithful)) == 0
        return raw

    def crc_check(self, bs, P, raw, faithful=False):
        ds = self.crc_data_size(bs, P)
        raw = np.ascontiguousarray(raw, np.uint8)
        nb = raw.size // bs
        data = np.zeros(nb * ds, np.uint8)
        st = np.zeros(nb, np.uint8)
        assert self.L.oracle_crc_check(bs, P, _p(raw), _p(data), _p(st), nb, int(faithful)) == 0
        return data, st

    # ---------------- Hamming ----------------
    def ham_data_size(self, bs):
        return self.L.oracle_hamming_data_size(bs)

    def ham_encode(self, bs, data, raw_old=None):
        ds = self.ham_data_size(bs)
        data = np.ascontiguousarray(data, np.uint8)
        nb = data.size // ds if ds else np.asarray(raw_old).size // bs  # power 0: no payload
        raw = np.zeros(nb * bs, np.uint8) if raw_old is None else np.array(raw_old, np.uint8, copy=True)
        self.L.oracle_hamming_encode(bs, _p(data), _p(raw), nb)
        return raw

    def ham_decode(self, bs, raw):
        ds = self.ham_data_size(bs)
        raw = np.ascontiguousarray(raw, np.uint8)
        nb = raw.size // bs
        data = np.zeros(nb * ds, np.uint8)
        st = np.zeros(nb, np.uint8)
        fixed = np.zeros(nb * bs, np.uint8)
        fb = np.zeros(nb, np.int32)
        self.L.oracle_hamming_decode(bs, _p(raw), _p(data), _p(st), _p(fixed), _p(fb), nb)
        return data, st, fixed, fb

    # ---------------- Parity ----------------
    def parity_encode(self, bs, data, raw_old=None):
        data = np.ascontiguousarray(data, np.uint8)
        nb = data.size // (bs - 1) if bs > 1 else np.asarray(raw_old).size  # 1-byte blocks: no payload
        raw = np.zeros(nb * bs, np.uint8) if raw_old is None else np.array(raw_old, np.uint8, copy=True)
        self.L.oracle_parity_encode(bs, _p(data), _p(raw), nb)
        return raw

    def parity_check(self, bs, raw):
        raw = np.ascontiguousarray(raw, np.uint8)
        nb = raw.size // bs
        data = np.zeros(nb * (bs - 1), np.uint8)
        st = np.zeros(nb, np.uint8)
        self.L.oracle_parity_check(bs, _p(raw), _p(data), _p(st), nb)
        return data, st


def _vote3(self, a, b, c, rec_bytes):
    a, b, c = (np.ascontiguousarray(x, np.uint8).reshape(-1) for x in (a, b, c))
    nrec = a.size // rec_bytes
    out = np.zeros(a.size, np.uint8)
    dmg = np.zeros(nrec, np.uint32)
    self.L.oracle_vote3(_p(a), _p(b), _p(c), _p(out), rec_bytes, nrec, _p(dmg))
    return out, dmg


Oracle.vote3 = _vote3


class OracleDevice:
    """Reference IBlockDevice semantics over an in-memory disk (oracle_dev_*)."""

    def __init__(self, oracle: Oracle, ecc_type, block_size, t=3, poly=0, disk_size=1 << 22):
        self.o = oracle
        self.disk = np.zeros(disk_size, np.uint8)
        self.log = np.zeros(1 << 16, np.int32)
        self.h = oracle.L.oracle_dev_create(int(ecc_type), block_size, t, poly, _p(self.disk), disk_size,
                                            _p(self.log), self.log.size)

    def __del__(self):
        try:
            self.o.L.oracle_dev_destroy(self.h)
        except Exception:
            pass

    def raw_block_size(self):
        return self.o.L.oracle_dev_raw_block_size(self.h)

    def data_size(self):
        return self.o.L.oracle_dev_data_size(self.h)

    def format(self, block):
        return self.o.L.oracle_dev_format(self.h, block)

    def read(self, block, offset, nbytes, capacity=None):
        cap = nbytes if capacity is None else capacity
        out = np.zeros(max(cap, nbytes, 1) + 4096, np.uint8)
        ln = c_size_t()
        rc = self.o.L.oracle_dev_read(self.h, block, offset, nbytes, cap, _p(out), ctypes.byref(ln))
        return rc, out[:ln.value].tobytes()

    def write(self, block, offset, data):
        d = np.frombuffer(bytes(data), np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        wr = c_size_t()
        rc = self.o.L.oracle_dev_write(self.h, block, offset, _p(d), len(data), ctypes.byref(wr))
        return rc, wr.value

    def log_entries(self):
        n = self.o.L.oracle_dev_log_len(self.h)
        return [int(x) for x in self.log[:n]]


def fnv1a64(b: bytes) -> int:
    h = 0xcbf29ce484222325
    for x in b:
        h ^= x
        h = (h * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h
