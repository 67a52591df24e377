"""Literal pure-Python restatement of the reference RS/CRC/Hamming code -- TEST ONLY.

A second, independent restatement used to cross-check oracle/ppfs_oracle.c on small cases
(including the reference's miscorrection behaviour with more than t errors).  It mirrors the
reference classes statement by statement (sizes, trimming, non-const operator[] extension),
with no shortcuts, so it is slow: use it for a few hundred blocks at most.

  GF256             lib/ecc_helpers/src/gf256.cpp
  PolynomialGF256   lib/ecc_helpers/src/polynomial_gf256.cpp
  ReedSolomon       lib/blockdevice/src/rs_block_device.cpp:95-280
  CrcPolynomial     lib/ecc_helpers/src/crc_polynomial.cpp:56-76
  Hamming           lib/blockdevice/src/hamming_block_device.cpp:21-230
"""
from __future__ import annotations

from typing import List, Tuple

# ---------------- GF256 ----------------
EXP = [0] * 256
LOG = [0] * 256
_x = 1
for _i in range(255):
    EXP[_i] = _x
    _x <<= 1
    if _x & 0x100:
        _x ^= 0x11D
EXP[255] = EXP[0]
for _i in range(255):
    LOG[EXP[_i]] = _i


def gmul(a, b):
    if a == 0 or b == 0:
        return 0
    s = LOG[a] + LOG[b]
    if s >= 255:
        s -= 255
    return EXP[s]


def gdiv(a, b):
    if a == 0 or b == 0:
        return 0
    d = LOG[a] - LOG[b]
    if d < 0:
        d += 255
    return EXP[d]


def ginv(a):
    if a == 0:
        return 0
    return EXP[255 - LOG[a]]


# ---------------- PolynomialGF256 ----------------
class Poly:
    MAX = 256

    def __init__(self, coeffs=()):
        self.c = [0] * Poly.MAX
        n = min(len(coeffs), Poly.MAX)
        self.c[:n] = list(coeffs)[:n]
        self.size = n
        self.trim()

    def trim(self):
        while self.size > 0 and self.c[self.size - 1] == 0:
            self.size -= 1

    def copy(self):
        p = Poly()
        p.c = list(self.c)
        p.size = self.size
        return p

    def add(self, o):
        n = max(self.size, o.size)
        return Poly([(self.c[i] if i < self.size else 0) ^ (o.c[i] if i < o.size else 0) for i in range(n)])

    def mul(self, o):
        if self.size == 0 or o.size == 0:
            return Poly()
        rs = self.size + o.size - 1
        assert rs <= Poly.MAX, "reference UB"
        r = [0] * rs
        for i in range(self.size):
            for j in range(o.size):
                r[i + j] ^= gmul(self.c[i], o.c[j])
        return Poly(r)

    def get(self, i):  # const operator[]
        return self.c[i] if i < self.size else 0

    def at(self, i):  # non-const operator[]: extends the size with zeros
        if i >= self.size:
            for j in range(self.size, i + 1):
                self.c[j] = 0
            self.size = i + 1
        return i

    def xk(self, k):
        assert k + self.size <= Poly.MAX, "reference UB"
        return Poly([0] * k + self.c[:self.size])

    def mod(self, d):
        if d.size == 0:
            return self.copy()
        rem = self.copy()
        lead = d.c[d.size - 1]
        while rem.size >= d.size:
            shift = rem.size - d.size
            f = gdiv(rem.c[rem.size - 1], lead)
            temp = Poly([0] * shift + [gmul(d.c[i], f) for i in range(d.size)])
            rem = rem.add(temp)
            rem.trim()
        return rem

    def evaluate(self, x):
        result, power = 0, 1
        for i in range(self.size):
            result = gmul(self.c[i], power) ^ result
            power = gmul(x, power)
        return result

    def derivative(self):
        ds = self.size - 1 if self.size > 0 else 0
        d = [0] * ds
        for i in range(1, self.size):
            d[i - 1] = self.c[i] if i % 2 else 0
        return Poly(d)


def rs_generator(t):
    g = Poly([1])
    power = 2
    for _ in range(2 * t):
        g = g.mul(Poly([power, 1]))
        power = gmul(power, 2)
    return g


def rs_sizes(block_size, t):
    n = min(block_size, 255)
    t = min(t, n // 2)
    return n, t


def rs_encode(block_size, t, data: bytes) -> bytes:
    n, t = rs_sizes(block_size, t)
    g = rs_generator(t)
    msg = Poly(list(data))
    sh = msg.xk(2 * t)
    enc = sh.add(sh.mod(g))
    return bytes(enc.get(i) for i in range(n))


def rs_decode(block_size, t, raw: bytes) -> Tuple[int, bytes, bytes]:
    """-> (status 0/1, payload, written-back bytes (code_word.size() of them; b'' when clean))"""
    n, t = rs_sizes(block_size, t)
    cw = Poly(list(raw))
    syn = []
    ok = True
    power = 2
    for _ in range(2 * t):
        s = cw.evaluate(power)
        syn.append(s)
        if s:
            ok = False
        power = gmul(power, 2)
    wb = b""
    if not ok:
        # _berlekampMassey :234-269
        sigma, B = Poly([1]), Poly([1])
        b, L, m = 1, 0, 1
        for nn in range(len(syn)):
            d = syn[nn]
            for i in range(1, L + 1):
                sigma.at(i)
                d ^= gmul(sigma.c[i], syn[nn - i])
            if d:
                T = sigma.copy()
                diff = B.mul(Poly([gdiv(d, b)])).xk(m)
                sigma = sigma.add(diff)
                if 2 * L <= nn:
                    L = nn + 1 - L
                    B, b, m = T, d, 1
                else:
                    m += 1
            else:
                m += 1
        locs = [ginv(i) for i in range(1, 256) if sigma.evaluate(i) == 0]
        S = Poly(syn)
        prod = S.mul(sigma)
        omega = Poly([prod.get(i) for i in range(len(syn))])
        dsig = sigma.derivative()
        vals = [gdiv(omega.evaluate(ginv(X)), dsig.evaluate(ginv(X))) for X in locs]
        for X, e in zip(locs, vals):
            pos = LOG[X]
            cw.at(pos)
            cw.c[pos] ^= e
        wb = bytes(cw.c[:cw.size])
    data = bytes(cw.get(2 * t + i) for i in range(n - 2 * t))
    return (0 if ok else 1), data, wb


# ---------------- CRC (bit arrays) ----------------
def crc_divide(P: int, bits: List[int]) -> List[int]:
    n = P.bit_length() - 1
    co = [(P >> (n - j)) & 1 for j in range(n + 1)]
    r = list(bits)
    for i in range(len(bits) - (n + 1)):  # crc_polynomial.cpp:63 -- one step short
        if not r[i]:
            continue
        for j in range(n + 1):
            r[i + j] ^= co[j]
    return r[len(r) - n:]


def bytes_to_bits(b: bytes) -> List[int]:
    return [(x >> (7 - k)) & 1 for x in b for k in range(8)]


def crc_stored_bits(P: int, data: bytes) -> List[int]:
    n = P.bit_length() - 1
    return crc_divide(P, bytes_to_bits(data) + [0] * n)


# ---------------- Hamming ----------------
def hamming_layout(block_size_power):
    bs = 1 << block_size_power
    ds = bs - -(-(block_size_power * 3 + 1) // 8)
    return bs, ds


def hamming_data_indices(bs, ds):
    out, cur = [], 0
    while len(out) < ds * 8:
        while (cur & (cur - 1)) == 0:
            cur += 1
        out.append(cur)
        cur += 1
    return out
