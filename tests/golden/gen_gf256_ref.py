"""Writes tests/golden/gf256_ref.npz from the REFERENCE's GF256 (lib/ecc_helpers/src/gf256.cpp),
compiled unmodified by oracle/Makefile into oracle/_ref/libppfs_ref_gf256.so.

Run in the build container (the reference tree is not on the GPU box):
    make -C oracle && python tests/golden/gen_gf256_ref.py

The fixture holds, as produced by the reference binary: the full 256 x 256 product and quotient
tables (a/0 = 0, gf256.cpp:56-64), the inverse table (inv(0) = 0, :76-81), the logarithm table
(log(0) = 0, :20-26, :72) and alpha^i for i = 0..255 (alpha = getPrimitiveElement() = 2, :83).
tests/test_oracle_kats.py checks oracle/ppfs_oracle.c against it exhaustively.
"""
import ctypes
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(ROOT, "oracle", "_ref", "libppfs_ref_gf256.so")
OUT = os.path.join(HERE, "gf256_ref.npz")


def dump(lib_path=LIB):
    L = ctypes.CDLL(lib_path)
    mul = np.zeros(65536, np.uint8)
    div = np.zeros(65536, np.uint8)
    inv = np.zeros(256, np.uint8)
    log = np.zeros(256, np.uint8)
    pw = np.zeros(256, np.uint8)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    L.ref_gf256_dump(p(mul), p(div), p(inv), p(log), p(pw))
    assert L.ref_gf256_add_mismatches() == 0, "reference + / - are not XOR"
    return {"mul": mul.reshape(256, 256), "div": div.reshape(256, 256), "inv": inv, "log": log, "pow": pw}


def main():
    if not os.path.exists(LIB):
        sys.exit(f"{LIB} missing: run `make -C oracle` in the container that holds /root/reference")
    t = dump()
    np.savez_compressed(OUT, **t)
    h = hashlib.sha256(b"".join(t[k].tobytes() for k in ("mul", "div", "inv", "log", "pow"))).hexdigest()
    print(f"wrote {OUT}: sha256(mul|div|inv|log|pow) = {h}")


if __name__ == "__main__":
    main()
