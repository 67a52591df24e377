#!/usr/bin/env python3
"""Kernel-time A/B helper: median encode / clean-decode / 1-error-decode times of one codec over
2^20 blocks with the library named by PPFS_ECC_LIB (no correctness checks: ablation builds may
compute wrong bytes on purpose).  Prints one JSON line.
usage: python3 tools/time_codec.py {rs3,rs16,hamming,crc,parity} [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from paritypartyfs_amd import ECC_CRC, ECC_HAMMING, ECC_PARITY, ECC_REED_SOLOMON, EccEngine, crc_implicit_to_explicit

name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
args = {"hamming": (ECC_HAMMING, 4096, 0, 0), "parity": (ECC_PARITY, 4096, 0, 0), "crc": (ECC_CRC, 4096, 0, crc_implicit_to_explicit(0x9960034C)),
        "rs3": (ECC_REED_SOLOMON, 512, 3, 0), "rs16": (ECC_REED_SOLOMON, 4096, 16, 0)}[name]
eng = EccEngine(args[0], args[1], args[2], crc_polynomial_explicit=args[3])
nb = 1 << 20
n, k = eng.raw_block_size, eng.data_size
data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device="cuda")
raw = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
out = torch.empty_like(data)
st = torch.empty(nb, dtype=torch.uint8, device="cuda")
col = raw.view(nb, n)[:, 100]


def timed(fn, pre=None):
    ts = []
    for i in range(reps + 3):
        if pre:
            pre()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


enc = timed(lambda: eng.encode(data, raw, nblocks=nb))
dec = timed(lambda: eng.decode(raw, out, st, write_back=True, nblocks=nb))


def flip():
    raw.view(nb, n)[:, 100] = col ^ 1


dec1 = timed(lambda: eng.decode(raw, out, st, write_back=True, nblocks=nb), flip)
print(json.dumps({"lib": os.path.basename(os.environ.get("PPFS_ECC_LIB", "libppfs_ecc.so")), "codec": name,
                  "encode_us": enc, "clean_decode_us": dec, "err1_decode_us": dec1}))
