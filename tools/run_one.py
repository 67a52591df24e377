#!/usr/bin/env python3
"""Run one codec's encode and decode on 2^20 blocks a few times (for rocprofv3 PMC passes).
usage: python3 tools/run_one.py {hamming,crc,parity,rs3,rs16} [block_size] [reps] [err]
err: flip one bit of raw byte 100 of every block before each decode (the 1-error decode)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from paritypartyfs_amd import ECC_CRC, ECC_HAMMING, ECC_PARITY, ECC_REED_SOLOMON, EccEngine, crc_implicit_to_explicit

name = sys.argv[1]
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
args = {"hamming": (ECC_HAMMING, bs, 0, 0), "parity": (ECC_PARITY, bs, 0, 0),
        "crc": (ECC_CRC, bs, 0, crc_implicit_to_explicit(0x9960034C)),
        "rs3": (ECC_REED_SOLOMON, 512, 3, 0), "rs16": (ECC_REED_SOLOMON, 4096, 16, 0)}[name]
eng = EccEngine(args[0], args[1], args[2], crc_polynomial_explicit=args[3])
nb = 1 << 20
n, k = eng.raw_block_size, eng.data_size
data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device="cuda")
raw = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
out = torch.empty_like(data)
st = torch.empty(nb, dtype=torch.uint8, device="cuda")
for _ in range(reps):
    eng.encode(data, raw, nblocks=nb)
err = len(sys.argv) > 4 and sys.argv[4] == "err"
col = raw.view(nb, n)[:, 100]
for _ in range(reps):
    if err:
        raw.view(nb, n)[:, 100] = col ^ 1
    eng.decode(raw, out, st, write_back=True, nblocks=nb)
torch.cuda.synchronize()
assert torch.equal(out, data)
print("ok", name, eng.kernel_name)
