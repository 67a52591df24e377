"""host_path_probe.py -- the host entry points' wall time, repeated: ppfs_ecc_{encode,decode}_host over
2^20 blocks of one config, pageable and page-locked caller buffers, each call timed `--reps` times
(bench.py's host_inclusive leg times one call of each).  Prints one JSON line per (mode, op) with
every rep's GiB/s (algorithmic bytes: data + codeword per block).  Diagnostic, not shipped:
    python tools/probes/host_path_probe.py [--block-size 512 --t 3 --reps 5 --modes pinned,pageable]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine, pinned  # noqa: E402

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--block-size", type=int, default=512)
    ap.add_argument("--t", type=int, default=3)
    ap.add_argument("--nblocks", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="pinned,pageable")
    ap.add_argument("--from-torch", action="store_true", help="payload from a device tensor's .cpu() (as bench.py)")
    a = ap.parse_args()
    eng = EccEngine(ECC_REED_SOLOMON, a.block_size, a.t, device=0)
    k, n, nb = eng.data_size, eng.raw_block_size, a.nblocks
    rng = np.random.default_rng(5)
    hd = rng.integers(0, 256, nb * k, dtype=np.uint8)
    if a.from_torch:
        import torch

        hd = torch.from_numpy(hd).to("cuda:0").cpu().numpy()
    hraw = np.empty(nb * n, np.uint8)
    hout = np.empty(nb * k, np.uint8)
    hst = np.empty(nb, np.uint8)
    alg = (k + n) * nb
    for mode in a.modes.split(","):
        ctx = pinned(hd, hraw, hout, hst) if mode == "pinned" else None
        if ctx:
            ctx.__enter__()
        try:
            res = {"encode": [], "decode_1err": [], "decode_clean": []}
            eng.encode_host(hd, hraw)
            good = hraw.copy()
            pos = np.arange(nb) * n + (np.arange(nb) * 37) % n
            for _ in range(a.reps):
                t0 = time.perf_counter()
                eng.encode_host(hd, hraw)
                res["encode"].append(alg / (time.perf_counter() - t0) / GIB)
                hraw[pos] ^= 0x5A
                t0 = time.perf_counter()
                eng.decode_host(hraw, hout, hst, write_back=True)
                res["decode_1err"].append(alg / (time.perf_counter() - t0) / GIB)
                assert np.array_equal(hraw, good) and np.array_equal(hout, hd) and int(hst.min()) == 1
                t0 = time.perf_counter()
                eng.decode_host(hraw, hout, hst, write_back=True)
                res["decode_clean"].append(alg / (time.perf_counter() - t0) / GIB)
                assert int(hst.max()) == 0
        finally:
            if ctx:
                ctx.__exit__(None, None, None)
        for op, v in res.items():
            print(json.dumps({"mode": mode, "op": op, "bs": a.block_size, "t": a.t,
                              "GiBps": [round(x, 2) for x in v], "best": round(max(v), 2)}), flush=True)


if __name__ == "__main__":
    main()
