#!/usr/bin/env python3
"""Standalone kernel timings of one engine build (PPFS_ECC_LIB), without output checks, for
ablation builds whose outputs are wrong on purpose (rs_wg.hpp MODE bits, tools/build_alt.sh).

usage: PPFS_ECC_LIB=... python tools/probes/kernel_ablate.py [--block-size 512 --t 3] [--tag name]
Prints one JSON line: median ms of L back-to-back launches, hot (same buffers) and cold (4 rotating
buffer sets), for encode and clean decode (status + write-back on).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--block-size", type=int, default=512)
    ap.add_argument("--t", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("PPFS_ECC_LIB", "default")))
    a = ap.parse_args()
    import torch

    import bench
    from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = EccEngine(ECC_REED_SOLOMON, a.block_size, a.t)
    n, k, nb = eng.raw_block_size, eng.data_size, a.blocks
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    R = 4
    d = [torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=g) for _ in range(R)]
    c = [torch.empty(nb * n, dtype=torch.uint8, device=dev) for _ in range(R)]
    o = [torch.empty(nb * k, dtype=torch.uint8, device=dev) for _ in range(R)]
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    ev = bench.HipEvents(a.launches + 1)

    def timed(fn, warm_s=0.3):
        t_end = time.perf_counter() + warm_s
        while time.perf_counter() < t_end:
            for i in range(8):
                fn(i)
            torch.cuda.synchronize()
        ev.record(0, s)
        for i in range(a.launches):
            fn(i)
            ev.record(i + 1, s)
        torch.cuda.synchronize()
        return round(float(np.median([ev.ms(i, i + 1) for i in range(a.launches)])) * 1e3, 2)

    res = {"tag": a.tag, "kernel": eng.kernel_name}
    res["enc_hot_us"] = timed(lambda i: eng.encode(d[0], c[0]))
    res["enc_cold_us"] = timed(lambda i: eng.encode(d[i % R], c[i % R]))
    for i in range(R):
        eng.encode(d[i], c[i])
    res["dec_hot_us"] = timed(lambda i: eng.decode(c[0], o[0], st, write_back=True))
    res["dec_cold_us"] = timed(lambda i: eng.decode(c[i % R], o[i % R], st, write_back=True))
    # one byte error per codeword, no write-back (the errors stay): the correction's cost
    res["dec_clean_nowb_hot_us"] = timed(lambda i: eng.decode(c[0], o[0], st, write_back=False))
    pos = torch.arange(nb, device=dev, dtype=torch.int64) * n + torch.randint(0, n, (nb,), device=dev, generator=g)
    bad = c[1].clone()
    bad[pos] ^= torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
    res["dec_1err_nowb_hot_us"] = timed(lambda i: eng.decode(bad, o[0], st, write_back=False))
    assert int((st == 1).sum().item()) == nb  # every block corrected
    alg = (n + k) * nb
    for key in ("enc_hot_us", "enc_cold_us", "dec_hot_us", "dec_cold_us", "dec_1err_nowb_hot_us"):
        res[key.replace("_us", "_frac")] = round(alg / (res[key] * 1e-6) / 8e12, 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
