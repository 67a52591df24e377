#!/usr/bin/env python3
"""Host-inclusive rates (BASELINE north_star: the path starts and ends in host memory).

RS(255,249) t=3, 2^20 blocks: encode_host, decode_host (1 error per block, payload + status out,
write-back) and scrub_host over numpy buffers, and decode_host / scrub_host of clean codewords, pageable (one CPU copy each way through the
library's pinned staging) and page-locked (ppfs_ecc_host_register: direct DMA).  GiB/s =
algorithmic bytes (payload + codeword per block) / wall time; median of --reps.  One JSON line
per (operation, memory kind).

--devices 0,0,...: run encode / decode through an EccGroup (ppfs_ecc_group_*: contiguous shards,
one host thread per listed device; the scrub rows are single-context).

usage: python3 tools/probes/bench_host.py [--blocks N] [--reps R] [--devices D0,D1,...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--devices", default=None)
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime order, see paritypartyfs_amd/_native.py)

    from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine, EccGroup, pinned

    nb = a.blocks
    eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
    devs = tuple(int(x) for x in a.devices.split(",")) if a.devices else None
    grp = EccGroup(ECC_REED_SOLOMON, 512, 3, devices=devs) if devs else eng
    n, k = eng.raw_block_size, eng.data_size
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, nb * k, dtype=np.uint8)
    raw = np.zeros(nb * n, np.uint8)
    eng.encode_host(data, raw)
    clean = raw.copy()
    pos = rng.integers(0, n, nb) + np.arange(nb) * n
    bad = clean.copy()
    bad[pos] ^= rng.integers(1, 256, nb, dtype=np.uint8)
    out = np.empty(nb * k, np.uint8)
    st = np.empty(nb, np.uint8)
    gib = 2.0 ** 30

    def timed(fn, prep):
        ts = []
        for _ in range(a.reps):
            prep()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    for kind in ("pageable", "pinned"):
        ctx = pinned(data, raw, out, st) if kind == "pinned" else None
        if ctx:
            ctx.__enter__()
        try:
            t_enc = timed(lambda: grp.encode_host(data, raw), lambda: None)
            assert np.array_equal(raw, clean)
            t_dec = timed(lambda: grp.decode_host(raw, out, st, write_back=True), lambda: np.copyto(raw, bad))
            assert np.array_equal(out, data) and np.array_equal(raw, clean) and bool((st == 1).all())
            t_scr = timed(lambda: eng.scrub_host(raw, nblocks=nb, status=st), lambda: np.copyto(raw, bad))
            assert np.array_equal(raw, clean)
            # clean codewords (the common read): nothing changes, no codeword comes back
            t_decc = timed(lambda: grp.decode_host(raw, out, st, write_back=True), lambda: None)
            assert np.array_equal(out, data) and np.array_equal(raw, clean) and not st.any()
            t_scrc = timed(lambda: eng.scrub_host(raw, nblocks=nb, status=st), lambda: None)
        finally:
            if ctx:
                ctx.__exit__(None, None, None)
        per = nb * (n + k)
        for op, t in (("encode_host", t_enc), ("decode_host", t_dec), ("scrub_host", t_scr),
                      ("decode_host_clean", t_decc), ("scrub_host_clean", t_scrc)):
            by = per if not op.startswith("scrub_host") else nb * n * 2
            print(json.dumps({"op": op, "memory": kind, "blocks": nb, "devices": list(devs) if devs and
                              not op.startswith("scrub") else [0], "ms": round(t * 1e3, 3),
                              "GiB_per_s": round(by / t / gib, 2)}), flush=True)


if __name__ == "__main__":
    main()
