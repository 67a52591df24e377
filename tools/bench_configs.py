#!/usr/bin/env python3
"""Per-configuration kernel throughput (device-resident), one JSON line per config.

BASELINE.json configs: cfg2/cfg3 RS(255,249) t=3 encode / 1-error decode, cfg4 Hamming and
CRC 0x9960034c at block_size 4096, cfg5 RS(255,223) t=16 (per-GPU shard of 2^20 blocks), plus
parity.  Each line: median kernel time over --reps launches (the kernels' dispatch-packet events),
algorithmic bytes per launch, GB/s and fraction of the 8 TB/s HBM peak.  Launches are timed
back to back (same kernel, same buffers) after a 0.3 s clock ramp, with fence-free HIP events.  A device-side round
trip check (decode(encode(x)) == x, status as expected) guards every config; bit-exactness vs
the oracle is tests/test_gpu_parity.py's job.

usage: python3 tools/bench_configs.py [--blocks N] [--reps R] [--only NAME]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 8000.0


def prewarm(fn, seconds):
    """Untimed back-to-back launches so the timed ones run at the sustained clock."""
    import time

    import torch

    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()


def timed_launch(he, i, fn):
    """One engine call whose kernel records events 2 i, 2 i + 1 from its own dispatch packet
    (ppfs_ecc_time_next_launch; bench.py's in-step timing): the kernel's duration, as rocprofv3
    reports it, without the launch gap."""
    from paritypartyfs_amd import _native

    L = _native.lib()
    L.ppfs_ecc_time_next_launch(he.ev[2 * i], he.ev[2 * i + 1])
    fn()
    L.ppfs_ecc_time_next_launch(None, None)


def med_ms(fn, reps, stream, warm_s=0.3):
    """Median kernel time over `reps` back-to-back launches (dispatch-packet events, timed_launch)."""
    import torch

    from bench import HipEvents

    prewarm(fn, warm_s)
    he = HipEvents(2 * reps)
    for i in range(reps):
        timed_launch(he, i, fn)
    torch.cuda.synchronize()
    r = float(np.median([he.ms(2 * i, 2 * i + 1) for i in range(reps)]))
    he.close()
    return r


# BASELINE.json configs measured by bench.py's `configs` leg (name, ecc_type, block_size, t, implicit CRC poly)
def baseline_configs():
    from paritypartyfs_amd import ECC_CRC, ECC_HAMMING, ECC_PARITY, ECC_REED_SOLOMON

    return [
        ("cfg2-3 rs255_t3 bs512", ECC_REED_SOLOMON, 512, 3, 0),
        ("cfg5 rs255_t16 bs4096", ECC_REED_SOLOMON, 4096, 16, 0),
        ("cfg4 hamming bs4096", ECC_HAMMING, 4096, 0, 0),
        ("cfg4 crc32 0x9960034c bs4096", ECC_CRC, 4096, 0, 0x9960034C),
        ("parity bs4096", ECC_PARITY, 4096, 0, 0),
        ("rs255_t8 bs255", ECC_REED_SOLOMON, 255, 8, 0),
    ]


def run_config(name, typ, bs, t, poly_implicit, nb, reps, stream, dev, warm_s=0.3):
    """One config over nb blocks: median back-to-back kernel times (encode, clean decode / check, and
    for RS / Hamming a 1-error decode with write-back, timed as bench.py's step times it: right after
    an untimed encode of the same batch and the one-byte-per-block injection -- round 4; it used to
    follow an untimed restore copy, which left other lines in the caches) and a device-side
    round-trip self-check.  Returns the JSON-able line."""
    import torch

    from bench import HipEvents
    from paritypartyfs_amd import ECC_HAMMING, ECC_REED_SOLOMON, EccEngine, crc_implicit_to_explicit

    poly = crc_implicit_to_explicit(poly_implicit) if poly_implicit else 0
    eng = EccEngine(typ, bs, t, crc_polynomial_explicit=poly, device=dev.index or 0)
    n, k = eng.raw_block_size, eng.data_size
    g = torch.Generator(device=dev)
    g.manual_seed(0x50504653)
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=g)
    raw = torch.zeros(nb * n, dtype=torch.uint8, device=dev)
    out = torch.empty(nb * k, dtype=torch.uint8, device=dev)
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    enc_ms = med_ms(lambda: eng.encode(data, raw, nblocks=nb), reps, stream, warm_s)
    clean = raw.clone()
    dec_clean_ms = med_ms(lambda: eng.decode(raw, out, st, write_back=True, nblocks=nb), reps, stream, warm_s)
    ok = bool(torch.equal(out, data)) and int(st.max()) == 0
    line = {"config": name, "blocks": nb, "raw": n, "data": k, "kernel_path": eng.kernel_name,
            "encode_ms": round(enc_ms, 4), "encode_GBps": round((k + n) * nb / enc_ms / 1e6, 1),
            "decode_clean_ms": round(dec_clean_ms, 4),
            "decode_clean_GBps": round((k + n) * nb / dec_clean_ms / 1e6, 1)}
    if typ == ECC_REED_SOLOMON or typ == ECC_HAMMING:
        pos = torch.arange(nb, device=dev, dtype=torch.int64) * n + torch.randint(0, n, (nb,), device=dev, generator=g)
        if typ == ECC_HAMMING:
            val = (1 << torch.randint(0, 8, (nb,), device=dev, generator=g)).to(torch.uint8)
        else:
            val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
        badb = clean[pos] ^ val  # the corrupted byte of every block

        def corrupt():  # as bench.py's step: fresh codewords by the encode, then one byte per block
            eng.encode(data, raw, nblocks=nb)
            raw.index_put_((pos,), badb)

        def dec1():
            corrupt()
            eng.decode(raw, out, st, write_back=True, nblocks=nb)

        prewarm(dec1, warm_s)
        he = HipEvents(2 * reps)
        for i in range(reps):
            corrupt()  # untimed: the decode is timed right after the encode + injection, in-step
            timed_launch(he, i, lambda: eng.decode(raw, out, st, write_back=True, nblocks=nb))
        torch.cuda.synchronize()
        dec_ms = float(np.median([he.ms(2 * i, 2 * i + 1) for i in range(reps)]))
        he.close()
        if typ == ECC_HAMMING:
            # a flip in an unused tail bit is not an error (status 0); every other one is
            ok = ok and bool(torch.equal(out, data)) and int(st.max()) <= 1
        else:
            ok = ok and bool(torch.equal(out, data)) and int(st.min()) == 1 and bool(torch.equal(raw, clean))
        line.update({"decode_1err_ms": round(dec_ms, 4), "decode_1err_GBps": round((k + n) * nb / dec_ms / 1e6, 1)})
    best = max(v for kk, v in line.items() if kk.endswith("GBps"))
    line["roofline_frac_encode"] = round(line["encode_GBps"] / PEAK, 4)
    line["roofline_frac_decode_clean"] = round(line["decode_clean_GBps"] / PEAK, 4)
    if "decode_1err_GBps" in line:
        line["roofline_frac_decode_1err"] = round(line["decode_1err_GBps"] / PEAK, 4)
    line["roofline_frac_best"] = round(best / PEAK, 4)
    line["roundtrip_ok"] = ok
    eng.close()
    del data, raw, out, st, clean
    torch.cuda.empty_cache()
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    import torch

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    for name, typ, bs, t, poly in baseline_configs():
        if a.only and a.only not in name:
            continue
        print(json.dumps(run_config(name, typ, bs, t, poly, a.blocks, a.reps, stream, dev)), flush=True)


if __name__ == "__main__":
    main()
