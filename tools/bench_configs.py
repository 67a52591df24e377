#!/usr/bin/env python3
"""Per-configuration kernel throughput (device-resident), one JSON line per config.

BASELINE.json configs: cfg2/cfg3 RS(255,249) t=3 encode / 1-error decode, cfg4 Hamming and
CRC 0x9960034c at block_size 4096, cfg5 RS(255,223) t=16 (per-GPU shard of 2^20 blocks), plus
parity.  Each line: median kernel time over --reps launches (the kernels' dispatch-packet events),
algorithmic bytes per launch, GB/s and fraction of the 8 TB/s HBM peak.

Cold caches (round 6): encodes and clean decodes rotate over buffer sets whose bytes between two
uses of one set exceed the 256 MiB Infinity Cache (MI355X_MICROARCH.md), so no launch reads its
input from the previous launch's lines (round 5 timed them on the same buffers: cfg5's 234 MB
payload then encoded 18 % faster than inside its own bench step).  1-error decodes are timed as
bench.py's step times them: right after an untimed encode of the same batch and the
one-byte-per-block injection.  `step_leg` times a whole bench step (encode -> inject -> decode)
of any RS shape, K steps back to back: bench.py reports it for cfg5 (configs[4]'s shard) beside
the headline, so the driver's line carries cfg5's in-step numbers.

A device-side round trip check (decode(encode(x)) == x, status as expected) guards every config;
bit-exactness vs the oracle is tests/test_gpu_parity.py's job.

usage: python3 tools/bench_configs.py [--blocks N] [--reps R] [--only NAME] [--step-leg]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 8000.0
IC_BYTES = 256 << 20  # Infinity Cache (MI355X_MICROARCH.md)


def rotation_sets(set_bytes, most=4):
    """Buffer sets to rotate over so that the bytes moved between two uses of one set are at least
    twice the Infinity Cache: (R - 1) x set_bytes > 512 MiB (one set when a single set is already 4x
    the cache, e.g. cfg4's 8.6 GB; RS(255,249) and RS(255,223) at 2^20 blocks: 3 sets)."""
    if set_bytes >= 4 * IC_BYTES:
        return 1
    r = 2
    while (r - 1) * set_bytes <= 2 * IC_BYTES and r < most:
        r += 1
    return r


def prewarm(fn, seconds):
    """Untimed back-to-back launches so the timed ones run at the sustained clock."""
    import time

    import torch

    t_end = time.perf_counter() + seconds
    i = 0
    while time.perf_counter() < t_end:
        for _ in range(8):
            fn(i)
            i += 1
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


def med_ms(fn, reps, warm_s=0.3, pre=None):
    """Median kernel time over `reps` launches fn(i) (dispatch-packet events, timed_launch); pre(i),
    untimed, is queued before launch i."""
    import torch

    from bench import HipEvents

    prewarm(lambda i: (pre(i) if pre else None, fn(i)), warm_s)
    he = HipEvents(2 * reps)
    for i in range(reps):
        if pre:
            pre(i)
        timed_launch(he, i, lambda: fn(i))
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


def _rate(nb, k, n, ms):
    return round((k + n) * nb / ms / 1e6, 1)


def config_line(name, nb, n, k, kernel_path, sets, enc_ms, dec_clean_ms, dec_1err_ms=None, ok=True):
    """The JSON line of one config from its kernel times (ms): GB/s and fraction of 8 TB/s per leg.
    Pure bookkeeping (tests/test_bench_records.py checks its fields on CPU)."""
    line = {"config": name, "blocks": nb, "raw": n, "data": k, "kernel_path": kernel_path,
            "cold_sets": sets,
            "encode_ms": round(enc_ms, 4), "encode_GBps": _rate(nb, k, n, enc_ms),
            "decode_clean_ms": round(dec_clean_ms, 4), "decode_clean_GBps": _rate(nb, k, n, dec_clean_ms)}
    if dec_1err_ms is not None:
        line.update({"decode_1err_ms": round(dec_1err_ms, 4), "decode_1err_GBps": _rate(nb, k, n, dec_1err_ms)})
    line["roofline_frac_encode"] = round(line["encode_GBps"] / PEAK, 4)
    line["roofline_frac_decode_clean"] = round(line["decode_clean_GBps"] / PEAK, 4)
    if dec_1err_ms is not None:
        line["roofline_frac_decode_1err"] = round(line["decode_1err_GBps"] / PEAK, 4)
    line["roundtrip_ok"] = bool(ok)
    return line


def run_config(name, typ, bs, t, poly_implicit, nb, reps, stream, dev, warm_s=0.3):
    """One config over nb blocks: median kernel times of the encode and the clean decode / check,
    each rotating over cold buffer sets (rotation_sets), and for RS / Hamming a 1-error decode with
    write-back timed in-step (after an untimed encode + injection of the same batch); a device-side
    round-trip self-check.  Returns the JSON-able line."""
    import torch

    from paritypartyfs_amd import ECC_HAMMING, ECC_REED_SOLOMON, EccEngine, crc_implicit_to_explicit

    poly = crc_implicit_to_explicit(poly_implicit) if poly_implicit else 0
    eng = EccEngine(typ, bs, t, crc_polynomial_explicit=poly, device=dev.index or 0)
    n, k = eng.raw_block_size, eng.data_size
    R = rotation_sets(nb * (k + n))
    g = torch.Generator(device=dev)
    g.manual_seed(0x50504653)
    data = [torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=g) for _ in range(R)]
    raw = [torch.zeros(nb * n, dtype=torch.uint8, device=dev) for _ in range(R)]
    out = [torch.empty(nb * k, dtype=torch.uint8, device=dev) for _ in range(R)]
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    enc_ms = med_ms(lambda i: eng.encode(data[i % R], raw[i % R], nblocks=nb), reps, warm_s)
    clean = raw[0].clone()
    dec_clean_ms = med_ms(lambda i: eng.decode(raw[i % R], out[i % R], st, write_back=True, nblocks=nb), reps, warm_s)
    ok = all(bool(torch.equal(out[j], data[j])) for j in range(R)) and int(st.max()) == 0
    dec_ms = None
    if typ == ECC_REED_SOLOMON or typ == ECC_HAMMING:
        pos = torch.arange(nb, device=dev, dtype=torch.int64) * n + torch.randint(0, n, (nb,), device=dev, generator=g)
        if typ == ECC_HAMMING:
            val = (1 << torch.randint(0, 8, (nb,), device=dev, generator=g)).to(torch.uint8)
        else:
            val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
        badb = clean[pos] ^ val  # the corrupted byte of every block of set 0

        def corrupt(i):  # as bench.py's step: fresh codewords by the encode, then one byte per block
            eng.encode(data[0], raw[0], nblocks=nb)
            raw[0].index_put_((pos,), badb)

        dec_ms = med_ms(lambda i: eng.decode(raw[0], out[0], st, write_back=True, nblocks=nb), reps, warm_s, pre=corrupt)
        if typ == ECC_HAMMING:
            # a flip in an unused tail bit is not an error (status 0); every other one is
            ok = ok and bool(torch.equal(out[0], data[0])) and int(st.max()) <= 1
        else:
            ok = ok and bool(torch.equal(out[0], data[0])) and int(st.min()) == 1 and bool(torch.equal(raw[0], clean))
    line = config_line(name, nb, n, k, eng.kernel_name, R, enc_ms, dec_clean_ms, dec_ms, ok)
    eng.close()
    del data, raw, out, st, clean
    torch.cuda.empty_cache()
    return line


def step_line(bs, t, nb, n, k, steps, enc_ms, dec_ms, inj_ms, step_ms, ok):
    """The JSON line of a step leg from its per-step kernel means (ms).  Pure bookkeeping."""
    alg = (k + n) * nb
    fr = lambda ms: round(alg / (ms * 1e-3) / 1e9 / PEAK, 4)  # noqa: E731
    return {"workload": f"RS({n},{k}) t={t} block_size={bs}: encode + 1-byte-error inject + decode with write-back",
            "blocks": nb, "steps": steps,
            "kernels_ms": {"encode": round(enc_ms, 5), "inject": round(inj_ms, 5), "decode": round(dec_ms, 5)},
            "in_step_frac": {"encode": fr(enc_ms), "decode": fr(dec_ms)},
            "ms_per_step": round(step_ms, 5),
            "GiBps": round(2 * alg / (step_ms * 1e-3) / (1 << 30), 3),
            "verified": bool(ok)}


def step_leg(bs, t, nb, steps, dev, stream, warm_s=0.5):
    """K bench steps of RS(block_size, t) back to back (bench.py's step: encode -> one-byte-per-block
    injection by the engine's kernel -> decode with write-back and status), each kernel timed by its
    dispatch-packet events, the step by stream events around the K steps."""
    import time

    import torch

    from bench import HipEvents
    from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine, _native, inject_bytes

    NL = _native.lib()
    eng = EccEngine(ECC_REED_SOLOMON, bs, t, device=dev.index or 0)
    n, k = eng.raw_block_size, eng.data_size
    g = torch.Generator(device=dev)
    g.manual_seed(0x50504653 ^ 0x5)
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=g)
    cw = torch.empty(nb * n, dtype=torch.uint8, device=dev)
    out = torch.empty(nb * k, dtype=torch.uint8, device=dev)
    status = torch.empty(nb, dtype=torch.uint8, device=dev)
    col = torch.randint(0, n, (nb,), device=dev, generator=g)
    val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
    eng.encode(data, cw, nblocks=nb)
    bad = cw[torch.arange(nb, device=dev, dtype=torch.int64) * n + col] ^ val
    col8 = col.to(torch.uint8)

    def step():
        eng.encode(data, cw, nblocks=nb)
        inject_bytes(cw, n, col8, bad, nblocks=nb)
        eng.decode(cw, out, status, write_back=True, nblocks=nb)

    t_end = time.perf_counter() + warm_s
    while time.perf_counter() < t_end:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
    he = HipEvents(4 * steps + 2)
    hk = HipEvents(4 * steps)
    he.record(4 * steps, stream)
    for i in range(steps):
        NL.ppfs_ecc_time_next_launch(hk.ev[4 * i], hk.ev[4 * i + 1])
        eng.encode(data, cw, nblocks=nb)
        NL.ppfs_ecc_time_next_launch(None, None)
        he.record(4 * i + 1, stream)
        inject_bytes(cw, n, col8, bad, nblocks=nb)
        he.record(4 * i + 2, stream)
        NL.ppfs_ecc_time_next_launch(hk.ev[4 * i + 2], hk.ev[4 * i + 3])
        eng.decode(cw, out, status, write_back=True, nblocks=nb)
        NL.ppfs_ecc_time_next_launch(None, None)
    he.record(4 * steps + 1, stream)
    torch.cuda.synchronize()
    enc = float(np.mean([hk.ms(4 * i, 4 * i + 1) for i in range(steps)]))
    dec = float(np.mean([hk.ms(4 * i + 2, 4 * i + 3) for i in range(steps)]))
    inj = float(np.mean([he.ms(4 * i + 1, 4 * i + 2) for i in range(steps)]))
    step_ms = he.ms(4 * steps, 4 * steps + 1) / steps
    he.close()
    hk.close()
    ok = bool(torch.equal(out, data)) and int(status.min()) == 1 and int(status.max()) == 1
    line = step_line(bs, t, nb, n, k, steps, enc, dec, inj, step_ms, ok)
    line["kernel_path"] = eng.stream_kernel_name(stream)
    eng.close()
    del data, cw, out, status
    torch.cuda.empty_cache()
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--step-leg", action="store_true", help="also the cfg5 step leg (bench.py's configs.cfg5_step)")
    a = ap.parse_args()
    import torch

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    for name, typ, bs, t, poly in baseline_configs():
        if a.only and a.only not in name:
            continue
        print(json.dumps(run_config(name, typ, bs, t, poly, a.blocks, a.reps, stream, dev)), flush=True)
    if a.step_leg:
        print(json.dumps(step_leg(4096, 16, a.blocks, a.reps, dev, stream)), flush=True)


if __name__ == "__main__":
    main()
