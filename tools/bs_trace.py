#!/usr/bin/env python3
"""Per-phase cycle breakdown of the 2t = 32 decode (rs_bs.hpp rs_bs_decode_kernel) inside the cfg5 step.

Needs the profiling build: tools/build_alt.sh --product trace -DPPFS_TK_TRACE=1, then
  PPFS_ECC_LIB=paritypartyfs_amd/_lib/alt/libppfs_ecc_trace.so python tools/bs_trace.py
Runs encode + 1-byte inject + decode-with-write-back steps (bench.py's cfg5 step), then reads the
last decode launch's per-wave phase sums and prints their means (cycles per wave, per tile, and
share), one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["prologue", "dma_wait", "cmodg", "s12_logs", "xp_confirm", "fix", "status", "emission", "free_dma"]
N = 13


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--clean", action="store_true", help="no injected errors")
    a = ap.parse_args()
    import torch

    from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine, _native, inject_bytes

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    eng = EccEngine(ECC_REED_SOLOMON, 4096, 16)
    n, k, nb = eng.raw_block_size, eng.data_size, a.blocks
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=g)
    cw = torch.empty(nb * n, dtype=torch.uint8, device=dev)
    out = torch.empty(nb * k, dtype=torch.uint8, device=dev)
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    col = torch.randint(0, n, (nb,), device=dev, generator=g).to(torch.uint8)
    val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)

    def step():
        eng.encode(data, cw, nblocks=nb)
        if not a.clean:
            inject_bytes(cw, n, col, val, nblocks=nb, xor=True)
        eng.decode(cw, out, st, write_back=True, nblocks=nb)

    t_end = time.perf_counter() + a.seconds
    while time.perf_counter() < t_end:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
    step()
    torch.cuda.synchronize()
    L = _native.lib()
    fn = L.ppfs_bs_trace_read
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(4096 * N, np.uint64)
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    tr = buf.reshape(4096, N)
    gw = np.nonzero(tr[:, 10] > 0)[0]  # wave index blockIdx * NW + wave (NW = 8)
    tr = tr[tr[:, 10] > 0]
    t0, t1 = tr[:, 11].astype(np.int64), tr[:, 12].astype(np.int64)  # 100 MHz realtime, per wave
    base = t0.min()
    xcd = (gw // 8) % 8  # workgroups go round-robin over the 8 XCDs
    per_xcd = {int(x): [round(float(np.percentile(t1[xcd == x] - base, q)) / 100.0, 1) for q in (0, 50, 100)]
               for x in range(8)}
    cu = gw // 8
    per_cu_spread = np.array([(t1[cu == c].max() - t1[cu == c].min()) / 100.0 for c in np.unique(cu)])
    tail = {"span_us": round((t1.max() - base) / 100.0, 2), "start_spread_us": round((t0.max() - base) / 100.0, 2),
            "end_us": {q: round(float(np.percentile(t1 - base, q)) / 100.0, 2) for q in (0, 10, 50, 90, 100)},
            "end_us_by_xcd_min_med_max": per_xcd,
            "within_cu_end_spread_us_median": round(float(np.median(per_cu_spread)), 2)}
    tr = tr.astype(np.float64)
    tot = tr[:, 10].mean()
    iters = tr[:, 9].sum()
    res = {"blocks": nb, "mode": "clean" if a.clean else "1-error", "waves": len(tr), "total_cycles": round(tot),
           "tiles_per_wave": round(tr[:, 9].mean(), 2),
           "share": {p: round(tr[:, i].mean() / tot, 3) for i, p in enumerate(PHASES)},
           "per_tile": {p: round(tr[:, i].sum() / max(1.0, iters)) for i, p in enumerate(PHASES) if i > 0},
           "realtime": tail}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
