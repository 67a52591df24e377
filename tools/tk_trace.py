#!/usr/bin/env python3
"""Per-phase cycle breakdown of the ticket-counter encode (rs_wg_tk.hpp) inside the bench step.

Needs the profiling build: tools/build_alt.sh --product trace -DPPFS_TK_TRACE=1, then
  PPFS_ECC_LIB=paritypartyfs_amd/_lib/alt/libppfs_ecc_trace.so python tools/tk_trace.py
Runs encode + inject + decode steps (bench.py's step) for --seconds, then reads the last encode
launch's per-workgroup sums (waves 0 and 1: wave 0 takes the tickets, wave 1 issues tile DMA) and
prints their means in cycles and as a share of the workgroup's time, one JSON line.
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

PHASES = ["prologue", "issue", "remainder", "barrier_B", "emission", "vm_wait", "barrier_A", "epilogue"]
PHASES_DEC = ["prologue", "issue", "remainder", "barrier_B", "correction", "emission", "vm_wait", "barrier_A"]
N = 12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--standalone", action="store_true", help="encode launches alone (no inject / decode)")
    a = ap.parse_args()
    import torch

    from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine, _native, inject_bytes

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
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
        if not a.standalone:
            inject_bytes(cw, n, col, val, nblocks=nb, xor=True)
            eng.decode(cw, out, st, write_back=True, nblocks=nb)

    t_end = time.perf_counter() + a.seconds
    while time.perf_counter() < t_end:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
    # the last launches' traces: the encode's and (in-step) the decode's sums of the final step
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    L = _native.lib()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    res = {"blocks": nb, "mode": "standalone" if a.standalone else "in-step"}

    def read(fname, wpc, phases, key):
        fn = getattr(L, fname)
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        buf = np.zeros(4096 * 2 * N, np.uint64)
        rc = fn(buf.ctypes.data, buf.nbytes)
        assert rc == 0, rc
        grid = wpc * cus
        tr = buf.reshape(4096, 2, N)[:grid].astype(np.float64)
        out = {"grid": grid}
        for w, name in ((0, "wave0"), (1, "wave1_dma")):
            t = tr[:, w, :]
            tot = t[:, 9].mean()
            out[name] = {"total_cycles": round(tot), "iterations": round(t[:, 8].mean(), 2),
                         "share": {p: round(t[:, i].mean() / tot, 3) for i, p in enumerate(phases)},
                         "per_iter": {p: round(t[:, i].sum() / max(1.0, t[:, 8].sum())) for i, p in enumerate(phases)
                                      if i > 0}}
        # workgroup ends on the realtime clock (wave 0's stamp): the tail
        t0, t1 = buf.reshape(4096, 2, N)[:grid, 0, 10].astype(np.int64), buf.reshape(4096, 2, N)[:grid, 0, 11].astype(np.int64)
        base = t0.min()
        xcd = np.arange(grid) % 8
        out["realtime"] = {"span_us": round((t1.max() - base) / 100.0, 2),
                           "end_us": {q: round(float(np.percentile(t1 - base, q)) / 100.0, 2) for q in (0, 10, 50, 90, 100)},
                           "end_us_by_xcd_min_med_max": {int(x): [round(float(np.percentile(t1[xcd == x] - base, q)) / 100.0, 1)
                                                             for q in (0, 50, 100)] for x in range(8)}}
        res[key] = out

    read("ppfs_tk_trace_read_t6", 2, PHASES, "encode")
    if not a.standalone:
        read("ppfs_tk_trace_dec_read_t6", 3, PHASES_DEC, "decode")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
