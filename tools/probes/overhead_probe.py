#!/usr/bin/env python3
"""Where does the timed region's fixed overhead come from?  (bench.py: wall ms_per_step exceeded
the device time of the same steps by 0.5-1 ms per 20-step region in r1/r2a.)

For K in a few sizes, eager steps of the bench workload, timed several ways:
  wall_sync      barrier-free bench form: torch.cuda.synchronize(); t0; K steps; synchronize(); t1
  wall_issue     host time to issue the K steps (t0 -> after the last launch returns)
  dev            fence-free HIP events around the same K steps (GPU time from first to last)
  wall_evspin    same steps, the end detected by spinning on hipEventQuery instead of a blocking sync
  first_lat      host time from t0 until an event recorded right after the FIRST kernel completes,
                 minus that kernel's device time (= the GPU start latency of the region)
Prints one JSON line per (variant, K).
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
    n, k = eng.raw_block_size, eng.data_size
    nb = 1 << 20
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=g)
    cw = torch.empty(nb * n, dtype=torch.uint8, device=dev)
    out = torch.empty(nb * k, dtype=torch.uint8, device=dev)
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    pos = torch.arange(nb, device=dev, dtype=torch.int64) * n + torch.randint(0, n, (nb,), device=dev, generator=g)
    eng.encode(data, cw)
    bad = cw[pos] ^ 0x5A
    s = torch.cuda.current_stream()
    L = ctypes.CDLL("libamdhip64.so")

    def step():
        eng.encode(data, cw)
        cw.index_put_((pos,), bad)
        eng.decode(cw, out, st, write_back=True)

    t_end = time.perf_counter() + 1.0
    while time.perf_counter() < t_end:
        for _ in range(16):
            step()
        torch.cuda.synchronize()
    ev = bench.HipEvents(4)
    for K in (1, 2, 5, 10, 20, 50):
        rows = {"wall_sync": [], "wall_issue": [], "dev": [], "wall_evspin": [], "first_lat": [], "sync_only": []}
        for rep in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev.record(0, s)
            for _ in range(K):
                step()
            ev.record(1, s)
            t_issue = time.perf_counter()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            rows["wall_sync"].append((t1 - t0) * 1e3)
            rows["wall_issue"].append((t_issue - t0) * 1e3)
            rows["dev"].append(ev.ms(0, 1))
            # end by spinning on the event
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(K):
                step()
            ev.record(2, s)
            while L.hipEventQuery(ev.ev[2]) != 0:
                pass
            rows["wall_evspin"].append((time.perf_counter() - t0) * 1e3)
            # GPU start latency: first encode, then spin until it is done
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev.record(0, s)
            eng.encode(data, cw)
            ev.record(3, s)
            while L.hipEventQuery(ev.ev[3]) != 0:
                pass
            t1 = time.perf_counter()
            rows["first_lat"].append((t1 - t0) * 1e3 - ev.ms(0, 3))
            # an empty synchronize
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            rows["sync_only"].append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"K": K, **{a: round(float(np.median(b)), 4) for a, b in rows.items()}}), flush=True)


if __name__ == "__main__":
    main()
