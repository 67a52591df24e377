#!/usr/bin/env python3
"""Does the bench step's fault injection hide behind the previous batch's decode?  Two buffer
sets; encode and decode on one stream, the injection on a second stream, so that batch k's
injection runs beside batch k-1's decode.  Prints one JSON line per form (ms per step, verified):
  seq   encode(A) inject(A) decode(A) per step, one stream (bench.py's form)
  pipe  S1: encode(X_k), decode(X_{k-1});  S2: inject(X_k) after encode(X_k); the decode of X_k
        waits for its injection (fence-free HIP events for the cross-stream waits)

usage: python tools/probes/inject_overlap_probe.py [--steps 40] [--block-size 512 --t 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--block-size", type=int, default=512)
    ap.add_argument("--t", type=int, default=3)
    a = ap.parse_args()
    import torch

    import bench
    from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine, inject_bytes

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    eng = EccEngine(ECC_REED_SOLOMON, a.block_size, a.t)
    n, k, nb = eng.raw_block_size, eng.data_size, a.blocks
    g = torch.Generator(device=dev)
    g.manual_seed(0x50504653)
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=g)
    col = torch.randint(0, n, (nb,), device=dev, generator=g)
    pos = torch.arange(nb, device=dev, dtype=torch.int64) * n + col
    col8 = col.to(torch.uint8)
    sets = [(torch.empty(nb * n, dtype=torch.uint8, device=dev), torch.empty(nb * k, dtype=torch.uint8, device=dev),
             torch.empty(nb, dtype=torch.uint8, device=dev)) for _ in range(2)]
    eng.encode(data, sets[0][0], nblocks=nb)
    bad = sets[0][0][pos] ^ torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    K = a.steps
    ev = bench.HipEvents(2 * K + 4)
    L = ev.L

    def wait(stream, i):
        rc = L.hipStreamWaitEvent(ctypes.c_void_p(stream.cuda_stream), ev.ev[i], ctypes.c_uint(0))
        assert rc == 0, rc

    def seq(kk):
        cw, out, st = sets[0]
        for _ in range(kk):
            eng.encode(data, cw, nblocks=nb, stream=s1)
            inject_bytes(cw, n, col8, bad, nblocks=nb, stream=s1)
            eng.decode(cw, out, st, write_back=True, nblocks=nb, stream=s1)

    def pipe(kk):
        # event 2i = encode(X_i) done (s1), 2i+1 = inject(X_i) done (s2)
        for i in range(kk + 1):
            if i < kk:
                cw = sets[i & 1][0]
                eng.encode(data, cw, nblocks=nb, stream=s1)
                ev.record(2 * i, s1)
                wait(s2, 2 * i)
                inject_bytes(cw, n, col8, bad, nblocks=nb, stream=s2)
                ev.record(2 * i + 1, s2)
            if i >= 1:
                cwp, outp, stp = sets[(i - 1) & 1]
                wait(s1, 2 * (i - 1) + 1)
                eng.decode(cwp, outp, stp, write_back=True, nblocks=nb, stream=s1)

    for name, fn in (("seq", seq), ("pipe", pipe), ("seq", seq), ("pipe", pipe)):
        t_end = time.perf_counter() + 0.5
        while time.perf_counter() < t_end:
            fn(4)
            torch.cuda.synchronize()
        for cw, out, st in sets:
            out.zero_()
            st.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(K)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / K * 1e3
        used = sets[:1] if name == "seq" else sets
        ok = all(bool(torch.equal(out, data)) and int(st.min()) == 1 and int(st.max()) == 1 for _, out, st in used)
        print(json.dumps({"form": name, "ms_per_step": round(ms, 4), "verified": ok, "steps": K,
                          "GiBps": round(2 * (n + k) * nb / (ms * 1e-3) / (1 << 30), 1)}), flush=True)
    ev.close()


if __name__ == "__main__":
    main()
