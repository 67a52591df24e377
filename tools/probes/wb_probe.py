"""wb_probe.py -- where a 1-error decode's extra time goes: the decode's own correction / write-back
work, or the one-byte-per-block injection that precedes it (its 2^20 partial-sector writes still
in flight or dirty in the caches when the decode reads the same lines).  Each variant is the
median kernel time of the decode (dispatch-packet events, tools/bench_configs.timed_launch) after:
  clean        encode                                   -> decode (write-back)
  clean_flush  encode, 1 GiB unrelated copy              -> decode
  err          encode, injection                         -> decode (write-back)   [bench_configs]
  err_nowb     encode, injection                         -> decode (no write-back)
  err_flush    encode, injection, 1 GiB unrelated copy   -> decode (write-back)
Diagnostic, not shipped:  python tools/probes/wb_probe.py [--only hamming|rs3|rs16]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from bench import HipEvents
    from paritypartyfs_amd import ECC_HAMMING, ECC_REED_SOLOMON, EccEngine
    from tools.bench_configs import prewarm, timed_launch

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--blocks", type=int, default=1 << 20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfgs = [("hamming", ECC_HAMMING, 4096, 0), ("rs3", ECC_REED_SOLOMON, 512, 3), ("rs16", ECC_REED_SOLOMON, 4096, 16)]
    fa = torch.empty(1 << 29, dtype=torch.uint8, device=dev)
    fb = torch.empty(1 << 29, dtype=torch.uint8, device=dev)
    for name, typ, bs, t in cfgs:
        if a.only and a.only != name:
            continue
        eng = EccEngine(typ, bs, t, device=0)
        n, k, nb = eng.raw_block_size, eng.data_size, a.blocks
        g = torch.Generator(device=dev)
        g.manual_seed(7)
        data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=g)
        raw = torch.zeros(nb * n, dtype=torch.uint8, device=dev)
        out = torch.empty(nb * k, dtype=torch.uint8, device=dev)
        st = torch.empty(nb, dtype=torch.uint8, device=dev)
        eng.encode(data, raw, nblocks=nb)
        clean = raw.clone()
        pos = torch.arange(nb, device=dev, dtype=torch.int64) * n + torch.randint(0, n, (nb,), device=dev, generator=g)
        if typ == ECC_HAMMING:
            val = (1 << torch.randint(0, 8, (nb,), device=dev, generator=g)).to(torch.uint8)
        else:
            val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
        badb = clean[pos] ^ val

        def enc():
            eng.encode(data, raw, nblocks=nb)

        def inj():
            raw.index_put_((pos,), badb)

        def flush():
            fb.copy_(fa)

        variants = {
            "clean": ([enc], True),
            "clean_flush": ([enc, flush], True),
            "err": ([enc, inj], True),
            "err_nowb": ([enc, inj], False),
            "err_flush": ([enc, inj, flush], True),
        }
        res = {}
        for vn, (pre, wb) in variants.items():
            def step():
                for f in pre:
                    f()
                eng.decode(raw, out, st, write_back=wb, nblocks=nb)

            prewarm(step, 0.3)
            he = HipEvents(2 * a.reps)
            for i in range(a.reps):
                for f in pre:
                    f()
                timed_launch(he, i, lambda: eng.decode(raw, out, st, write_back=wb, nblocks=nb))
            torch.cuda.synchronize()
            res[vn] = round(float(np.median([he.ms(2 * i, 2 * i + 1) for i in range(a.reps)])) * 1e3, 1)
            he.close()
            assert torch.equal(out, data), (name, vn)
        print(json.dumps({"config": name, "blocks": nb, "decode_us": res}), flush=True)
        eng.close()
        del data, raw, out, st, clean
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
