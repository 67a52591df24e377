#!/usr/bin/env python3
"""Does running step k+1's encode beside step k's decode (two buffer sets, two streams) raise the
throughput of the encode + inject + decode step?  Prints one JSON line: ms per step with one stream
(the bench's form) and with the steps alternating over two streams, both verified.

usage: python tools/probes/overlap_probe.py [--steps 40] [--blocks 1048576]
"""
import argparse
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
    a = ap.parse_args()
    import torch

    from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine

    dev = torch.device("cuda", 0)
    eng = EccEngine(ECC_REED_SOLOMON, 512, 3)
    n, k, nb = eng.raw_block_size, eng.data_size, a.blocks
    g = torch.Generator(device=dev)
    g.manual_seed(0x50504653)
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=g)
    err_pos = torch.arange(nb, device=dev, dtype=torch.int64) * n + torch.randint(0, n, (nb,), device=dev, generator=g)
    err_val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
    sets = []
    for _ in range(2):
        cw = torch.empty(nb * n, dtype=torch.uint8, device=dev)
        sets.append((cw, torch.empty(nb * k, dtype=torch.uint8, device=dev), torch.empty(nb, dtype=torch.uint8, device=dev)))
    eng.encode(data, sets[0][0], nblocks=nb)
    bad = sets[0][0][err_pos] ^ err_val
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    default = torch.cuda.current_stream()

    def step(i, two):
        if two == "default":
            cw, out, st = sets[0]
            eng.encode(data, cw, nblocks=nb)
            cw.index_put_((err_pos,), bad)
            eng.decode(cw, out, st, write_back=True, nblocks=nb)
            return
        s = streams[i & 1] if two else streams[0]
        cw, out, st = sets[i & 1] if two else sets[0]
        with torch.cuda.stream(s):
            eng.encode(data, cw, nblocks=nb, stream=s)
            cw.index_put_((err_pos,), bad)
            eng.decode(cw, out, st, write_back=True, nblocks=nb, stream=s)

    res = {"default_is_null": default.cuda_stream == 0}
    for rnd in range(3):
        for two in ("default", False, True):
            t_end = time.perf_counter() + 0.3
            while time.perf_counter() < t_end:
                for i in range(8):
                    step(i, two)
                torch.cuda.synchronize()
            for i in range(5):
                step(i, two)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                step(i, two)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            ok = all(bool(torch.equal(o, data)) and int(s.min()) == 1 and int(s.max()) == 1
                     for (_, o, s) in (sets if two is True else sets[:1]))
            key = "default_stream" if two == "default" else ("two_streams" if two else "one_stream")
            res.setdefault(key, []).append(round(ms, 4))
            res.setdefault("verified", True)
            res["verified"] &= ok
    gib = 2 * nb * (k + n) / 2**30
    res["GiBps_one"] = [round(gib / (m / 1e3), 1) for m in res["one_stream"]]
    res["GiBps_two"] = [round(gib / (m / 1e3), 1) for m in res["two_streams"]]
    res["GiBps_default"] = [round(gib / (m / 1e3), 1) for m in res["default_stream"]]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
