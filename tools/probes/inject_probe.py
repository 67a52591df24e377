#!/usr/bin/env python3
"""Cost of the bench step's error injection (one wrong byte per codeword, 2^20 codewords) in
different torch forms.  Prints one JSON line per form: median us over 50 launches."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import bench

    dev = torch.device("cuda", 0)
    nb, n = 1 << 20, 255
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    cw = torch.randint(0, 256, (nb * n,), dtype=torch.uint8, device=dev, generator=g)
    col = torch.randint(0, n, (nb,), device=dev, generator=g)
    pos = torch.arange(nb, device=dev, dtype=torch.int64) * n + col
    bad = cw[pos] ^ torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)
    v2 = cw.view(nb, n)
    col2 = col.view(nb, 1)
    bad2 = bad.view(nb, 1)
    rows = torch.arange(nb, device=dev)
    from paritypartyfs_amd import inject_bytes

    col8 = col.to(torch.uint8)
    xv = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=g)  # XOR twice: net no change
    forms = {
        "ppfs_inject": lambda: inject_bytes(cw, n, col8, bad),
        "ppfs_inject_xor2": lambda: (inject_bytes(cw, n, col8, xv, xor=True), inject_bytes(cw, n, col8, xv, xor=True)),
        "index_put_int64": lambda: cw.index_put_((pos,), bad),
        "scatter_dim1": lambda: v2.scatter_(1, col2, bad2),
        "adv_index_2d": lambda: v2.index_put_((rows, col), bad),
    }
    ref = None
    s = torch.cuda.current_stream()
    ev = bench.HipEvents(51)
    for name, f in forms.items():
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        ev.record(0, s)
        for i in range(50):
            f()
            ev.record(i + 1, s)
        torch.cuda.synchronize()
        us = float(np.median([ev.ms(i, i + 1) for i in range(50)])) * 1e3
        chk = int(torch.sum(cw[pos] != bad).item())
        print(json.dumps({"form": name, "median_us": round(us, 2), "mismatches": chk}), flush=True)


if __name__ == "__main__":
    main()
