#!/usr/bin/env python3
"""bench.py -- device-resident RS encode+decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]/[2]): ecc_type=reed_solomon, block_size=512,
rs_correctable_bytes=3 -> RS(255,249) (the reference clamps codewords to 255 B,
rs_block_device.cpp:57), 2^20 blocks per GPU, synthetic uniform payloads.

One step = encode(2^20 payloads -> codewords)            [rs255 encode kernel]
         + inject exactly one byte error into every codeword (one torch scatter of wrong bytes)
         + decode(codewords -> payloads, status, in-place write-back)   [rs255 decode kernel]
value = algorithmic bytes of all ranks (encode 504 B + decode 504 B per block) / step time.

Multi-GPU: one process per GPU (torchrun).  Blocks are independent, so each rank owns its own
2^20-block shard ("scaling": "weak"); the only collectives are the barrier around the timed
region and the max-over-ranks of the elapsed time (not on the data path).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--graph-steps", type=int, default=10, help="steps captured per hipGraph")
    ap.add_argument("--blocks", type=int, default=1 << 20, help="blocks per GPU")
    ap.add_argument("--block-size", type=int, default=512)
    ap.add_argument("--t", type=int, default=3)
    ap.add_argument("--prewarm-s", type=float, default=1.0, help="untimed clock ramp before the warmup steps")
    ap.add_argument("--no-graph", dest="graph", action="store_false", help="eager launches instead of one hipGraph per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-blocks", type=int, default=1 << 18)
    ap.add_argument("--host-inclusive", action="store_true", help="also time the pinned H2D+kernel+D2H path")
    ap.add_argument("--verify", action="store_true", help="check a sample of outputs against the oracle")
    return ap.parse_args()


def cpu_baseline(bs, t, nblocks, seed=1234):
    """Oracle ('port') timed on host cores over a bounded sample (rank 0, N=1 only)."""
    from concurrent.futures import ThreadPoolExecutor

    from tests.oracle_lib import Oracle

    o = Oracle()
    n, k, _ = o.rs_sizes(bs, t)
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, nblocks * k, dtype=np.uint8)
    cores = min(16, os.cpu_count() or 1)
    parts = np.array_split(np.arange(nblocks), cores)
    bufs = []
    for p in parts:
        bufs.append(np.ascontiguousarray(data.reshape(nblocks, k)[p]).reshape(-1))
    pos = rng.integers(0, n, nblocks)
    val = rng.integers(1, 256, nblocks, dtype=np.uint8)
    o.rs_encode(bs, t, data[:k])  # tables initialised before threads start

    def enc(i):
        return o.rs_encode(bs, t, bufs[i])

    t0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:
        cws = list(ex.map(enc, range(cores)))
    t_enc = time.perf_counter() - t0
    bads = []
    for i, p in enumerate(parts):
        c = cws[i].reshape(-1, n).copy()
        c[np.arange(len(p)), pos[p]] ^= val[p]
        bads.append(c.reshape(-1))

    def dec(i):
        return o.rs_decode(bs, t, bads[i])

    t0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:
        list(ex.map(dec, range(cores)))
    t_dec = time.perf_counter() - t0
    alg = (k + n) * nblocks
    return {
        "value": round(2 * alg / (t_enc + t_dec) / GIB, 4),
        "unit": "GiB/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{nblocks} RS({n},{k}) blocks: encode + 1-byte-error decode, oracle/ppfs_oracle.c "
                  f"on {cores} host threads over disjoint block ranges",
        "encode_blocks_per_s": round(nblocks / t_enc),
        "decode_blocks_per_s": round(nblocks / t_dec),
    }


class HipEvents:
    """Timing events without the system-scope fence (hipEventDisableSystemFence): a default event
    record writes back and invalidates the caches, which charges the previous kernel's dirty lines
    to the next interval and slows the kernel after it.  Created through libamdhip64 directly
    (torch's events use the default flags)."""

    FLAGS = 0x20000000  # hipEventDisableSystemFence (hip_runtime_api.h)

    def __init__(self, n):
        import ctypes
        self.ct = ctypes
        self.L = ctypes.CDLL("libamdhip64.so")
        self.ev = [ctypes.c_void_p() for _ in range(n)]
        for e in self.ev:
            rc = self.L.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(self.FLAGS))
            assert rc == 0, f"hipEventCreateWithFlags: {rc}"

    def record(self, i, stream):
        rc = self.L.hipEventRecord(self.ev[i], self.ct.c_void_p(stream.cuda_stream))
        assert rc == 0, f"hipEventRecord: {rc}"

    def ms(self, i, j):
        f = self.ct.c_float()
        rc = self.L.hipEventElapsedTime(self.ct.byref(f), self.ev[i], self.ev[j])
        assert rc == 0, f"hipEventElapsedTime: {rc}"
        return f.value


def timed_steps(step, steps, world, sync, device=None):
    """Time exactly `steps` calls of step() between barrier + sync on both sides; returns the
    MAX elapsed seconds over ranks (every rank gets the same value).  The barrier and the
    max-reduce are the only collectives: nothing on the data path."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return elapsed


def load_traffic(path=os.path.join(ROOT, "profiles", "pmc_latest.json")):
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine

    eng = EccEngine(ECC_REED_SOLOMON, args.block_size, args.t, device=dev.index)
    n, k = eng.raw_block_size, eng.data_size
    nb = args.blocks
    gen = torch.Generator(device=dev)
    gen.manual_seed(0x50504653 ^ rank)  # "PPFS" ^ rank
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=gen)
    cw = torch.empty(nb * n, dtype=torch.uint8, device=dev)
    out = torch.empty(nb * k, dtype=torch.uint8, device=dev)
    status = torch.empty(nb, dtype=torch.uint8, device=dev)
    # one error per codeword: position uniform in [0,255), value uniform in [1,255]
    err_pos = (torch.arange(nb, device=dev, dtype=torch.int64) * n
               + torch.randint(0, n, (nb,), device=dev, generator=gen))
    err_val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen)
    stream = torch.cuda.current_stream()
    # The payloads never change, so every step's clean codewords are identical: the corrupted
    # byte of block b is always clean[b, pos_b] ^ val_b.  Precompute it once; the per-step
    # injection is then a single scatter of 2^20 wrong bytes into the fresh codewords.
    eng.encode(data, cw, nblocks=nb)
    bad_bytes = cw[err_pos] ^ err_val
    torch.cuda.synchronize()

    def inject():
        cw.index_put_((err_pos,), bad_bytes)

    def step():
        eng.encode(data, cw, nblocks=nb)
        inject()
        eng.decode(cw, out, status, write_back=True, nblocks=nb)

    for _ in range(2):  # eager once (also loads every kernel) before any capture
        step()
    torch.cuda.synchronize()
    run = step
    graph = None
    group = max(1, args.graph_steps)
    if args.graph:
        # hipGraphs of whole steps: `group` consecutive steps per graph (one replay = `group` full
        # encode + inject + decode steps, no host launch overhead and no graph boundary between
        # them); K = q * group + r timed steps run as q group replays + r single-step replays.
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        graph_g = graph
        if group > 1:
            graph_g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph_g):
                for _ in range(group):
                    step()
        run = graph.replay

    def run_steps(k):
        if graph is None or group == 1:
            for _ in range(k):
                run()
            return
        for _ in range(k // group):
            graph_g.replay()
        for _ in range(k % group):
            graph.replay()

    # Clock ramp: a GPU that was idle runs its first milliseconds of work at lower clocks (the first
    # ~50 ms of back-to-back launches measured up to 25 % slower on MI355X).  Run the same step,
    # untimed, for --prewarm-s seconds before the W warmup steps, so the K timed steps see the
    # sustained clock a production scrub / FUSE stream runs at.  Nothing here is reused later.
    t_end = time.perf_counter() + args.prewarm_s
    while time.perf_counter() < t_end:
        run_steps(32)
        torch.cuda.synchronize()
    run_steps(args.warmup)
    torch.cuda.synchronize()
    if args.warmup > 0:
        # cheap device-side self-check of the last warmup step: every block corrected, payload restored
        ok = bool(torch.equal(out, data)) and int(status.min()) == 1 and int(status.max()) == 1
        if not ok:
            print(json.dumps({"error": "verification failed"}), file=sys.stderr)
            sys.exit(3)

    elapsed = timed_steps(lambda: run_steps(args.steps), 1, world, torch.cuda.synchronize, dev)

    # Kernel durations (roofline.achieved): eager steps bracketed by fence-free HIP events on the
    # launch stream, all K queued before one synchronize (host issue ~30 us/step << device time),
    # so an event pair brackets its kernel plus the ~1-2 us dependent-launch boundary.
    he = HipEvents(4 * args.steps + 2)
    t_issue = time.perf_counter()
    for i in range(args.steps):
        he.record(4 * i, stream)
        eng.encode(data, cw, nblocks=nb)
        he.record(4 * i + 1, stream)
        inject()
        he.record(4 * i + 2, stream)
        eng.decode(cw, out, status, write_back=True, nblocks=nb)
        he.record(4 * i + 3, stream)
    t_issue = (time.perf_counter() - t_issue) / args.steps
    torch.cuda.synchronize()
    enc_ms = [he.ms(4 * i, 4 * i + 1) for i in range(args.steps)]
    inj_ms = [he.ms(4 * i + 1, 4 * i + 2) for i in range(args.steps)]
    dec_ms = [he.ms(4 * i + 2, 4 * i + 3) for i in range(args.steps)]
    enc_avg, dec_avg, inj_avg = float(np.mean(enc_ms)), float(np.mean(dec_ms)), float(np.mean(inj_ms))
    # device time of the timed region itself (same K steps again, two events around them)
    he.record(4 * args.steps, stream)
    run_steps(args.steps)
    he.record(4 * args.steps + 1, stream)
    torch.cuda.synchronize()
    gpu_ms_per_step = he.ms(4 * args.steps, 4 * args.steps + 1) / args.steps
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]

    # device copy reference peak (same bytes as one encode: read k, write n per block)
    cp_src = torch.empty(nb * (k + n) // 2, dtype=torch.uint8, device=dev)
    cp_dst = torch.empty_like(cp_src)
    for _ in range(3):
        cp_dst.copy_(cp_src)
    ev[4].record(stream)
    for _ in range(10):
        cp_dst.copy_(cp_src)
    ev[5].record(stream)
    ev[5].synchronize()
    torch_copy_gbs = 2 * cp_src.numel() / (ev[4].elapsed_time(ev[5]) / 10 * 1e-3) / 1e9
    # the engine's full-grid 16-byte copy kernel (ppfs_copy_device): the HBM ceiling this access
    # shape reaches, timed like the kernels (fence-free events on the launch stream, median)
    from paritypartyfs_amd import device_copy

    for _ in range(3):
        device_copy(cp_dst, cp_src, stream=stream)
    hc = HipEvents(20)
    for i in range(10):
        hc.record(2 * i, stream)
        device_copy(cp_dst, cp_src, stream=stream)
        hc.record(2 * i + 1, stream)
    torch.cuda.synchronize()
    copy_ms = float(np.median([hc.ms(2 * i, 2 * i + 1) for i in range(10)]))
    copy_gbs = 2 * cp_src.numel() / (copy_ms * 1e-3) / 1e9
    del cp_src, cp_dst

    alg_per_block = k + n  # 504 B for RS(255,249), both for encode and decode
    if (args.block_size, args.t) == (512, 3):
        cfg_ref = "BASELINE configs[1]+[2]"
    elif (args.block_size, args.t) == (4096, 16):
        cfg_ref = "BASELINE configs[4], one GPU's shard"
    else:
        cfg_ref = "not a BASELINE config"
    total_bytes = 2 * alg_per_block * nb * world * args.steps
    value = total_bytes / elapsed / GIB
    ms_per_step = elapsed / args.steps * 1e3

    dom_ms = max(enc_avg, dec_avg)
    which = "decode" if dec_avg >= enc_avg else "encode"
    kn = eng.kernel_name
    if kn.startswith("rs255-wg"):
        dom_name = f"rs_wg_{which}_kernel<{n - k}>"
    elif kn.startswith("rs255-pair"):  # 16 < 2t <= 32 (rs_pair.hpp)
        dom_name = f"rs_pair_{'decode' if which == 'decode' else 'encode_img'}_kernel<{n - k}>"
    elif kn.startswith("rs255-slice8") and which == "encode" and n - k == 16:
        dom_name = f"rs_solo_encode_img_kernel<{n - k}>"
    else:
        dom_name = f"rs255_{which}_kernel<{n - k}>"
    achieved = alg_per_block * nb / (dom_ms * 1e-3) / 1e9
    traffic = None
    pmc = load_traffic()
    kp = (pmc or {}).get("kernels", {}).get(dom_name)
    if kp and kp.get("blocks") == nb:
        traffic = round(kp["hbm_bytes_per_launch"])  # profiles/pmc_latest.json, tools/pmc_summary.py

    host_incl = None
    if args.host_inclusive and rank == 0:
        hd = data.cpu().numpy()
        hraw = np.empty(nb * n, np.uint8)
        hout = np.empty(nb * k, np.uint8)
        hst = np.empty(nb, np.uint8)
        eng.encode_host(hd, hraw)
        t1 = time.perf_counter()
        eng.encode_host(hd, hraw)
        t2 = time.perf_counter()
        eng.decode_host(hraw, hout, hst, write_back=True)
        t3 = time.perf_counter()
        host_incl = {"encode_GiBps": round(alg_per_block * nb / (t2 - t1) / GIB, 3),
                     "decode_GiBps": round(alg_per_block * nb / (t3 - t2) / GIB, 3)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.block_size, args.t, min(args.cpu_sample_blocks, nb))

    if rank == 0:
        line = {
            "metric": "device-resident GiB/s: RS encode+decode, 512 B blocks, 1 M-block batch",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": f"RS({n},{k}) t={args.t} block_size={args.block_size}: encode + 1-byte-error "
                            f"inject + decode with write-back, {nb} blocks per GPU ({cfg_ref})",
                "blocks_per_gpu": nb,
                "global_blocks": nb * world,
                "parallelism": f"shard{world}",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom_name,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": alg_per_block * nb,
                "avg_launch_ms": round(dom_ms, 5),
            },
            "cpu_baseline": cpu,
            "kernels_ms": {"encode": round(enc_avg, 5), "inject": round(inj_avg, 5), "decode": round(dec_avg, 5)},
            "encode_GBps": round(alg_per_block * nb / (enc_avg * 1e-3) / 1e9, 1),
            "decode_GBps": round(alg_per_block * nb / (dec_avg * 1e-3) / 1e9, 1),
            "device_copy_GBps": round(copy_gbs, 1),
            "device_copy_kernel": "ppfs_copy_device (full-grid 16-B copy, same bytes as one encode)",
            "torch_copy_GBps": round(torch_copy_gbs, 1),
            # payload rate beside the algorithmic one, and the dominant kernel
            # against the device-to-device copy measured above
            "payload_GiBps": round(value * k / alg_per_block, 3),
            "roofline_frac_of_device_copy": round(achieved / copy_gbs, 4) if copy_gbs else None,
            "host_inclusive": host_incl,
            "kernel_path": eng.kernel_name,
            "launch": f"hipGraph of {group} steps" if graph is not None else "eager",
            "host_issue_us_per_eager_step": round(t_issue * 1e6, 1),
            "device_ms_per_step": round(gpu_ms_per_step, 4),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
