#!/usr/bin/env python3
"""bench.py -- device-resident RS encode+decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]/[2]): ecc_type=reed_solomon, block_size=512,
rs_correctable_bytes=3 -> RS(255,249) (the reference clamps codewords to 255 B,
rs_block_device.cpp:57), 2^20 blocks per GPU, synthetic uniform payloads.
`--block-size 4096 --t 16` runs configs[4]'s RS(255,223) shard instead (2^20 blocks per GPU).

One step = encode(2^20 payloads -> codewords)            [rs255 encode kernel]
         + inject exactly one byte error into every codeword (the engine's inject kernel stores
           the precomputed wrong byte of every block; --inject torch: torch's index_put_)
         + decode(codewords -> payloads, status, in-place write-back)   [rs255 decode kernel]
value = algorithmic bytes of all ranks (encode k+n B + decode n+k B per block) / step time.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` (N > 1, no torchrun env) starts
`torch.distributed.run` with N ranks as a child process before anything touches a GPU and exits
with its code; under torchrun (WORLD_SIZE set) each rank runs its own shard.  Blocks are
independent, so every rank owns a 2^20-block shard ("scaling": "weak"); the only collectives are
the barrier around the timed region and the max-over-ranks of the elapsed time (not on the data
path).  `--dry-run-cpu` replaces the engine by a CPU stand-in (gloo, no GPU) to exercise exactly
this launch / timing path in tests; its numbers are not measurements.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "device-resident GiB/s: RS encode+decode, 512 B blocks, 1 M-block batch"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (ranks); default: WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--launch", choices=("eager", "graph"), default="eager",
                    help="eager launches (default) or one hipGraph per --graph-steps steps")
    ap.add_argument("--graph-steps", type=int, default=10, help="steps captured per hipGraph (--launch graph)")
    ap.add_argument("--blocks", type=int, default=1 << 20, help="blocks per GPU")
    ap.add_argument("--block-size", type=int, default=512)
    ap.add_argument("--t", type=int, default=3)
    ap.add_argument("--inject", choices=("engine", "engine-xor", "torch"), default="engine",
                    help="fault-injection form: the engine's one-byte-per-block kernel storing the "
                         "precomputed wrong byte (engine) or XORing the error value in (engine-xor: "
                         "load + store), or torch index_put_")
    ap.add_argument("--prewarm-s", type=float, default=1.0, help="untimed clock ramp before the warmup steps")
    ap.add_argument("--standalone-launches", type=int, default=30, help="back-to-back launches per kernel")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", dest="configs", action="store_false",
                    help="skip the per-config kernel leg (BASELINE configs[3] Hamming / CRC bs 4096 and "
                         "configs[4] RS(255,223), rank 0 at N=1, outside the timed region)")
    ap.add_argument("--config-reps", type=int, default=20)
    ap.add_argument("--cpu-sample-blocks", type=int, default=1 << 20)
    ap.add_argument("--cpu-faithful-blocks", type=int, default=1 << 18)
    ap.add_argument("--no-host-inclusive", dest="host_inclusive", action="store_false",
                    help="skip the H2D + kernel + D2H leg (rank 0, N=1)")
    ap.add_argument("--host-reps", type=int, default=3, help="host_inclusive: calls per (mode, op); best reported")
    ap.add_argument("--dry-run-cpu", action="store_true", help="CPU stand-in for the engine (launcher tests)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal on a box with fewer GPUs than ranks: rank r uses GPU r %% count and the "
                         "barrier / max-reduce run over gloo (RCCL needs one GPU per rank); the line then "
                         "checks the multi-rank path on real kernels, not scaling")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------
# launcher: N ranks as a child process (nothing has touched a GPU yet)
# ------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(nranks: int, argv) -> int:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


# ------------------------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the oracle on the host cores
# ------------------------------------------------------------------------------------------
def _pool_time(fn, nparts):
    from concurrent.futures import ThreadPoolExecutor

    t0 = time.perf_counter()
    with ThreadPoolExecutor(nparts) as ex:
        res = list(ex.map(fn, range(nparts)))
    return time.perf_counter() - t0, res


def usable_cpus():
    """CPUs this process may actually use: the affinity mask, capped by the cgroup's CPU quota
    (a GPU box's job sees the whole machine in os.cpu_count() but gets a share of it).  Returns
    (cores, detail dict) -- the detail says where the figure came from."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    cores = min(aff, quota) if quota else aff
    return cores, {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota}


# the reference's own CPU path (sources compiled unmodified, g++ -O2, 8-vCPU
# Xeon, 8 threads), quoted -- not measured in this run
REF_QUOTED = {
    (512, 3): {"encode_blocks_per_s": 19899, "decode_1err_blocks_per_s": 349701, "threads": 8},
    (4096, 16): {"encode_blocks_per_s": 15552, "decode_1err_blocks_per_s": 126088, "threads": 8},
}


def cpu_baseline(bs, t, nblocks, nfaithful, seed=1234):
    """Two CPU columns on the same synthetic workload (encode, then a 1-byte-error decode), one
    thread per usable core over disjoint block ranges (the ctypes calls release the GIL):
      value / "port": the oracle's table-driven codec (LFSR encode, table syndromes; blocks with
          a non-zero syndrome run the restated reference decode) -- the strong CPU baseline;
      "faithful": the reference's algorithm restated over C arrays (schoolbook long-division
          encode, Horner syndromes, BM / 255-point root search / Forney), SURVEY 8(d)'s
          "reference-faithful variant", on a smaller sample.  Faithful to the algorithm, not to the
          cost: it omits writeBlock's old-block read + decode (rs_block_device.cpp:61-93) and
          PolynomialGF256's 256-entry temporaries (polynomial_gf256.cpp:101-127);
      "reference_quoted": the reference's own per-call rates from BASELINE.md section 2 (not
          measured here)."""
    from tests.oracle_lib import Oracle

    o = Oracle()
    n, k, _ = o.rs_sizes(bs, t)
    cores, cpu_detail = usable_cpus()
    rng = np.random.default_rng(seed)

    def run(nb, enc_fn, dec_fn):
        data = rng.integers(0, 256, nb * k, dtype=np.uint8)
        parts = np.array_split(np.arange(nb), cores)
        bufs = [np.ascontiguousarray(data.reshape(nb, k)[p]).reshape(-1) for p in parts]
        pos = rng.integers(0, n, nb)
        val = rng.integers(1, 256, nb, dtype=np.uint8)
        enc_fn(data[:k])  # tables initialised before the threads start
        t_enc, cws = _pool_time(lambda i: enc_fn(bufs[i]), cores)
        bads = []
        for i, p in enumerate(parts):
            c = cws[i].reshape(-1, n).copy()
            c[np.arange(len(p)), pos[p]] ^= val[p]
            bads.append(c.reshape(-1))
        t_dec, outs = _pool_time(lambda i: dec_fn(bads[i]), cores)
        ok = all(np.array_equal(outs[i][0], bufs[i]) for i in range(cores))
        return t_enc, t_dec, ok

    te, td, ok = run(nblocks, lambda d: o.rs_encode_table(bs, t, d), lambda r: o.rs_decode_table(bs, t, r))
    fe, fd, fok = run(nfaithful, lambda d: o.rs_encode(bs, t, d), lambda r: o.rs_decode(bs, t, r))
    alg = k + n
    quoted = None
    if (bs, t) in REF_QUOTED:
        qr = REF_QUOTED[(bs, t)]
        qe, qd = qr["encode_blocks_per_s"], qr["decode_1err_blocks_per_s"]
        quoted = {
            "value": round(2 * alg / (1 / qe + 1 / qd) / GIB, 5),
            "unit": "GiB/s",
            "encode_blocks_per_s": qe,
            "decode_1err_blocks_per_s": qd,
            "threads": qr["threads"],
            "kind": "reference (quoted, not measured in this run)",
            "source": "BASELINE.md section 2: the reference's writeBlock (old-block read + decode + encode, "
                      "rs_block_device.cpp:61-117) and readBlock with 1 error (:25-50,119-183), compiled "
                      "unmodified (g++ -O2), 8-vCPU Xeon, 8 threads, +-30 %",
        }
    return {
        "value": round(2 * alg * nblocks / (te + td) / GIB, 4),
        "unit": "GiB/s",
        "cores": cores,
        "cores_detail": cpu_detail,
        "kind": "port",
        "sample": f"{nblocks} RS({n},{k}) blocks (the whole workload): encode + 1-byte-error decode, "
                  f"oracle/ppfs_oracle.c table codec on {cores} host threads over disjoint block ranges",
        "encode_blocks_per_s": round(nblocks / te),
        "decode_blocks_per_s": round(nblocks / td),
        "verified": bool(ok),
        "faithful": {
            "value": round(2 * alg * nfaithful / (fe + fd) / GIB, 4),
            "unit": "GiB/s",
            "cores": cores,
            "kind": "port (reference algorithm, C arrays)",
            "sample": f"{nfaithful} RS({n},{k}) blocks: schoolbook long-division encode + Horner-syndrome / BM / "
                      f"255-point root search / Forney decode (restated rs_block_device.cpp:95-280 over C arrays; "
                      f"without writeBlock's old-block read + decode and PolynomialGF256's temporaries, so "
                      f"faster than the reference's own code)",
            "encode_blocks_per_s": round(nfaithful / fe),
            "decode_blocks_per_s": round(nfaithful / fd),
            "verified": bool(fok),
        },
        "reference_quoted": quoted,
    }


# ------------------------------------------------------------------------------------------
# timing helpers
# ------------------------------------------------------------------------------------------
def _hip_ok(rc, what):
    """A HIP runtime call's status, checked explicitly (not by assert: `python -O` would drop the call)."""
    if rc != 0:
        raise RuntimeError(f"{what}: hipError {rc}")


class HipEvents:
    """Timing events without the system-scope fence (hipEventDisableSystemFence): a default event
    record writes back and invalidates the caches, which charges the previous kernel's dirty lines
    to the next interval and slows the kernel after it.  Created through the HIP runtime torch
    loaded (same library instance as the engine's launches)."""

    FLAGS = 0x20000000  # hipEventDisableSystemFence (hip_runtime_api.h)

    def __init__(self, n):
        import ctypes
        self.ct = ctypes
        self.L = ctypes.CDLL("libamdhip64.so")
        self.ev = [ctypes.c_void_p() for _ in range(n)]
        for e in self.ev:
            _hip_ok(self.L.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(self.FLAGS)), "hipEventCreateWithFlags")

    def record(self, i, stream):
        _hip_ok(self.L.hipEventRecord(self.ev[i], self.ct.c_void_p(stream.cuda_stream)), "hipEventRecord")

    def ms(self, i, j):
        f = self.ct.c_float()
        _hip_ok(self.L.hipEventElapsedTime(self.ct.byref(f), self.ev[i], self.ev[j]), "hipEventElapsedTime")
        return f.value

    def close(self):
        for e in self.ev:
            self.L.hipEventDestroy(e)


def timed_steps(step, steps, world, sync, device=None, pre=None, bar_group=None):
    """Time exactly `steps` calls of step() between barrier + sync on both sides; returns the
    MAX elapsed seconds over ranks (every rank gets the same value).  The barrier and the
    max-reduce are the only collectives: nothing on the data path.

    pre(): untimed work queued BEFORE the barrier (warm-up steps), so that the GPU is busy while
    the ranks meet -- an RCCL barrier idles the host for long enough that an idle GPU drops its
    clocks, and the first timed steps then ran ~15 % slow (r3c: 0.2675 vs 0.2294 ms per step under
    torchrun at WORLD_SIZE=1 with the barrier on an idle GPU).  The synchronize after the barrier
    drains pre()'s work; the region starts from a busy, clocked-up GPU.  bar_group: the process group
    of the barriers (a gloo group beside RCCL: an RCCL barrier's kernel waits for the work queued on
    the current stream, so the host reached the region's synchronize only after the GPU had drained
    and idled -- r3e, 0.2553 vs 0.2258 ms per step of device time under torchrun at WORLD_SIZE=1)."""
    import torch
    import torch.distributed as dist

    # under torchrun the collectives run whenever a process group exists, also at WORLD_SIZE=1:
    # `torchrun --nproc-per-node 1 bench.py` then executes exactly the RCCL code of the 8-GPU run
    coll = world > 1 or (dist.is_available() and dist.is_initialized())
    if pre is not None:
        pre()
    if coll:
        dist.barrier(group=bar_group)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    if coll:
        dist.barrier(group=bar_group)
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return elapsed


def lib_sha256():
    from paritypartyfs_amd import _native

    h = hashlib.sha256()
    with open(_native.LIB_PATH, "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def load_traffic(kernel, nblocks, path=os.path.join(ROOT, "profiles", "pmc_latest.json")):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_summary.py), used
    only when it was collected on THIS build of the library (sha256 of libppfs_ecc.so) for the
    same kernel and block count; otherwise None (never a stale figure)."""
    try:
        with open(path) as f:
            pmc = json.load(f)
    except Exception:
        return None, "no profiles/pmc_latest.json"
    kp = pmc.get("kernels", {}).get(kernel)
    if not kp or kp.get("blocks") != nblocks:
        return None, f"pmc_latest.json ({pmc.get('tag')}) has no {kernel} over {nblocks} blocks"
    if pmc.get("lib_sha256") != lib_sha256():
        return None, f"pmc_latest.json ({pmc.get('tag')}) was collected on another build of libppfs_ecc.so"
    return round(kp["hbm_bytes_per_launch"]), f"rocprofv3 PMC {pmc.get('tag')} (same library build)"


def host_link_ceilings(dev, nb, k, n, reps=3):
    """The host link measured on this box: hipMemcpyAsync between hipHostMalloc'd
    (page-locked) and device memory, H2D only, D2H only, and both at once on two non-blocking streams,
    over the bytes the host entry points move -- encode: k B in, n B out per block; 1-error decode
    with write-back: n B in, k + n B out (payload + every changed codeword).  Best of `reps`; rates in
    GB/s of bytes moved, ceilings in algorithmic GiB/s (k + n B per block, the unit of the *_host
    rates).  Straight HIP calls (ctypes, the runtime torch loaded), as the engine's own copies."""
    import ctypes

    import torch

    torch.cuda.synchronize()
    L = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
    big = (k + n) * nb
    h_in, h_out, d_in, d_out = vp(), vp(), vp(), vp()
    streams = [vp(), vp()]
    try:
        _hip_ok(L.hipHostMalloc(ctypes.byref(h_in), ctypes.c_size_t(big), 0), "hipHostMalloc")
        _hip_ok(L.hipHostMalloc(ctypes.byref(h_out), ctypes.c_size_t(big), 0), "hipHostMalloc")
        _hip_ok(L.hipMalloc(ctypes.byref(d_in), ctypes.c_size_t(big)), "hipMalloc")
        _hip_ok(L.hipMalloc(ctypes.byref(d_out), ctypes.c_size_t(big)), "hipMalloc")
        for st in streams:
            _hip_ok(L.hipStreamCreateWithFlags(ctypes.byref(st), 1), "hipStreamCreateWithFlags")  # non-blocking
        H2D, D2H = 1, 2  # hipMemcpyHostToDevice, hipMemcpyDeviceToHost

        def copy(dst, src, nbytes, kind, st):
            _hip_ok(L.hipMemcpyAsync(dst, src, ctypes.c_size_t(nbytes), kind, st), "hipMemcpyAsync")

        def best(fn):
            ts = []
            for _ in range(reps):
                fn()  # one untimed pass each time: both directions' DMA engines warm
                for st in streams:
                    _hip_ok(L.hipStreamSynchronize(st), "hipStreamSynchronize")
                t0 = time.perf_counter()
                fn()
                for st in streams:
                    _hip_ok(L.hipStreamSynchronize(st), "hipStreamSynchronize")
                ts.append(time.perf_counter() - t0)
            return min(ts)

        def both(b_in, b_out, chunk=8 << 20):
            # the two directions in 8 MiB pieces, issued alternately on their own streams (one copy of
            # each direction in flight at a time, as the engine's host path overlaps its chunks)
            o_in = o_out = 0
            while o_in < b_in or o_out < b_out:
                if o_in < b_in:
                    m = min(chunk, b_in - o_in)
                    copy(vp(d_in.value + o_in), vp(h_in.value + o_in), m, H2D, streams[0])
                    o_in += m
                if o_out < b_out:
                    m = min(chunk, b_out - o_out)
                    copy(vp(h_out.value + o_out), vp(d_out.value + o_out), m, D2H, streams[1])
                    o_out += m

        t_h2d = best(lambda: copy(d_in, h_in, k * nb, H2D, streams[0]))
        t_d2h = best(lambda: copy(h_out, d_out, n * nb, D2H, streams[1]))
        t_enc = best(lambda: both(k * nb, n * nb))
        t_dec = best(lambda: both(n * nb, (k + n) * nb))
        # a decode whose write-back comes back as a patch list (api.cpp patch_slots: 2 slots of 4 B
        # per block for RS(255, k)) moves n B in, k + 8 B out
        t_decp = best(lambda: both(n * nb, (k + 8) * nb))
    finally:
        for st in streams:
            if st.value:
                L.hipStreamDestroy(st)
        for p_ in (h_in, h_out):
            if p_.value:
                L.hipHostFree(p_)
        for p_ in (d_in, d_out):
            if p_.value:
                L.hipFree(p_)
    alg = (k + n) * nb
    return {
        "h2d_GBps": round(k * nb / t_h2d / 1e9, 2),
        "d2h_GBps": round(n * nb / t_d2h / 1e9, 2),
        "bidir_encode_bytes_GBps": round((k + n) * nb / t_enc / 1e9, 2),
        "bidir_decode_bytes_GBps": round((k + 2 * n) * nb / t_dec / 1e9, 2),
        "encode_ceiling_GiBps": round(alg / t_enc / GIB, 3),
        "decode_1err_ceiling_GiBps": round(alg / t_dec / GIB, 3),
        "decode_1err_patch_ceiling_GiBps": round(alg / t_decp / GIB, 3),
        "method": "hipMemcpyAsync between hipHostMalloc'd and hipMalloc'd buffers; both directions at once: 8 MiB "
                  f"pieces issued alternately on two non-blocking streams; best of {reps}",
    }


# SURVEY 6 (measured in the dev container, 8-vCPU Xeon, reference sources at -O2, one thread):
# RS(255,249) writeBlock (encode, incl. the old-block decode) and readBlock (clean decode) rates
REF_CPU_CFG1 = {"writeBlock_blocks_per_s": 2422, "readBlock_clean_blocks_per_s": 95162,
                "source": "SURVEY.md 6: reference C++ compiled here, 1 thread, HeapDisk, dev container (not the GPU box)"}


def cfg1_leg(min_s=0.05, timeout_s=240):
    """BASELINE configs[0] (performance_tests/bench_blockdevice.cpp:12-110 on the GPU-backed C++
    adapter, tests/cpp/bench_blockdevice.cpp, built by __graft_entry__.build): per-block readBlock /
    writeBlock of RS(255,249) over 4096 blocks and the batched readBlocks / writeBlocks, plus the
    reference bench's raw / crc(0xea) / hamming(2^8) / rs(t=16) sweep over 1..256-byte calls on
    256-byte blocks, beside the reference CPU rates.  A child process (it opens its own context)."""
    exe = os.path.join(ROOT, "tests", "cpp", "_build", "bench_blockdevice")
    if not os.path.exists(exe):
        return {"error": "tests/cpp/_build/bench_blockdevice not built (__graft_entry__.build)"}
    try:
        r = subprocess.run([exe, str(min_s)], capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"error": f"bench_blockdevice exceeded {timeout_s} s"}
    if r.returncode != 0:
        return {"error": f"bench_blockdevice rc {r.returncode}: {r.stderr[-300:]}"}
    rows = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    out = {"sweep": {}, "reference_cpu": REF_CPU_CFG1}
    for row in rows:
        name = row.get("bench", "")
        if name.startswith("BM_BlockDevice_"):
            op, rest = name[len("BM_BlockDevice_"):].split("/", 1)
            dev_, n = rest.split("/")
            d = out["sweep"].setdefault(dev_.replace("_test", ""), {})
            rate = row.get("BytesRead_per_s", row.get("BytesWritten_per_s"))
            d[f"{op.lower()}_{n}"] = {"us_per_call": row["us_per_call"], "KiB_per_s": round(rate / 1024.0, 1),
                                      "ok": row["ok"]}
        elif name.startswith("cfg1"):
            out["rs255_249_4096_blocks"] = {k_: v for k_, v in row.items() if k_ != "bench"}
        elif name.startswith("MappedFileDisk"):
            out["mapped_file_disk_2p20_blocks"] = {k_: v for k_, v in row.items() if k_ != "bench"}
    c = out.get("rs255_249_4096_blocks")
    if c:
        out["per_block_read_vs_reference_cpu"] = round(c["per_block_read_blocks_per_s"]
                                                       / REF_CPU_CFG1["readBlock_clean_blocks_per_s"], 2)
        out["per_block_write_vs_reference_cpu"] = round(c["per_block_write_blocks_per_s"]
                                                        / REF_CPU_CFG1["writeBlock_blocks_per_s"], 2)
    out["note"] = ("BASELINE configs[0]: the reference bench's calls through the C++ IBlockDevice adapter on the GPU "
                   "(per-block calls served by the resident server kernel); KiB_per_s as google/benchmark's "
                   "BytesRead / BytesWritten counters; outside the timed region")
    return out


def rank_fields(mine, alg_step_bytes, world, elapsed_s, steps):
    """SURVEY 8(e) fields of an N-rank line, made on every rank (all_gather over the default group;
    the ranks reach this point together, after the timed region):
      per_rank_kernels_ms: every rank's in-step kernel means (min / max over ranks, and each rank's),
        so one SCALE run shows whether a slow GPU or the launch path set the max-over-ranks time;
      aggregate_frac: sum over ranks of the algorithmic bytes of the timed steps / the timed region
        (max over ranks) / (N x the per-GPU HBM peak) -- the job's fraction of N GPUs' bandwidth."""
    import torch.distributed as dist

    gathered = [mine]
    if dist.is_available() and dist.is_initialized():
        gathered = [None] * dist.get_world_size()
        dist.all_gather_object(gathered, mine)
    gathered = sorted(gathered, key=lambda g: g["rank"])
    per = {}
    for key in ("encode", "decode"):
        vals = [g[key] for g in gathered]
        per[key] = {"min": round(min(vals), 5), "max": round(max(vals), 5), "by_rank": [round(v, 5) for v in vals]}
    total = alg_step_bytes * world * steps
    agg = total / elapsed_s / 1e9 / (world * HBM_PEAK_GBS)
    return per, {"aggregate_frac": round(agg, 4), "aggregate_peak_GBps": world * HBM_PEAK_GBS,
                 "aggregate_bytes": total, "ranks_reporting": len(gathered)}


# ------------------------------------------------------------------------------------------
# dry run: the launch / timing path with a CPU stand-in for the engine (tests only)
# ------------------------------------------------------------------------------------------
def dry_run(args, world, rank):
    import torch.distributed as dist

    if world > 1 or os.environ.get("WORLD_SIZE"):
        dist.init_process_group("gloo")
    buf = np.zeros(1 << 16, np.uint8)

    part_s = {"encode": [], "decode": []}

    def step():  # stand-in work: no ECC, no GPU ("encode" = the XOR, "decode" = the sleep)
        t0 = time.perf_counter()
        np.bitwise_xor(buf, 1, out=buf)
        t1 = time.perf_counter()
        time.sleep(0.001 * (rank + 1))
        part_s["encode"].append(t1 - t0)
        part_s["decode"].append(time.perf_counter() - t1)

    for _ in range(args.warmup):
        step()
    elapsed = timed_steps(step, args.steps, world, lambda: None, None)
    mine = {"rank": rank, "block_size": args.block_size, "t": args.t, "blocks": args.blocks,
            "encode": float(np.mean(part_s["encode"])) * 1e3, "decode": float(np.mean(part_s["decode"])) * 1e3}
    gathered = [mine]
    if dist.is_initialized():
        gathered = [None] * dist.get_world_size()
        dist.all_gather_object(gathered, mine)
    # the N-rank fields of the real line, over the stand-in's times and the workload's byte count
    # (RS codeword n = min(block_size, 255), k = n - 2t: rs_block_device.cpp:57)
    n = min(args.block_size, 255)
    k = n - 2 * args.t
    per_rank, agg = rank_fields(mine, 2 * (k + n) * args.blocks, world, elapsed, args.steps)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry_run": True, "value": None, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                          "scaling": "weak", "note": "CPU stand-in for the engine: launcher / timing test only",
                          "config": {"workload": f"RS({n},{k}) t={args.t} block_size={args.block_size} (stand-in)",
                                     "blocks_per_gpu": args.blocks, "global_blocks": args.blocks * world,
                                     "parallelism": f"shard{world}"},
                          "per_rank_kernels_ms": per_rank, **agg,
                          # what every rank parsed: the driver's argv must reach the ranks unchanged
                          "rank_args": [{k: g[k] for k in ("rank", "block_size", "t", "blocks")} for g in gathered]}),
              flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


# ------------------------------------------------------------------------------------------
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        # the driver's command form `python bench.py --gpus N`: start N ranks, report their line
        return launch_ranks(args.gpus, argv)
    world = int(env_world or 1)
    if args.gpus is not None and args.gpus != world:
        print(json.dumps({"error": f"--gpus {args.gpus} but WORLD_SIZE={world}"}), file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run_cpu:
        dry_run(args, world, rank)
        return 0

    import torch
    import torch.distributed as dist

    red_dev = None  # where the max-reduce of the elapsed time lives (the GPU for RCCL)
    if env_world is not None and args.share_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dist.init_process_group("gloo")
        red_dev = torch.device("cpu")
    elif env_world is not None:
        # under torchrun -- the driver's N-GPU form, and also at WORLD_SIZE=1 -- always RCCL with
        # its barrier and the GPU max-reduce, so a 1-GPU `torchrun --nproc-per-node 1` run executes
        # exactly the code of the 8-GPU scaling run
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    # the timed region's barriers over gloo (CPU) beside RCCL, which keeps the max-reduce (timed_steps)
    bar_group = dist.new_group(backend="gloo") if dist.is_initialized() and dist.get_backend() == "nccl" else None
    dev = torch.device("cuda", torch.cuda.current_device())
    red_dev = red_dev or dev
    # Every launch of the run goes to one created stream, not the legacy null stream (which orders
    # each launch against the other blocking streams): 0-1.7 % per step across two boxes
    # (tools/probes/overlap_probe.py; running consecutive steps on two streams gained nothing either).
    torch.cuda.set_stream(torch.cuda.Stream(dev))

    from paritypartyfs_amd import ECC_REED_SOLOMON, EccEngine, device_copy, pinned

    eng = EccEngine(ECC_REED_SOLOMON, args.block_size, args.t, device=dev.index)
    n, k = eng.raw_block_size, eng.data_size
    nb = args.blocks
    gen = torch.Generator(device=dev)
    gen.manual_seed(0x50504653 ^ rank)  # "PPFS" ^ rank: every rank its own shard
    data = torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=gen)
    cw = torch.empty(nb * n, dtype=torch.uint8, device=dev)
    out = torch.empty(nb * k, dtype=torch.uint8, device=dev)
    status = torch.empty(nb, dtype=torch.uint8, device=dev)
    # one error per codeword: position uniform in [0,255), value uniform in [1,255]
    err_col = torch.randint(0, n, (nb,), device=dev, generator=gen)
    err_pos = torch.arange(nb, device=dev, dtype=torch.int64) * n + err_col
    err_val = torch.randint(1, 256, (nb,), dtype=torch.uint8, device=dev, generator=gen)
    stream = torch.cuda.current_stream()
    # The payloads never change, so every step's clean codewords are identical: the corrupted
    # byte of block b is always clean[b, pos_b] ^ val_b.  Precompute it once; the per-step
    # injection is then a single scatter of 2^20 wrong bytes into the fresh codewords.
    eng.encode(data, cw, nblocks=nb)
    clean_cw = cw.clone()
    bad_bytes = cw[err_pos] ^ err_val
    err_col8 = err_col.to(torch.uint8)
    torch.cuda.synchronize()

    # Every launch goes to torch's CURRENT stream at call time (no stream captured here): inside
    # torch.cuda.graph() that is the capture stream, so --launch graph captures the injection too.
    if args.inject == "engine":
        from paritypartyfs_amd import inject_bytes

        def inject():
            inject_bytes(cw, n, err_col8, bad_bytes, nblocks=nb)
    elif args.inject == "engine-xor":
        from paritypartyfs_amd import inject_bytes

        def inject():
            inject_bytes(cw, n, err_col8, err_val, nblocks=nb, xor=True)
    else:
        def inject():
            cw.index_put_((err_pos,), bad_bytes)

    def step():
        eng.encode(data, cw, nblocks=nb)
        inject()
        eng.decode(cw, out, status, write_back=True, nblocks=nb)

    for _ in range(2):  # eager once (also loads every kernel) before any capture
        step()
    torch.cuda.synchronize()
    group = max(1, args.graph_steps)
    graph = graph_g = None
    if args.launch == "graph":
        # hipGraphs of whole steps: `group` consecutive steps per graph; K = q * group + r timed
        # steps run as q group replays + r single-step replays
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        graph_g = graph
        if group > 1:
            graph_g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph_g):
                for _ in range(group):
                    step()

    def run_steps(kk):
        if graph is None:
            for _ in range(kk):
                step()
            return
        for _ in range(kk // group):
            graph_g.replay()
        for _ in range(kk % group):
            graph.replay()

    # Clock ramp: a GPU that was idle runs its first milliseconds of work at lower clocks (the first
    # ~50 ms of back-to-back launches measured up to 25 % slower on MI355X).  Run the same step,
    # untimed, for --prewarm-s seconds before the W warmup steps, so the K timed steps see the
    # sustained clock a production scrub / FUSE stream runs at.  Nothing here is reused later.
    def rewarm(seconds):
        t_end = time.perf_counter() + seconds
        while time.perf_counter() < t_end:
            run_steps(8)
            torch.cuda.synchronize()

    rewarm(args.prewarm_s)
    # The W warmup steps are queued right before the barrier and run straight into the timed
    # region: nothing but the barrier (while they run) and the synchronize the region starts with
    # lies between them (an idle GPU drops its clocks within a millisecond or two and the next steps
    # run slower while they ramp back: r2c, 0.311 ms per step after a host-side check vs 0.25 back
    # to back).  The self-check runs after the region.
    elapsed = timed_steps(lambda: run_steps(args.steps), 1, world, torch.cuda.synchronize, red_dev,
                          pre=lambda: run_steps(args.warmup), bar_group=bar_group)
    # the same timed region again, 3 times (reported beside the measurement, never as `value`):
    # shows whether the measured region was representative of back-to-back regions
    repeats = [timed_steps(lambda: run_steps(args.steps), 1, world, torch.cuda.synchronize, red_dev,
                           pre=lambda: run_steps(max(2, args.warmup)), bar_group=bar_group) / args.steps * 1e3
               for _ in range(3)]
    # device-side self-check of the last timed step: every block corrected, payload restored
    ok = bool(torch.equal(out, data)) and int(status.min()) == 1 and int(status.max()) == 1
    if not ok:
        print(json.dumps({"error": "verification failed"}), file=sys.stderr)
        return 3

    # ---- everything below is outside the timed region ----
    # (1) in-step kernel durations (roofline.achieved): eager steps bracketed by fence-free HIP
    # events on the launch stream, all K queued before one synchronize
    K = args.steps
    # every measurement below starts from the sustained clock again (the self-check idled the GPU)
    rewarm(0.3)
    # Two measures per kernel: (a) events recorded on the stream around each call (they include the
    # launch gap before the kernel starts), (b) the kernel's own dispatch-packet timestamps
    # (ppfs_ecc_time_next_launch: hipExtLaunchKernel start / stop events, what rocprofv3's kernel
    # trace measures).  roofline.achieved uses (b), so that it agrees with the committed rocprofv3
    # summary of the same kernel; (a) is reported beside it.
    from paritypartyfs_amd import _native

    NL = _native.lib()
    he = HipEvents(4 * K + 2)
    hk = HipEvents(4 * K)
    t_issue = time.perf_counter()
    for i in range(K):
        he.record(4 * i, stream)
        NL.ppfs_ecc_time_next_launch(hk.ev[4 * i], hk.ev[4 * i + 1])
        eng.encode(data, cw, nblocks=nb)
        NL.ppfs_ecc_time_next_launch(None, None)
        he.record(4 * i + 1, stream)
        inject()
        he.record(4 * i + 2, stream)
        NL.ppfs_ecc_time_next_launch(hk.ev[4 * i + 2], hk.ev[4 * i + 3])
        eng.decode(cw, out, status, write_back=True, nblocks=nb)
        NL.ppfs_ecc_time_next_launch(None, None)
        he.record(4 * i + 3, stream)
    t_issue = (time.perf_counter() - t_issue) / K
    torch.cuda.synchronize()
    enc_ev = [he.ms(4 * i, 4 * i + 1) for i in range(K)]
    inj_ms = [he.ms(4 * i + 1, 4 * i + 2) for i in range(K)]
    dec_ev = [he.ms(4 * i + 2, 4 * i + 3) for i in range(K)]
    enc_ms = [hk.ms(4 * i, 4 * i + 1) for i in range(K)]
    dec_ms = [hk.ms(4 * i + 2, 4 * i + 3) for i in range(K)]
    hk.close()
    enc_avg, dec_avg, inj_avg = float(np.mean(enc_ms)), float(np.mean(dec_ms)), float(np.mean(inj_ms))
    enc_ev_avg, dec_ev_avg = float(np.mean(enc_ev)), float(np.mean(dec_ev))
    # every rank's kernel means (min / max over ranks) and the job's fraction of N x peak
    per_rank, agg = rank_fields({"rank": rank, "encode": enc_avg, "decode": dec_avg}, 2 * (k + n) * nb, world,
                                elapsed, args.steps)
    # device time of the timed region's launch form (same K steps again, two events around them)
    he.record(4 * K, stream)
    run_steps(K)
    he.record(4 * K + 1, stream)
    torch.cuda.synchronize()
    gpu_ms_per_step = he.ms(4 * K, 4 * K + 1) / K
    he.close()

    # (2) standalone kernels: L back-to-back launches of one kernel, fence-free events between
    # them (the north-star measurement: RS encode over the 1 M-block batch on its own).  "hot":
    # every launch on the same buffers, so part of the 261 MB input can still sit in the 256 MB
    # Infinity Cache from the previous launch; "cold": the launches rotate over R independent
    # buffer sets (R x 0.5 GB), so every launch reads its input from HBM.
    L = max(3, args.standalone_launches)
    R = 4
    hs = HipEvents(L + 1)
    hsk = HipEvents(2 * L)
    sa_events = {}  # launch-to-launch stream-event intervals, reported beside the kernel times

    def time_launches(fn, key):
        # kernel durations from the dispatch packets (as in-step above); the stream-event intervals
        # between consecutive launches also contain the gap between kernels
        for i in range(3):
            fn(i)
        hs.record(0, stream)
        for i in range(L):
            NL.ppfs_ecc_time_next_launch(hsk.ev[2 * i], hsk.ev[2 * i + 1])
            fn(i)
            NL.ppfs_ecc_time_next_launch(None, None)
            hs.record(i + 1, stream)
        torch.cuda.synchronize()
        sa_events[key] = round(float(np.median([hs.ms(i, i + 1) for i in range(L)])), 5)
        return [hsk.ms(2 * i, 2 * i + 1) for i in range(L)]

    rewarm(0.3)
    enc_sa = time_launches(lambda i: eng.encode(data, cw, nblocks=nb), "encode_ms_median")
    assert torch.equal(cw, clean_cw), "standalone encode output differs"
    # clean decode (status + write-back enabled, nothing to correct): the read path of a scrub
    rewarm(0.3)
    eng.encode(data, cw, nblocks=nb)
    dec_sa = time_launches(lambda i: eng.decode(cw, out, status, write_back=True, nblocks=nb), "clean_decode_ms_median")
    d_rot = [data] + [torch.randint(0, 256, (nb * k,), dtype=torch.uint8, device=dev, generator=gen)
                      for _ in range(R - 1)]
    c_rot = [torch.empty(nb * n, dtype=torch.uint8, device=dev) for _ in range(R)]
    o_rot = [torch.empty(nb * k, dtype=torch.uint8, device=dev) for _ in range(R)]
    rewarm(0.3)
    enc_cold = time_launches(lambda i: eng.encode(d_rot[i % R], c_rot[i % R], nblocks=nb), "cold_encode_ms_median")
    rewarm(0.3)
    dec_cold = time_launches(lambda i: eng.decode(c_rot[i % R], o_rot[i % R], status, write_back=True, nblocks=nb),
                             "cold_clean_decode_ms_median")
    assert torch.equal(o_rot[1], d_rot[1]), "standalone decode output differs"
    del d_rot, c_rot, o_rot
    hs.close()
    hsk.close()

    # (3) device copy ceiling: the engine's full-grid 16-byte copy kernel over the bytes of one
    # encode (read k, write n per block), timed like the kernels
    cp_src = torch.empty(nb * (k + n) // 2, dtype=torch.uint8, device=dev)
    cp_dst = torch.empty_like(cp_src)
    rewarm(0.3)
    for _ in range(3):
        device_copy(cp_dst, cp_src, stream=stream)
    hc = HipEvents(21)
    hc.record(0, stream)
    for i in range(20):
        device_copy(cp_dst, cp_src, stream=stream)
        hc.record(i + 1, stream)
    torch.cuda.synchronize()
    copy_ms = float(np.median([hc.ms(i, i + 1) for i in range(20)]))
    copy_gbs = 2 * cp_src.numel() / (copy_ms * 1e-3) / 1e9
    # the same copy rotating over 4 source / destination pairs (source bytes from HBM)
    cps = [(torch.empty_like(cp_src), torch.empty_like(cp_src)) for _ in range(3)] + [(cp_src, cp_dst)]
    for i in range(3):
        device_copy(cps[i % 4][1], cps[i % 4][0], stream=stream)
    hc.record(0, stream)
    for i in range(20):
        device_copy(cps[i % 4][1], cps[i % 4][0], stream=stream)
        hc.record(i + 1, stream)
    torch.cuda.synchronize()
    copy_cold_gbs = 2 * cp_src.numel() / (float(np.median([hc.ms(i, i + 1) for i in range(20)])) * 1e-3) / 1e9
    hc.close()
    del cp_src, cp_dst, cps

    alg_per_block = k + n  # 504 B for RS(255,249), both for encode and decode
    alg_launch = alg_per_block * nb
    if (args.block_size, args.t) == (512, 3):
        cfg_ref = "BASELINE configs[1]+[2]"
    elif (args.block_size, args.t) == (4096, 16):
        cfg_ref = "BASELINE configs[4], one GPU's shard"
    else:
        cfg_ref = "not a BASELINE config"
    total_bytes = 2 * alg_launch * world * K
    value = total_bytes / elapsed / GIB
    ms_per_step = elapsed / K * 1e3

    def kname(which):
        kn = eng.kernel_name
        if kn.startswith("rs255-wg-tk"):  # 2t <= 8: ticket kernels (rs_wg_tk.hpp); tkenc: encode only
            tk = which == "encode" or not kn.startswith("rs255-wg-tkenc")
            return f"rs_wg_{which}{'_tk' if tk else ''}_kernel<{n - k}>"
        if kn.startswith("rs255-wg"):
            return f"rs_wg_{which}_kernel<{n - k}>"
        if kn.startswith("rs255-bs"):  # 2t = 32 (rs_bs.hpp)
            return f"rs_bs_{which}_kernel<{n - k}>"
        if kn.startswith("rs255-w1"):  # 2t <= 8, wave-independent ablation (rs_w1.hpp)
            return f"rs_w1_{which}_kernel<{n - k}>"
        if kn.startswith("rs255-pair"):  # 16 < 2t <= 32 (rs_pair.hpp)
            return f"rs_pair_{'decode' if which == 'decode' else 'encode_img'}_kernel<{n - k}>"
        if kn.startswith("rs255-slice8") and which == "encode" and n - k == 16:
            return f"rs_solo_encode_img_kernel<{n - k}>"
        return f"rs255_{which}_kernel<{n - k}>"

    which = "decode" if dec_avg >= enc_avg else "encode"
    dom_ms = max(enc_avg, dec_avg)
    dom_name = kname(which)
    achieved = alg_launch / (dom_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(dom_name, nb)
    frac = lambda ms: round(alg_launch / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)  # noqa: E731

    # (4) host-inclusive rate (north_star: the path starts and ends in host memory): H2D + kernel
    # + D2H through the engine's host entry points, pageable and page-locked, rank 0 at N=1
    host_incl = None
    if args.host_inclusive and rank == 0 and world == 1:
        hd = data.cpu().numpy()
        hraw = np.empty(nb * n, np.uint8)
        hout = np.empty(nb * k, np.uint8)
        hst = np.empty(nb, np.uint8)
        host_incl = {}
        for mode in ("pageable", "pinned"):
            ctx = pinned(hd, hraw, hout, hst) if mode == "pinned" else None
            if ctx:
                ctx.__enter__()
            t_enc, t_dec, ok = [], [], True
            pos = np.arange(nb) * n + (np.arange(nb) * 37) % n
            try:
                eng.encode_host(hd, hraw)  # staging warm
                for _ in range(args.host_reps):  # best of host_reps: one ~20 ms call is at the mercy of the host
                    t1 = time.perf_counter()
                    eng.encode_host(hd, hraw)
                    t_enc.append(time.perf_counter() - t1)
                    hraw[pos] ^= 0x5A  # one error per block
                    t1 = time.perf_counter()
                    eng.decode_host(hraw, hout, hst, write_back=True)
                    t_dec.append(time.perf_counter() - t1)
                    ok = ok and bool(np.array_equal(hout, hd)) and int(hst.min()) == 1
            finally:
                if ctx:
                    ctx.__exit__(None, None, None)
            host_incl[mode] = {"encode_GiBps": round(alg_launch / min(t_enc) / GIB, 3),
                               "decode_1err_GiBps": round(alg_launch / min(t_dec) / GIB, 3), "verified": ok,
                               "reps": args.host_reps}
        try:
            host_incl["link"] = host_link_ceilings(dev, nb, k, n)
        except RuntimeError as e:  # a failed link measurement must not cost the headline line
            host_incl["link"] = {"error": str(e)}
        lk = host_incl["link"]
        for mode in ("pageable", "pinned") if "error" not in lk else ():
            # each call's copies alone, both directions at once over page-locked memory: the ceiling
            # the host path can reach (decode with write-back also returns every changed codeword)
            host_incl[mode]["encode_frac_of_link"] = round(host_incl[mode]["encode_GiBps"] / lk["encode_ceiling_GiBps"], 3)
            host_incl[mode]["decode_1err_frac_of_link"] = round(host_incl[mode]["decode_1err_GiBps"]
                                                                / lk["decode_1err_ceiling_GiBps"], 3)
            # the same against the copies the call makes now (write-back as a patch list, round 6)
            host_incl[mode]["decode_1err_frac_of_patch_link"] = round(host_incl[mode]["decode_1err_GiBps"]
                                                                      / lk["decode_1err_patch_ceiling_GiBps"], 3)
        host_incl["note"] = ("ppfs_ecc_{encode,decode}_host over the same 2^20 blocks: H2D + kernel + D2H wall "
                             "time (best of reps calls), algorithmic bytes; never `value`; *_frac_of_link = rate / "
                             "the call's copies alone over page-locked memory (link) when every changed codeword "
                             "comes back whole (n in, k + n out); *_frac_of_patch_link = against the copies of the "
                             "patch-list write-back the engine uses (n in, k + 8 out)")

    # (5) the other BASELINE configs (driver-visible per-config kernel rates): configs[3] Hamming and
    # CRC 0x9960034c at block_size 4096 and configs[4] RS(255,223), 2^20 blocks each, back-to-back
    # launches of one kernel with a round-trip self-check (tools/bench_configs.py run_config)
    cfg_lines = None
    if args.configs and rank == 0 and world == 1:
        from tools.bench_configs import baseline_configs, run_config

        want = {"cfg4 hamming bs4096": "cfg4_hamming_bs4096", "cfg4 crc32 0x9960034c bs4096": "cfg4_crc_0x9960034c_bs4096",
                "cfg5 rs255_t16 bs4096": "cfg5_rs255_223_bs4096", "cfg2-3 rs255_t3 bs512": "cfg2_3_rs255_249_bs512"}
        cfg_lines = {}
        for name, typ, cbs, ct, poly in baseline_configs():
            if name not in want:
                continue  # (the bench's own workload stays in: its 1-error decode, timed in-step style,
                # must agree with kernels_ms.decode)
            cfg_lines[want[name]] = run_config(name, typ, cbs, ct, poly, 1 << 20, args.config_reps, stream, dev)
        if (args.block_size, args.t) != (4096, 16):
            # configs[4]'s shard in its own bench step (encode -> inject -> decode, K steps): the
            # in-step fractions rocprofv3's profile of `--block-size 4096 --t 16` reproduces
            from tools.bench_configs import step_leg

            cfg_lines["cfg5_step"] = step_leg(4096, 16, 1 << 20, max(10, args.config_reps), dev, stream)
        cfg_lines["note"] = ("BASELINE configs measured outside the timed region: median kernel time over launches "
                             "of one kernel over 2^20 blocks (each kernel's dispatch-packet start / stop), algorithmic "
                             "bytes (payload + raw per block) / time, fraction of 8 TB/s; encodes and clean decodes "
                             "rotate over cold_sets buffer sets (inputs from HBM, not the Infinity Cache); each "
                             "1-error decode is timed right after an untimed encode of the same batch and a "
                             "one-byte-per-block injection, as in the headline step; cfg5_step = configs[4]'s shard "
                             "in its own bench step (per-step kernel means); roundtrip_ok = decode(encode(x)) == x "
                             "with the expected statuses")

    # (6) BASELINE configs[0]: the reference's bench_blockdevice workload on the C++ adapter
    cfg1 = cfg1_leg() if args.configs and rank == 0 and world == 1 else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.block_size, args.t, min(args.cpu_sample_blocks, nb),
                           min(args.cpu_faithful_blocks, nb))

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": K,
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
            **({"rehearsal": f"{world} ranks sharing {torch.cuda.device_count()} GPU(s), barrier / max-reduce "
                             "over gloo: the multi-rank path on real kernels, not a scaling figure"}
               if world > 1 and args.share_gpu else {}),
            "roofline": {
                "bound": "hbm",
                "kernel": dom_name,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": alg_launch,
                "avg_launch_ms": round(dom_ms, 5),
                "timing": "in-step launches, the kernel's dispatch-packet start / stop (hipExtLaunchKernel events, "
                          "as rocprofv3's kernel trace); stream events around the call: kernels_ms_stream_events",
            },
            "cpu_baseline": cpu,
            "configs": cfg_lines,
            "cfg1": cfg1,
            "kernels_ms": {"encode": round(enc_avg, 5), "inject": round(inj_avg, 5), "decode": round(dec_avg, 5)},
            "in_step_frac": {"encode": frac(enc_avg), "decode": frac(dec_avg)},
            # the timed region's algorithmic bytes over all ranks / (N x 8 TB/s), and the
            # in-step kernel means of every rank (rank 0's are kernels_ms)
            **agg,
            "per_rank_kernels_ms": per_rank,
            "kernels_ms_stream_events": {"encode": round(enc_ev_avg, 5), "decode": round(dec_ev_avg, 5),
                                         "in_step_frac_encode": frac(enc_ev_avg), "in_step_frac_decode": frac(dec_ev_avg)},
            "standalone": {
                "launches": L,
                "encode_ms_median": round(float(np.median(enc_sa)), 5),
                "encode_ms_mean": round(float(np.mean(enc_sa)), 5),
                "encode_frac": frac(float(np.median(enc_sa))),
                "clean_decode_ms_median": round(float(np.median(dec_sa)), 5),
                "clean_decode_frac": frac(float(np.median(dec_sa))),
                "cold_encode_ms_median": round(float(np.median(enc_cold)), 5),
                "cold_encode_frac": frac(float(np.median(enc_cold))),
                "cold_clean_decode_ms_median": round(float(np.median(dec_cold)), 5),
                "cold_clean_decode_frac": frac(float(np.median(dec_cold))),
                "stream_event_intervals_ms": sa_events,
                "note": "back-to-back launches of one kernel outside the timed region, each kernel's duration "
                        "from its dispatch packet (stream_event_intervals_ms: fence-free events between the "
                        "launches, gaps included) (north-star: >= 70 % on RS t=3 encode over 1 M blocks); hot = "
                        "same buffers every launch (input partly Infinity-Cache resident), cold = launches "
                        f"rotate over {R} buffer sets (input from HBM)",
            },
            "device_copy_GBps": round(copy_gbs, 1),
            "device_copy_cold_GBps": round(copy_cold_gbs, 1),
            "device_copy_kernel": "ppfs_copy_device (full-grid 16-B copy, same bytes as one encode)",
            # payload rate beside the algorithmic one, and the dominant kernel
            # against the device-to-device copy measured above
            "payload_GiBps": round(value * k / alg_per_block, 3),
            "roofline_frac_of_device_copy": round(achieved / copy_gbs, 4) if copy_gbs else None,
            "host_inclusive": host_incl,
            "kernel_path": eng.stream_kernel_name(stream),
            "collectives": ("rccl max-reduce, gloo barriers" if dist.is_initialized() and dist.get_backend() == "nccl"
                            else "gloo" if dist.is_initialized() else "none (single process, no torchrun)"),
            "launch": f"hipGraph of {group} steps" if graph is not None else "eager",
            "host_issue_us_per_eager_step": round(t_issue * 1e6, 1),
            "device_ms_per_step": round(gpu_ms_per_step, 4),
            "repeat_ms_per_step": [round(x, 4) for x in repeats],
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
