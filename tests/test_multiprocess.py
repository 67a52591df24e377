"""N>1 path on CPU: two gloo ranks run bench.py's timed region (tests the barrier / max-over-ranks
timing the driver's multi-GPU bench relies on; the data path has no collective to test)."""
import os
import socket
import sys
import time

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    # rank r's step sleeps (r+1) * 20 ms: the reported time must be the slowest rank's
    el = bench.timed_steps(lambda: time.sleep(0.02 * (rank + 1)), 3, world, lambda: None, None)
    q.put((rank, el))
    dist.destroy_process_group()


def test_gloo_world2_max_over_ranks():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    res = dict(q.get() for _ in range(world))
    assert abs(res[0] - res[1]) < 1e-9  # every rank reports the max
    assert res[0] >= 3 * 0.02 * world * 0.95


def test_bench_gpus2_launches_two_ranks():
    """The driver's command form `python bench.py --gpus 2` starts two ranks itself (torchrun as a
    child process) and reports n_gpus 2 with the slowest rank's time.  The engine is replaced by
    bench.py's CPU stand-in (--dry-run-cpu, gloo): this exercises the launcher, the barrier and the
    max-over-ranks, not the kernels."""
    import json
    import subprocess

    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5",
                        "--warmup", "1", "--dry-run-cpu"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 2 and line["dry_run"] and line["steps"] == 5
    assert line["ms_per_step"] >= 2.0 * 0.95  # rank 1's stand-in sleeps 2 ms per step
    # SURVEY 8(e) fields of the N-rank line: every rank's kernel times, the job's fraction of N x peak
    per = line["per_rank_kernels_ms"]
    assert line["ranks_reporting"] == 2 and len(per["decode"]["by_rank"]) == 2
    assert per["decode"]["min"] <= per["decode"]["max"] and per["decode"]["max"] >= 2.0 * 0.95
    assert per["decode"]["by_rank"][1] > per["decode"]["by_rank"][0]  # rank 1 sleeps twice as long
    assert line["aggregate_peak_GBps"] == 2 * 8000.0
    exp = line["aggregate_bytes"] / (line["ms_per_step"] * 1e-3 * 5) / 1e9 / (2 * 8000.0)
    assert line["aggregate_bytes"] == 2 * 504 * (1 << 20) * 2 * 5
    assert abs(line["aggregate_frac"] - exp) <= 1e-3 * exp + 1e-4


def test_bench_gpus2_argv_reaches_every_rank():
    """The driver's configs[4] form `python bench.py --gpus 2 --block-size 4096 --t 16`: the launcher
    passes the argv to every rank unchanged (each rank reports what it parsed, all_gather over gloo)."""
    import json
    import subprocess

    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--block-size", "4096", "--t", "16", "--blocks", "12345", "--dry-run-cpu"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    ranks = sorted(line["rank_args"], key=lambda a: a["rank"])
    assert [a["rank"] for a in ranks] == [0, 1]
    assert all(a["block_size"] == 4096 and a["t"] == 16 and a["blocks"] == 12345 for a in ranks)


def test_bench_torchrun_world1_runs_collectives():
    """Under torchrun at WORLD_SIZE=1 the timed region still runs the barrier and the max-reduce (the
    code path of the N-GPU run); here with the CPU stand-in over gloo."""
    import json
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--dry-run-cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=dict(os.environ))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert line["n_gpus"] == 1 and len(line["rank_args"]) == 1


def test_bench_rejects_world_mismatch():
    import subprocess

    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--dry-run-cpu"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_bench_gpus4_cfg5_shape():
    """configs[4]'s command shape at four ranks, `python bench.py --gpus 4 --block-size 4096 --t 16`
    (CPU stand-in over gloo): every rank reports, the job's blocks are 4 x 2^20 RS(255,223)
    codewords, and aggregate_frac is taken against 4 x 8 TB/s."""
    import json
    import subprocess

    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "3", "--warmup", "1",
                        "--block-size", "4096", "--t", "16", "--dry-run-cpu"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 4 and line["ranks_reporting"] == 4
    assert line["config"]["global_blocks"] == 4 * (1 << 20) and line["config"]["blocks_per_gpu"] == 1 << 20
    assert "RS(255,223)" in line["config"]["workload"]
    per = line["per_rank_kernels_ms"]
    assert all(len(per[key]["by_rank"]) == 4 for key in ("encode", "decode"))
    assert per["decode"]["by_rank"][3] > per["decode"]["by_rank"][0]  # rank r's stand-in sleeps (r + 1) ms
    assert line["aggregate_peak_GBps"] == 4 * 8000.0
    assert line["aggregate_bytes"] == 2 * 478 * (1 << 20) * 4 * 3
    exp = line["aggregate_bytes"] / (line["ms_per_step"] * 1e-3 * 3) / 1e9 / (4 * 8000.0)
    assert abs(line["aggregate_frac"] - exp) <= 1e-3 * exp + 1e-4
    assert sorted(a["rank"] for a in line["rank_args"]) == [0, 1, 2, 3]
    assert all(a["block_size"] == 4096 and a["t"] == 16 for a in line["rank_args"])
