#!/bin/bash
# Round 5: the N > 1 bench path rehearsed on the one-GPU box (two ranks sharing the card over RCCL,
# --share-gpu): the multi-rank JSON line (per-rank kernel times, aggregate fraction) end to end
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 2 --share-gpu --steps 30 --warmup 5 --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5n2_bench.json 2> gpurun_out/r5n2_bench.err || { tail -20 gpurun_out/r5n2_bench.err; exit 1; }
tail -1 gpurun_out/r5n2_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','n_gpus','ms_per_step','aggregate_frac','per_rank_kernels_ms','ranks_reporting','collectives') if k in d})"
