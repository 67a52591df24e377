#!/bin/bash
# GPU box (round 3): records of the current tree in two parts, each one gpurun call.
#   part A: normal GPU suite, checked GPU suite (PPFS_ECC_DEBUG + PPFS_ECC_SYNC_CHECK), smoke, the
#           driver's default bench line, a torchrun world-1 line (the RCCL branch SCALE runs)
#   part B: rocprofv3 trace + PMC of the default bench, the cfg5 bench line, per-config kernel rates
# Usage: tools/gpu_r3g.sh <tag> A|B     (build first: __graft_entry__.build(), tools/build_alt.sh
#        --product debug -DPPFS_ECC_DEBUG=1)
set -o pipefail
TAG=${1:-r3g}
PART=${2:-A}
mkdir -p gpurun_out
if [ "$PART" = A ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_gputest.log 2>&1
  rc=$?; tail -2 gpurun_out/${TAG}_gputest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_gputest.log | head -20; exit $rc; }
  timeout -k 10 600 bash tools/gpu_debug_suite.sh ${TAG}_debug_suite || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('kernels_ms'))"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/${TAG}_torchrun1_bench.json 2> gpurun_out/${TAG}_torchrun1_bench.err
  rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_torchrun1_bench.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_torchrun1_bench.json').read().strip().splitlines()[-1]); print('torchrun', d['value'], d['ms_per_step'], d.get('collectives'))"
else
  timeout -k 10 900 bash tools/profile_box.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; tail gpurun_out/${TAG}_prof.log; exit 1; }
  echo profiled
  timeout -k 10 300 python bench.py --block-size 4096 --t 16 > gpurun_out/${TAG}_bench_cfg5.json 2> gpurun_out/${TAG}_bench_cfg5.err || { tail -3 gpurun_out/${TAG}_bench_cfg5.err; exit 1; }
  echo bench_cfg5
  timeout -k 10 300 python tools/bench_configs.py > gpurun_out/${TAG}_configs.jsonl 2> gpurun_out/${TAG}_configs.err || { tail gpurun_out/${TAG}_configs.err; exit 1; }
  echo configs
fi
