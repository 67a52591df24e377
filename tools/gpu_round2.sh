#!/bin/bash
# GPU box (round 2): full GPU suite (fault guard on), the default bench line, the graph-launch
# variant of the same line, then rocprofv3 trace + PMC passes of the bench.
# Usage: tools/gpu_round2.sh <tag> [skip-prof]
set -o pipefail
TAG=${1:-r2}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/${TAG}_pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; tail -c 3000 gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --launch graph --no-cpu-baseline --no-host-inclusive > gpurun_out/${TAG}_bench_graph.json 2> gpurun_out/${TAG}_bench_graph.err || exit 1
[ "$2" = "skip-prof" ] && exit 0
timeout -k 10 900 bash tools/profile_box.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; tail gpurun_out/${TAG}_prof.log; exit 1; }
echo done
