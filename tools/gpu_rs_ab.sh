#!/bin/bash
# GPU box: RS correctness on the current build, then the bench A/B against alt builds.
# Usage: VARIANTS="base ..." tools/gpu_rs_ab.sh <tag>
set -o pipefail
TAG=${1:-rsab}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hygiene.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rs or full_size or group or destroy" > gpurun_out/${TAG}_t.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_t.log | head; exit $rc; }
bash tools/ab_bench.sh $TAG
