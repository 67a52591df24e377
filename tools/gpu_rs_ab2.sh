#!/bin/bash
# GPU box: RS tests on the current build, standalone kernel A/B and bench A/B against alt builds.
set -o pipefail
TAG=${1:-rsab}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hygiene.py tests/test_gpu_block_device.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rs or full_size or group or destroy or scrub or block" > gpurun_out/${TAG}_t.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_t.log | head; exit $rc; }
bash tools/gpu_kablate.sh ${TAG}_k || exit 1
bash tools/ab_bench.sh ${TAG}_b
