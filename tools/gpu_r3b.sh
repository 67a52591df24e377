#!/bin/bash
# GPU box (round 3): normal-build GPU suite, then the same suite on the bounds- and copy-checked
# PPFS_ECC_DEBUG build (tools/build_alt.sh --product debug -DPPFS_ECC_DEBUG=1).
set -o pipefail
TAG=${1:-r3b}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_gputest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_gputest.log | head -20; exit $rc; }
timeout -k 10 900 bash tools/gpu_debug_suite.sh ${TAG}_debug || exit 1
