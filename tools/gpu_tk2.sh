#!/bin/bash
# GPU box: the ticket decode (default build) against the encode-only ticket build (alt tkenc):
# GPU suite on the default build, then kernel and bench A/B.  Usage: tools/gpu_tk2.sh <tag>
set -o pipefail
TAG=${1:-tk2}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/gpu_dyn2.sh $TAG tkenc || exit 1
timeout -k 10 900 bash tools/gpu_ab_bench.sh "" tkenc || exit 1
