#!/bin/bash
# GPU box: early DMA in the byte-slice cfg5 kernels (default build) against the build without it
# (alt noed): GPU suite, then cfg5 bench A/B.  Usage: tools/gpu_ed.sh <tag>
set -o pipefail
TAG=${1:-ed}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/gpu_ab_bench.sh "--block-size 4096 --t 16" noed || exit 1
