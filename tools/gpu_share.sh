#!/bin/bash
# GPU box: the multi-rank bench path on real kernels with N ranks sharing the box's one GPU
# (bench.py --share-gpu: gloo barrier / max-reduce).  Usage: tools/gpu_share.sh <tag>
set -o pipefail
TAG=${1:-share}
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --share-gpu --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive \
      > gpurun_out/${TAG}_n$n.json 2> gpurun_out/${TAG}_n$n.err || { tail -20 gpurun_out/${TAG}_n$n.err; exit 1; }
  tail -c 700 gpurun_out/${TAG}_n$n.json; echo
done
