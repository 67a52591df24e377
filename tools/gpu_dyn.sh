#!/bin/bash
# GPU box: dynamic-tile encode (PPFS_WG_DYN) -- GPU suite on the dyn build, kernel-only A/B of
# the skeletons (MODE 0) and full kernels, then the bench line A/B.  Usage: tools/gpu_dyn.sh <tag>
set -o pipefail
TAG=${1:-dyn}
mkdir -p gpurun_out
A=$PWD/paritypartyfs_amd/_lib/alt
PPFS_ECC_LIB=$A/libppfs_ecc_dyn.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "(rs or RS or server or parity) and not group and not host" > gpurun_out/${TAG}_test.log 2>&1 || { tail -30 gpurun_out/${TAG}_test.log; exit 1; }
tail -1 gpurun_out/${TAG}_test.log
for r in 1 2; do
for v in default dyn st_m0 dyn_m0; do
  if [ $v = default ]; then L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; else L=$A/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 120 python tools/kernel_ablate.py --tag $v >> gpurun_out/${TAG}_kablate.jsonl 2>> gpurun_out/${TAG}_kablate.err || { tail -5 gpurun_out/${TAG}_kablate.err; exit 1; }
  tail -1 gpurun_out/${TAG}_kablate.jsonl
done
done
R=3 VARIANTS="dyn" bash tools/ab_bench_full.sh ${TAG}ab
