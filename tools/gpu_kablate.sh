#!/bin/bash
# GPU box: tools/kernel_ablate.py over the current build and alt builds, rounds interleaved.
# Usage: VARIANTS="a b" tools/gpu_kablate.sh <tag> [kernel_ablate args]
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for r in 1 2; do
for v in new ${VARIANTS}; do
  if [ $v = new ]; then L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; else L=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 120 python tools/kernel_ablate.py --tag $v "$@" >> gpurun_out/${TAG}.jsonl 2>> gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  tail -1 gpurun_out/${TAG}.jsonl
done
done
