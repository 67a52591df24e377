#!/bin/bash
# GPU box: kernel-only A/B of the dynamic-tile encode variants.  Usage: tools/gpu_dyn2.sh <tag> <variants...>
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
A=$PWD/paritypartyfs_amd/_lib/alt
for r in 1 2; do
for v in default "$@"; do
  if [ $v = default ]; then L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; else L=$A/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 120 python tools/kernel_ablate.py --tag $v >> gpurun_out/${TAG}_kablate.jsonl 2>> gpurun_out/${TAG}_kablate.err || { tail -5 gpurun_out/${TAG}_kablate.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_kablate.jsonl').read().strip().splitlines()[-1]); print(d['tag'], 'enc hot/cold', d['enc_hot_us'], d['enc_cold_us'], 'dec hot/cold', d['dec_hot_us'], d['dec_cold_us'])"
done
done
