#!/bin/bash
# GPU box: parity of an alt build (RS device tests) then kernel + bench A/B against the current build.
# Usage: VARIANTS="rp4" tools/gpu_rp.sh <tag>
set -o pipefail
TAG=$1
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
      --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_hygiene.py > gpurun_out/${TAG}_pytest_$v.log 2>&1 \
      || { tail -30 gpurun_out/${TAG}_pytest_$v.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest_$v.log
done
VARIANTS="${VARIANTS}" bash tools/gpu_kablate.sh ${TAG}_k || exit 1
VARIANTS="${VARIANTS}" bash tools/ab_bench.sh ${TAG}_ab || exit 1
