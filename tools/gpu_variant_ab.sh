#!/bin/bash
# GPU box: parity tests selected by -k on each variant build (_lib/alt/libppfs_ecc_<v>.so), then the
# interleaved bench A/B (tools/ab_bench.sh) of the current build against them.
# Usage: VARIANTS="a b" KSEL="<pytest -k expr>" tools/gpu_variant_ab.sh <tag> [bench args]
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so timeout -k 10 300 python -u -m pytest tests -x -q \
      --timeout 120 --timeout-method thread -m gpu -k "$KSEL" > gpurun_out/${TAG}_${v}_tests.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/${TAG}_${v}_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 bash tools/ab_bench.sh ${TAG}_ab "$@" > gpurun_out/${TAG}_ab.txt 2>&1 || { tail gpurun_out/${TAG}_ab.txt; exit 1; }
cat gpurun_out/${TAG}_ab.txt
