#!/bin/bash
# GPU box: RS GPU tests on each variant build, then interleaved bench A/B rounds for the default
# (t = 3) line and the cfg5 (t = 16) line.
# Usage: V3="a b" V16="c d" KSEL3="<-k expr>" tools/gpu_ab2.sh <tag>   (builds: tools/build_alt.sh)
set -o pipefail
TAG=${1:-ab2}
mkdir -p gpurun_out
for v in ${V3} ${V16}; do
  PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
      --timeout 120 --timeout-method thread -m gpu -k "${KSEL:-rs}" > gpurun_out/${TAG}_${v}_tests.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/${TAG}_${v}_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
if [ -n "$V3" ]; then
  VARIANTS="$V3" timeout -k 10 600 bash tools/ab_bench.sh ${TAG}_t3 > gpurun_out/${TAG}_t3.txt 2>&1 || { tail gpurun_out/${TAG}_t3.txt; exit 1; }
  cat gpurun_out/${TAG}_t3.txt
fi
if [ -n "$V16" ]; then
  VARIANTS="$V16" timeout -k 10 600 bash tools/ab_bench.sh ${TAG}_t16 --block-size 4096 --t 16 > gpurun_out/${TAG}_t16.txt 2>&1 || { tail gpurun_out/${TAG}_t16.txt; exit 1; }
  cat gpurun_out/${TAG}_t16.txt
fi
