#!/bin/bash
# GPU box (round 3): cfg5 decode variants (t = 16 RS GPU tests on each, then the interleaved cfg5
# bench A/B), and the phase traces of the t = 3 encode / decode and the 2t = 32 decode.
# Usage: VARIANTS="d12 d10 ..." tools/gpu_r3h.sh <tag>     (variants built by tools/build_alt.sh)
set -o pipefail
TAG=${1:-r3h}
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
      --timeout 120 --timeout-method thread -m gpu -k "rs and 16" > gpurun_out/${TAG}_${v}_tests.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/${TAG}_${v}_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 bash tools/ab_bench.sh ${TAG}_cfg5ab --block-size 4096 --t 16 > gpurun_out/${TAG}_cfg5ab.txt 2>&1 || { tail gpurun_out/${TAG}_cfg5ab.txt; exit 1; }
cat gpurun_out/${TAG}_cfg5ab.txt
if [ -f paritypartyfs_amd/_lib/alt/libppfs_ecc_trace.so ]; then
  T=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_trace.so
  PPFS_ECC_LIB=$T timeout -k 10 120 python tools/tk_trace.py > gpurun_out/${TAG}_tktrace.jsonl 2>&1 || { tail gpurun_out/${TAG}_tktrace.jsonl; exit 1; }
  PPFS_ECC_LIB=$T timeout -k 10 120 python tools/tk_trace.py --standalone >> gpurun_out/${TAG}_tktrace.jsonl 2>&1 || { tail gpurun_out/${TAG}_tktrace.jsonl; exit 1; }
  PPFS_ECC_LIB=$T timeout -k 10 120 python tools/bs_trace.py > gpurun_out/${TAG}_bstrace.jsonl 2>&1 || { tail gpurun_out/${TAG}_bstrace.jsonl; exit 1; }
  cat gpurun_out/${TAG}_tktrace.jsonl gpurun_out/${TAG}_bstrace.jsonl
fi
