#!/bin/bash
# GPU box: CRC (and Hamming) tests on each variant build, then interleaved per-config kernel rates
# (tools/bench_configs.py --only crc) of the current build ("new") and the variants.
# Usage: VARIANTS="a b" tools/gpu_crc_ab.sh <tag>
set -o pipefail
TAG=${1:-crcab}
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
      --timeout 120 --timeout-method thread -m gpu -k "crc or full_size" > gpurun_out/${TAG}_${v}_tests.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/${TAG}_${v}_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do
for v in new ${VARIANTS}; do
  if [ $v = new ]; then L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; else L=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 120 python tools/bench_configs.py --only crc > gpurun_out/${TAG}_${v}_$r.jsonl 2>> gpurun_out/${TAG}.err || exit 1
  python3 -c "
import json
for l in open('gpurun_out/${TAG}_${v}_$r.jsonl'):
    d = json.loads(l)
    print('%8s r$r %-28s enc %.4f ms  chk %.4f ms' % ('$v', d['config'], d.get('encode_ms', 0), d.get('decode_clean_ms', 0)))"
done
done
