#!/bin/bash
# Round 5: the t <= 4 decode with a single error's HBM write-back stored after wave 0's emission (lease lib
# tkwb: -DPPFS_TK_LATE_WB=1; GPU RS tests on it first) against the same build without (base): bench steps, interleaved
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
PPFS_ECC_LIB=$L/libppfs_ecc_tkwb.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "rs or RS or 255 or lifecycle or scrub" > gpurun_out/r5tkwb_test.log 2>&1 || { tail -5 gpurun_out/r5tkwb_test.log; exit 1; }
tail -1 gpurun_out/r5tkwb_test.log
for r in 1 2 3 4 5; do
  for lib in $L/libppfs_ecc_base.so $L/libppfs_ecc_tkwb.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5tkwb_tmp.json 2> gpurun_out/r5tkwb_bench.err || { tail -5 gpurun_out/r5tkwb_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5tkwb_tmp.json >> gpurun_out/r5tkwb_ab.jsonl
  done
done
cat gpurun_out/r5tkwb_ab.jsonl
