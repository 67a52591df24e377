#!/bin/bash
# Round 5: RS decodes with the status bytes stored after the tile's emission (lease libs: rslate = both
# knobs, for the GPU suite; tklate: -DPPFS_TK_LATE_ST=1, the t <= 4 decode; bslate: -DPPFS_BS_LATE_ST=1,
# the cfg5 decode) against the same build without (base): bench steps, interleaved
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
PPFS_ECC_LIB=$L/libppfs_ecc_rslate.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5rsl_test.log 2>&1 || { tail -5 gpurun_out/r5rsl_test.log; exit 1; }
tail -1 gpurun_out/r5rsl_test.log
for r in 1 2 3; do
  for lib in $L/libppfs_ecc_base.so $L/libppfs_ecc_tklate.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5rsl_tmp.json 2> gpurun_out/r5rsl_bench.err || { tail -5 gpurun_out/r5rsl_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5rsl_tmp.json >> gpurun_out/r5rsl_tk_ab.jsonl
  done
  for lib in $L/libppfs_ecc_base.so $L/libppfs_ecc_bslate.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py --block-size 4096 --t 16 --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5rsl_tmp.json 2> gpurun_out/r5rsl_bench.err || { tail -5 gpurun_out/r5rsl_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5rsl_tmp.json >> gpurun_out/r5rsl_bs_ab.jsonl
  done
done
cat gpurun_out/r5rsl_tk_ab.jsonl gpurun_out/r5rsl_bs_ab.jsonl
