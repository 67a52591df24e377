#!/bin/bash
# Round 5: cfg5 decode with the single error's HBM write-back deferred to after the tile's emission
# (lease lib bswb: -DPPFS_BS_LATE_WB=1; GPU suite on it first) and a second look at the t <= 4 decode's late
# status bytes (tklate: -DPPFS_TK_LATE_ST=1), against the same build without (base): bench steps, interleaved
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
PPFS_ECC_LIB=$L/libppfs_ecc_bswb.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "rs or RS or t16 or 255" > gpurun_out/r5rswb_test.log 2>&1 || { tail -5 gpurun_out/r5rswb_test.log; exit 1; }
tail -1 gpurun_out/r5rswb_test.log
for r in 1 2 3 4; do
  for lib in $L/libppfs_ecc_base.so $L/libppfs_ecc_tklate.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5rswb_tmp.json 2> gpurun_out/r5rswb_bench.err || { tail -5 gpurun_out/r5rswb_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5rswb_tmp.json >> gpurun_out/r5rswb_tk_ab.jsonl
  done
done
for r in 1 2 3; do
  for lib in $L/libppfs_ecc_base.so $L/libppfs_ecc_bswb.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py --block-size 4096 --t 16 --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5rswb_tmp.json 2> gpurun_out/r5rswb_bench.err || { tail -5 gpurun_out/r5rswb_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5rswb_tmp.json >> gpurun_out/r5rswb_bs_ab.jsonl
  done
done
cat gpurun_out/r5rswb_tk_ab.jsonl gpurun_out/r5rswb_bs_ab.jsonl
