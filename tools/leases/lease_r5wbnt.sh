#!/bin/bash
# Round 5: the RS decodes' corrected-byte write-backs as non-temporal byte stores (lease lib wbnt:
# -DPPFS_WB_NT=1; RS GPU tests on it first) against the same build without (base): headline and cfg5 bench steps, interleaved
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
PPFS_ECC_LIB=$L/libppfs_ecc_wbnt.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "rs or RS or 255 or t16 or scrub" > gpurun_out/r5wbnt_test.log 2>&1 || { tail -5 gpurun_out/r5wbnt_test.log; exit 1; }
tail -1 gpurun_out/r5wbnt_test.log
for r in 1 2 3; do
  for lib in $L/libppfs_ecc_base.so $L/libppfs_ecc_wbnt.so; do
    for cfg in "" "--block-size 4096 --t 16"; do
      PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py $cfg --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/r5wbnt_tmp.json 2> gpurun_out/r5wbnt_bench.err || { tail -5 gpurun_out/r5wbnt_bench.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'cfg': sys.argv[4], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5wbnt_tmp.json "${cfg:-t3}" >> gpurun_out/r5wbnt_ab.jsonl
    done
  done
done
cat gpurun_out/r5wbnt_ab.jsonl
