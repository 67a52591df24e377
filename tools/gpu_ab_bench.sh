# GPU box: bench A/B of alternative library builds: tools/gpu_ab_bench.sh "<bench args>" variant...
set -o pipefail
mkdir -p gpurun_out
ARGS=$1; shift
for v in default "$@" default "$@"; do
  if [ $v = default ]; then L=""; else L=paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 200 python bench.py $ARGS --no-cpu-baseline --no-host-inclusive > gpurun_out/bench_ab.log 2>&1 || { tail -3 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['kernels_ms'], d['standalone']['clean_decode_ms_median'], d['standalone']['cold_clean_decode_ms_median'])" | tee -a gpurun_out/bench_ab.txt
done
