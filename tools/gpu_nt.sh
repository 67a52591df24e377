# GPU box: non-temporal write-back / inject stores -- decode tests on the wbnt build, bench A/B (t=3 and t=16)
set -o pipefail
mkdir -p gpurun_out
PPFS_ECC_LIB=paritypartyfs_amd/_lib/alt/libppfs_ecc_both.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hygiene.py -x -q --timeout 120 --timeout-method thread -m gpu -k "decode or inject or many_tiles or full_size" > gpurun_out/pytest_nt.log 2>&1
rc=$?; echo "both: $(tail -1 gpurun_out/pytest_nt.log)"; [ $rc -eq 0 ] || exit $rc
for cfg in "--t 3" "--block-size 4096 --t 16"; do
for v in default wbnt injnt both default; do
  if [ $v = default ]; then L=""; else L=paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 200 python bench.py $cfg --no-cpu-baseline --no-host-inclusive > gpurun_out/bench_nt.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/bench_nt.log').read().strip().splitlines()[-1]); print('$cfg $v', d['value'], d['ms_per_step'], d['kernels_ms'], d['repeat_ms_per_step'])" | tee -a gpurun_out/bench_nt.txt
done
done
