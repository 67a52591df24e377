# round 6, lease k: deferred-correction cfg5 decode (rs_bs.hpp rs_bs_decode_dc_kernel) -- parity tests on
# the DMA form (dc2, lease library), then the cfg5 bench step A/B: shipped / dc2 (NBUF 1) / dc1 (NBUF 0)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/paritypartyfs_amd/_lib/lease
PPFS_ECC_LIB=$L/libppfs_ecc_dc2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_block_device.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r6k_dc2_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6k_dc2_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r6k_cfg5_dc_ab.jsonl; : > $out
for rnd in 1 2; do
for v in base dc2 dc1; do
  if [ $v = base ]; then lib=""; else lib="PPFS_ECC_LIB=$L/libppfs_ecc_$v.so"; fi
  env $lib timeout -k 10 200 python bench.py --block-size 4096 --t 16 --steps 50 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/r6k_tmp.json 2>/dev/null || { echo "fail $v"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r6k_tmp.json').read().strip().splitlines()[-1]);print(json.dumps({'variant':'$v','round':$rnd,'value':d['value'],'ms_per_step':d['ms_per_step'],'kernels_ms':d['kernels_ms'],'in_step_frac':d['in_step_frac']}))" >> $out
done
done
cat $out
