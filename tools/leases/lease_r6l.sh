# round 6, lease l: cfg5 encode with register prefetch of the next tile (NBUF 0, tickets) vs the
# shipped single-image DMA encode (NBUF 1) in the cfg5 bench step, 3 interleaved rounds; t16 parity
# tests on the variant
set -o pipefail
mkdir -p gpurun_out
L=$PWD/paritypartyfs_amd/_lib/lease
PPFS_ECC_LIB=$L/libppfs_ecc_enc0.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "16 or 4096" > gpurun_out/r6l_enc0_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6l_enc0_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r6l_cfg5_enc_ab.jsonl; : > $out
for rnd in 1 2 3; do
for v in base enc0; do
  if [ $v = base ]; then lib=""; else lib="PPFS_ECC_LIB=$L/libppfs_ecc_$v.so"; fi
  env $lib timeout -k 10 200 python bench.py --block-size 4096 --t 16 --steps 50 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/r6l_tmp.json 2>/dev/null || { echo "fail $v"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r6l_tmp.json').read().strip().splitlines()[-1]);print(json.dumps({'variant':'$v','round':$rnd,'value':d['value'],'ms_per_step':d['ms_per_step'],'kernels_ms':d['kernels_ms'],'in_step_frac':d['in_step_frac']}))" >> $out
done
done
cat $out
