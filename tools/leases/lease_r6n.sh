# round 6, lease n: cfg5 decode with the general path called between two tile loops (no callee-saved
# VGPRs in the tile loop: 8-wave kernel 155 own VGPRs, was 249), which lets it run more waves:
# t16 parity tests on the shipped 8-wave form and the 12-wave form, then the cfg5 bench step A/B:
# old (round-6 final) / base (8 waves) / w12p (12, register prefetch, tables in L2) / w12d (12, DMA) /
# w11p (11, GF in LDS) / w10p (10, GF + XP rows in LDS), 2 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
L=$PWD/paritypartyfs_amd/_lib/lease
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "16 or 4096" > gpurun_out/r6n_base_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6n_base_tests.log; [ $rc -eq 0 ] || exit $rc
PPFS_ECC_LIB=$L/libppfs_ecc_w12p.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "16 or 4096" > gpurun_out/r6n_w12p_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6n_w12p_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r6n_cfg5_waves_ab.jsonl; : > $out
for rnd in 1 2; do
for v in old base w12p w12d w11p w10p; do
  if [ $v = base ]; then lib=""; else lib="PPFS_ECC_LIB=$L/libppfs_ecc_$v.so"; fi
  env $lib timeout -k 10 200 python bench.py --block-size 4096 --t 16 --steps 50 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/r6n_tmp.json 2>gpurun_out/r6n_tmp.err || { echo "fail $v"; tail -5 gpurun_out/r6n_tmp.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r6n_tmp.json').read().strip().splitlines()[-1]);print(json.dumps({'variant':'$v','round':$rnd,'value':d['value'],'ms_per_step':d['ms_per_step'],'kernels_ms':d['kernels_ms'],'in_step_frac':d['in_step_frac']}))" >> $out
done
done
cat $out
