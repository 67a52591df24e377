# round 6, lease r: the cfg5 chain with the row's payload bytes in registers (rs_bs.hpp
# bs_remainder_rows: copied out of the image once per tile, chunks by DPP from the holder lane; no
# per-step row reads) -- t16 parity tests on the variant, then the cfg5 bench step A/B: base /
# rows3 (encode + decode) / rows1 (encode only) / rows2 (decode only), 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
L=$PWD/paritypartyfs_amd/_lib/lease
PPFS_ECC_LIB=$L/libppfs_ecc_rows3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "16 or 4096" > gpurun_out/r6r_rows3_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6r_rows3_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r6r_cfg5_rows_ab.jsonl; : > $out
for rnd in 1 2 3; do
for v in base rows3 rows1 rows2; do
  if [ $v = base ]; then lib=""; else lib="PPFS_ECC_LIB=$L/libppfs_ecc_$v.so"; fi
  env $lib timeout -k 10 200 python bench.py --block-size 4096 --t 16 --steps 50 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/r6r_tmp.json 2>gpurun_out/r6r_tmp.err || { echo "fail $v"; tail -5 gpurun_out/r6r_tmp.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r6r_tmp.json').read().strip().splitlines()[-1]);print(json.dumps({'variant':'$v','round':$rnd,'value':d['value'],'ms_per_step':d['ms_per_step'],'kernels_ms':d['kernels_ms'],'in_step_frac':d['in_step_frac']}))" >> $out
done
done
cat $out
