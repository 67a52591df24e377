# GPU box: wave-independent t<=4 kernels -- RS parity tests per variant library, kernel timings, bench A/B
set -o pipefail
mkdir -p gpurun_out
for v in ${W1_VARIANTS:-w1 w1rp}; do
  PPFS_ECC_LIB=paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rs" > gpurun_out/pytest_w1_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/pytest_w1_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in default ${W1_KVARIANTS:-w1 w1rp w1m0} default; do
  if [ $v = default ]; then L=""; else L=paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 200 python tools/kernel_ablate.py --block-size 512 --t 3 --tag $v >> gpurun_out/w1_kablate.jsonl 2>gpurun_out/w1_kablate.err || { tail gpurun_out/w1_kablate.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/w1_kablate.jsonl'):
    d=json.loads(l); print(d['tag'], d['enc_hot_us'], d['enc_cold_us'], d['dec_hot_us'], d['dec_cold_us'], d['dec_1err_nowb_hot_us'])"
for v in default ${W1_BVARIANTS:-w1 w1rp} default; do
  if [ $v = default ]; then L=""; else L=paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-inclusive > gpurun_out/bench_w1_$v.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/bench_w1_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['kernels_ms'], d['standalone']['encode_ms_median'], d['standalone']['cold_encode_ms_median'])"
done
