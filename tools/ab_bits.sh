set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "crc or hamming or parity or bit" > gpurun_out/bits_t.log 2>&1
rc=$?; tail -3 gpurun_out/bits_t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in base new; do
  if [ $v = base ]; then L=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_base.so; else L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; fi
  for c in hamming crc32 parity; do
    PPFS_ECC_LIB=$L timeout -k 10 120 python tools/bench_configs.py --only $c > gpurun_out/abdpp_${v}_${c}_$r.log 2>&1 || exit 1
  done
done
done
grep -h config gpurun_out/abdpp_* | cut -c1-400
