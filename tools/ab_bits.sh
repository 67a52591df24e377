# GPU box: bit-codec tests (CRC / Hamming / parity, incl. block-device sequences) on the current
# build, then a cfg4 A/B of the current build against _lib/alt/libppfs_ecc_base.so (codecs: $@)
set -o pipefail
mkdir -p gpurun_out
CODECS=${@:-hamming crc32 parity}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_block_device.py -x -q --timeout 120 --timeout-method thread -m gpu -k "crc or hamming or parity or bit or full_size" > gpurun_out/bits_t.log 2>&1
rc=$?; tail -3 gpurun_out/bits_t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in base new; do
  if [ $v = base ]; then L=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_base.so; else L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; fi
  for c in $CODECS; do
    PPFS_ECC_LIB=$L timeout -k 10 120 python tools/bench_configs.py --only $c > gpurun_out/abbf_${v}_${c}_$r.log 2>&1 || exit 1
  done
done
done
for f in gpurun_out/abbf_*; do echo $f; grep config $f | cut -c150-360; done
