# GPU box: bit-codec tests on the current build, then cfg4 rates of builds that differ in blocks
# per wave (BF_BPW for Hamming / parity; base = HEAD build): _lib/alt/libppfs_ecc_<v>.so, two rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_block_device.py tests/test_vote_scrub.py -x -q --timeout 120 --timeout-method thread -m gpu -k "crc or hamming or parity or bit or full_size or scrub" > gpurun_out/bpw_t.log 2>&1
rc=$?; tail -2 gpurun_out/bpw_t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in ${VARIANTS:-base new bf2 bf4}; do
  if [ $v = new ]; then L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; else L=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 150 python tools/bench_configs.py --only bs4096 > gpurun_out/abbpw_${v}_$r.log 2>&1 || exit 1
done
done
for f in gpurun_out/abbpw_*; do echo $f; grep -v cfg5 $f | grep config | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('  ', d['config'][:14], d['encode_ms'], d['decode_clean_ms'], d.get('decode_1err_ms'))"; done
