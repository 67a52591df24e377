# round 5, lease c: cfg5 log-domain single-error confirmation and encode register prefetch; CRC at
# 5 waves per SIMD; the driver's bench line (host link in chunked duplex copies)
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
for v in logchk encrp; do
  PPFS_ECC_LIB=$L/libppfs_ecc_$v.so timeout -k 10 300 $PYT tests/test_gpu_parity.py -k "rs and 4096" > gpurun_out/r5c_${v}_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r5c_${v}_pytest.log; [ $rc -eq 0 ] || exit $rc
done
PPFS_ECC_LIB=$L/libppfs_ecc_crcw5.so timeout -k 10 300 $PYT tests/test_gpu_parity.py -k crc > gpurun_out/r5c_crcw5_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r5c_crcw5_pytest.log; [ $rc -eq 0 ] || exit $rc
ab() { # tag only libs...
  local tag=$1 only=$2; shift 2
  for r in 1 2; do
    for lib in "$@"; do
      PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only "$only" > gpurun_out/r5c_tmp.jsonl 2>gpurun_out/r5c_ab.err || { tail -5 gpurun_out/r5c_ab.err; return 1; }
      python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5c_tmp.jsonl >> gpurun_out/r5c_${tag}_ab.jsonl
    done
  done
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d['lib'], d['round'], d['config'], {k: v for k, v in d.items() if k.endswith('_ms')})" gpurun_out/r5c_${tag}_ab.jsonl
}
P=paritypartyfs_amd/_lib/libppfs_ecc.so
ab cfg5 cfg5 $P $L/libppfs_ecc_logchk.so $L/libppfs_ecc_encrp.so || exit 1
ab cfg4 cfg4 $P $L/libppfs_ecc_crcw5.so || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r5c_bench.json 2> gpurun_out/r5c_bench.err || { tail -5 gpurun_out/r5c_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r5c_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['in_step_frac'],d['roofline']['traffic'],json.dumps(d['host_inclusive']))"
