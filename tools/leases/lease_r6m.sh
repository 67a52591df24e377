# round 6, lease m: XCD-contiguous block ranges for the streaming CRC / Hamming / parity kernels
# (bit_fast.hip bf_wg, PPFS_AB_XCD=1) vs the dispatch order -- bit-kernel parity tests on the variant,
# then the cfg4 configs leg, 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
L=$PWD/paritypartyfs_amd/_lib/lease
PPFS_ECC_LIB=$L/libppfs_ecc_xcd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "crc or ham or parity" > gpurun_out/r6m_xcd_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6m_xcd_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r6m_xcd_ab.jsonl; : > $out
for rnd in 1 2 3; do
for v in base xcd; do
  if [ $v = base ]; then lib=""; else lib="PPFS_ECC_LIB=$L/libppfs_ecc_$v.so"; fi
  for cfg in hamming crc parity; do
    env $lib timeout -k 10 200 python tools/bench_configs.py --only $cfg > gpurun_out/r6m_tmp.json 2>/dev/null || { echo "fail $v $cfg"; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/r6m_tmp.json').read().strip().splitlines()[-1]);print(json.dumps({'variant':'$v','round':$rnd,**{k:v for k,v in d.items() if k.endswith('_ms') or k.startswith('roofline') or k=='config'}}))" >> $out
  done
done
done
cat $out
