# round 6, lease v: Hamming decode wave caps 20 / 24 / 28 / none and parity check caps 11-16 (after lease u),
# tests on the candidate
set -o pipefail
mkdir -p gpurun_out
L=$PWD/paritypartyfs_amd/_lib/lease
for v in w1; do
  PPFS_ECC_LIB=$L/libppfs_ecc_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "hamming or parity" > gpurun_out/r6v_tests_$v.log 2>&1; rc=$?
  echo "$v $(tail -1 gpurun_out/r6v_tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
out=gpurun_out/r6v_bitfast_shapes_ab.jsonl; : > $out
for rnd in 1 2 3; do
for v in base w1 w2 w3 w4; do
  if [ $v = base ]; then lib=""; else lib="PPFS_ECC_LIB=$L/libppfs_ecc_$v.so"; fi
  for c in hamming parity; do
  env $lib timeout -k 10 200 python tools/bench_configs.py --only $c > gpurun_out/r6v_tmp.jsonl 2>gpurun_out/r6v_tmp.err || { echo "fail $v"; tail -5 gpurun_out/r6v_tmp.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r6v_tmp.jsonl'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(json.dumps({'variant':'$v','round':$rnd,'config':d.get('config'),'encode_ms':d.get('encode_ms'),'decode_clean_ms':d.get('decode_clean_ms'),'decode_1err_ms':d.get('decode_1err_ms')}))" >> $out
  done
done
done
cat $out
