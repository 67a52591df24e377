# round 6, lease t: CRC check shapes around 4-wave workgroups (WV x blocks per wave), 3 interleaved rounds
# CRC tests on each variant first
set -o pipefail
mkdir -p gpurun_out
L=$PWD/paritypartyfs_amd/_lib/lease
for v in c44; do
  PPFS_ECC_LIB=$L/libppfs_ecc_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "crc" > gpurun_out/r6t_tests_$v.log 2>&1; rc=$?
  echo "$v $(tail -1 gpurun_out/r6t_tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
out=gpurun_out/r6t_crc_shapes_ab.jsonl; : > $out
for rnd in 1 2 3; do
for v in base c42 c44 c48 c34 c64 c84; do
  if [ $v = base ]; then lib=""; else lib="PPFS_ECC_LIB=$L/libppfs_ecc_$v.so"; fi
  env $lib timeout -k 10 200 python tools/bench_configs.py --only crc > gpurun_out/r6t_tmp.jsonl 2>gpurun_out/r6t_tmp.err || { echo "fail $v"; tail -5 gpurun_out/r6t_tmp.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r6t_tmp.jsonl'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(json.dumps({'variant':'$v','round':$rnd,'config':d.get('config'),'encode_ms':d.get('encode_ms'),'decode_clean_ms':d.get('decode_clean_ms'),'roofline_frac_encode':d.get('roofline_frac_encode'),'roofline_frac_decode_clean':d.get('roofline_frac_decode_clean')}))" >> $out
done
done
cat $out
