# round 6, lease w: the Hamming encode's payload loads non-temporal again (round 5 dropped them for the
# 1-error decode timed right after), in the cold configs leg with the XCD-local ranges; Hamming tests first
set -o pipefail
mkdir -p gpurun_out
L=$PWD/paritypartyfs_amd/_lib/lease
PPFS_ECC_LIB=$L/libppfs_ecc_hnt.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "hamming" > gpurun_out/r6w_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r6w_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r6w_ham_nt_ab.jsonl; : > $out
for rnd in 1 2 3; do
for v in base hnt; do
  if [ $v = base ]; then lib=""; else lib="PPFS_ECC_LIB=$L/libppfs_ecc_$v.so"; fi
  env $lib timeout -k 10 200 python tools/bench_configs.py --only hamming > gpurun_out/r6w_tmp.jsonl 2>gpurun_out/r6w_tmp.err || { echo "fail $v"; tail -5 gpurun_out/r6w_tmp.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r6w_tmp.jsonl'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(json.dumps({'variant':'$v','round':$rnd,'config':d.get('config'),'encode_ms':d.get('encode_ms'),'decode_clean_ms':d.get('decode_clean_ms'),'decode_1err_ms':d.get('decode_1err_ms')}))" >> $out
done
done
cat $out
