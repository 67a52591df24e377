# round 5, lease l: Hamming decode correcting from registers (no LDS read-back behind lgkmcnt(0)),
# Hamming oracle tests, then cfg4 A/B against the committed build
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ham" > gpurun_out/r5l_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5l_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in $L/libppfs_ecc_base.so $P; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only "cfg4 hamming" > gpurun_out/r5l_tmp.jsonl 2>gpurun_out/r5l_ab.err || { tail -5 gpurun_out/r5l_ab.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5l_tmp.jsonl >> gpurun_out/r5l_ham_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5l_ham_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d['config'], {k: v for k, v in d.items() if k.endswith('_ms') or 'frac' in k})"
