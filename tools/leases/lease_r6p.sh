# round 6, lease p: the injection's 32-byte read-modify-write with a thread's four sector loads issued
# before any store (variant 1) vs the shipped byte stores: headline bench step, 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
for v in 1; do
  PPFS_AB_INJ=$v timeout -k 10 200 python -u -m pytest tests/test_gpu_hygiene.py -x -q --timeout 120 --timeout-method thread -m gpu -k "inject" > gpurun_out/r6p_tests_$v.log 2>&1; rc=$?
  tail -1 gpurun_out/r6p_tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
out=gpurun_out/r6p_inject_ab.jsonl; : > $out
for rnd in 1 2 3; do
for v in 0 1; do
  PPFS_AB_INJ=$v timeout -k 10 200 python bench.py --steps 50 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/r6p_tmp.json 2>gpurun_out/r6p_tmp.err || { echo "fail $v"; tail -5 gpurun_out/r6p_tmp.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r6p_tmp.json').read().strip().splitlines()[-1]);print(json.dumps({'variant':'$v','round':$rnd,'value':d['value'],'ms_per_step':d['ms_per_step'],'kernels_ms':d['kernels_ms'],'in_step_frac':d['in_step_frac'],'verified':d.get('verified')}))" >> $out
done
done
cat $out
