# round 6, lease o: the bench step's injection as an aligned 16 / 32 / 64-byte read-modify-write of
# the piece holding the byte (pieces wholly inside the block; byte stores at the block edges) vs the
# shipped byte stores: headline bench step, 3 interleaved rounds; injection tests under each variant
set -o pipefail
mkdir -p gpurun_out
for v in 16 32 64; do
  PPFS_AB_INJ=$v timeout -k 10 200 python -u -m pytest tests/test_gpu_hygiene.py -x -q --timeout 120 --timeout-method thread -m gpu -k "inject" > gpurun_out/r6o_tests_$v.log 2>&1; rc=$?
  tail -1 gpurun_out/r6o_tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
out=gpurun_out/r6o_inject_ab.jsonl; : > $out
for rnd in 1 2 3; do
for v in 0 16 32 64; do
  PPFS_AB_INJ=$v timeout -k 10 200 python bench.py --steps 50 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/r6o_tmp.json 2>gpurun_out/r6o_tmp.err || { echo "fail $v"; tail -5 gpurun_out/r6o_tmp.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r6o_tmp.json').read().strip().splitlines()[-1]);print(json.dumps({'variant':'$v','round':$rnd,'value':d['value'],'ms_per_step':d['ms_per_step'],'kernels_ms':d['kernels_ms'],'in_step_frac':d['in_step_frac'],'verified':d.get('verified')}))" >> $out
done
done
cat $out
