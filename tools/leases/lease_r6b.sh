# round 6, lease b: after the switch clean-up and the bench legs (cold configs, cfg5 step, cfg1) --
# GPU suite, smoke, the driver's bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r6b_gputest.log 2>&1; rc=$?
tail -3 gpurun_out/r6b_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6b_smoke.log 2>&1 || { tail -5 gpurun_out/r6b_smoke.log; exit 1; }
tail -1 gpurun_out/r6b_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r6b_bench.json 2> gpurun_out/r6b_bench.err || { tail -5 gpurun_out/r6b_bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r6b_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['in_step_frac'])
for k,v in d['configs'].items():
    if isinstance(v, dict): print(k, {kk: vv for kk, vv in v.items() if 'frac' in kk or kk in ('kernels_ms','ms_per_step','cold_sets','roundtrip_ok','verified')})
print('cfg1', json.dumps(d['cfg1'].get('rs255_249_4096_blocks')), d['cfg1'].get('per_block_read_vs_reference_cpu'))
print('host', json.dumps({m: d['host_inclusive'][m] for m in ('pinned','pageable')}))
PY
