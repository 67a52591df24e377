# round 5, lease zb: cross-XCD ticket stealing at the batch end (t <= 4 ticket kernels, cfg5 waves):
# RS oracle tests, bench step A/B, cfg5 A/B, tails
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "rs" > gpurun_out/r5zb_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5zb_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in $L/libppfs_ecc_nosteal.so $P; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5zb_tmp.json 2> gpurun_out/r5zb_bench.err || { tail -5 gpurun_out/r5zb_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5zb_tmp.json >> gpurun_out/r5zb_steal_ab.jsonl
  done
done
cat gpurun_out/r5zb_steal_ab.jsonl
for r in 1 2; do
  for lib in $L/libppfs_ecc_nosteal.so $P; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only cfg5 > gpurun_out/r5zb_tmp.jsonl 2>gpurun_out/r5zb_ab.err || { tail -5 gpurun_out/r5zb_ab.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5zb_tmp.jsonl >> gpurun_out/r5zb_cfg5_steal_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5zb_cfg5_steal_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d['roundtrip_ok'], {k: v for k, v in d.items() if k.endswith('_ms')})"
PPFS_ECC_LIB=$L/libppfs_ecc_trace.so timeout -k 10 300 python tools/tk_trace.py > gpurun_out/r5zb_tk_tail.jsonl 2> gpurun_out/r5zb.err || { tail -5 gpurun_out/r5zb.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r5zb_tk_tail.jsonl').read())
for k in ('encode','decode'): print(k, json.dumps(d[k]['realtime']))"
PPFS_ECC_LIB=$L/libppfs_ecc_trace.so timeout -k 10 300 python tools/bs_trace.py > gpurun_out/r5zb_bs_tail.jsonl 2> gpurun_out/r5zb.err || { tail -5 gpurun_out/r5zb.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r5zb_bs_tail.jsonl').read()); print('cfg5 decode', json.dumps(d['realtime']))"
