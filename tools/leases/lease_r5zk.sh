# round 5, lease zk: cfg5 waves moving on to other XCDs' counters when theirs runs dry (LDS mask of
# dry counters per workgroup, moves out of line): t = 16 oracle tests, cfg5 A/B, tails
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_lifecycle.py -k "16 or t16 or ticket or graph" > gpurun_out/r5zk_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5zk_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in $L/libppfs_ecc_bsnosteal.so $P; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only cfg5 > gpurun_out/r5zk_tmp.jsonl 2>gpurun_out/r5zk_ab.err || { tail -5 gpurun_out/r5zk_ab.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5zk_tmp.jsonl >> gpurun_out/r5zk_cfg5_steal_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5zk_cfg5_steal_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d['roundtrip_ok'], {k: v for k, v in d.items() if k.endswith('_ms')})"
for m in "" "--clean"; do
  PPFS_ECC_LIB=$L/libppfs_ecc_trace.so timeout -k 10 300 python tools/bs_trace.py $m >> gpurun_out/r5zk_cfg5_tail.jsonl 2> gpurun_out/r5zk.err || { tail -5 gpurun_out/r5zk.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/r5zk_cfg5_tail.jsonl'):
    d=json.loads(l); print(d['mode'], d['realtime']['span_us'], d['realtime']['end_us'], d['realtime']['end_us_by_xcd_min_med_max'])"
