# round 5, lease x: cfg5 kernels taking tiles by per-XCD ticket per wave (vs the static walk):
# t = 16 oracle tests, cfg5 A/B, the decode's per-wave end times with tickets
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "16 or t16 or ticket" > gpurun_out/r5x_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5x_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in $L/libppfs_ecc_bsstatic.so $P; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only cfg5 > gpurun_out/r5x_tmp.jsonl 2>gpurun_out/r5x_ab.err || { tail -5 gpurun_out/r5x_ab.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5x_tmp.jsonl >> gpurun_out/r5x_cfg5_tickets_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5x_cfg5_tickets_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d['roundtrip_ok'], {k: v for k, v in d.items() if k.endswith('_ms') or k.startswith('roofline_frac_')})"
for m in "" "--clean"; do
  PPFS_ECC_LIB=$L/libppfs_ecc_trace.so timeout -k 10 300 python tools/bs_trace.py $m >> gpurun_out/r5x_cfg5_tail_tickets.jsonl 2> gpurun_out/r5x.err || { tail -5 gpurun_out/r5x.err; exit 1; }
done
cat gpurun_out/r5x_cfg5_tail_tickets.jsonl | cut -c1-1200
