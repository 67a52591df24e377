# round 5, lease t: wave priorities -- t <= 4 ticket kernels (every wave raised from barrier B to the
# next remainder phase) on the bench step; bit kernels (around the first loads) on cfg4
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2 3; do
  for lib in $P $L/libppfs_ecc_tkeprio.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5t_tmp.json 2> gpurun_out/r5t_bench.err || { tail -5 gpurun_out/r5t_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5t_tmp.json >> gpurun_out/r5t_tk_eprio_ab.jsonl
  done
done
cat gpurun_out/r5t_tk_eprio_ab.jsonl
for r in 1 2; do
  for lib in $P $L/libppfs_ecc_bfprio1.so $L/libppfs_ecc_bfprio2.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only "cfg4" > gpurun_out/r5t_tmp.jsonl 2>gpurun_out/r5t_ab.err || { tail -5 gpurun_out/r5t_ab.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5t_tmp.jsonl >> gpurun_out/r5t_bf_prio_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5t_bf_prio_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d['config'][:10], d['roundtrip_ok'], {k: v for k, v in d.items() if k.endswith('_ms')})"
