# round 5, lease r: wave priorities -- cfg5 decode (correction + emission, or everything but the
# chain) and encode (emission + DMA), t = 3 decode (wave 0 through the corrections)
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2 3; do
  for lib in $P $L/libppfs_ecc_prio2.so $L/libppfs_ecc_prio4.so $L/libppfs_ecc_prio4e.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only cfg5 > gpurun_out/r5r_tmp.jsonl 2>gpurun_out/r5r_ab.err || { tail -5 gpurun_out/r5r_ab.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5r_tmp.jsonl >> gpurun_out/r5r_cfg5_prio_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5r_cfg5_prio_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d['roundtrip_ok'], {k: v for k, v in d.items() if k.endswith('_ms')})"
for r in 1 2 3; do
  for lib in $P $L/libppfs_ecc_tkprio.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5r_tmp.json 2> gpurun_out/r5r_bench.err || { tail -5 gpurun_out/r5r_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5r_tmp.json >> gpurun_out/r5r_tk_prio_ab.jsonl
  done
done
cat gpurun_out/r5r_tk_prio_ab.jsonl
