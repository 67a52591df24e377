# round 5, lease zi: cfg5 decode waves with tickets + priorities in place -- 8 waves register
# prefetch (shipped), 8 / 9 / 10 waves single image (GF + XP rows in LDS, S12 from L2), 12 waves
# (every correction table in L2; 46 VGPRs spilled)
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2; do
  for lib in $P $L/libppfs_ecc_d8n1.so $L/libppfs_ecc_d9.so $L/libppfs_ecc_d10.so $L/libppfs_ecc_d12.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only cfg5 > gpurun_out/r5zi_tmp.jsonl 2>gpurun_out/r5zi_ab.err || { tail -5 gpurun_out/r5zi_ab.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5zi_tmp.jsonl >> gpurun_out/r5zi_cfg5_waves_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5zi_cfg5_waves_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d['roundtrip_ok'], {k: v for k, v in d.items() if k.endswith('_ms')})"
