# round 5, lease zg: the step's 4.7 us gaps after the encode / decode (end-of-kernel system-scope
# release, hip_ext.h) -- output store policies: nt (shipped), plain, nt sc1, sc0 sc1, nt sc0 sc1
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2; do
  for lib in $P $L/libppfs_ecc_tkst0.so $L/libppfs_ecc_stp2.so $L/libppfs_ecc_stp3.so $L/libppfs_ecc_stp4.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5zg_tmp.json 2> gpurun_out/r5zg_bench.err || { tail -5 gpurun_out/r5zg_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'device_ms_per_step': d['device_ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5zg_tmp.json >> gpurun_out/r5zg_store_policy_ab.jsonl
  done
done
cat gpurun_out/r5zg_store_policy_ab.jsonl
