# round 5, lease k: the bench step's one-byte injection in reverse block order (the encode's last
# codeword lines are the ones still in the Infinity Cache) vs forward
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2 3; do
  for lib in $P $L/libppfs_ecc_injrev.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python bench.py --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5k_tmp.json 2> gpurun_out/r5k_bench.err || { tail -5 gpurun_out/r5k_bench.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels_ms': d['kernels_ms']}))" $(basename $lib) $r gpurun_out/r5k_tmp.json >> gpurun_out/r5k_inject_rev_ab.jsonl
  done
done
cat gpurun_out/r5k_inject_rev_ab.jsonl
