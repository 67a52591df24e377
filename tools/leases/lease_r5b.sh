# round 5, lease b: the driver's bench line (host link via hipMemcpyAsync), cfg5 decode at 11 / 12
# waves (S12 / XP / GF tables out of LDS), the cfg5 decode phase trace, rocprofv3 profile + PMC
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
timeout -k 10 600 python bench.py > gpurun_out/r5b_bench.json 2> gpurun_out/r5b_bench.err || { tail -5 gpurun_out/r5b_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r5b_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['in_step_frac'],json.dumps(d['host_inclusive']))"
for r in 1 2; do
  for lib in paritypartyfs_amd/_lib/libppfs_ecc.so $L/libppfs_ecc_d11t1n1.so $L/libppfs_ecc_d12t2n1.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only cfg5 > gpurun_out/r5b_tmp.jsonl 2>gpurun_out/r5b_cfg5.err || { tail -5 gpurun_out/r5b_cfg5.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5b_tmp.jsonl | tee -a gpurun_out/r5b_cfg5_ab.jsonl | cut -c1-300
  done
done
for m in "" "--clean"; do
  PPFS_ECC_LIB=$L/libppfs_ecc_trace.so timeout -k 10 120 python tools/bs_trace.py $m >> gpurun_out/r5b_cfg5_phase_trace.jsonl 2>gpurun_out/r5b_trace.err || { tail -5 gpurun_out/r5b_trace.err; exit 1; }
done
cat gpurun_out/r5b_cfg5_phase_trace.jsonl
timeout -k 10 900 bash tools/profile_box.sh r5b --no-configs > gpurun_out/r5b_prof.log 2>&1 || { echo "profile failed"; tail gpurun_out/r5b_prof.log; exit 1; }
tail -5 gpurun_out/r5b_prof.log
