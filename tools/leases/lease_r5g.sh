# round 5, lease g: why bench.py's host leg reads lower than host_path_probe.py on the same path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/probes/host_path_probe.py --modes pinned,pageable --reps 3 > gpurun_out/r5g_probe.jsonl 2>&1 || { tail -5 gpurun_out/r5g_probe.jsonl; exit 1; }
timeout -k 10 300 python tools/probes/host_path_probe.py --modes pinned --reps 3 --from-torch > gpurun_out/r5g_probe_torch.jsonl 2>&1 || { tail -5 gpurun_out/r5g_probe_torch.jsonl; exit 1; }
cat gpurun_out/r5g_probe.jsonl gpurun_out/r5g_probe_torch.jsonl | grep -v decode_clean
for v in "--no-cpu-baseline" ""; do
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-configs $v > gpurun_out/r5g_bench.json 2> gpurun_out/r5g_bench.err || { tail -5 gpurun_out/r5g_bench.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r5g_bench.json').read().strip().splitlines()[-1]);h=d['host_inclusive'];print('$v', h['pinned'], h['pageable'])"
done
