# round 5, lease zf: the step's launch gaps from a kernel trace (consecutive kernels' end -> start)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5zf -o run -- python3 bench.py --steps 40 --warmup 5 --no-configs --no-cpu-baseline --no-host-inclusive > gpurun_out/r5zf_trace.log 2>&1 || { tail -20 gpurun_out/r5zf_trace.log; exit 1; }
python3 - <<'PY' > gpurun_out/r5zf_gaps.json
import csv, glob, json, statistics
f = glob.glob('/tmp/r5zf/**/run_kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
ks = [(r['Kernel_Name'][:40], int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows]
gaps = {}
for a, b in zip(ks, ks[1:]):
    g = (b[1] - a[2]) / 1000.0
    if -5 < g < 50:
        key = a[0].split('(')[0][-28:] + ' -> ' + b[0].split('(')[0][-28:]
        gaps.setdefault(key, []).append(g)
out = {k: {"n": len(v), "median_us": round(statistics.median(v), 2), "min_us": round(min(v), 2)} for k, v in gaps.items() if len(v) >= 10}
print(json.dumps(out, indent=1))
PY
cat gpurun_out/r5zf_gaps.json
