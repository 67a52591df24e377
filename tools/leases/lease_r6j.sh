# round 6, lease j: zero-copy patch writes into a page-locked caller image -- full GPU suite, host
# probe (t = 3 and t = 16), the driver's bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r6j_gputest.log 2>&1; rc=$?
tail -3 gpurun_out/r6j_gputest.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r6j_host.jsonl; : > $out
timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned,pageable --reps 5 2>/dev/null >> $out || exit 1
timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned --reps 5 --block-size 4096 --t 16 2>/dev/null >> $out || exit 1
cat $out
timeout -k 10 600 python bench.py > gpurun_out/r6j_bench.json 2> gpurun_out/r6j_bench.err || { tail -5 gpurun_out/r6j_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6j_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['in_step_frac']);h=d['host_inclusive'];print({m: h[m] for m in ('pinned','pageable')})"
