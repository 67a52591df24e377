# round 5, lease u: host path with one stream per pipeline stage (H2D / kernels / D2H) and three
# staging slots; the full GPU suite, then the driver's bench line (host_inclusive vs the link)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5u_gputest.log 2>&1; rc=$?
tail -3 gpurun_out/r5u_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r5u_bench.json 2> gpurun_out/r5u_bench.err || { tail -5 gpurun_out/r5u_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r5u_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['in_step_frac'],d['roofline']['traffic'],json.dumps(d['host_inclusive']))"
