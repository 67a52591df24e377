# round 6, lease a: baseline of the round-5 build on today's box -- the driver's bench line and the cfg5 step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err || { tail -5 gpurun_out/r6a_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6a_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['in_step_frac'])"
timeout -k 10 300 python bench.py --block-size 4096 --t 16 --no-cpu-baseline --no-configs --no-host-inclusive > gpurun_out/r6a_cfg5.json 2> gpurun_out/r6a_cfg5.err || { tail -5 gpurun_out/r6a_cfg5.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6a_cfg5.json').read().strip().splitlines()[-1]);print(d['value'],d['in_step_frac'])"
