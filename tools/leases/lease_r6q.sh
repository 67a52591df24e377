# round 6, lease q: the driver's bench command on the shipped library (its line's `traffic` now from
# pmc_latest.json of this build), then multi-rank rehearsals on the one GPU: 2 ranks at the headline
# shape and 4 ranks at configs[4]'s per-GPU shape (--block-size 4096 --t 16), barrier + max-reduce over RCCL
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r6q_bench.json 2> gpurun_out/r6q_bench.err || { tail -5 gpurun_out/r6q_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6q_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['in_step_frac'],d['roofline']['traffic'],d['roofline'].get('traffic_source'))"
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --steps 20 > gpurun_out/r6q_n2.json 2> gpurun_out/r6q_n2.err || { tail -5 gpurun_out/r6q_n2.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6q_n2.json').read().strip().splitlines()[-1]);print(d['n_gpus'],d['value'],d.get('aggregate_frac'),d['config'])"
timeout -k 10 300 python bench.py --gpus 4 --share-gpu --steps 10 --block-size 4096 --t 16 > gpurun_out/r6q_n4_cfg5.json 2> gpurun_out/r6q_n4_cfg5.err || { tail -5 gpurun_out/r6q_n4_cfg5.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6q_n4_cfg5.json').read().strip().splitlines()[-1]);print(d['n_gpus'],d['value'],d.get('aggregate_frac'),d['config'])"
