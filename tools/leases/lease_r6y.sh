# round 6, lease y: the driver's N-GPU launch form at N = 1 (torchrun, RCCL barrier + max-reduce on the
# GPU, the same code as the 8-GPU scaling run), headline and configs[4] shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6y_torchrun1.json 2> gpurun_out/r6y_torchrun1.err || { tail -5 gpurun_out/r6y_torchrun1.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6y_torchrun1.json').read().strip().splitlines()[-1]);print(d['n_gpus'],d['value'],d['in_step_frac'],d.get('aggregate_frac'),d['collectives'] if 'collectives' in d else '')"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --steps 20 --warmup 5 --block-size 4096 --t 16 > gpurun_out/r6y_torchrun1_cfg5.json 2> gpurun_out/r6y_torchrun1_cfg5.err || { tail -5 gpurun_out/r6y_torchrun1_cfg5.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6y_torchrun1_cfg5.json').read().strip().splitlines()[-1]);print(d['n_gpus'],d['value'],d['in_step_frac'],d.get('aggregate_frac'))"
