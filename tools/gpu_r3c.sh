#!/bin/bash
# GPU box (round 3): the default bench line (with the configs leg), interleaved A/B of the engine
# builds on the bench line, the graph-launch line and a torchrun world-1 run of the RCCL branch.
set -o pipefail
TAG=${1:-r3c}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; tail -c 400 gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
VARIANTS="${AB:-r3base}" timeout -k 10 900 bash tools/ab_bench.sh ${TAG}_ab > gpurun_out/${TAG}_ab.txt 2>&1 || { tail gpurun_out/${TAG}_ab.txt; exit 1; }
cat gpurun_out/${TAG}_ab.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --launch graph --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/${TAG}_bench_graph.json 2> gpurun_out/${TAG}_bench_graph.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench_graph.err; exit $rc; }
echo graph_ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/${TAG}_torchrun1_bench.json 2> gpurun_out/${TAG}_torchrun1_bench.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_torchrun1_bench.err; exit $rc; }
echo torchrun_ok
