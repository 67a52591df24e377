#!/bin/bash
# GPU box (round 3, first session): normal-build GPU suite, the same suite on the bounds- and
# copy-checked PPFS_ECC_DEBUG build, the default bench line (with the configs leg), the graph-launch
# line (inject on the capture stream), and a torchrun world-1 run of the RCCL branch.
set -o pipefail
TAG=${1:-r3b}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_gputest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_gputest.log | head -20; exit $rc; }
timeout -k 10 900 bash tools/gpu_debug_suite.sh ${TAG}_debug || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; tail -c 600 gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --launch graph --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/${TAG}_bench_graph.json 2> gpurun_out/${TAG}_bench_graph.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench_graph.err; exit $rc; }
echo graph_ok
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/${TAG}_torchrun1_bench.json 2> gpurun_out/${TAG}_torchrun1_bench.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_torchrun1_bench.err; exit $rc; }
echo torchrun_ok
