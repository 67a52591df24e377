# GPU box, full round refresh: GPU suite, bench profile (trace + PMC), per-config rates, rs16 PMC, host rates, default bench line. Usage: tools/gpu_round_full.sh <tag>
TAG=${1:-r1i}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/profile_box.sh $TAG > gpurun_out/prof.log 2>&1 || { echo "profile failed"; tail gpurun_out/prof.log; exit 1; }
echo profiled
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || { echo "configs failed"; tail gpurun_out/configs_$TAG.err; exit 1; }
echo configs
timeout -k 10 300 bash tools/pmc_py.sh rs16_$TAG $GRAFT_REPO_ROOT/tools/run_one.py rs16 > gpurun_out/pmc_rs16_$TAG.log 2>&1 || { echo "pmc failed"; cat gpurun_out/pmc_rs16_$TAG.log; exit 1; }
echo pmc
timeout -k 10 300 python tools/bench_host.py > gpurun_out/host_$TAG.jsonl 2> gpurun_out/host_$TAG.err || { echo "host failed"; tail gpurun_out/host_$TAG.err; exit 1; }
echo host
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-600; exit $rc
