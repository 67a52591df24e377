# GPU box: per-config kernel rates and the t=16 PMC passes (tag $1)
set -o pipefail
TAG=${1:-r1h}
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || { echo "configs failed"; tail gpurun_out/configs_$TAG.err; exit 1; }
timeout -k 10 300 bash tools/pmc_py.sh rs16_$TAG $GRAFT_REPO_ROOT/tools/run_one.py rs16 > gpurun_out/pmc_rs16_$TAG.log 2>&1 || { echo "pmc failed"; cat gpurun_out/pmc_rs16_$TAG.log; exit 1; }
cut -c1-420 gpurun_out/configs_$TAG.jsonl
