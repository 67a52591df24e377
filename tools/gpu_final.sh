# GPU box, final records of a build: GPU suite, smoke, rocprofv3 trace + PMC of the default bench, the
# driver's default bench line, the cfg5 bench line, per-config kernel rates, the cfg5 PMC.
# Usage: tools/gpu_final.sh <tag>
TAG=${1:-final}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 bash tools/profile_box.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; tail gpurun_out/${TAG}_prof.log; exit 1; }
echo profiled
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -3 gpurun_out/${TAG}_bench.log; exit 1; }
echo bench
timeout -k 10 300 python bench.py --block-size 4096 --t 16 > gpurun_out/${TAG}_bench_cfg5.log 2>&1 || { tail -3 gpurun_out/${TAG}_bench_cfg5.log; exit 1; }
echo bench_cfg5
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/${TAG}_configs.jsonl 2> gpurun_out/${TAG}_configs.err || { tail gpurun_out/${TAG}_configs.err; exit 1; }
echo configs
timeout -k 10 300 bash tools/pmc_py.sh rs16_$TAG $GRAFT_REPO_ROOT/tools/run_one.py rs16 > gpurun_out/${TAG}_pmc_rs16.log 2>&1 || { cat gpurun_out/${TAG}_pmc_rs16.log; exit 1; }
echo pmc_rs16
