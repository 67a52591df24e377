# GPU box: full GPU test suite, rocprofv3 profile (trace + PMC passes), then the default bench line
set -o pipefail
TAG=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/profile_box.sh $TAG > gpurun_out/prof.log 2>&1 || { echo "profile failed"; tail gpurun_out/prof.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; exit $rc
