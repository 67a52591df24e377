# GPU box: RS parity tests, then the bench (kernel times in the JSON line)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "rs" > gpurun_out/pytest_rs.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_rs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -2 gpurun_out/bench.log; exit $rc
