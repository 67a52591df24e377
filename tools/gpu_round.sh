set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && cat gpurun_out/bench.log | tail -3 &&
timeout -k 10 600 bash tools/profile_box.sh r1c > gpurun_out/prof.log 2>&1; echo prof=$?
