# round 5, lease ze: lifecycle tests (graph replays with t = 16 per-wave tickets), host-path tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lifecycle.py tests/test_gpu_parity.py -k "graph or host or ticket or lifecycle or stream" > gpurun_out/r5ze_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5ze_pytest.log; exit $rc
