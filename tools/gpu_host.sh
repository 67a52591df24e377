# GPU box: host-path tests (write-back fetch, pinned / pageable, block devices, scrub) + host rates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_block_device.py tests/test_vote_scrub.py tests/test_cpp_adapter.py -x -q --timeout 200 --timeout-method thread -m gpu -k "host or block or scrub or cpp or rmw" > gpurun_out/host_t.log 2>&1
rc=$?; tail -3 gpurun_out/host_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_host.py > gpurun_out/host_b.jsonl 2> gpurun_out/host_b.err || { tail gpurun_out/host_b.err; exit 1; }
cat gpurun_out/host_b.jsonl
