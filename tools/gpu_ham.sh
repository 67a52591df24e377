#!/bin/bash
# GPU box: full GPU suite, then the reference's block-device bench cases (per-block latency).
set -o pipefail
TAG=${1:-ham}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 tests/cpp/_build/bench_blockdevice 0.2 > gpurun_out/${TAG}_bench_blockdevice.jsonl 2> gpurun_out/${TAG}_bench_blockdevice.err || { tail gpurun_out/${TAG}_bench_blockdevice.err; exit 1; }
grep -i "ham\|crc" gpurun_out/${TAG}_bench_blockdevice.jsonl | head -40
