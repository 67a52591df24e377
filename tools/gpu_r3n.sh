#!/bin/bash
# GPU box (round 3): default bench line (kernel timing from dispatch packets), rocprofv3 trace + PMC of
# the same build, cfg5 bench line, phase traces of the t = 3 encode / decode and the 2t = 32 decode.
set -o pipefail
TAG=${1:-r3n}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_ms'], d['kernels_ms_stream_events'])"
timeout -k 10 300 python bench.py --block-size 4096 --t 16 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/${TAG}_bench_cfg5.json 2> gpurun_out/${TAG}_bench_cfg5.err || { tail -5 gpurun_out/${TAG}_bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench_cfg5.json').read().strip().splitlines()[-1]); print('cfg5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_ms'], d['kernels_ms_stream_events'])"
timeout -k 10 900 bash tools/profile_box.sh $TAG --no-configs > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; tail gpurun_out/${TAG}_prof.log; exit 1; }
grep -E "encode_tk|decode_tk" gpurun_out/prof_${TAG}/trace_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
T=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_trace.so
PPFS_ECC_LIB=$T timeout -k 10 120 python tools/tk_trace.py 2>/dev/null > gpurun_out/${TAG}_tktrace.jsonl || { tail gpurun_out/${TAG}_tktrace.jsonl; exit 1; }
PPFS_ECC_LIB=$T timeout -k 10 120 python tools/bs_trace.py 2>/dev/null > gpurun_out/${TAG}_bstrace.jsonl || { tail gpurun_out/${TAG}_bstrace.jsonl; exit 1; }
cat gpurun_out/${TAG}_tktrace.jsonl gpurun_out/${TAG}_bstrace.jsonl
