#!/bin/bash
# GPU box (round 3): normal + checked GPU suites, bench A/B of engine builds (AB="..." variants in
# _lib/alt), the encode phase trace, and a torchrun world-1 line.
set -o pipefail
TAG=${1:-r3f}
mkdir -p gpurun_out
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_gputest.log 2>&1
  rc=$?; tail -2 gpurun_out/${TAG}_gputest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_gputest.log | head -20; exit $rc; }
  timeout -k 10 600 bash tools/gpu_debug_suite.sh ${TAG}_debug || exit 1
fi
if [ -n "$AB" ]; then
  VARIANTS="$AB" timeout -k 10 900 bash tools/ab_bench.sh ${TAG}_ab $ABARGS > gpurun_out/${TAG}_ab.txt 2>&1 || { tail gpurun_out/${TAG}_ab.txt; exit 1; }
  cat gpurun_out/${TAG}_ab.txt
fi
for TR in trace trace0; do
  [ -f paritypartyfs_amd/_lib/alt/libppfs_ecc_$TR.so ] || continue
  PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$TR.so timeout -k 10 120 python tools/tk_trace.py > gpurun_out/${TAG}_$TR.jsonl 2>/dev/null || { tail gpurun_out/${TAG}_$TR.jsonl; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/${TAG}_$TR.jsonl'):
    d = json.loads(l)
    for k in ('encode', 'decode'):
        for w in ('wave0', 'wave1_dma'):
            if k in d:
                print('$TR', d['mode'], k, w, d[k][w]['total_cycles'], d[k][w]['per_iter'])"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/${TAG}_torchrun1_bench.json 2> gpurun_out/${TAG}_torchrun1_bench.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_torchrun1_bench.err; exit $rc; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_torchrun1_bench.json').read().strip().splitlines()[-1]); print('torchrun', d['value'], d['ms_per_step'], d['device_ms_per_step'], d['repeat_ms_per_step'], d['collectives'])"
