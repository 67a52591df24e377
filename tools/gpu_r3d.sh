#!/bin/bash
# GPU box (round 3): GPU suite on the normal and the checked build, CRC config A/B, cfg5 bench A/B,
# torchrun world-1 run with the barrier-while-busy timing.
set -o pipefail
TAG=${1:-r3d}
mkdir -p gpurun_out
[ -n "$SKIP_SUITE" ] || { timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_gputest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_gputest.log | head -20; exit $rc; }; }
timeout -k 10 600 bash tools/gpu_debug_suite.sh ${TAG}_debug || exit 1
for v in new crc1 crc1nf bfpf r3base new crc1 crc1nf bfpf r3base; do
  if [ $v = new ]; then L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; else L=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 120 python tools/bench_configs.py --only crc >> gpurun_out/${TAG}_crc_$v.jsonl 2>> gpurun_out/${TAG}_crc.err || exit 1
done
tail -n 2 gpurun_out/${TAG}_crc_*.jsonl | cut -c1-400
VARIANTS="nosect" timeout -k 10 600 bash tools/ab_bench.sh ${TAG}_cfg5ab --block-size 4096 --t 16 > gpurun_out/${TAG}_cfg5ab.txt 2>&1 || { tail gpurun_out/${TAG}_cfg5ab.txt; exit 1; }
cat gpurun_out/${TAG}_cfg5ab.txt
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/${TAG}_torchrun1_bench.json 2> gpurun_out/${TAG}_torchrun1_bench.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_torchrun1_bench.err; exit $rc; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_torchrun1_bench.json').read().strip().splitlines()[-1]); print('torchrun', d['value'], d['ms_per_step'], d['device_ms_per_step'], d['repeat_ms_per_step'], d['collectives'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-configs > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print('plain', d['value'], d['ms_per_step'], d['device_ms_per_step'], d['repeat_ms_per_step'], d['kernels_ms'])"
PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_trace.so timeout -k 10 120 python tools/tk_trace.py > gpurun_out/${TAG}_tktrace.jsonl 2>&1 || { tail gpurun_out/${TAG}_tktrace.jsonl; exit 1; }
PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_trace.so timeout -k 10 120 python tools/tk_trace.py --standalone >> gpurun_out/${TAG}_tktrace.jsonl 2>&1 || { tail gpurun_out/${TAG}_tktrace.jsonl; exit 1; }
cat gpurun_out/${TAG}_tktrace.jsonl
