# round 5, lease i: pageable host path -- persistent copy pool at 4 / 8 / 12 / 16 threads vs a
# thread spawn per copy (4 threads); then the GPU suite
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2; do
  for v in "spawn 4" "pool 4" "pool 8" "pool 12" "pool 16"; do
    set -- $v
    lib=$P; [ $1 = spawn ] && lib=$L/libppfs_ecc_spawn.so
    PPFS_ECC_COPY_THREADS=$2 PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/probes/host_path_probe.py --modes pageable --reps 3 --from-torch > gpurun_out/r5i_tmp.jsonl 2>gpurun_out/r5i_probe.err || { tail -5 gpurun_out/r5i_probe.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'variant': sys.argv[1], 'threads': int(sys.argv[2]), 'round': int(sys.argv[3]), **json.loads(l)})) for l in open(sys.argv[4])]" $1 $2 $r gpurun_out/r5i_tmp.jsonl >> gpurun_out/r5i_pageable_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5i_pageable_ab.jsonl'):
    d=json.loads(l); print(d['variant'], d['threads'], d['round'], d['op'], d['GiBps'])"
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5i_gputest.log 2>&1; rc=$?
tail -3 gpurun_out/r5i_gputest.log; exit $rc
