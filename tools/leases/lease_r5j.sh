# round 5, lease j: the box's CPU share, and the pageable host path over copy-pool sizes 6-14
set -o pipefail
mkdir -p gpurun_out
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:64])"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -i "numa\|model name\|socket\|thread\|core"; } > gpurun_out/r5j_cpu.txt 2>&1
cat gpurun_out/r5j_cpu.txt
for r in 1 2; do
  for n in 6 8 10 12 14; do
    PPFS_ECC_COPY_THREADS=$n timeout -k 10 300 python tools/probes/host_path_probe.py --modes pageable --reps 3 --from-torch > gpurun_out/r5j_tmp.jsonl 2>gpurun_out/r5j_probe.err || { tail -5 gpurun_out/r5j_probe.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'threads': int(sys.argv[1]), 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $n $r gpurun_out/r5j_tmp.jsonl >> gpurun_out/r5j_pageable_threads.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5j_pageable_threads.jsonl'):
    d=json.loads(l); print(d['threads'], d['round'], d['op'], d['GiBps'])"
