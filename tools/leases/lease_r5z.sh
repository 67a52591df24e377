# round 5, lease z: t = 3 ticket kernels' workgroup end times (trace build): how much is tail
set -o pipefail
mkdir -p gpurun_out
PPFS_ECC_LIB=paritypartyfs_amd/_lib/lease/libppfs_ecc_trace.so timeout -k 10 300 python tools/tk_trace.py > gpurun_out/r5z_tk_tail.jsonl 2> gpurun_out/r5z.err || { tail -5 gpurun_out/r5z.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r5z_tk_tail.jsonl').read())
for k in ('encode','decode'): print(k, json.dumps(d[k]['realtime']))"
