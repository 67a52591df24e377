# round 5, lease h: host path with two streams (H2D | kernels + D2H) vs four (one per stage), in a
# torch process and a torch-free one, then bench.py's host leg and the full GPU suite
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2; do
  for lib in $L/libppfs_ecc_4stream.so $P; do
    for ft in "" "--from-torch"; do
      PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/probes/host_path_probe.py --modes pinned,pageable --reps 3 $ft > gpurun_out/r5h_tmp.jsonl 2>gpurun_out/r5h_probe.err || { tail -5 gpurun_out/r5h_probe.err; exit 1; }
      python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'torch': sys.argv[2] != '', 'round': int(sys.argv[3]), **json.loads(l)})) for l in open(sys.argv[4])]" $(basename $lib) "$ft" $r gpurun_out/r5h_tmp.jsonl >> gpurun_out/r5h_host_ab.jsonl
    done
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5h_host_ab.jsonl'):
    d=json.loads(l)
    if d['op']!='decode_clean': print(d['lib'][12:], d['torch'], d['round'], d['mode'], d['op'], d['GiBps'])"
for r in 1 2; do
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-configs --no-cpu-baseline > gpurun_out/r5h_bench.json 2> gpurun_out/r5h_bench.err || { tail -5 gpurun_out/r5h_bench.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r5h_bench.json').read().strip().splitlines()[-1]);h=d['host_inclusive'];print(h['pinned'], h['pageable'])"
done
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5h_gputest.log 2>&1; rc=$?
tail -3 gpurun_out/r5h_gputest.log; exit $rc
