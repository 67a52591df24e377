# round 6, lease i: patch-list write-back with the orig copy on the input stream -- host-path GPU
# tests, the patch A/B once more, and the driver's bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "host or scrub or group or vote" > gpurun_out/r6i_hosttests.log 2>&1; rc=$?
tail -3 gpurun_out/r6i_hosttests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r6i_host_patch_ab.jsonl; : > $out
for v in "" "PPFS_ECC_PATCH=0"; do
  echo "{\"variant\": \"$v\"}" >> $out
  env $v timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned,pageable --reps 5 2>/dev/null >> $out || { tail -5 $out; exit 1; }
  echo "{\"variant\": \"t16 $v\"}" >> $out
  env $v timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned --reps 5 --block-size 4096 --t 16 2>/dev/null >> $out || exit 1
done
cat $out
timeout -k 10 600 python bench.py > gpurun_out/r6i_bench.json 2> gpurun_out/r6i_bench.err || { tail -5 gpurun_out/r6i_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6i_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['in_step_frac']);print(json.dumps(d['host_inclusive']))"
