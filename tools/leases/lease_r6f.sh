# round 6, lease f: 64 Ki host chunks + ramped fill / drain -- host-path GPU tests, then A/B vs no ramp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "host or scrub or group or vote" > gpurun_out/r6f_hosttests.log 2>&1; rc=$?
tail -3 gpurun_out/r6f_hosttests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r6f_host_ramp_ab.jsonl; : > $out
for v in "" "PPFS_ECC_NO_RAMP=1" "" "PPFS_ECC_NO_RAMP=1"; do
  echo "{\"variant\": \"$v\"}" >> $out
  env $v timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned,pageable --reps 5 2>/dev/null >> $out || { tail -5 $out; exit 1; }
done
cat $out
