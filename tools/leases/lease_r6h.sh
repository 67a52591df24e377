# round 6, lease h: decode write-back returned as patch lists (vote.hip patch_list_kernel) -- host-path
# GPU tests, then A/B against whole-codeword returns (PPFS_ECC_PATCH=0), page-locked and pageable
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "host or scrub or group or vote" > gpurun_out/r6h_hosttests.log 2>&1; rc=$?
tail -3 gpurun_out/r6h_hosttests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r6h_host_patch_ab.jsonl; : > $out
for v in "" "PPFS_ECC_PATCH=0" "" "PPFS_ECC_PATCH=0"; do
  echo "{\"variant\": \"$v\"}" >> $out
  env $v timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned,pageable --reps 5 2>/dev/null >> $out || { tail -5 $out; exit 1; }
done
echo '{"variant": "t16"}' >> $out
timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned --reps 5 --block-size 4096 --t 16 2>/dev/null >> $out || exit 1
echo '{"variant": "t16 PPFS_ECC_PATCH=0"}' >> $out
PPFS_ECC_PATCH=0 timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned --reps 5 --block-size 4096 --t 16 2>/dev/null >> $out || exit 1
cat $out
