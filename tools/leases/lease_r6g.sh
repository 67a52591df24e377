# round 6, lease g: host path A/B -- staging slots 3 / 4, with and without the ramped chunks (page-locked)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r6g_host_slots_ab.jsonl; : > $out
for rnd in 1 2; do
for v in "PPFS_ECC_NO_RAMP=1" "PPFS_ECC_SLOTS=4 PPFS_ECC_NO_RAMP=1" "" "PPFS_ECC_SLOTS=4"; do
  echo "{\"variant\": \"$v\"}" >> $out
  env $v timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned --reps 7 2>/dev/null >> $out || { tail -5 $out; exit 1; }
done
done
cat $out
