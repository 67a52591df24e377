# round 6, lease e: host path chunk size sweep (page-locked), after r6d (64 Ki blocks: +5-6 %)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r6e_host_chunks.jsonl; : > $out
for v in 65536 98304 131072 196608 262144 32768 131072 65536; do
  echo "{\"chunk_blocks\": $v}" >> $out
  PPFS_ECC_CHUNK_BLOCKS=$v timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned,pageable --reps 5 2>/dev/null >> $out || { tail -5 $out; exit 1; }
done
cat $out
