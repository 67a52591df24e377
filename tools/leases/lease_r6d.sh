# round 6, lease d: host path staging shapes (chunk size, decode codewords on the H2D stream), page-locked
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r6d_host_shapes.jsonl; : > $out
for v in "" "PPFS_ECC_HOST_SPLIT=1" "PPFS_ECC_CHUNK_BLOCKS=65536" "PPFS_ECC_CHUNK_BLOCKS=16384" "PPFS_ECC_HOST_SPLIT=1 PPFS_ECC_CHUNK_BLOCKS=65536" "" "PPFS_ECC_HOST_SPLIT=1"; do
  echo "{\"variant\": \"$v\"}" >> $out
  env $v timeout -k 10 120 python tools/probes/host_path_probe.py --modes pinned --reps 5 >> $out 2>&1 || { tail -5 $out; exit 1; }
done
cat $out
