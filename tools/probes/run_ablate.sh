set -o pipefail
mkdir -p gpurun_out
for b in stream_ablate stream_ablate2 rs_ablate rs_ablate_dec; do
  echo "== $b"; timeout -k 10 120 ./tools/probes/$b.bin || exit 1
done
