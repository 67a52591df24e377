# A/B of library builds on one codec's kernel times (tools/time_codec.py), interleaved, N rounds:
#   bash tools/ab_codec.sh TAG CODEC N LIB1 LIB2 ...
set -o pipefail
TAG=$1; C=$2; N=$3; shift 3
mkdir -p gpurun_out
for r in $(seq 1 $N); do
    for L in "$@"; do
        PPFS_ECC_LIB=$L timeout -k 10 180 python tools/time_codec.py $C 30 | tee -a gpurun_out/${TAG}_${C}_ab.jsonl || exit 1
    done
done
