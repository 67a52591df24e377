# round 5, lease zj: cfg5 decode phase trace on the shipped kernels (tickets + priorities)
set -o pipefail
mkdir -p gpurun_out
for m in "" "--clean"; do
  PPFS_ECC_LIB=paritypartyfs_amd/_lib/lease/libppfs_ecc_trace.so timeout -k 10 300 python tools/bs_trace.py $m >> gpurun_out/r5zj_cfg5_phase_trace.jsonl 2> gpurun_out/r5zj.err || { tail -5 gpurun_out/r5zj.err; exit 1; }
done
cut -c1-700 gpurun_out/r5zj_cfg5_phase_trace.jsonl
