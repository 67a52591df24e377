# round 5, lease w: cfg5 decode per-wave start / end (trace build): how much of the kernel is tail
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
for m in "" "--clean"; do
  PPFS_ECC_LIB=$L/libppfs_ecc_trace.so timeout -k 10 300 python tools/bs_trace.py $m >> gpurun_out/r5w_cfg5_tail.jsonl 2> gpurun_out/r5w.err || { tail -5 gpurun_out/r5v.err; exit 1; }
done
cat gpurun_out/r5w_cfg5_tail.jsonl
