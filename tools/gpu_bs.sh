# GPU box: byte-slice t=16 kernels -- GPU suite, then kernel timings of encode variants, then the cfg5 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_bs.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_bs.log; [ $rc -eq 0 ] || exit $rc
for v in ${BS_VARIANTS:-default enc12 enc10 default}; do
  if [ $v = default ]; then L=""; else L=paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 200 python tools/kernel_ablate.py --block-size 4096 --t 16 --tag $v >> gpurun_out/bs_kablate.jsonl 2>gpurun_out/bs_kablate.err || { tail gpurun_out/bs_kablate.err; exit 1; }
done
cat gpurun_out/bs_kablate.jsonl
timeout -k 10 300 python bench.py --block-size 4096 --t 16 --no-host-inclusive > gpurun_out/bench_bs_cfg5.log 2>&1; rc=$?; tail -1 gpurun_out/bench_bs_cfg5.log | cut -c1-1500; exit $rc
