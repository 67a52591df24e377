# GPU box: RS tests on the current build and on variant $1 (alt lib), then cfg5 A/B
set -o pipefail
mkdir -p gpurun_out
V=${1:-nw4}
A=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$V.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rs or full_size" > gpurun_out/pair_t.log 2>&1
rc=$?; tail -2 gpurun_out/pair_t.log; [ $rc -eq 0 ] || exit $rc
PPFS_ECC_LIB=$A timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rs or full_size" > gpurun_out/pair_t_$V.log 2>&1
rc=$?; tail -2 gpurun_out/pair_t_$V.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in new $V; do
  if [ $v = new ]; then L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; else L=$A; fi
  PPFS_ECC_LIB=$L timeout -k 10 120 python tools/bench_configs.py --only ${ONLY:-t16} > gpurun_out/abpair_${v}_$r.log 2>&1 || exit 1
done
done
for f in gpurun_out/abpair_*; do echo $f; grep config $f | cut -c150-330; done
