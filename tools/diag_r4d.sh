# one-off diagnostic (round 4): A/B of the round-3 and current libraries on one box, then the
# destroy-beside-a-server lifecycle test on each library with the create steps traced
set -o pipefail
mkdir -p gpurun_out
R3=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_r3.so
NEW=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so
bash tools/gpu.sh r4d ab=$R3,$NEW,1 || exit 1
PT="python -u -m pytest tests/test_gpu_lifecycle.py -k destroy_does_not_wait -x -v -s --timeout 120 --timeout-method thread -m gpu"
PPFS_ECC_TRACE=1 timeout -k 10 150 $PT > gpurun_out/r4d_life_new.log 2>&1; rc=$?
echo "new lifecycle rc=$rc"; tail -3 gpurun_out/r4d_life_new.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
PPFS_ECC_LIB=$R3 timeout -k 10 150 $PT > gpurun_out/r4d_life_r3.log 2>&1; rc=$?
echo "r3 lifecycle rc=$rc"; tail -3 gpurun_out/r4d_life_r3.log
exit 0
