# round 6: the GPU suite on the bounds-checked build (PPFS_ECC_DEBUG: every kernel access range-checked, faults counted per test)
set -o pipefail
mkdir -p gpurun_out
PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/lease/libppfs_ecc_debug.so timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r6x_debug_suite.log 2>&1; rc=$?
tail -3 gpurun_out/r6x_debug_suite.log; exit $rc
