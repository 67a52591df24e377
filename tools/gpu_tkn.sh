#!/bin/bash
# GPU box: ring depth of the ticket encode (alt tkn3 / tkn4, rs_wg_tk_ablate.hpp) against the
# shipped kernel: RS parity tests on tkn4, then bench A/B.  Usage: tools/gpu_tkn.sh <tag>
set -o pipefail
TAG=${1:-tkn}
mkdir -p gpurun_out
PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_tkn4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hygiene.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rs or streams" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash tools/gpu_ab_bench.sh "" tkn3 tkn4 || exit 1
