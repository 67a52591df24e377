#!/bin/bash
# GPU box: the whole -m gpu suite on the PPFS_ECC_DEBUG build (csrc/dbg.hpp: every kernel
# bounds-checks its global accesses against the extents its launch implies, counts and skips the
# ones outside; tests/conftest.py fails a test whose kernels counted any), with PPFS_ECC_SYNC_CHECK=1
# (every device entry point synchronizes and reports its own asynchronous errors).
# Build first: tools/build_alt.sh --product debug -DPPFS_ECC_DEBUG=1
set -o pipefail
TAG=${1:-debug}
mkdir -p gpurun_out
PPFS_ECC_LIB=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_debug.so PPFS_ECC_SYNC_CHECK=1 \
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_pytest.log
grep -m 20 "PPFS_ECC_DEBUG" gpurun_out/${TAG}_pytest.log
exit $rc
