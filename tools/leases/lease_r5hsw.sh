#!/bin/bash
# Round 5: Hamming decode workgroup shape / wave cap re-tuned after the early image and late status stores
# (lease libs h2x16: 2-wave workgroups; h4x12 / h4x20: 4-wave at 12 / 20 waves per CU; h8x16: 8-wave) against
# the shipped 4-wave x 16 (base); Hamming GPU tests on each, then the configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
for v in h2x16 h4x12 h4x20 h8x16; do
    PPFS_ECC_LIB=$L/libppfs_ecc_$v.so timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "hamming or Hamming" > gpurun_out/r5hsw_test_$v.log 2>&1 || { tail -5 gpurun_out/r5hsw_test_$v.log; exit 1; }
    tail -1 gpurun_out/r5hsw_test_$v.log
done
for r in 1 2; do
    for v in base h2x16 h4x12 h4x20 h8x16; do
        PPFS_ECC_LIB=$L/libppfs_ecc_$v.so timeout -k 10 200 python -u tools/bench_configs.py --only hamming | sed "s|^|{\"lib\": \"$v\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5hsw_cfg_ab.jsonl || exit 1
    done
done
