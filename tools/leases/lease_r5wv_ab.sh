#!/bin/bash
# Round 5: Hamming / parity kernels in one-wave workgroups, waves per CU capped at 6 / 8 / 12 / 16
# (lease libs wv1_*), against the shipped 4-wave workgroups; configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
B=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2; do
    for L in $B paritypartyfs_amd/_lib/lease/libppfs_ecc_wv1_{6,8,12,16}.so; do
        for c in hamming parity; do
            PPFS_ECC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only $c | sed "s|^|{\"lib\": \"$(basename $L)\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5wv_cfg_ab.jsonl || exit 1
        done
    done
done
