#!/bin/bash
# Round 5: Hamming / parity workgroup shapes and wave caps, second sweep (lease libs s*), against
# the shipped build; configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
B=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2; do
    for L in $B paritypartyfs_amd/_lib/lease/libppfs_ecc_s{10,12,14,4b,2}.so; do
        for c in hamming parity; do
            PPFS_ECC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only $c | sed "s|^|{\"lib\": \"$(basename $L)\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5wv2_cfg_ab.jsonl || exit 1
        done
    done
done
