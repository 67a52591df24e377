#!/bin/bash
# Round 5: CRC check and encode workgroup shapes, second sweep (lease libs d1-d6) on
# the compact 14 KiB map staging, against the shipped 4 x 4; configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
B=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2; do
    for L in $B paritypartyfs_amd/_lib/lease/libppfs_ecc_d{1,2,3,4,5,6}.so; do
        PPFS_ECC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only crc | sed "s|^|{\"lib\": \"$(basename $L)\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5crc2_cfg_ab.jsonl || exit 1
    done
done
