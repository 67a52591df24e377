#!/bin/bash
# Round 5: CRC check and encode workgroup shapes, 8-bit piece maps in the check (lease libs g0-g3: 2x4, 4x4, 6x4, 8x2) on
# the compact 14 KiB map staging, against the shipped 4 x 4; configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
B=paritypartyfs_amd/_lib/libppfs_ecc.so
for r in 1 2; do
    for L in $B paritypartyfs_amd/_lib/lease/libppfs_ecc_g{0,1,2,3}.so; do
        PPFS_ECC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only crc | sed "s|^|{\"lib\": \"$(basename $L)\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5crc5_cfg_ab.jsonl || exit 1
    done
done
