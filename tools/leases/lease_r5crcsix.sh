#!/bin/bash
# Round 5: CRC encode on 6-bit piece / Horner maps (lease libs crcsix: -DPPFS_CRC_ENC_SIX=1, 92 VGPRs, 25 KiB
# image; crcsix6: the same at 6 waves per SIMD) against the shipped 8-bit maps (base): CRC GPU tests on each,
# then the configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
for v in crcsix crcsix6; do
    PPFS_ECC_LIB=$L/libppfs_ecc_$v.so timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "crc or CRC" > gpurun_out/r5six_test_$v.log 2>&1 || { tail -5 gpurun_out/r5six_test_$v.log; exit 1; }
    tail -1 gpurun_out/r5six_test_$v.log
done
for r in 1 2 3; do
    for v in base crcsix crcsix6; do
        PPFS_ECC_LIB=$L/libppfs_ecc_$v.so timeout -k 10 200 python -u tools/bench_configs.py --only crc | sed "s|^|{\"lib\": \"$v\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5six_cfg_ab.jsonl || exit 1
    done
done
