#!/bin/bash
# Round 5: status bytes and corrected-byte write-backs of the Hamming decode and the CRC / parity checks
# stored after the payload emission (lease lib latest: -DPPFS_BF_LATE_ST=1) against the same build without
# (base): the GPU tests of those codecs on the variant, then the configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
PPFS_ECC_LIB=paritypartyfs_amd/_lib/lease/libppfs_ecc_latest.so timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "hamming or crc or parity or Hamming or CRC" > gpurun_out/r5late_test.log 2>&1 || { tail -5 gpurun_out/r5late_test.log; exit 1; }
tail -1 gpurun_out/r5late_test.log
for r in 1 2 3; do
    for L in paritypartyfs_amd/_lib/lease/libppfs_ecc_{base,latest}.so; do
        for c in hamming crc parity; do
            PPFS_ECC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only $c | sed "s|^|{\"lib\": \"$(basename $L)\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5late_cfg_ab.jsonl || exit 1
        done
    done
done
