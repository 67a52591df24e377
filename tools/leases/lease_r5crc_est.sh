#!/bin/bash
# Round 5: CRC / parity kernels with their output stores issued before the CRC / parity computation (lease
# libs crcest: -DPPFS_CRC_ENC_EARLY_ST=1; crccst: -DPPFS_CRC_CHK_EARLY_ST=1, check at 97 VGPRs; parest:
# -DPPFS_PAR_CHK_EARLY_ST=1) against the same build without (base): the GPU parity tests of each variant's
# codec, then the configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
for v in crcest:crc crccst:crc parest:parity; do
    K=${v#*:}; v=${v%:*}
    PPFS_ECC_LIB=paritypartyfs_amd/_lib/lease/libppfs_ecc_$v.so timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k $K > gpurun_out/r5est_test_$v.log 2>&1 || { tail -5 gpurun_out/r5est_test_$v.log; exit 1; }
    tail -1 gpurun_out/r5est_test_$v.log
done
for r in 1 2 3; do
    for L in paritypartyfs_amd/_lib/lease/libppfs_ecc_{base,crcest,crccst}.so; do
        PPFS_ECC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only crc | sed "s|^|{\"lib\": \"$(basename $L)\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5est_cfg_ab.jsonl || exit 1
    done
done
for r in 1 2 3; do
    for L in paritypartyfs_amd/_lib/lease/libppfs_ecc_{base,parest}.so; do
        PPFS_ECC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only parity | sed "s|^|{\"lib\": \"$(basename $L)\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5est_par_ab.jsonl || exit 1
    done
done
