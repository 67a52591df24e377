#!/bin/bash
# Round 5: CRC kernels with register prefetch of the wave's next block (lease libs crcpf: -DPPFS_CRC_CHK_PF=1,
# check 127 VGPRs; crcepf: -DPPFS_CRC_ENC_PF=1, encode 95 VGPRs) against the same build without (base); configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
    for L in paritypartyfs_amd/_lib/lease/libppfs_ecc_{base,crcpf,crcepf}.so; do
        PPFS_ECC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only crc | sed "s|^|{\"lib\": \"$(basename $L)\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5cpf_cfg_ab.jsonl || exit 1
    done
done
