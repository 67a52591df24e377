#!/bin/bash
# Round 5: Hamming decode with the LDS image stores issued before the syndrome reduction
# (lease lib hamei: -DPPFS_HAM_DEC_EARLY_IMG=1) against the same build without it (base); configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
    for L in paritypartyfs_amd/_lib/lease/libppfs_ecc_{base,hamei}.so; do
        PPFS_ECC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only hamming | sed "s|^|{\"lib\": \"$(basename $L)\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5hei_cfg_ab.jsonl || exit 1
    done
done
