#!/bin/bash
# Round 5: NT payload loads in the Hamming / parity encodes (shipped lib) vs without (encld0),
# configs leg of cfg4 Hamming and parity, interleaved
set -o pipefail
mkdir -p gpurun_out
N=paritypartyfs_amd/_lib/libppfs_ecc.so
O=paritypartyfs_amd/_lib/lease/libppfs_ecc_encld0.so
for r in 1 2 3; do
    for L in $N $O; do
        for c in hamming parity; do
            PPFS_ECC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only $c | sed "s|^|{\"lib\": \"$(basename $L)\", \"r\": $r, \"line\": |; s|$|}|" >> gpurun_out/r5nt_cfg_ab.jsonl || exit 1
        done
    done
done
