#!/bin/bash
# Round 5: (a) CRC check on 8-bit piece maps (lease libs g0-g3: 2x4, 4x4, 6x4, 8x2 workgroup x blocks);
# (b) Hamming decode emission unrolled (h1: 2, h2: 4; h3: 4 at 12 waves per CU; h4 / h5: 4 in
# one-wave workgroups at 16 / 12 waves per CU) -- against the shipped build, configs leg, interleaved
set -o pipefail
mkdir -p gpurun_out
B=paritypartyfs_amd/_lib/libppfs_ecc.so
run() { PPFS_ECC_LIB=$1 timeout -k 10 200 python -u tools/bench_configs.py --only $2 | sed "s|^|{\"lib\": \"$(basename $1)\", \"r\": $3, \"line\": |; s|$|}|" >> gpurun_out/r5mix_cfg_ab.jsonl; }
for r in 1 2; do
    for L in $B paritypartyfs_amd/_lib/lease/libppfs_ecc_g{0,1,2,3}.so; do run $L crc $r || exit 1; done
    for L in $B paritypartyfs_amd/_lib/lease/libppfs_ecc_h{1,2,3,4,5}.so; do run $L hamming $r || exit 1; done
done
