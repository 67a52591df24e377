# round 4: staged encode emission -- RS parity, A/B against the round-3 library, phase trace
set -o pipefail
A=$PWD/paritypartyfs_amd/_lib/alt
bash tools/gpu.sh r4f rs ab=$A/libppfs_ecc_r3.so,$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so,2 tktrace
