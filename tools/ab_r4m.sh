# round 4 A/Bs: cfg5 with four lanes per block (rs_bs4.hpp: parity, then kernel times), the
# write-back of a fix's 64-byte region (Hamming; t <= 4 RS decode: parity + bench), bit kernels
# with blocks per wave + prefetch
set -o pipefail
MAIN=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so
ALT=$PWD/paritypartyfs_amd/_lib/alt
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py"
PPFS_ECC_LIB=$ALT/libppfs_ecc_bsquad.so timeout -k 10 600 $PYT -k "rs and (16 or 4096 or t16)" > gpurun_out/r4m_bsquad_rs.log 2>&1 || { tail -15 gpurun_out/r4m_bsquad_rs.log; exit 1; }
tail -1 gpurun_out/r4m_bsquad_rs.log
bash tools/ab_codec.sh r4m rs16 2 $MAIN $ALT/libppfs_ecc_bsquad.so || exit 1
PPFS_ECC_LIB=$ALT/libppfs_ecc_bsquade.so timeout -k 10 600 $PYT -k "rs and (16 or 4096 or t16)" > gpurun_out/r4m_bsquade_rs.log 2>&1 || { tail -15 gpurun_out/r4m_bsquade_rs.log; exit 1; }
tail -1 gpurun_out/r4m_bsquade_rs.log
bash tools/ab_codec.sh r4m_enc rs16 2 $MAIN $ALT/libppfs_ecc_bsquade.so || exit 1
bash tools/ab_codec.sh r4m hamming 2 $MAIN $ALT/libppfs_ecc_hamwb64.so $ALT/libppfs_ecc_bpw2pf.so || exit 1
bash tools/ab_codec.sh r4m crc 1 $MAIN $ALT/libppfs_ecc_bpw2pf.so || exit 1
PPFS_ECC_LIB=$ALT/libppfs_ecc_rswb64.so timeout -k 10 600 $PYT -k rs > gpurun_out/r4m_rswb64_rs.log 2>&1 || { tail -5 gpurun_out/r4m_rswb64_rs.log; exit 1; }
tail -1 gpurun_out/r4m_rswb64_rs.log
bash tools/gpu.sh r4m ab=$MAIN,$ALT/libppfs_ecc_rswb64.so,2 || exit 1
