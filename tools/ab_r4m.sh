# round 4: write-back as a 64-byte region instead of a lone byte -- Hamming decode (kernel times)
# and the t <= 4 RS decode (parity tests + in-step bench A/B)
set -o pipefail
MAIN=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so
ALT=$PWD/paritypartyfs_amd/_lib/alt
bash tools/ab_codec.sh r4m hamming 3 $MAIN $ALT/libppfs_ecc_hamwb64.so || exit 1
PPFS_ECC_LIB=$ALT/libppfs_ecc_rswb64.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k rs > gpurun_out/r4m_rswb64_rs.log 2>&1 || { tail -5 gpurun_out/r4m_rswb64_rs.log; exit 1; }
tail -1 gpurun_out/r4m_rswb64_rs.log
bash tools/gpu.sh r4m ab=$MAIN,$ALT/libppfs_ecc_rswb64.so,3 || exit 1
