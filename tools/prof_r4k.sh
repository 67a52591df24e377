# round 4: cfg4 parity tests + A/B + PMC (tools/prof_cfg4.sh), the cfg5 half-chain timing ablation,
# the t=3 decode 8-byte-window variant (parity + bench A/B), then the default bench's rocprofv3 trace
# + PMC passes (tools/profile_box.sh)
set -o pipefail
TAG=${1:-r4k}
ALT=$PWD/paritypartyfs_amd/_lib/alt
MAIN=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so
bash tools/gpu.sh ${TAG} tests=crc+or+hamming || exit 1
timeout -k 10 900 bash tools/prof_cfg4.sh ${TAG} || exit 1
for r in 1 2; do
    for L in $MAIN $ALT/libppfs_ecc_bshalf.so; do
        PPFS_ECC_LIB=$L timeout -k 10 120 python tools/time_codec.py rs16 | tee -a gpurun_out/${TAG}_bshalf_ab.jsonl || exit 1
    done
done
PPFS_ECC_LIB=$ALT/libppfs_ecc_decw64.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k rs > gpurun_out/${TAG}_decw64_rs.log 2>&1 || { tail -5 gpurun_out/${TAG}_decw64_rs.log; exit 1; }
tail -1 gpurun_out/${TAG}_decw64_rs.log
bash tools/gpu.sh ${TAG} ab=$MAIN,$ALT/libppfs_ecc_decw64.so,2 || exit 1
timeout -k 10 1000 bash tools/profile_box.sh ${TAG} --no-configs > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -3 gpurun_out/${TAG}_prof.log
