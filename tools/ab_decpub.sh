# round 4: decode ticket published after barrier C with the single-error write-backs deferred there
# (decpub) vs the final build: RS parity + lifecycle, in-step bench A/B, phase traces
set -o pipefail
MAIN=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so
ALT=$PWD/paritypartyfs_amd/_lib/alt
PPFS_ECC_LIB=$ALT/libppfs_ecc_decpub.so timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_lifecycle.py tests/test_gpu_block_device.py -k "rs or ticket or stream or slot or recycled or Reed" > gpurun_out/r4s_decpub_rs.log 2>&1 || { tail -15 gpurun_out/r4s_decpub_rs.log; exit 1; }
tail -1 gpurun_out/r4s_decpub_rs.log
bash tools/gpu.sh r4s ab=$MAIN,$ALT/libppfs_ecc_decpub.so,3 || exit 1
PPFS_ECC_LIB=$ALT/libppfs_ecc_decpubtrace.so timeout -k 10 120 python tools/tk_trace.py 2> /dev/null > gpurun_out/r4s_decpub_tktrace.jsonl || { tail gpurun_out/r4s_decpub_tktrace.jsonl; exit 1; }
cut -c1-2500 gpurun_out/r4s_decpub_tktrace.jsonl
