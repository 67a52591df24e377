# round 4: tickets taken at the end of an iteration and published after barrier B of the next
# (tkend) vs the current build: RS parity + lifecycle on tkend, in-step bench A/B, phase traces
set -o pipefail
MAIN=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so
ALT=$PWD/paritypartyfs_amd/_lib/alt
PPFS_ECC_LIB=$ALT/libppfs_ecc_tkend.so timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_lifecycle.py -k "rs or ticket or stream or slot or recycled" > gpurun_out/r4q_tkend_rs.log 2>&1 || { tail -15 gpurun_out/r4q_tkend_rs.log; exit 1; }
tail -1 gpurun_out/r4q_tkend_rs.log
bash tools/gpu.sh r4q ab=$MAIN,$ALT/libppfs_ecc_tkend.so,3 || exit 1
PPFS_ECC_LIB=$ALT/libppfs_ecc_tkendtrace.so timeout -k 10 120 python tools/tk_trace.py 2> /dev/null > gpurun_out/r4q_tkend_tktrace.jsonl || { tail gpurun_out/r4q_tkend_tktrace.jsonl; exit 1; }
cat gpurun_out/r4q_tkend_tktrace.jsonl | cut -c1-1500
