# one-off diagnostic (round 4): the destroy-beside-a-server lifecycle test hangs in a fresh process
# (round-3 library too).  Variants: more hardware queues, the server on a high-priority stream,
# no server (launch path).
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest tests/test_gpu_lifecycle.py -k destroy_does_not_wait -x -v -s --timeout 60 --timeout-method thread -m gpu"
for v in "GPU_MAX_HW_QUEUES=8" "PPFS_ECC_SRV_PRIO=1" "PPFS_ECC_SERVER=0" "PPFS_ECC_NONE=1"; do
    tag=${v%%=*}
    env PPFS_ECC_TRACE=1 $v timeout -k 10 100 $PT > gpurun_out/r4g_$tag.log 2>&1; rc=$?
    echo "$v rc=$rc $(grep -c 'server: launch' gpurun_out/r4g_$tag.log) launches"; tail -2 gpurun_out/r4g_$tag.log
    [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
done
exit 0
