#!/bin/bash
# Runs ON the GPU box (via gpurun): rocprofv3 kernel trace + separate PMC passes for bench.py.
# Usage: tools/profile_box.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-r1}; shift
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/prof_$TAG
mkdir -p $OUT
sha256sum $ROOTDIR/paritypartyfs_amd/_lib/libppfs_ecc.so | cut -d' ' -f1 > $OUT/lib.sha256
cd /tmp && export TMPDIR=/tmp
B="python3 $ROOTDIR/bench.py --steps 50 --warmup 5 --prewarm-s 0.3 --no-cpu-baseline --no-host-inclusive $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- $B > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- $B > $OUT/fetch.log 2>&1 || { echo "fetch failed"; tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- $B > $OUT/write.log 2>&1 || { echo "write failed"; tail -20 $OUT/write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $OUT/sq -o sq --output-format csv -- $B > $OUT/sq.log 2>&1 || { echo "sq failed"; tail -20 $OUT/sq.log; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/sq2 -o sq2 --output-format csv -- $B > $OUT/sq2.log 2>&1 || { echo "sq2 failed"; tail -20 $OUT/sq2.log; }
find $OUT -name "*.csv" | head -50
echo done
