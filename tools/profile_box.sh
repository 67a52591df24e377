#!/bin/bash
# Runs ON the GPU box (via gpurun): rocprofv3 kernel trace + separate PMC passes for bench.py.
# Raw rocprofv3 output stays in /tmp; only the kernel stats, the per-kernel counter medians
# (tools/pmc_reduce.py), the library hash and the logs go to gpurun_out/prof_<tag>.
# Usage: tools/profile_box.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-r1}; shift
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/prof_$TAG
RAW=/tmp/prof_$TAG
mkdir -p $OUT $RAW
sha256sum $ROOTDIR/paritypartyfs_amd/_lib/libppfs_ecc.so | cut -d' ' -f1 > $OUT/lib.sha256
cd /tmp && export TMPDIR=/tmp
B="python3 $ROOTDIR/bench.py --steps 50 --warmup 5 --prewarm-s 0.3 --no-cpu-baseline --no-host-inclusive $*"
# the same bench command untraced first: its line is what the trace's averages must reproduce (the
# tracer adds ~4 us to every dispatch-packet interval the bench itself measures under it)
timeout -k 10 300 $B > $OUT/untraced.log 2>&1 || { echo "untraced bench failed"; tail -20 $OUT/untraced.log; exit 1; }
grep '^{"metric"' $OUT/untraced.log | tail -1 > $OUT/bench_line_untraced.json || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $RAW/trace -o trace --output-format csv -- $B > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
cp $RAW/trace/trace_kernel_stats.csv $OUT/
python3 $ROOTDIR/tools/trace_reduce.py $RAW/trace/trace_kernel_trace.csv $OUT/trace_durations.json || echo "trace_reduce failed"
grep '^{"metric"' $OUT/trace.log | tail -1 > $OUT/bench_line.json || true # the traced run's own bench line
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $RAW/fetch -o fetch --output-format csv -- $B > $OUT/fetch.log 2>&1 || { echo "fetch failed"; tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $RAW/write -o write --output-format csv -- $B > $OUT/write.log 2>&1 || { echo "write failed"; tail -20 $OUT/write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $RAW/sq -o sq --output-format csv -- $B > $OUT/sq.log 2>&1 || { echo "sq failed"; tail -20 $OUT/sq.log; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $RAW/sq2 -o sq2 --output-format csv -- $B > $OUT/sq2.log 2>&1 || { echo "sq2 failed"; tail -20 $OUT/sq2.log; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $RAW/sq3 -o sq3 --output-format csv -- $B > $OUT/sq3.log 2>&1 || { echo "sq3 failed"; tail -20 $OUT/sq3.log; }
python3 $ROOTDIR/tools/pmc_reduce.py $RAW $OUT/counters_median.json || exit 1
rm -rf $RAW
ls -la $OUT
echo done
