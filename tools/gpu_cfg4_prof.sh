# GPU box: rocprofv3 kernel trace (--stats) and FETCH/WRITE/SQ PMC passes of the cfg4 streaming
# kernels (Hamming, CRC 0x9960034c, parity; bs 4096, 2^20 blocks).  Usage: tools/gpu_cfg4_prof.sh <tag>
set -o pipefail
TAG=${1:-r1}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOTDIR/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in hamming crc parity; do
  OUT=$ROOTDIR/gpurun_out/cfg4_${TAG}_$c
  mkdir -p $OUT
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $ROOTDIR/tools/run_one.py $c 4096 10 > $OUT/trace.log 2>&1 || { echo "trace $c failed"; tail -5 $OUT/trace.log; exit 1; }
done
timeout -k 10 300 bash $ROOTDIR/tools/pmc_py.sh cfg4_${TAG}_ham $ROOTDIR/tools/run_one.py hamming > $ROOTDIR/gpurun_out/pmc_cfg4_ham.log 2>&1 || { echo "pmc ham failed"; cat $ROOTDIR/gpurun_out/pmc_cfg4_ham.log; exit 1; }
timeout -k 10 300 bash $ROOTDIR/tools/pmc_py.sh cfg4_${TAG}_crc $ROOTDIR/tools/run_one.py crc > $ROOTDIR/gpurun_out/pmc_cfg4_crc.log 2>&1 || { echo "pmc crc failed"; cat $ROOTDIR/gpurun_out/pmc_cfg4_crc.log; exit 1; }
echo done
