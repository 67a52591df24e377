# round 6, lease bb: RS(255,249) decode write-backs straight into a page-locked caller image (the decode
# kernel stores its corrections there: no codeword copy, no patch kernel) -- the GPU suite on the new
# library, then the host-path probe, old (second final build) vs new, page-locked, 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r6bb_gputest.log 2>&1; rc=$?
tail -2 gpurun_out/r6bb_gputest.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/paritypartyfs_amd/_lib/lease
out=gpurun_out/r6bb_host_wbdirect_ab.jsonl; : > $out
for rnd in 1 2 3; do
for v in old new; do
  if [ $v = new ]; then lib=""; else lib="PPFS_ECC_LIB=$L/libppfs_ecc_$v.so"; fi
  echo "{\"variant\": \"$v\", \"round\": $rnd}" >> $out
  env $lib timeout -k 10 300 python tools/probes/host_path_probe.py --modes pinned --reps 5 >> $out 2> gpurun_out/r6bb_tmp.err || { echo "fail $v"; tail -5 gpurun_out/r6bb_tmp.err; exit 1; }
done
done
cat $out
