# round 5, lease e: host path A/B (a stream per slot vs a stream per stage), 5 reps per call, then a
# copy/kernel trace of the page-locked calls
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
for lib in $L/libppfs_ecc_2slot.so paritypartyfs_amd/_lib/libppfs_ecc.so; do
  echo "== $lib"
  PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/probes/host_path_probe.py >> gpurun_out/r5e_host.jsonl 2>gpurun_out/r5e_host.err || { tail -5 gpurun_out/r5e_host.err; exit 1; }
  tail -6 gpurun_out/r5e_host.jsonl
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r5e_trace -o run -- python tools/probes/host_path_probe.py --modes pinned --reps 2 > gpurun_out/r5e_trace.log 2>&1 || { tail -20 gpurun_out/r5e_trace.log; exit 1; }
find gpurun_out/r5e_trace -name "*.csv" | head
