# round-4 final build: GPU suite, smoke, the driver's bench, configs, then an A/B against the build
# before the 5-bit field encode tables (r4r), the phase traces, and the rocprofv3 records
set -o pipefail
TAG=${1:-r4t}
bash tools/gpu.sh ${TAG} tests smoke benchfull configs ab=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_r4r.so,$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so,2 tktrace || exit 1
timeout -k 10 1000 bash tools/profile_box.sh ${TAG} --no-configs > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -3 gpurun_out/${TAG}_prof.log
