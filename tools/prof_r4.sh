# round-4 records on the final build: rocprofv3 kernel trace + PMC passes of the default bench and of
# the cfg5 bench (each beside an untraced run of the same command), then cfg4 (A/B vs round 3 + PMC)
set -o pipefail
TAG=${1:-r4p}
timeout -k 10 1000 bash tools/profile_box.sh ${TAG} --no-configs > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -3 gpurun_out/${TAG}_prof.log
timeout -k 10 1000 bash tools/profile_box.sh ${TAG}_cfg5 --no-configs --block-size 4096 --t 16 > gpurun_out/${TAG}_cfg5_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_cfg5_prof.log; exit 1; }
tail -3 gpurun_out/${TAG}_cfg5_prof.log
timeout -k 10 900 bash tools/prof_cfg4.sh ${TAG} || exit 1
