# round-4 profiles: rocprofv3 kernel trace + PMC passes of the default bench and of the cfg5 bench
set -o pipefail
timeout -k 10 1000 bash tools/profile_box.sh ${1:-r4i} --no-configs > gpurun_out/${1:-r4i}_prof.log 2>&1 || { tail -20 gpurun_out/${1:-r4i}_prof.log; exit 1; }
tail -3 gpurun_out/${1:-r4i}_prof.log
timeout -k 10 1000 bash tools/profile_box.sh ${1:-r4i}_cfg5 --no-configs --block-size 4096 --t 16 > gpurun_out/${1:-r4i}_cfg5_prof.log 2>&1 || { tail -20 gpurun_out/${1:-r4i}_cfg5_prof.log; exit 1; }
tail -3 gpurun_out/${1:-r4i}_cfg5_prof.log
