# round 5, lease zh: pageable host path with non-temporal (streaming) staging copies vs memcpy;
# host-path GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_block_device.py tests/test_vote_scrub.py -k "host or scrub or vote or group" > gpurun_out/r5zh_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5zh_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for nt in 0 1; do
    PPFS_ECC_COPY_NT=$nt timeout -k 10 300 python tools/probes/host_path_probe.py --modes pageable --reps 3 --from-torch > gpurun_out/r5zh_tmp.jsonl 2>gpurun_out/r5zh_probe.err || { tail -5 gpurun_out/r5zh_probe.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'copy_nt': int(sys.argv[1]), 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $nt $r gpurun_out/r5zh_tmp.jsonl >> gpurun_out/r5zh_copy_nt_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5zh_copy_nt_ab.jsonl'):
    d=json.loads(l); print(d['copy_nt'], d['round'], d['op'], d['GiBps'])"
