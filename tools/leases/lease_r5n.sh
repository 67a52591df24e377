# round 5, lease n: Hamming decode write-back as the corrected byte's whole 128-byte line (from
# registers) vs the lone byte store; oracle tests, write-back probe, cfg4 A/B
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_block_device.py -k "ham" > gpurun_out/r5n_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5n_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in $L/libppfs_ecc_base.so $P; do
  PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/probes/wb_probe.py --only hamming > gpurun_out/r5n_tmp.jsonl 2>gpurun_out/r5n_probe.err || { tail -5 gpurun_out/r5n_probe.err; exit 1; }
  echo "$(basename $lib) $(cat gpurun_out/r5n_tmp.jsonl)" | tee -a gpurun_out/r5n_wb_probe.txt
done
for r in 1 2; do
  for lib in $L/libppfs_ecc_base.so $P; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only "cfg4 hamming" > gpurun_out/r5n_tmp.jsonl 2>gpurun_out/r5n_ab.err || { tail -5 gpurun_out/r5n_ab.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5n_tmp.jsonl >> gpurun_out/r5n_ham_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5n_ham_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], {k: v for k, v in d.items() if k.endswith('_ms') or 'frac_dec' in k})"
