# round 5, lease y: CRC check map staging by LDS-DMA with the first block's loads right behind
# (vs plain loads + barrier + block loads): CRC oracle tests, cfg4 CRC A/B
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
P=paritypartyfs_amd/_lib/libppfs_ecc.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_block_device.py -k "crc" > gpurun_out/r5y_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5y_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in $L/libppfs_ecc_crcplain.so $P; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only "cfg4 crc" > gpurun_out/r5y_tmp.jsonl 2>gpurun_out/r5y_ab.err || { tail -5 gpurun_out/r5y_ab.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5y_tmp.jsonl >> gpurun_out/r5y_crc_dma_stage_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5y_crc_dma_stage_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d['roundtrip_ok'], {k: v for k, v in d.items() if k.endswith('_ms') or k.startswith('roofline_frac_')})"
