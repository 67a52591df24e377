# round 5, lease a: tiny Hamming / parity tests + C++ adapter, the driver's bench line (host link),
# cfg5 ILP2 chain ablation, CRC per-position maps (oracle tests on the variant, cfg4 A/B)
set -o pipefail
mkdir -p gpurun_out
L=paritypartyfs_amd/_lib/lease
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $PYT tests > gpurun_out/r5a_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5a_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/bs_chain_probe.bin > gpurun_out/r5a_chain_probe.jsonl 2>&1; rc=$?; cat gpurun_out/r5a_chain_probe.jsonl; [ $rc -eq 0 ] || exit $rc
PPFS_ECC_LIB=$L/libppfs_ecc_crcpp.so timeout -k 10 300 $PYT tests/test_gpu_parity.py -k crc > gpurun_out/r5a_crcpp_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5a_crcpp_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r5a_benchfull.json 2> gpurun_out/r5a_benchfull.err || { tail -5 gpurun_out/r5a_benchfull.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r5a_benchfull.json').read().strip().splitlines()[-1]);print(d['value'],d['in_step_frac'],d['host_inclusive'])"
for r in 1 2; do
  for lib in paritypartyfs_amd/_lib/libppfs_ecc.so $L/libppfs_ecc_crcpp.so; do
    PPFS_ECC_LIB=$lib timeout -k 10 300 python tools/bench_configs.py --only cfg4 > gpurun_out/r5a_cfg4_tmp.jsonl 2>gpurun_out/r5a_cfg4.err || { tail -5 gpurun_out/r5a_cfg4.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $lib) $r gpurun_out/r5a_cfg4_tmp.jsonl >> gpurun_out/r5a_cfg4_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5a_cfg4_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], d.get('name'), {k: v for k, v in d.items() if 'frac' in k})"
for v in splitrd rp; do
  PPFS_ECC_LIB=$L/libppfs_ecc_$v.so timeout -k 10 300 $PYT tests/test_gpu_parity.py -k "rs and 4096" > gpurun_out/r5a_${v}_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5a_${v}_pytest.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_codec.sh r5a rs16 3 paritypartyfs_amd/_lib/libppfs_ecc.so $L/libppfs_ecc_rp.so $L/libppfs_ecc_splitrd.so $L/libppfs_ecc_n1.so $L/libppfs_ecc_ilp2n1.so || exit 1
# last: unaligned 16-byte global stores (a misaligned-access fault would end the lease here)
timeout -k 10 120 tools/row_store_probe.bin > gpurun_out/r5a_row_store_probe.jsonl 2>&1; rc=$?; cat gpurun_out/r5a_row_store_probe.jsonl; [ $rc -eq 0 ] || exit $rc
