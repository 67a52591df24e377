# GPU box: byte-slice t=16 variants -- t=16 parity subset per variant library, then kernel timings, then the cfg5 bench line
set -o pipefail
mkdir -p gpurun_out
SEL='4096-16 or cfg5_rs_t16 or rs4096t16'
for v in ${BS_VARIANTS:-encrp decrp enc12 enc12rp}; do
  PPFS_ECC_LIB=paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "$SEL" > gpurun_out/pytest_bs_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/pytest_bs_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in default ${BS_VARIANTS:-encrp decrp enc12 enc12rp} default; do
  if [ $v = default ]; then L=""; else L=paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 200 python tools/kernel_ablate.py --block-size 4096 --t 16 --tag $v >> gpurun_out/bs_kablate2.jsonl 2>gpurun_out/bs_kablate.err || { tail gpurun_out/bs_kablate.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/bs_kablate2.jsonl'):
    d=json.loads(l); print(d['tag'], d['enc_hot_us'], d['enc_cold_us'], d['dec_hot_us'], d['dec_cold_us'], d['dec_1err_nowb_hot_us'])"
