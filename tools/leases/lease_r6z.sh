# round 6, lease z: timing ablation of the cfg5 decode's single-error path (wrong bytes on purpose in
# noboth): noxp = the XP-row confirmation's 16 exp lookups skipped (the 1-error batch still decodes
# right), noboth = also the S12 lookups (garbage positions); configs leg --only cfg5, 3 rounds
set -o pipefail
mkdir -p gpurun_out
L=$PWD/paritypartyfs_amd/_lib/lease
out=gpurun_out/r6z_cfg5_corr_ablation.jsonl; : > $out
for rnd in 1 2 3; do
for v in base noxp noboth; do
  if [ $v = base ]; then lib=""; else lib="PPFS_ECC_LIB=$L/libppfs_ecc_$v.so"; fi
  env $lib timeout -k 10 200 python tools/bench_configs.py --only cfg5 > gpurun_out/r6z_tmp.jsonl 2>gpurun_out/r6z_tmp.err || { echo "fail $v"; tail -5 gpurun_out/r6z_tmp.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r6z_tmp.jsonl'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(json.dumps({'variant':'$v','round':$rnd,'encode_ms':d.get('encode_ms'),'decode_clean_ms':d.get('decode_clean_ms'),'decode_1err_ms':d.get('decode_1err_ms'),'ok':d.get('roundtrip_ok')}))" >> $out
done
done
cat $out
