#!/bin/bash
# GPU box: A/B of engine builds on the bench line (current build = "new", others
# _lib/alt/libppfs_ecc_<v>.so), rounds interleaved.  Usage: VARIANTS="a b" tools/ab_bench.sh <tag> [bench args]
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
for v in new ${VARIANTS}; do
  if [ $v = new ]; then L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; else L=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-configs \
      --standalone-launches 20 --prewarm-s 0.5 "$@" > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
  python3 - gpurun_out/${TAG}_${v}_$r.json $v $r <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k, s = d["kernels_ms"], d["standalone"]
print(f"{sys.argv[2]:>8} r{sys.argv[3]} value {d['value']:8.1f} step {d['ms_per_step']:.4f} | in-step enc {k['encode']*1e3:6.1f} inj {k['inject']*1e3:5.1f} dec {k['decode']*1e3:6.1f} us | standalone enc {s['encode_ms_median']*1e3:6.1f} dec {s['clean_decode_ms_median']*1e3:6.1f} cold enc {s['cold_encode_ms_median']*1e3:6.1f} dec {s['cold_clean_decode_ms_median']*1e3:6.1f} us | copy {d['device_copy_GBps']} cold {d['device_copy_cold_GBps']}")
PY
done
done
