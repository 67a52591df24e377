#!/bin/bash
# GPU box: A/B of engine builds on the DEFAULT bench line (as the driver runs it, minus the CPU
# and host legs), R rounds interleaved.  Usage: R=3 VARIANTS="a b" tools/ab_bench_full.sh <tag>
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 ${R:-3}); do
for v in new ${VARIANTS}; do
  if [ $v = new ]; then L=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; else L=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_$v.so; fi
  PPFS_ECC_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-inclusive "$@" > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
  python3 - gpurun_out/${TAG}_${v}_$r.json $v $r <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k, s = d["kernels_ms"], d["standalone"]
print(f"{sys.argv[2]:>8} r{sys.argv[3]} value {d['value']:8.1f} rep {d.get('repeat_ms_per_step')} | frac {d['roofline']['frac']:.4f} in-step enc {k['encode']*1e3:6.1f} dec {k['decode']*1e3:6.1f} | sa enc {s['encode_ms_median']*1e3:6.1f} dec {s['clean_decode_ms_median']*1e3:6.1f} cold enc {s['cold_encode_ms_median']*1e3:6.1f} dec {s['cold_clean_decode_ms_median']*1e3:6.1f}")
PY
done
done
