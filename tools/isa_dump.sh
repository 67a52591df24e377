#!/bin/bash
# Dumps the gfx950 device assembly of every product translation unit into $1 (one .s per TU and
# 2t instance), so that a source clean-up can be checked to leave the shipped ISA unchanged:
#   tools/isa_dump.sh /tmp/isa_a; <edit>; tools/isa_dump.sh /tmp/isa_b; diff -r /tmp/isa_a /tmp/isa_b
set -e
OUT=$(realpath -m "$1"); mkdir -p "$OUT"
cd "$(dirname "$0")/../paritypartyfs_amd/csrc"
F="--offload-arch=gfx950 -O3 -std=c++17 -Wno-inline-asm -Wno-unused-function --cuda-device-only -S"
for t in 2 4 6 8 10 16 32; do
  /opt/rocm/bin/hipcc $F -DPPFS_T2=$t rs_fast_inst.hip -o "$OUT/rs_fast_t$t.s" &
done
for s in rs_kernels bit_kernels bit_fast vote; do
  /opt/rocm/bin/hipcc $F $s.hip -o "$OUT/$s.s" &
done
wait
# drop lines that name source files or the compiler build (not code)
sed -i -e '/\.file\s/d' -e '/\.ident/d' -e '/^\s*\.loc\s/d' -e '/amdhsa.printf/d' -e 's/__hip_cuid_[0-9a-f]*/__hip_cuid_X/g' "$OUT"/*.s
