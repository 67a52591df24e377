#!/bin/bash
# Kernel resources of a built library: LDS, scratch, SGPRs, VGPRs, VGPR spills per kernel (gfx950
# code object notes).  Usage: tools/kres.sh [lib.so] [name filter regex]
LIB=$(realpath ${1:-paritypartyfs_amd/_lib/libppfs_ecc.so}); PAT=${2:-.}
D=$(mktemp -d) && cd $D && cp $LIB l.so && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading l.so >/dev/null 2>&1
for o in *gfx950*; do /opt/rocm/lib/llvm/bin/llvm-readelf --notes $o; done | python3 -c "
import re,sys
cur=None; rows=[]
for line in sys.stdin:
    m=re.match(r'\s+\.(group_segment_fixed_size|name|private_segment_fixed_size|sgpr_count|vgpr_count|vgpr_spill_count):\s+(\S+)',line)
    if not m: continue
    k,v=m.groups()
    if k=='group_segment_fixed_size': cur={}; rows.append(cur)
    cur[k]=v
for r in rows:
    n=r.get('name','?')
    if re.search(sys.argv[1], n): print('lds %6s scratch %4s sgpr %3s vgpr %3s spill %s  %s' % (r.get('group_segment_fixed_size'), r.get('private_segment_fixed_size'), r.get('sgpr_count'), r.get('vgpr_count'), r.get('vgpr_spill_count'), n[:110]))
" "$PAT"
rm -rf $D
