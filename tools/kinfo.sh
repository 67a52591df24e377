#!/bin/bash
# Register / LDS / scratch use of the kernels in one RS instantiation: tools/kinfo.sh <T2> <name regex> [hipcc flags]
T2=$1; RE=$2; shift 2
cd "$(dirname "$0")/../paritypartyfs_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-inline-asm --cuda-device-only -S -DPPFS_T2=$T2 "$@" rs_fast_inst.hip -o /tmp/kinfo_$$.s || exit 1
awk -v re="$RE" '/^\t\.amdhsa_kernel /{name=$2; f=(name ~ re)} f&&/next_free_vgpr|group_segment_fixed_size|private_segment_fixed_size/{print substr(name,1,48), $1, $2} /\.end_amdhsa_kernel/{f=0}' /tmp/kinfo_$$.s
rm -f /tmp/kinfo_$$.s
