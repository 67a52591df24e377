#!/bin/bash
# Builds a variant of the engine into paritypartyfs_amd/_lib/alt/libppfs_ecc_<name>.so (load it with
# PPFS_ECC_LIB=...):
#   tools/build_alt.sh <name> '<extra hipcc flags>'            ablation build: the RS fast path from
#       tools/ablations/rs_fast_inst_ablate.hip (every PPFS_* switch of rounds 1-2, the headers in
#       tools/ablations/)
#   tools/build_alt.sh --product <name> '<extra hipcc flags>'  the shipped dispatch with extra flags
#       (e.g. the bounds-checked build: --product debug -DPPFS_ECC_DEBUG=1)
# _lib/alt/ stays on this machine (.gpurunignore); a leading --lease puts the library into
# _lib/lease/ instead, which travels to the GPU box (A/B baselines, trace builds a lease loads).
set -e
DIR=alt
if [ "$1" = "--lease" ]; then
    DIR=lease
    shift
fi
INST=../../tools/ablations/rs_fast_inst_ablate.hip
INC="-I. -I../../tools/ablations"
if [ "$1" = "--product" ]; then
    INST=rs_fast_inst.hip
    INC=""
    shift
fi
N=$1; shift
cd "$(dirname "$0")/../paritypartyfs_amd/csrc"
make -j8 OUT=../_lib/$DIR/libppfs_ecc_$N.so OBJDIR=../_lib/alt/obj_$N RS_INST=$INST EXTRA="$INC $*" >/dev/null
echo "built _lib/$DIR/libppfs_ecc_$N.so ($INST $*)"
