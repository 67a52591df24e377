#!/bin/bash
# Builds an ablation variant of the engine: tools/build_alt.sh <name> '<extra hipcc flags>'
#   -> paritypartyfs_amd/_lib/alt/libppfs_ecc_<name>.so (load it with PPFS_ECC_LIB=...)
set -e
N=$1; shift
cd "$(dirname "$0")/../paritypartyfs_amd/csrc"
make -j8 OUT=../_lib/alt/libppfs_ecc_$N.so OBJDIR=../_lib/alt/obj_$N EXTRA="$*" >/dev/null
echo "built _lib/alt/libppfs_ecc_$N.so ($*)"
