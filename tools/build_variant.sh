#!/bin/bash
# Build an A/B variant of libtvfem.so from patched sources (the library has no
# compile-time or environment switches): copies csrc/ to a scratch directory,
# applies the sed expression, builds, and installs tvfem/libtvfem<SUFFIX>.so.
#   bash tools/build_variant.sh SUFFIX 'sed expression' [file under csrc/]
set -e
SUF=$1; EXPR=$2; FILE=${3:-tv_cg.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/tvfem_var_$SUF
rm -rf $W && mkdir -p $W/tvfem
cp -r $ROOT/fem-glass-tempering_amd/csrc $ROOT/fem-glass-tempering_amd/Makefile $W/
sed -i "s#-I../include#-I$ROOT/include#; s#\.\./include/tvfem.h#$ROOT/include/tvfem.h#" $W/Makefile
sed -i "$EXPR" $W/csrc/$FILE
(cd $W && make -j8 >/dev/null)
cp $W/tvfem/libtvfem.so $ROOT/fem-glass-tempering_amd/tvfem/libtvfem$SUF.so
echo "built libtvfem$SUF.so"
