#!/bin/bash
# Isolated march timings (tools/march_variants.py) for library variants, interleaved, 2 repetitions.
#   bash tools/gpu_mv.sh TAG "suffix ..." [extra args]   (suffix "base" = libtvfem.so)
set -o pipefail
TAG=$1; LIBS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for v in $LIBS; do
    s=$v; [ "$v" = base ] && s=""
    TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 120 python3 tools/march_variants.py "$@" > $OUT/mv_${v}_$rep.log 2>&1 || { tail -5 $OUT/mv_${v}_$rep.log; exit 1; }
    grep MARCH $OUT/mv_${v}_$rep.log
  done
done
