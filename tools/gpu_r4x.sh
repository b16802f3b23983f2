#!/bin/bash
# Round-4 session X: the gated post-solve group in the distributed multigrid
# solve -- partition / loopback / unstructured-partition tests, then A/B of
# the per-rank shares against the committed library (_head).
set -o pipefail
TAG=${1:-r4x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_partition.py tests/test_loopback.py tests/test_upartition.py -m gpu -x -v -s -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests.log | head -30; exit $rc; }
for rep in 1 2; do
for spec in "s8 --share 8" "s4 --share 4" "s2 --share 2"; do
  set -- $spec; tag=$1; shift
  for v in base _head; do
    s=$v; [ "$v" = base ] && s=""
    TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $OUT/b_${tag}_${v}_$rep.json 2> $OUT/b_${tag}_${v}_$rep.err || { tail -5 $OUT/b_${tag}_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${tag}_${v}_$rep.json'));print('$tag $v', round(d['ms_per_step'],3), d['config']['krylov_its_per_step'])"
  done
done
done
