#!/bin/bash
# Round-4 session W: the post-solve group for the Jacobi solves (KSPCG and the
# single-reduction form) -- the full GPU suite, then A/B against the committed
# library (_head): C2, C3 (single-reduction), C4 Jacobi (KSPCG), C4 GMG.
set -o pipefail
TAG=${1:-r4w}
OUT=gpurun_out/$TAG
mkdir -p $OUT
[ -n "$SKIPT" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests.log | head -30; exit $rc; }
for rep in 1 2; do
for spec in "c2 --cells 100,100,10 --thermal-only" "c3 --cells 200,200,25 --pc jacobi" "c4j --pc jacobi --steps 5" "c4"; do
  set -- $spec; tag=$1; shift
  for v in base _head; do
    s=$v; [ "$v" = base ] && s=""
    TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $OUT/b_${tag}_${v}_$rep.json 2> $OUT/b_${tag}_${v}_$rep.err || { tail -5 $OUT/b_${tag}_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${tag}_${v}_$rep.json'));print('$tag $v', round(d['ms_per_step'],3), d['config']['krylov_its_per_step'])"
  done
done
done
