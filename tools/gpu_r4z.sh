#!/bin/bash
# Round-4 session V: the post-solve group (dx, Newton update, ||dx||) queued
# behind every multigrid batch, gated on the device state -- A/B against the
# committed library (_head): C4, C3 (Jacobi, GMG), C2, share/8; the tests.
set -o pipefail
TAG=${1:-r4u}
OUT=gpurun_out/$TAG
mkdir -p $OUT
[ -n "$SKIPT" ] || timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_multigrid.py tests/test_fullsize.py tests/test_golden.py tests/test_gpu_configs.py tests/test_loopback.py tests/test_paper_mode.py tests/test_output.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests.log | head -30; exit $rc; }
[ -n "$SKIPT" ] || timeout -k 10 900 python -u -m pytest tests/test_partition.py tests/test_upartition.py tests/test_amg.py tests/test_unstructured.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests_part.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests_part.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests_part.log | head -30; exit $rc; }
for rep in 1 2; do
for spec in "c4" "c3g --cells 200,200,25 --pc gmg" "c5 --family DG --cells 200,200,25"; do
  set -- $spec; tag=$1; shift
  for v in base _head; do
    s=$v; [ "$v" = base ] && s=""
    TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $OUT/b_${tag}_${v}_$rep.json 2> $OUT/b_${tag}_${v}_$rep.err || { tail -5 $OUT/b_${tag}_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${tag}_${v}_$rep.json'));print('$tag $v', round(d['ms_per_step'],3), d['config']['krylov_its_per_step'])"
  done
done
done
