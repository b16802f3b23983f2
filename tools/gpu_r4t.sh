#!/bin/bash
# Round-4 session T: side-face stencils on grids up to kStenMaxNodes -- A/B of
# the per-rank shares (/2 off, /4 and /8 on), C3 with GMG (on) and C4 (off)
# against the committed library (_head); the GMG parity tests.
set -o pipefail
TAG=${1:-r4t}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_multigrid.py tests/test_golden.py tests/test_gpu_configs.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests.log | head -30; exit $rc; }
for rep in 1 2; do
for spec in "s8 --share 8" "s4 --share 4" "c3g --cells 200,200,25 --pc gmg" "s2 --share 2"; do
  set -- $spec; tag=$1; shift
  for v in base _head; do
    s=$v; [ "$v" = base ] && s=""
    TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $OUT/b_${tag}_${v}_$rep.json 2> $OUT/b_${tag}_${v}_$rep.err || { tail -5 $OUT/b_${tag}_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${tag}_${v}_$rep.json'));print('$tag $v', round(d['ms_per_step'],3), d['config']['krylov_its_per_step'], {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"
  done
done
done
