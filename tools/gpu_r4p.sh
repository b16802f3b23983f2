#!/bin/bash
# Round-4 session P: single-round-trip march prologue + lagged PCG logic on
# partitions -- A/B isolated timings against the previous library
# (libtvfem_old.so), the parity tests (operator / multigrid / full-size /
# golden / partitioned GMG + loopback), C4, C3 and share/8 bench lines.
set -o pipefail
TAG=${1:-r4p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_mv.sh $TAG "base _old" || exit 1
TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem_wgt.so timeout -k 10 120 python3 tools/wgtrace/run.py > $OUT/wgt.log 2>&1 || { tail -5 $OUT/wgt.log; exit 1; }
grep -E "^\[" $OUT/wgt.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_multigrid.py tests/test_fullsize.py tests/test_golden.py tests/test_loopback.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 900 python -u -m pytest tests/test_partition.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "gmg or vcycle or single_partition" > $OUT/tests_part.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests_part.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests_part.log | head -20; exit $rc; }
for v in base _old; do
  s=$v; [ "$v" = base ] && s=""
  L=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so
  TVFEM_LIB=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$v.log 2>&1 || { tail -5 $OUT/bench_$v.log; exit 1; }
  echo "c4 $v $(tail -1 $OUT/bench_$v.log | cut -c1-200)"
  TVFEM_LIB=$L timeout -k 10 300 python3 bench.py --cells 200,200,25 --pc jacobi --steps 30 --warmup 3 --no-cpu-baseline > $OUT/bench_c3_$v.log 2>&1 || { tail -5 $OUT/bench_c3_$v.log; exit 1; }
  echo "c3 $v $(tail -1 $OUT/bench_c3_$v.log | cut -c1-200)"
  TVFEM_LIB=$L timeout -k 10 300 python3 bench.py --share 8 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_s8_$v.log 2>&1 || { tail -5 $OUT/bench_s8_$v.log; exit 1; }
  echo "s8 $v $(tail -1 $OUT/bench_s8_$v.log | cut -c1-200)"
done
