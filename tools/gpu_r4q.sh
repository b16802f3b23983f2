#!/bin/bash
# Round-4 session Q: the column-band XCD tile mapping and the tail-split chunk layout (kTailSplit 1 = production
# candidate, _ts0 = uniform chunks, _ts2 = two chunks re-split into three):
# _head = the committed library; isolated march timings, the workgroup
# timeline, parity, C4 and C3 bench lines.
set -o pipefail
TAG=${1:-r4q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_mv.sh $TAG "base _ts0 _ts2 _head" || exit 1
TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem_wgt.so timeout -k 10 120 python3 tools/wgtrace/run.py > $OUT/wgt.log 2>&1 || { tail -5 $OUT/wgt.log; exit 1; }
grep -E "^\[" $OUT/wgt.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_multigrid.py tests/test_fullsize.py tests/test_golden.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests.log | head -20; exit $rc; }
for rep in 1 2; do
for v in base _ts0 _ts2 _head; do
  s=$v; [ "$v" = base ] && s=""
  L=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so
  TVFEM_LIB=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_${v}_$rep.log 2>&1 || { tail -5 $OUT/bench_${v}_$rep.log; exit 1; }
  echo "c4 $v $(tail -1 $OUT/bench_${v}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), {k: round(v.get("ms",0)*1e3,1) for k,v in d.get("kernels",{}).items()}, "flushed", round(d["roofline"]["hbm_flushed"]["ms_per_launch"]*1e3,1))')"
done
done
for v in base _head; do
  s=$v; [ "$v" = base ] && s=""
  TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 300 python3 bench.py --cells 200,200,25 --pc jacobi --steps 30 --warmup 3 --no-cpu-baseline > $OUT/bench_c3_$v.log 2>&1 || { tail -5 $OUT/bench_c3_$v.log; exit 1; }
  echo "c3 $v $(tail -1 $OUT/bench_c3_$v.log | cut -c150-250)"
done
