#!/bin/bash
# Round-4 session S: side-face stencils inside the marching launch (no face
# workgroups, no k_cg_addfaces, no k_mg_post_faces pass) -- A/B isolated
# timings against the committed library (_head), the parity tests, C4 and
# share/8 bench lines.
set -o pipefail
TAG=${1:-r4s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
[ -n "$SKIPMV" ] || bash tools/gpu_mv.sh $TAG "base _head" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_multigrid.py tests/test_fullsize.py tests/test_golden.py tests/test_loopback.py tests/test_gpu_configs.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 900 python -u -m pytest tests/test_partition.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "gmg or vcycle or single_partition or dirichlet or host_edit" > $OUT/tests_part.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests_part.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests_part.log | head -30; exit $rc; }
for rep in 1 2; do
for v in base _head; do
  s=$v; [ "$v" = base ] && s=""
  L=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so
  TVFEM_LIB=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err || { tail -5 $OUT/bench_${v}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_${v}_$rep.json'));r=d['roofline'];print('c4 $v', round(d['ms_per_step'],3), d['config']['krylov_its_per_step'], {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()}, 'frac', round(r['frac'],3), 'flushed', round(r['hbm_flushed']['ms_per_launch']*1e3,1))"
done
done
for v in base _head; do
  s=$v; [ "$v" = base ] && s=""
  TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 300 python3 bench.py --share 8 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_s8_$v.json 2> $OUT/bench_s8_$v.err || { tail -5 $OUT/bench_s8_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_s8_$v.json'));print('s8 $v', round(d['ms_per_step'],3), {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"
done
