#!/bin/bash
# Round-4 session Y: the visco update with the next dof's inputs prefetched --
# isolated update timings (tools/visco_modes.py) and C4 bench lines, A/B
# against the committed library (_head); the parity tests that read the
# viscoelastic state.
set -o pipefail
TAG=${1:-r4y}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_paper_mode.py tests/test_fullsize.py tests/test_golden.py tests/test_gpu_configs.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests.log | head -30; exit $rc; }
for rep in 1 2; do
  for v in base _head; do
    s=$v; [ "$v" = base ] && s=""
    TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 200 python3 tools/visco_modes.py --steps 1 --reps 30 > $OUT/vm_${v}_$rep.log 2>&1 || { tail -3 $OUT/vm_${v}_$rep.log; exit 1; }
    echo "visco $v $(grep VISCO_MODE $OUT/vm_${v}_$rep.log | cut -c1-110)"
    TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b_c4_${v}_$rep.json 2> $OUT/b_c4_${v}_$rep.err || { tail -5 $OUT/b_c4_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_c4_${v}_$rep.json'));print('c4 $v', round(d['ms_per_step'],3), round(d['kernels']['visco_update']['ms']*1e3,1))"
  done
done
