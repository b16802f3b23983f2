#!/bin/bash
# Round-4: the DG tile's load addresses from the host's iteration parity (the
# solver state tested after the prologue's loads) -- the GPU suites that run
# DG, then C5 A/B against the committed library (_head).
set -o pipefail
TAG=${1:-r4dg2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_multigrid.py tests/test_gpu_configs.py tests/test_partition.py tests/test_paper_mode.py tests/test_output.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests.log | head -30; exit $rc; }
for rep in 1 2 3; do
  for v in base _head; do
    s=$v; [ "$v" = base ] && s=""
    TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 300 python3 bench.py --family DG --cells 200,200,25 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b_c5_${v}_$rep.json 2> $OUT/b_c5_${v}_$rep.err || { tail -5 $OUT/b_c5_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_c5_${v}_$rep.json'));print('c5 $v', round(d['ms_per_step'],3), d['config']['krylov_its_per_step'], {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"
  done
done
