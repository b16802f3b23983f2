#!/bin/bash
# A/B of one experiment switch on the C4 (and C5) GMG bench lines.
# Usage (via gpurun): bash tools/gpu_ab2.sh TAG 'ENV=val ...'
set -o pipefail
TAG=${1:-ab}; AENV=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_multigrid.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { grep -E "^E |Error|FAILED" $OUT/tests.log | head -20; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -1
for fam in CG DG; do
  if [ $fam = CG ]; then cells=400,400,50; else cells=200,200,25; fi
  timeout -k 10 300 python3 bench.py --pc gmg --family $fam --cells $cells --steps 5 --warmup 1 --kernel-reps 3 --no-cpu-baseline > $OUT/b_${fam}_A.json 2> $OUT/b_${fam}_A.err || exit 1
  timeout -k 10 300 env TVFEM_EXPERIMENTS=1 $AENV python3 bench.py --pc gmg --family $fam --cells $cells --steps 5 --warmup 1 --kernel-reps 3 --no-cpu-baseline > $OUT/b_${fam}_B.json 2> $OUT/b_${fam}_B.err || exit 1
  python3 -c "
import json
for v in 'AB':
    d=json.load(open('$OUT/b_${fam}_'+v+'.json'))
    print('$fam', v, round(d['ms_per_step'],3), 'ms/step', d['config']['krylov_its_per_step'], 'its', {k:round(x['ms']*1e3,1) for k,x in d['kernels'].items()})
"
done
