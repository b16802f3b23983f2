#!/bin/bash
# A/B of the DG1 multigrid at C5: default vs an experiment switch (bench lines only).
# Usage (via gpurun): bash tools/gpu_dgab.sh TAG SWITCH [bench args]
set -o pipefail
TAG=${1:-dgab}; SW=${2:-TVFEM_MG_UNFUSED}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --pc gmg --steps 5 --warmup 1 --kernel-reps 3 --no-cpu-baseline --family DG --cells 200,200,25 "$@" > $OUT/b_a.json 2> $OUT/b_a.err || exit 1
TVFEM_EXPERIMENTS=1 env $SW=1 timeout -k 10 300 python3 bench.py --pc gmg --steps 5 --warmup 1 --kernel-reps 3 --no-cpu-baseline --family DG --cells 200,200,25 "$@" > $OUT/b_b.json 2> $OUT/b_b.err || exit 1
for f in a b; do python3 -c "
import json
d=json.loads(open('$OUT/b_$f.json').read().strip().splitlines()[-1]); c=d['config']
print('$f', round(d['ms_per_step'],3), c.get('krylov_its_per_step'), {k:round(v['ms']*1000,1) for k,v in d['kernels'].items()})
"; done
