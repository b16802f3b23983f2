#!/bin/bash
# Experiment-switch sweep (TVFEM_EXPERIMENTS=1) of bench lines at given shapes.
# Usage (via gpurun): bash tools/gpu_knobs.sh TAG "cells [bench args]" "ENV=.. ENV=.." ...
set -o pipefail
TAG=$1; shift
SHAPE=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for envs in "" "$@"; do
  i=$((i+1))
  echo "[knobs] $SHAPE :: $envs"
  env TVFEM_EXPERIMENTS=1 $envs timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --kernel-reps 5 --cells $SHAPE > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b$i.json'));print(round(d['ms_per_step'],3), 'ms/step', d['config']['krylov_its_per_step'], 'its', {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"
done
