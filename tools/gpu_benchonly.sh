#!/bin/bash
# Bench lines only (no tests): for each shape, the given --pcg forms.
# Usage (via gpurun): bash tools/gpu_benchonly.sh TAG "pcg forms" "cells[ args]" ...
set -o pipefail
TAG=$1; shift
FORMS=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for spec in "$@"; do
  for pcg in $FORMS; do
    i=$((i+1))
    echo "[bench] $spec --pcg $pcg"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --kernel-reps 5 --pcg $pcg --cells $spec > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b$i.json'));print(round(d['ms_per_step'],3), 'ms/step', d['config']['krylov_its_per_step'], 'its', {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"
  done
done
