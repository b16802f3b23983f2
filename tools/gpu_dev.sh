#!/bin/bash
# Development GPU session: full parity suite, then bench lines at the given
# shapes for both Krylov forms.  Usage (via gpurun): bash tools/gpu_dev.sh TAG "cells[ args]" ...
set -o pipefail
TAG=${1:-dev}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "[gpu_dev] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -rs --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -2
grep -h "^\[parity\]" $OUT/tests.log > $OUT/parity_lines.txt
[ $rc -ne 0 ] && { grep -E "^E |Error|FAILED" $OUT/tests.log | head -30; exit $rc; }
i=0
for spec in "$@"; do
  for pcg in single kspcg; do
    i=$((i+1))
    echo "[gpu_dev] bench $spec --pcg $pcg"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --kernel-reps 5 --pcg $pcg --cells $spec > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b$i.json'));print(round(d['ms_per_step'],3), 'ms/step', d['config']['krylov_its_per_step'], 'its', {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"
  done
done
