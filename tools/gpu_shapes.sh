#!/bin/bash
# Bench lines of the strong-scaling per-rank shapes of C4 and of C2/C3/C4 on
# one GPU (no CPU baseline), after a quick parity subset.
# Usage (via gpurun): bash tools/gpu_shapes.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-shapes}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
K=${2:-"time_steps or in_solve or march_edge or partitioned_run"}
echo "[gpu_shapes] tests -k $K"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for spec in "n8 400,50,50" "C3 200,200,25" "C2 100,100,10 --thermal-only" "C4 400,400,50"; do
  set -- $spec
  tag=$1; cells=$2; shift 2
  echo "[gpu_shapes] bench $tag"
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --cells $cells "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -5 $OUT/bench_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$tag.json'));print('$tag', round(d['ms_per_step'],3), 'ms/step', d['config']['krylov_its_per_step'], 'its', {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"
done
