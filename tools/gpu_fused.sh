#!/bin/bash
# fused coarse-level launch: multigrid parity tests, then C4 / C3 / C5 A/B lines
set -o pipefail
OUT=gpurun_out/${1:-fused}
mkdir -p $OUT
line() { python3 -c "import json;d=json.load(open('$1'));print('$2', round(d['ms_per_step'],3), 'ms/step', d['config'].get('krylov_its_per_step'), 'its', {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"; }
timeout -k 10 600 python -u -m pytest tests/test_multigrid.py tests/test_fullsize.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for spec in "C4off 400,400,50 -1" "C4f4 400,400,50 400000" "C4def 400,400,50 0" "C3off 200,200,25 -1" "C3def 200,200,25 0"; do
  set -- $spec; tag=$1; cells=$2; fz=$3
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --pc gmg --cells $cells --mg-fused-nodes $fz > $OUT/bench_$tag.$rep.json 2> $OUT/bench_$tag.$rep.err || { tail -5 $OUT/bench_$tag.$rep.err; exit 1; }
  line $OUT/bench_$tag.$rep.json $tag
done
done
for spec in "C5off -1" "C5def 0"; do
  set -- $spec; tag=$1; fz=$2
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --family DG --cells 200,200,25 --mg-fused-nodes $fz > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -5 $OUT/bench_$tag.err; exit 1; }
  line $OUT/bench_$tag.json $tag
done
