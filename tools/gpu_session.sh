#!/bin/bash
# One GPU session of the round: optional focused tests first, then the whole
# GPU suite, then the C4 bench line.  Usage (via gpurun):
#   bash tools/gpu_session.sh TAG [pytest -k expr for the focused run]
set -o pipefail
TAG=${1:-session}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ -n "$2" ]; then
  echo "[session] focused: $2"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -rs --timeout 300 --timeout-method thread -k "$2" > $OUT/focused.log 2>&1
  rc=$?; tail -4 $OUT/focused.log
  [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/focused.log | head -20; exit $rc; }
fi
echo "[session] full GPU suite"
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -4 $OUT/tests.log
grep -h "^\[parity\]\|^\[c3\|^\[fullsize\]" $OUT/tests.log > $OUT/parity_lines.txt
grep -E "FAILED|ERROR" $OUT/tests.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
echo "[session] bench C4"
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -5 $OUT/bench_c4.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c4.json'));print('C4', round(d['ms_per_step'],3), 'ms/step', d['config']['krylov_its_per_step'], 'its, frac', round(d['roofline']['frac'],3))"
exit $rc
