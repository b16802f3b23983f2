#!/bin/bash
# Multigrid development session: GMG tests, a profiled C4 bench (kernel trace)
# and a plain C4 bench line.  Usage (via gpurun): bash tools/gpu_mg.sh TAG [bench args]
set -o pipefail
TAG=${1:-mg}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest tests/test_multigrid.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed|\[gmg\]" $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "^E |Error" $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --pc gmg --steps 3 --warmup 1 --kernel-reps 3 --no-cpu-baseline "$@" > $OUT/b_prof.json 2> $OUT/b_prof.err || exit 1
timeout -k 10 400 python3 bench.py --pc gmg --steps 5 --warmup 1 --kernel-reps 5 --no-cpu-baseline "$@" > $OUT/b_gmg.json 2> $OUT/b_gmg.err
[ -n "$MG_EXTRA" ] && timeout -k 10 400 python3 bench.py --pc gmg --steps 5 --warmup 1 --kernel-reps 5 --no-cpu-baseline $MG_EXTRA > $OUT/b_extra.json 2> $OUT/b_extra.err
exit 0
