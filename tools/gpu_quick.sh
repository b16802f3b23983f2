#!/bin/bash
# Quick GPU check: the named test files, then the GMG C4 session summary.
# Usage (via gpurun): bash tools/gpu_quick.sh TAG test_file...
set -o pipefail
TAG=${1:-quick}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q -s -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -1
[ $rc -ne 0 ] && { grep -E "^E |Error|FAILED" $OUT/tests.log | head -30; exit $rc; }
bash tools/gpu_mg.sh $TAG
