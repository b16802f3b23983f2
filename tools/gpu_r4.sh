#!/bin/bash
# Round-4 GPU session: the named pytest selection, then an interleaved A/B of
# library builds on bench configs.  Usage (via gpurun):
#   bash tools/gpu_r4.sh TAG "test files" "suffix:label ..." "tag|bench args;..." ["pytest -k expression"]
set -o pipefail
TAG=$1; TESTS=$2; LIBS=$3; CFGS=$4
K=()
[ -n "$5" ] && K=(-k "$5")
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ -n "$TESTS" ]; then
  timeout -k 10 700 python -u -m pytest $TESTS "${K[@]}" -m gpu -x -v -s -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?
  grep -E "passed|failed" $OUT/tests.log | tail -1
  [ $rc -ne 0 ] && { grep -E "^E |Error|FAILED" $OUT/tests.log | head -30; exit $rc; }
fi
[ -n "$LIBS" ] && bash tools/gpu_ab.sh $TAG "$LIBS" "$CFGS"
exit $?
