#!/bin/bash
# Round-4 session M: the complete-J march (front face workgroups + face pass):
# isolated timings first, then the operator / multigrid / full-size parity tests.
set -o pipefail
OUT=gpurun_out/${1:-r4m}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 python3 tools/march_variants.py > $OUT/mv.log 2>&1 || { tail -20 $OUT/mv.log; exit 1; }
grep MARCH $OUT/mv.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_multigrid.py tests/test_fullsize.py tests/test_golden.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && grep -E "^E " $OUT/tests.log | head -20
exit $rc
