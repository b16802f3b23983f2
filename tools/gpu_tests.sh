#!/bin/bash
# GPU parity suite only.  Usage (via gpurun): bash tools/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
K=()
[ -n "$2" ] && K=(-k "$2")
echo "[gpu_tests] pytest -m gpu ${K[*]}"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -rs --timeout 400 --timeout-method thread "${K[@]}" > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
grep -h "^\[parity\]" $OUT/tests.log | sort | uniq | head -40 > $OUT/parity_lines.txt
exit $rc
