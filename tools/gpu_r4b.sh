#!/bin/bash
# Round-4 GPU session: the whole GPU suite (no -x: every failure listed), an
# interleaved A/B of library builds (tools/gpu_ab.sh), then rocprofv3 kernel
# traces of bench configurations with the step-window busy / idle accounting.
#   bash tools/gpu_r4b.sh TAG "suffix:label ..." "tag|bench args;..." "tag|bench args;..."(traces)
set -o pipefail
TAG=$1; LIBS=$2; CFGS=$3; TRC=$4
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -8
grep -h "^\[parity\]" $OUT/tests.log > $OUT/parity_lines.txt
[ $rc -gt 1 ] && exit $rc   # 1 = test failures (listed above); anything else: stop here
if [ -n "$LIBS" ]; then bash tools/gpu_ab.sh $TAG "$LIBS" "$CFGS" || exit 1; fi
if [ -n "$TRC" ]; then
  IFS=';' read -r -a TS <<< "$TRC"
  for spec in "${TS[@]}"; do
    t=${spec%%|*}; args=${spec#*|}
    IFS=' ' read -r -a argv <<< "$args"
    mkdir -p $OUT/tr_$t
    timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_$t/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline "${argv[@]}" > $OUT/tr_$t/b.json 2> $OUT/tr_$t/b.err || { tail -5 $OUT/tr_$t/b.err; exit 1; }
    f=$(find $OUT/tr_$t/prof -name "run_kernel_trace.csv" | head -1)
    echo "== trace $t: $args"
    python3 tools/trace_gaps.py "$f" > $OUT/tr_$t/gaps.txt 2>&1; head -40 $OUT/tr_$t/gaps.txt
  done
fi
exit $rc
