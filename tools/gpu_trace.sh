#!/bin/bash
# rocprofv3 kernel traces of bench configurations: "tag|bench args" pairs in $TRACES
set -o pipefail
OUT=gpurun_out/${1:-trace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
IFS=';'
for spec in $TRACES; do
  tag=${spec%%|*}; args=${spec#*|}
  mkdir -p $OUT/$tag
  IFS=' ' read -r -a argv <<< "$args"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$tag/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline "${argv[@]}" > $OUT/$tag/b_gmg.json 2> $OUT/$tag/b.err || { tail -5 $OUT/$tag/b.err; exit 1; }
  f=$(find $OUT/$tag/prof -name "run_kernel_trace.csv" | head -1); mv "$f" $OUT/$tag/prof/run_kernel_trace.csv 2>/dev/null
  echo "== $tag: $args"; python3 tools/mg_summary.py $OUT/$tag 28
done
