#!/bin/bash
# Session check: GPU parity suite, the default bench line and the multigrid
# kernel trace summary.  (RCCL refuses two ranks on one device -- ncclCommInitRank
# returns "invalid usage" -- so its transport cannot be rehearsed on one GPU.)
set -o pipefail
OUT=gpurun_out/t1
mkdir -p $OUT
bash tools/gpu_tests.sh t1 || exit 1
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
MG_EXTRA="" bash tools/gpu_mg.sh mg2 > /dev/null 2>&1 && python3 tools/mg_summary.py gpurun_out/mg2 12
