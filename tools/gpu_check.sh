#!/bin/bash
# One GPU session: parity tests, PMC traffic of the hot kernels, bench under rocprofv3 stats.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "[gpu_check] tests" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 && tail -3 $OUT/tests.log && \
echo "[gpu_check] pmc fetch" && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 tools/pmc_kernels.py > $OUT/pmc_fetch.log 2>&1 && \
echo "[gpu_check] pmc write" && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 tools/pmc_kernels.py > $OUT/pmc_write.log 2>&1 && \
python3 tools/pmc_summarize.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_matvec_400x400x50_n1.json > $OUT/pmc_summary.log 2>&1 && \
cp $OUT/pmc_matvec_400x400x50_n1.json profiles/ && \
echo "[gpu_check] bench" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python3 bench.py > $OUT/bench.json 2> $OUT/bench.err && \
cat $OUT/bench.json
[ $? -eq 0 ] && \
python3 tools/profile_summary.py $OUT/prof_bench $OUT/bench.json $OUT/profile_summary.json > $OUT/profile_summary.log 2>&1 && \
echo "[gpu_check] bench (no profiler)" && \
timeout -k 10 600 python3 bench.py > $OUT/bench_plain.json 2> $OUT/bench_plain.err && \
cat $OUT/bench_plain.json
