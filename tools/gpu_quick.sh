#!/bin/bash
# Short GPU session: parity tests, then bench.py under a rocprofv3 kernel trace
# and the bench/trace cross-check.  Usage (via gpurun): bash tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "[gpu_quick] tests" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 && tail -1 $OUT/tests.log && \
echo "[gpu_quick] bench" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err && \
python3 tools/profile_summary.py $OUT/prof_bench $OUT/bench.json $OUT/profile_summary.json > $OUT/profile_summary.log 2>&1 && \
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['ms_per_step'],{k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"
