#!/bin/bash
# The non-headline configurations of BASELINE.json on one GPU (C2 thermal-only,
# C3 coupled, C5 DG1 coupled): one bench line each.  Usage: bash tools/job_configs.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-configs}
mkdir -p $OUT
echo "[configs] C2" && timeout -k 10 300 python3 bench.py --cells 100,100,10 --thermal-only --steps 10 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err && \
echo "[configs] C3" && timeout -k 10 300 python3 bench.py --cells 200,200,25 --steps 10 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err && \
echo "[configs] C5" && timeout -k 10 400 python3 bench.py --cells 200,200,25 --family DG --steps 5 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err && \
for f in c2 c3 c5; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',d['config']['workload'],round(d['value']/1e6,1),'M/s',round(d['ms_per_step'],2),'ms',d['config']['krylov_its_per_step'],{k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"; done
