#!/bin/bash
# scratch GPU job (changes per experiment)
set -o pipefail
OUT=gpurun_out/${1:-tmp}
mkdir -p $OUT
echo "[tmp] tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 && tail -1 $OUT/tests.log && \
echo "[tmp] C5" && timeout -k 10 400 python3 bench.py --cells 200,200,25 --family DG --steps 5 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err && \
python3 -c "import json;d=json.load(open('$OUT/c5.json'));print(round(d['ms_per_step'],2),'ms',d['config']['krylov_its_per_step'],{k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"
