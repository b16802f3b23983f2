#!/bin/bash
# scratch GPU job (changes per experiment)
set -o pipefail
OUT=gpurun_out/${1:-tmp}
mkdir -p $OUT
echo "[tmp] tests rows 12" && TVFEM_MARCH_ROWS=12 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 && tail -1 $OUT/tests.log && \
for r in 12 8; do
echo "[tmp] C4 rows $r" && TVFEM_MARCH_ROWS=$r timeout -k 10 400 python3 bench.py --no-cpu-baseline > $OUT/c4_$r.json 2> $OUT/c4_$r.err && \
python3 -c "import json;d=json.load(open('$OUT/c4_$r.json'));print(round(d['ms_per_step'],3),'ms',d['config']['krylov_its_per_step'],{k:(round(v['ms']*1e3,1),round(v['ms_isolated']*1e3,1)) for k,v in d['kernels'].items()})" || exit 1
done
