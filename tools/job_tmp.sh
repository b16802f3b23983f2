#!/bin/bash
# scratch GPU job (changes per experiment)
set -o pipefail
OUT=gpurun_out/${1:-tmp}
mkdir -p $OUT
for v in 512 768; do
echo "[tmp] C4 vec blocks $v" && TVFEM_VEC_BLOCKS=$v timeout -k 10 400 python3 bench.py --no-cpu-baseline > $OUT/c4_$v.json 2> $OUT/c4_$v.err && \
python3 -c "import json;d=json.load(open('$OUT/c4_$v.json'));print(round(d['ms_per_step'],3),'ms',d['config']['krylov_its_per_step'],{k:(round(v['ms']*1e3,1),round(v['ms_isolated']*1e3,1)) for k,v in d['kernels'].items()})" || exit 1
done
