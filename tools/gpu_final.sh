#!/bin/bash
# Round-end check on the final tree: the GPU suite, smoke(), the default bench line.
set -o pipefail
OUT=gpurun_out/${1:-r4end}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('bench', round(d['ms_per_step'],3), round(d['value']/1e6,1), 'M/s frac', round(r['frac'],3), 'flushed', round(r['hbm_flushed']['frac'],3), 'cpu', d['cpu_baseline']['value'])"
