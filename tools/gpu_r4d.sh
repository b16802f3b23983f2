#!/bin/bash
# Round-4 session D: mixed-family partition tests (+ a mutation run without the
# ghost refresh, expected to fail), the counter list of this box, and the visco
# update's speed in N separate processes (tools/visco_modes.py).
#   bash tools/gpu_r4d.sh TAG NPROC
set -o pipefail
TAG=$1; NP=${2:-8}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests/test_partition.py -m gpu -v -s --timeout 200 --timeout-method thread -k mixed > $OUT/mixed.log 2>&1
echo "mixed rc=$?"; grep -E "^\[partition\]|PASSED|FAILED" $OUT/mixed.log | cut -c1-400
TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem_norefresh.so timeout -k 10 200 python -u -m pytest tests/test_partition.py -m gpu -v -s --timeout 150 --timeout-method thread -k mixed_families_host_edit > $OUT/mutation.log 2>&1
echo "mutation (no ghost refresh) rc=$? (1 expected)"; grep -E "AssertionError|PASSED|FAILED" $OUT/mutation.log | cut -c1-400 | head -5
timeout -k 10 60 rocprofv3 --list-avail > $OUT/counters.txt 2>&1; echo "list-avail rc=$?"
for i in $(seq 1 $NP); do
  timeout -k 10 120 python3 tools/visco_modes.py > $OUT/vm_$i.log 2>&1 || { tail -5 $OUT/vm_$i.log; exit 1; }
  grep VISCO_MODE $OUT/vm_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().split(' ',1)[1]); print('proc', $i, 'visco', d['visco_ms'], d['visco_ms_again'], 'jx', d['jx_ms'], {k: v['mod_2MiB'] for k, v in d['fields'].items()})"
done
