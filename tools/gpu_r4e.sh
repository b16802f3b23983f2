#!/bin/bash
# Round-4 session E: the mixed-family host-edit test and its mutation (no ghost
# refresh: must fail), then the visco update's speed and the effective GPU
# clock (GRBM cycles / kernel-trace duration) in N separate processes.
#   bash tools/gpu_r4e.sh TAG NPROC
set -o pipefail
TAG=$1; NP=${2:-12}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python -u -m pytest tests/test_partition.py -m gpu -v -s --timeout 150 --timeout-method thread -k mixed_families_host_edit > $OUT/edit.log 2>&1
echo "host edit rc=$?"; grep -E "^\[partition\]|PASSED|FAILED" $OUT/edit.log | cut -c1-300
TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem_norefresh.so timeout -k 10 200 python -u -m pytest tests/test_partition.py -m gpu -v -s --timeout 150 --timeout-method thread -k mixed_families_host_edit > $OUT/mutation.log 2>&1
echo "mutation (no ghost refresh) rc=$? (1 expected)"; grep -E "^\[partition\]|PASSED|FAILED" $OUT/mutation.log | cut -c1-300 | head -5
for i in $(seq 1 $NP); do
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pm_$i -o run --output-format csv -- python3 tools/visco_modes.py --reps 20 > $OUT/vm_$i.log 2>&1 || { tail -5 $OUT/vm_$i.log; exit 1; }
  grep VISCO_MODE $OUT/vm_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().split(' ',1)[1]); print('proc', $i, 'visco', d['visco_ms'], d['visco_ms_again'], 'jx', d['jx_ms'])"
  python3 tools/clock_summary.py $OUT/pm_$i
done
