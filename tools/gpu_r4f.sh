#!/bin/bash
# Round-4 session F: the mixed-family host-edit test in paper mode and its
# mutation (no ghost refresh: must fail); the cube-tile J x probe, flushed and warm.
set -o pipefail
OUT=gpurun_out/${1:-r4f}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python -u -m pytest tests/test_partition.py -m gpu -v -s --timeout 150 --timeout-method thread -k mixed_families_host_edit > $OUT/edit.log 2>&1
echo "host edit rc=$?"; grep -E "^\[partition\]|PASSED|FAILED" $OUT/edit.log | cut -c1-300
TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem_norefresh.so timeout -k 10 200 python -u -m pytest tests/test_partition.py -m gpu -v -s --timeout 150 --timeout-method thread -k mixed_families_host_edit > $OUT/mutation.log 2>&1
echo "mutation (no ghost refresh) rc=$? (1 expected)"; grep -E "^\[partition\]|PASSED|FAILED" $OUT/mutation.log | cut -c1-300 | head -5
timeout -k 10 120 tools/probe/cube_probe f > $OUT/cube_flushed.txt 2>&1; echo "cube flushed rc=$?"; cat $OUT/cube_flushed.txt
timeout -k 10 120 tools/probe/cube_probe > $OUT/cube_warm.txt 2>&1; echo "cube warm rc=$?"; cat $OUT/cube_warm.txt
