#!/bin/bash
# Round-4: DG tile addressing fix (wave-uniform layer base) -- C5 A/B against
# the committed library (_head), the DG parity tests, the DG PMC passes.
set -o pipefail
TAG=${1:-r4dg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for rep in 1 2; do
for v in base _head; do
  s=$v; [ "$v" = base ] && s=""
  TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$s.so timeout -k 10 300 python3 bench.py --family DG --cells 200,200,25 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c5_${v}_$rep.json 2> $OUT/bench_c5_${v}_$rep.err || { tail -5 $OUT/bench_c5_${v}_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_c5_${v}_$rep.json'));print('c5 $v', round(d['ms_per_step'],3), {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()}, 'frac', round(d['roofline']['frac'],3))"
done
done
timeout -k 10 900 python -u -m pytest tests/test_multigrid.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_fullsize.py tests/test_partition.py tests/test_loopback.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "dg or DG or mixed" > $OUT/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $OUT/tests.log | head -20; exit $rc; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr -d $OUT/pmc_DG_gmg_$ctr -o run --output-format csv -- python3 tools/pmc_kernels.py --pc gmg --family DG --cells 200,200,25 > $OUT/pmc_DG_gmg_$ctr.log 2>&1 || { tail -5 $OUT/pmc_DG_gmg_$ctr.log; exit 1; }
done
python3 tools/pmc_summarize.py $OUT/pmc_DG_gmg_FETCH_SIZE $OUT/pmc_DG_gmg_WRITE_SIZE $OUT/pmc_pcg_matvec_fused_DG_200x200x25_n1_gmg.json dg_matvec_fused > $OUT/pmc_summary.log 2>&1 || exit 1
grep -A4 '"dg_matvec_fused"' $OUT/pmc_pcg_matvec_fused_DG_200x200x25_n1_gmg.json
