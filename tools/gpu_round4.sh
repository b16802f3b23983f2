#!/bin/bash
# Round-4 GPU evidence (same parts as round 3), in two calls (each fits gpurun's 20-minute limit):
#   bash tools/gpu_round4.sh TAG A   -- GPU suite, PMC FETCH / WRITE passes of the
#        GMG solve (C4 CG, C5 DG), the C4 bench under a rocprofv3 kernel trace
#   bash tools/gpu_round4.sh TAG B   -- bench lines: C4 (with the CPU baseline),
#        C2 / C3 / C5, the Jacobi lines, the per-rank GMG shares of C4 (n2/n4/n8)
set -o pipefail
TAG=${1:-round}
PART=${2:-A}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { echo "[gpu_round4] $*"; }
line() { python3 -c "import json;d=json.load(open('$1'));print('$2', round(d['ms_per_step'],3), 'ms/step', d['config'].get('newton_its_per_step'), d['config']['krylov_its_per_step'], 'its', {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()}, 'frac', round(d['roofline']['frac'],3))"; }
if [ $PART = T ]; then  # the GPU suite only
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log
  grep -h "^\[parity\]\|^\[c3\|^\[fullsize\]\|^\[amg\]\|upartition\]" $OUT/tests.log > $OUT/parity_lines.txt
  grep -E "FAILED|ERROR" $OUT/tests.log | head -20
  exit $rc
fi
if [ $PART = P ]; then  # march probe, a focused test, the C3 GMG line
  timeout -k 10 180 tools/probe/build/march_probe f > $OUT/probe_f.txt 2>&1 || { tail -5 $OUT/probe_f.txt; exit 1; }
  grep -E "copy|G R=8|A R=8 store=1 xcd=1|max" $OUT/probe_f.txt
  timeout -k 10 300 python -u -m pytest tests/test_partition.py -m gpu -k output -v -s --timeout 200 --timeout-method thread > $OUT/ftest.log 2>&1; tail -2 $OUT/ftest.log
  for spec in "C3g 200,200,25 --pc gmg" "C3 200,200,25"; do
    set -- $spec; tag=$1; cells=$2; shift 2
    timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --cells $cells "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -5 $OUT/bench_$tag.err; exit 1; }
    line $OUT/bench_$tag.json $tag
  done
  exit 0
fi
if [ $PART = X ]; then  # A/B of library builds (TVFEM_LIB), interleaved: "lib-suffix config" pairs in $XPAIRS
  for rep in 1 2; do
    for pair in $XPAIRS; do
      v=${pair%%:*}; cfg=${pair##*:}; [ "$v" = base ] && v=""
      case $cfg in C4) args="";; C5) args="--family DG --cells 200,200,25";; C3) args="--cells 200,200,25 --pc gmg";; esac
      [ -f fem-glass-tempering_amd/tvfem/libtvfem$v.so ] || continue
      o=$OUT/bench_x$v.$cfg.$rep
      TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$v.so timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline $args > $o.json 2> $o.err || { tail -5 $o.err; exit 1; }
      python3 -c "import json;d=json.load(open('$o.json'));r=d['roofline'];print('lib$v $cfg', round(d['ms_per_step'],3), {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()}, 'flushed', round(r['hbm_flushed']['ms_per_launch']*1e3,1))"
    done
  done
  exit 0
fi
if [ $PART = A ]; then
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log
  grep -h "^\[parity\]\|^\[c3\|^\[fullsize\]" $OUT/tests.log > $OUT/parity_lines.txt
  grep -E "FAILED|ERROR" $OUT/tests.log | head -20
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  for fam in CG DG; do
    if [ $fam = CG ]; then cells=400,400,50; else cells=200,200,25; fi
    for ctr in FETCH_SIZE WRITE_SIZE; do
      step "pmc $fam gmg $ctr"
      timeout -s KILL 300 rocprofv3 --pmc $ctr -d $OUT/pmc_${fam}_gmg_$ctr -o run --output-format csv -- python3 tools/pmc_kernels.py --pc gmg --family $fam --cells $cells > $OUT/pmc_${fam}_gmg_$ctr.log 2>&1 || { tail -5 $OUT/pmc_${fam}_gmg_$ctr.log; exit 1; }
    done
    dom=pcg_matvec_fused; [ $fam = DG ] && dom=dg_matvec_fused
    f=pmc_pcg_matvec_fused_${fam}_${cells//,/x}_n1_gmg.json
    python3 tools/pmc_summarize.py $OUT/pmc_${fam}_gmg_FETCH_SIZE $OUT/pmc_${fam}_gmg_WRITE_SIZE $OUT/$f $dom > $OUT/pmc_${fam}_gmg_summary.log 2>&1 || exit 1
    cp $OUT/$f profiles/
  done
  step "bench C4 under rocprofv3 --kernel-trace --stats"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -5 $OUT/bench_prof.err; exit 1; }
  python3 tools/profile_summary.py $OUT/prof_bench $OUT/bench_prof.json $OUT/profile_summary.json > $OUT/profile_summary.log 2>&1
  line $OUT/bench_prof.json C4prof
  exit $rc
fi
if [ $PART = C ]; then  # the unstructured algebraic multigrid
  step "amg tests"
  timeout -k 10 600 python -u -m pytest tests/test_amg.py tests/test_unstructured.py tests/test_upartition.py -m gpu -v -s -rs --timeout 300 --timeout-method thread > $OUT/amg_tests.log 2>&1
  rc=$?; tail -3 $OUT/amg_tests.log; grep -h "^\[amg\]" $OUT/amg_tests.log
  [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/amg_tests.log | head -20; exit $rc; }
  for spec in "UMamg --pc amg" "UMjac --pc jacobi"; do
    set -- $spec; tag=$1; shift 1
    step "bench distorted $tag"
    timeout -k 10 600 python3 bench.py --mesh distorted --steps 5 --warmup 1 --kernel-reps 5 --no-cpu-baseline "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -5 $OUT/bench_$tag.err; exit 1; }
    line $OUT/bench_$tag.json $tag
  done
  exit 0
fi
if [ $PART = S ]; then  # per-rank shares of C4 (the distributed GMG, transport stubbed)
  if [ -x tools/probe/build/march_probe ]; then
    step "march probe (flushed, warm)"
    timeout -k 10 180 tools/probe/build/march_probe f > $OUT/probe_f.txt 2>&1 && timeout -k 10 180 tools/probe/build/march_probe > $OUT/probe_w.txt 2>&1 || { tail -5 $OUT/probe_f.txt; exit 1; }
    grep -E "copy|R=8 store=1 xcd=1|D 2 rows|max" $OUT/probe_f.txt
  fi
  step "C3 GMG under rocprofv3 --kernel-trace"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_c3g -o run --output-format csv -- python3 bench.py --cells 200,200,25 --pc gmg --steps 5 --warmup 1 --kernel-reps 3 --no-cpu-baseline > $OUT/bench_c3g_prof.json 2> $OUT/bench_c3g_prof.err || { tail -5 $OUT/bench_c3g_prof.err; exit 1; }
  for spec in "n2 400,400,50 --share 2" "n4 400,400,50 --share 4" "n8 400,400,50 --share 8" "n8j 400,400,50 --share 8 --pc jacobi"; do
    set -- $spec; tag=$1; cells=$2; shift 2
    step "bench $tag"
    timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --cells $cells "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -5 $OUT/bench_$tag.err; exit 1; }
    line $OUT/bench_$tag.json $tag
  done
  exit 0
fi
step "bench C4 (CPU baseline: the C/OpenMP port with the same GMG)"
timeout -k 10 600 python3 bench.py > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -5 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
for spec in "C2 100,100,10 --thermal-only" "C3 200,200,25" "C3g 200,200,25 --pc gmg" "C5 200,200,25 --family DG" "C4j 400,400,50 --pc jacobi" "n2 400,400,50 --share 2" "n4 400,400,50 --share 4" "n8 400,400,50 --share 8"; do
  set -- $spec; tag=$1; cells=$2; shift 2
  step "bench $tag"
  timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --cells $cells "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -5 $OUT/bench_$tag.err; exit 1; }
  line $OUT/bench_$tag.json $tag
done
