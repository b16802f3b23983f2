#!/bin/bash
# The one GPU-session runner (replaces the per-session scripts of rounds 1-4).
#   bash tools/gpu_run.sh TAG MODE...      modes run in order; the first failure ends the call
# Modes:
#   tests            the GPU suite (pytest -m gpu; PYTEST_K narrows it with -k)
#   bench            bench lines: BENCHES="tag|bench args;tag|args;..." (default: the C4 line with
#                    the CPU baseline); every line prints ms/step, Newton / Krylov counts, kernels
#   trace            rocprofv3 --kernel-trace of bench configs: TRACES="tag|args;..." + the idle-gap
#                    accounting of one step window (tools/trace_gaps.py)
#   stats            the C4 bench under rocprofv3 --kernel-trace --stats (profile summary)
#   pmc              FETCH_SIZE / WRITE_SIZE passes of the GMG solve (C4 CG, C5 DG), one pass each
#   ab               interleaved A/B of library builds: LIBS="suffix ..." (base = libtvfem.so) x
#                    BENCHES; each variant library runs PYTEST_AB (default: the step-parity subset)
#                    first, so a variant that is wrong never gets a timing line
#   loopback         the RCCL loopback check + the per-pattern latency table (tools/loopback_check.py)
set -o pipefail
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { echo "[gpu_run $TAG] $*"; }
line() {
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["config"]
r = d.get("roofline") or {}
fl = (r.get("hbm_flushed") or {}).get("ms_per_launch")
print(sys.argv[2], round(d["ms_per_step"], 3), "ms/step", c.get("newton_its_per_step"), c.get("krylov_its_per_step"), "its",
      {k: round(v["ms"] * 1e3, 1) for k, v in d.get("kernels", {}).items()},
      "frac", round(r.get("frac", 0.0), 3), "flushed_us", None if fl is None else round(fl * 1e3, 1))
EOF
}
run_bench() {  # tag, lib suffix, args...
  local tag=$1 v=$2; shift 2
  local o=$OUT/bench_${tag}${v:+_$v}
  TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$v.so timeout -k 10 600 python3 bench.py "$@" > $o.json 2> $o.err ||
    { tail -5 $o.err; return 1; }
  line $o.json "${tag}${v:+ lib$v}"
}
for MODE in "$@"; do
  case $MODE in
    tests)
      step "GPU suite ${PYTEST_K:+(-k $PYTEST_K)}"
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s -rs --timeout 300 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/tests.log 2>&1
      rc=$?; tail -3 $OUT/tests.log
      grep -h "^\[parity\]\|^\[c3\|^\[fullsize\]\|^\[amg\]\|upartition\]" $OUT/tests.log > $OUT/parity_lines.txt
      if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR|Error" $OUT/tests.log | head -20; exit $rc; fi
      ;;
    bench)
      IFS=';' read -r -a CFGS <<< "${BENCHES:-c4|--steps 20 --warmup 2}"
      for cfg in "${CFGS[@]}"; do
        tag=${cfg%%|*}; IFS=' ' read -r -a argv <<< "${cfg#*|}"
        step "bench $tag"
        run_bench $tag "" "${argv[@]}" || exit 1
      done
      ;;
    trace)
      IFS=';' read -r -a CFGS <<< "${TRACES:?TRACES}"
      for cfg in "${CFGS[@]}"; do
        tag=${cfg%%|*}; IFS=' ' read -r -a argv <<< "${cfg#*|}"
        step "trace $tag"
        mkdir -p $OUT/tr_$tag
        timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/tr_$tag/prof -o run --output-format csv -- \
          python3 bench.py --no-cpu-baseline "${argv[@]}" > $OUT/tr_$tag/b.json 2> $OUT/tr_$tag/b.err ||
          { tail -5 $OUT/tr_$tag/b.err; exit 1; }
        f=$(find $OUT/tr_$tag/prof -name "run_kernel_trace.csv" | head -1)
        mv "$f" $OUT/tr_$tag/run_kernel_trace.csv
        line $OUT/tr_$tag/b.json $tag
        python3 tools/trace_gaps.py $OUT/tr_$tag/run_kernel_trace.csv > $OUT/tr_$tag/gaps.txt 2>&1
        head -30 $OUT/tr_$tag/gaps.txt
      done
      ;;
    stats)
      step "C4 bench under rocprofv3 --kernel-trace --stats"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -5 $OUT/bench_prof.err; exit 1; }
      python3 tools/profile_summary.py $OUT/prof_bench $OUT/bench_prof.json $OUT/profile_summary.json > $OUT/profile_summary.log 2>&1
      line $OUT/bench_prof.json C4prof
      ;;
    pmc)
      for fam in CG DG; do
        if [ $fam = CG ]; then cells=400,400,50; else cells=200,200,25; fi
        for ctr in FETCH_SIZE WRITE_SIZE; do
          step "pmc $fam gmg $ctr"
          timeout -s KILL 300 rocprofv3 --pmc $ctr -d $OUT/pmc_${fam}_gmg_$ctr -o run --output-format csv -- \
            python3 tools/pmc_kernels.py --pc gmg --family $fam --cells $cells > $OUT/pmc_${fam}_gmg_$ctr.log 2>&1 ||
            { tail -5 $OUT/pmc_${fam}_gmg_$ctr.log; exit 1; }
          step "pmc $fam jx $ctr"
          timeout -s KILL 300 rocprofv3 --pmc $ctr -d $OUT/pmc_${fam}_jx_$ctr -o run --output-format csv -- \
            python3 tools/pmc_kernels.py --jx-only --family $fam --cells $cells > $OUT/pmc_${fam}_jx_$ctr.log 2>&1 ||
            { tail -5 $OUT/pmc_${fam}_jx_$ctr.log; exit 1; }
        done
        dom=pcg_matvec_fused; [ $fam = DG ] && dom=dg_matvec_fused
        f=pmc_pcg_matvec_fused_${fam}_${cells//,/x}_n1_gmg.json
        python3 tools/pmc_summarize.py $OUT/pmc_${fam}_gmg_FETCH_SIZE $OUT/pmc_${fam}_gmg_WRITE_SIZE $OUT/$f $dom \
          $OUT/pmc_${fam}_jx_FETCH_SIZE $OUT/pmc_${fam}_jx_WRITE_SIZE > $OUT/pmc_${fam}_gmg_summary.log 2>&1 || exit 1
      done
      ;;
    ab)
      IFS=';' read -r -a CFGS <<< "${BENCHES:?BENCHES}"
      for v in ${LIBS:?LIBS}; do
        if [ "$v" = base ]; then continue; fi
        step "parity subset on libtvfem$v.so"
        TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
          --timeout 200 --timeout-method thread -k "${PYTEST_AB:-steps or partition or vcycle or fullsize}" \
          > $OUT/ab_tests_$v.log 2>&1 || { echo "variant $v FAILED its parity subset"; tail -15 $OUT/ab_tests_$v.log; exit 1; }
        tail -1 $OUT/ab_tests_$v.log
      done
      for rep in 1 2; do
        for v in $LIBS; do
          if [ "$v" = base ]; then v=""; fi
          for cfg in "${CFGS[@]}"; do
            tag=${cfg%%|*}; IFS=' ' read -r -a argv <<< "${cfg#*|}"
            run_bench ${tag}_$rep "$v" --no-cpu-baseline "${argv[@]}" || exit 1
          done
        done
      done
      ;;
    loopback)
      step "RCCL loopback"
      timeout -k 10 600 python3 tools/loopback_check.py > $OUT/loopback.txt 2>&1 || { tail -20 $OUT/loopback.txt; exit 1; }
      tail -40 $OUT/loopback.txt
      ;;
    *) echo "unknown mode $MODE"; exit 2 ;;
  esac
done
