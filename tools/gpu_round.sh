#!/bin/bash
# Round-end GPU session: parity suite, PMC traffic (separate FETCH / WRITE
# passes) of the C4 and C5 hot kernels, the C4 bench under a rocprofv3 kernel
# trace + the trace cross-check, the plain C4 bench line, and the C2/C3/C5 and
# per-rank-share bench lines.  Usage (via gpurun): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { echo "[gpu_round] $*"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s -rs --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -1
grep -h "^\[parity\]" $OUT/tests.log > $OUT/parity_lines.txt
for fam in CG DG; do
  if [ $fam = CG ]; then cells=400,400,50; dom=pcg_matvec_fused; key=pcg_matvec_fused; else cells=200,200,25; dom=dg_matvec_fused; key=pcg_matvec_fused; fi
  step "pmc $fam fetch"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_${fam}_fetch -o run --output-format csv -- python3 tools/pmc_kernels.py --family $fam --cells $cells > $OUT/pmc_${fam}_fetch.log 2>&1 || exit 1
  step "pmc $fam write"
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_${fam}_write -o run --output-format csv -- python3 tools/pmc_kernels.py --family $fam --cells $cells > $OUT/pmc_${fam}_write.log 2>&1 || exit 1
  python3 tools/pmc_summarize.py $OUT/pmc_${fam}_fetch $OUT/pmc_${fam}_write $OUT/pmc_${key}_${fam}_${cells//,/x}_n1.json $dom > $OUT/pmc_${fam}_summary.log 2>&1 || exit 1
  cp $OUT/pmc_${key}_${fam}_${cells//,/x}_n1.json profiles/
done
step "pmc distorted-hex fetch / write"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_UM_fetch -o run --output-format csv -- python3 tools/pmc_kernels.py --mesh distorted > $OUT/pmc_UM_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_UM_write -o run --output-format csv -- python3 tools/pmc_kernels.py --mesh distorted > $OUT/pmc_UM_write.log 2>&1 || exit 1
python3 tools/pmc_summarize.py $OUT/pmc_UM_fetch $OUT/pmc_UM_write $OUT/pmc_jacobian_apply_unstructured_CG_400x400x50_n1.json jacobian_apply_unstructured > $OUT/pmc_UM_summary.log 2>&1 || exit 1
cp $OUT/pmc_jacobian_apply_unstructured_CG_400x400x50_n1.json profiles/
step "bench distorted-hex C4 under rocprofv3 --kernel-trace --stats"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_distorted -o run --output-format csv -- python3 bench.py --mesh distorted --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_distorted_prof.json 2> $OUT/bench_distorted_prof.err || { tail -5 $OUT/bench_distorted_prof.err; exit 1; }
timeout -k 10 600 python3 bench.py --mesh distorted --steps 5 --warmup 1 > $OUT/bench_distorted.json 2> $OUT/bench_distorted.err || { tail -5 $OUT/bench_distorted.err; exit 1; }
step "bench C4 under rocprofv3 --kernel-trace --stats"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python3 bench.py > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -5 $OUT/bench_prof.err; exit 1; }
python3 tools/profile_summary.py $OUT/prof_bench $OUT/bench_prof.json $OUT/profile_summary.json > $OUT/profile_summary.log 2>&1
step "bench C5 under rocprofv3 --kernel-trace"
timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/prof_c5 -o run --output-format csv -- python3 bench.py --family DG --cells 200,200,25 --steps 5 --warmup 1 --kernel-reps 3 --no-cpu-baseline > $OUT/bench_c5_prof.json 2> $OUT/bench_c5_prof.err || { tail -5 $OUT/bench_c5_prof.err; exit 1; }
step "bench C4 plain"
timeout -k 10 600 python3 bench.py > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -5 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
# n8 / n4 / n2: one rank's share of the C4 slab partition, with the partitioned
# path's solver (Jacobi; single-reduction CG up to 3M owned nodes, KSPCG above); C4j / C5j: the Jacobi-PCG lines
for spec in "C2 100,100,10 --thermal-only" "C3 200,200,25" "C5 200,200,25 --family DG" "C5j 200,200,25 --family DG --pc jacobi --no-cpu-baseline" "C4j 400,400,50 --pc jacobi --no-cpu-baseline" "n8 400,50,50 --pc jacobi --pcg single --no-cpu-baseline" "n4 400,100,50 --pc jacobi --pcg single --no-cpu-baseline" "n2 400,200,50 --pc jacobi --pcg kspcg --no-cpu-baseline"; do
  set -- $spec; tag=$1; cells=$2; shift 2
  step "bench $tag"
  timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --cells $cells "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -5 $OUT/bench_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$tag.json'));print('$tag', round(d['ms_per_step'],3), 'ms/step', d['config']['krylov_its_per_step'], 'its', {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()})"
done
step "bench C3 with output"
mkdir -p /tmp/tvout && timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --cells 200,200,25 --output /tmp/tvout > $OUT/bench_C3_output.json 2> $OUT/bench_C3_output.err && rm -rf /tmp/tvout
python3 -c "import json;d=json.load(open('$OUT/bench_C3_output.json'));print('C3+output', round(d['ms_per_step'],3))"
