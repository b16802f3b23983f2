#!/bin/bash
# A/B of experiment switches on bench lines (kernel table + flushed J x).
# Usage (via gpurun): bash tools/gpu_ab.sh TAG "ARGS" "VAR=V ..." ["VAR=V ..." ...]
#   ARGS: bench arguments shared by every variant; "-" = the defaults
set -o pipefail
TAG=$1; ARGS=$2; shift 2
[ "$ARGS" = "-" ] && ARGS=""
OUT=gpurun_out/$TAG
mkdir -p $OUT
n=0
for V in "$@"; do
  n=$((n+1))
  [ "$V" = "-" ] && V=""
  env TVFEM_EXPERIMENTS=1 $V timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --kernel-reps 5 --no-cpu-baseline $ARGS > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -5 $OUT/b_$n.err; exit 1; }
  python3 - "$OUT/b_$n.json" "$V" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]; fl = d["roofline"].get("hbm_flushed", {})
print(f"[{sys.argv[2] or 'default'}] {d['ms_per_step']:.3f} ms/step its {c.get('krylov_its_per_step')} "
      f"flushed {fl.get('ms_per_launch', 0)*1000:.1f}us frac {fl.get('frac', 0):.3f} "
      + str({k: round(v['ms'] * 1000, 1) for k, v in d['kernels'].items()}), flush=True)
PY
done
