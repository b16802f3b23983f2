#!/bin/bash
# A/B of library builds, interleaved: $1 = tag, $2 = "suffix:label ..." (suffix "base" = libtvfem.so), $3 = bench configs "tag|args;..."
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
IFS=';' read -r -a CFGS <<< "$3"
for rep in 1 2; do
  for lib in $2; do
    v=${lib%%:*}; [ "$v" = base ] && v=""
    for cfg in "${CFGS[@]}"; do
      tag=${cfg%%|*}; args=${cfg#*|}
      IFS=' ' read -r -a argv <<< "$args"
      o=$OUT/b${v}_${tag}_$rep
      TVFEM_LIB=$PWD/fem-glass-tempering_amd/tvfem/libtvfem$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline "${argv[@]}" > $o.json 2> $o.err || { tail -5 $o.err; exit 1; }
      python3 -c "import json;d=json.load(open('$o.json'));print('lib$v', '$tag', round(d['ms_per_step'],3), d['config'].get('krylov_its_per_step'), {k:round(v['ms']*1e3,1) for k,v in d['kernels'].items()}, 'flushed', round(d['roofline']['hbm_flushed']['ms_per_launch']*1e3,1))"
    done
  done
done
