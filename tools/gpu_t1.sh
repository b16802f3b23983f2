#!/bin/bash
# Session check: GPU parity suite, the default bench line, and a one-GPU
# rehearsal of the RCCL transport (two ranks sharing GPU 0, where RCCL allows it).
set -o pipefail
OUT=gpurun_out/t1
mkdir -p $OUT
bash tools/gpu_tests.sh t1 || exit 1
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 180 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29731 \
  tools/partition_check.py --comm rccl0 --cells 12,48,6 > $OUT/rccl0.log 2>&1
echo "rccl0 rc=$?"
grep -h "PARTITION_CHECK\|Duplicate\|NCCL\|rror" $OUT/rccl0.log | head -20
