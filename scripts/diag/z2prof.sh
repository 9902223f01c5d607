#!/bin/bash
set -euo pipefail
OUT=gpurun_out/z2prof; mkdir -p $OUT
for MODE in zero_2 zero_3; do
MMPT_CPROFILE=$OUT/$MODE MMPT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29712 bench.py --gpus 2 --model tiny-mm --steps 2 --warmup 1 \
    --global-batch 16 --micro-batch 4 --text-len 47 --no-cpu-baseline --no-yardstick --sharding $MODE > $OUT/$MODE.json 2> $OUT/$MODE.err
done
head -60 $OUT/zero_2.rank0.txt
