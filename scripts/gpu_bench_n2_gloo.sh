#!/bin/bash
# Rehearsal of bench.py's N > 1 path (torch.distributed.run launch, RANK / WORLD_SIZE, barrier,
# max-over-ranks timing, DDP gradient exchange) with two ranks sharing the one GPU over gloo.
set -euo pipefail
OUT=gpurun_out/n2; mkdir -p $OUT
MMPT_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 \
    --global-batch 64 --micro-batch 16 --no-cpu-baseline > $OUT/bench_n2.json 2> $OUT/bench_n2.err \
    || { tail -30 $OUT/bench_n2.err; exit 1; }
cat $OUT/bench_n2.json
