#!/bin/bash
# Rehearsal of bench.py's N > 1 path (torch.distributed.run launch, RANK / WORLD_SIZE, barrier,
# max-over-ranks timing, the exchange of each mode, the per-rank comm busy / exposed fields)
# with two ranks sharing the one GPU over gloo: ddp, zero_2, zero_3.
set -euo pipefail
OUT=gpurun_out/n2; mkdir -p $OUT
PORT=29517
for MODE in ddp zero_2 zero_3; do
  SH=""; [ "$MODE" != ddp ] && SH="--sharding $MODE"
  PORT=$((PORT+1))
  MMPT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $PORT bench.py --gpus 2 --steps 2 --warmup 1 \
      --global-batch 32 --micro-batch 8 --no-cpu-baseline --no-yardstick $SH > $OUT/bench_n2_$MODE.json 2> $OUT/bench_n2_$MODE.err \
      || { tail -30 $OUT/bench_n2_$MODE.err; exit 1; }
  grep '^{' $OUT/bench_n2_$MODE.json > $OUT/line_$MODE.json; python -c "import json,sys; d=json.load(open('$OUT/line_$MODE.json')); print('$MODE', d['value'], d['config']['parallelism'], json.dumps(d['comm']))"
done
