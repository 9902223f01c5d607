#!/bin/bash
# Round-3 bench lines beyond the headline on one GPU, each workload's micro-batch by the
# reference's find_max_mbs_pow2 rule (bench.py probes where no footprint is measured):
# C2 (Pythia-1B @ 2049, batch 1024), C5 (CLIP-L/14-336 + Pythia-2.8B) plain and as BASELINE
# configures it (ZeRO-3 + host offload), llava-pretrain; then the N>1 rehearsal (two gloo ranks
# on the one GPU, tiny model: the launch / exchange / comm-accounting path of ddp, zero_2, zero_3).
set -euo pipefail
OUT=gpurun_out/configs_r03; mkdir -p "$OUT"
run() {
  local tag=$1; shift
  timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err" \
      || { tail -20 "$OUT/$tag.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));c=d['config'];print('$tag',d['value'],d['ms_per_step'],d['mfu'],c['micro_batch'],c.get('micro_batch_rule'),d['max_memory_reserved_gb'],d.get('training_days'))"
}
[ -n "${SKIP_CFG:-}" ] || run c2 --model pythia-1b --steps 2 --warmup 1
[ -n "${SKIP_CFG:-}" ] || run c5 --model clip-l14-336-pythia-2.8b --steps 2 --warmup 1
[ -n "${SKIP_CFG:-}" ] || run c5_z3_off --model clip-l14-336-pythia-2.8b --steps 2 --warmup 1 --sharding zero_3 --offload
[ -n "${SKIP_CFG:-}" ] || run llava_pretrain --model llava-pretrain --steps 3 --warmup 1
PORT=29617
for MODE in ddp zero_2 zero_3; do
  SH=""; [ "$MODE" != ddp ] && SH="--sharding $MODE"
  PORT=$((PORT+1))
  MMPT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $PORT bench.py --gpus 2 --model tiny-mm --steps 2 --warmup 1 \
      --global-batch 16 --micro-batch 4 --text-len 47 --no-cpu-baseline --no-yardstick $SH > $OUT/n2_$MODE.json 2> $OUT/n2_$MODE.err \
      || { tail -30 $OUT/n2_$MODE.err; exit 1; }
  grep '^{' $OUT/n2_$MODE.json > $OUT/n2_line_$MODE.json
  python -c "import json; d=json.load(open('$OUT/n2_line_$MODE.json')); print('$MODE', d['value'], d['config']['parallelism'], json.dumps(d['comm'])[:300])"
done
