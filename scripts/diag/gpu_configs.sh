#!/bin/bash
# BASELINE configs beyond the headline (one GPU): C5 (CLIP-L/14-336 + Pythia-2.8B) plain and
# with ZeRO-3 + offload, and C4's per-GPU work (Pythia-1B, 128 samples, ZeRO-3 + AC).
set -euo pipefail
OUT=gpurun_out/configs
mkdir -p "$OUT"
run() {
  local tag=$1; shift
  timeout -k 10 500 python -u bench.py --no-cpu-baseline "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err" \
      || { tail -20 "$OUT/$tag.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag',d['value'],d['ms_per_step'],d['mfu'],d['loss'],d['max_memory_reserved_gb'])"
}
run c5 --model clip-l14-336-pythia-2.8b --micro-batch 32 --steps 2 --warmup 1
run c5_z3_off --model clip-l14-336-pythia-2.8b --micro-batch 32 --steps 1 --warmup 1 --sharding zero_3 --offload
run c4_1gpu --model pythia-1b --text-len 2049 --micro-batch 16 --global-batch 128 --steps 1 --warmup 1 --sharding zero_3 --activation-checkpointing
