#!/bin/bash
# Round-2 bench lines on one MI355X: C2 (Pythia-1B @ 2049) and C5 (CLIP-L/14-336 + Pythia-2.8B)
# with their CPU baselines, the real llava-pretrain (CLIP-L/14-336 + Llama-3.2-1B, tower and
# LLM frozen), the headline workload under zero_2 and zero_3++, and the default headline line.
set -euo pipefail
OUT=gpurun_out/cfg2
mkdir -p "$OUT"
run() {
  local tag=$1; local lim=$2; shift 2
  timeout -k 10 "$lim" python -u bench.py "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err" \
      || { tail -20 "$OUT/$tag.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag',d['value'],d['ms_per_step'],d['mfu'],d.get('training_days'),d['max_memory_reserved_gb'])"
}
run c2 400 --model pythia-1b --no-cpu-variants
run c5 500 --model clip-l14-336-pythia-2.8b --micro-batch 32 --steps 2 --warmup 1 --no-cpu-variants
run llava_pretrain 400 --model llava-pretrain --no-cpu-baseline
run zero2 300 --sharding zero_2 --no-cpu-baseline
run zero3pp 400 --sharding zero_3++ --no-cpu-baseline
run headline 400
