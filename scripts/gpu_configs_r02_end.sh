#!/bin/bash
# End-of-round-2 bench lines for the other configurations (final kernels): C2, C5, llava-pretrain.
set -euo pipefail
OUT=gpurun_out/cfg_end
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
run headline 300 --no-cpu-baseline
