#!/bin/bash
# Offload lines after the vectorised host Adam: the offload GPU tests, C3 + offload (DDP and
# ZeRO-3), C5 + ZeRO-3 + offload, and the headline line for the same box.
set -euo pipefail
OUT=gpurun_out/off2
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_sharding_gpu.py tests/test_rccl_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -k "offload" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
run() {
  local tag=$1; local lim=$2; shift 2
  timeout -k 10 "$lim" python -u bench.py "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err" \
      || { tail -20 "$OUT/$tag.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag',d['value'],d['ms_per_step'],d['mfu'],d['max_memory_reserved_gb'])"
}
run offload 300 --offload --no-cpu-baseline
run zero3_offload 300 --sharding zero_3 --offload --no-cpu-baseline
run c5_z3_offload 500 --model clip-l14-336-pythia-2.8b --micro-batch 32 --steps 2 --warmup 1 --sharding zero_3 --offload --no-cpu-baseline
run headline 300 --no-cpu-baseline
