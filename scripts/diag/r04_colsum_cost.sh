#!/bin/bash
# Step-time cost of the qkv bias column sums: bench unpatched vs with them skipped (diagnostic).
set -euo pipefail
OUT=gpurun_out/colsum_r04; mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$OUT/base_$i.json" 2> "$OUT/base_$i.err"
  timeout -k 10 400 python -u scripts/diag/r04_colsum_cost.py --no-cpu-baseline > "$OUT/skip_$i.json" 2> "$OUT/skip_$i.err"
done
echo colsum done
