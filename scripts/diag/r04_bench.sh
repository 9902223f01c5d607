#!/bin/bash
# The default bench line twice on one box (box-to-box clocks differ by up to ~10%; the line
# carries the clock and the 8192^3 yardstick so runs can be compared).
set -euo pipefail
OUT=gpurun_out/r04_bench_${1:-a}; mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || { tail -20 "$OUT/bench_$i.err"; exit 1; }
done
echo bench done
