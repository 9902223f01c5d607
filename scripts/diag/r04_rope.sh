#!/bin/bash
# attention backward + rope backward at the bench shape: fused into the dK / dQ epilogues vs the
# attention backward followed by the rope kernel (bench_attn's pythia_bench line), twice.
set -euo pipefail
OUT=gpurun_out/rope_r04; mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
done
echo rope done
