#!/bin/bash
# D = 256 register-ring depths after the slab layout: forward V^T (VD 3 -> 4) and K (SD 2 -> 3)
# fragment rings, dQ-from-dS K^T ring (KD 3 -> 4); attention microbench alternated, twice.
set -euo pipefail
OUT=gpurun_out/depth_r04; mkdir -p "$OUT"
D=multimodal_llm_pretraining_amd/lib/diag
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/base_$i.json" 2> "$OUT/base_$i.err"
  for v in vd4 sd3 kd4; do
    MMPT_LIB=$D/libmmpt_$v.so timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/${v}_$i.json" 2> "$OUT/${v}_$i.err"
  done
done
echo depth done
