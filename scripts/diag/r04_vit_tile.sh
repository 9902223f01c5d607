#!/bin/bash
# ViT-shape GEMMs (K = 768 / 3072, T = 256 x 197 tokens): gemm4p (default) vs the 128x128
# two-workgroups-per-CU kernel (MMPT_GEMM_TILE=128), two alternating runs each.
set -euo pipefail
OUT=gpurun_out/r04_vit_${1:-a}; mkdir -p "$OUT"
ARGS="--tokens 180992 --iters 10 --no-ref --bias --only vit_fc1_fwd_big,vit_qkv_fwd,vit_fc2_fwd,vit_o_fwd,vit_qkv_dx,vit_fc1_dx,vit_fc2_dx"
for r in 1 2; do
  timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/d$r.jsonl" 2> "$OUT/d.err"
  MMPT_GEMM_TILE=128 timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/t$r.jsonl" 2> "$OUT/t.err"
done
python3 - "$OUT" <<'PY'
import json, sys
d = sys.argv[1]
names = ["d1", "t1", "d2", "t2"]
runs = [{r["shape"]: r for r in map(json.loads, open(f"{d}/{n}.jsonl"))} for n in names]
print(f"{'shape':18s} " + " ".join(f"{n:>18s}" for n in names) + "  (us, TF/s)")
for k in runs[0]:
    print(f"{k:18s} " + " ".join(f"{r[k]['mmpt_us']:9.1f} {r[k]['mmpt_tflops']:7.1f}" for r in runs))
PY
