#!/bin/bash
# CU start skew A/B (MMPT_GEMM_SKEW: every other CU of an XCD starts s_sleep-127 x N later, so
# the two halves' epilogue write bursts alternate instead of coinciding).
set -euo pipefail
TAG=${1:-a}
OUT=gpurun_out/r04_skew_${TAG}; mkdir -p "$OUT"
S=${2:-fc1_fwd_gelu,fc2_dx_dgelu_cs,qkv_fwd,lm_head_fwd,fc2_fwd_resid,sq8192}
ARGS="--tokens 180992 --iters 10 --no-ref --bias --only $S"
for k in 0 4 7 14 0; do
  MMPT_GEMM_SKEW=$k timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/skew$k.jsonl" 2> "$OUT/skew$k.err"
done
python3 - "$OUT" <<'PY'
import json, sys
d = sys.argv[1]
names = ["skew0", "skew4", "skew7", "skew14"]
runs = [{r["shape"]: r for r in map(json.loads, open(f"{d}/{n}.jsonl"))} for n in names]
print(f"{'shape':18s} " + " ".join(f"{n:>18s}" for n in names) + "  (us, TF/s)")
for k in runs[0]:
    print(f"{k:18s} " + " ".join(f"{r[k]['mmpt_us']:9.1f} {r[k]['mmpt_tflops']:7.1f}" for r in runs))
PY
