#!/bin/bash
# GEMM A/B on the GPU box: element-wise GEMM tests, then the bench-size shape timings with
# the current kernel and with MMPT_GEMM_PERSIST=0 (one workgroup per tile).
# Usage: bash scripts/gpu_gemm_ab.sh <tag> [shape-list]
set -euo pipefail
TAG=$1
ONLY=${2:-}
OUT=gpurun_out/ab_${TAG}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k gemm > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
ARGS="--tokens 180992 --iters 5 --no-ref"
[ -n "$ONLY" ] && ARGS="$ARGS --only $ONLY"
timeout -k 10 300 python -u scripts/bench_gemm.py $ARGS > "$OUT/new.jsonl" 2> "$OUT/new.err"
MMPT_GEMM_PERSIST=0 timeout -k 10 300 python -u scripts/bench_gemm.py $ARGS > "$OUT/old.jsonl" 2> "$OUT/old.err"
python - "$OUT" <<'PY'
import json, sys
d = sys.argv[1]
new = {r["shape"]: r for r in map(json.loads, open(f"{d}/new.jsonl"))}
old = {r["shape"]: r for r in map(json.loads, open(f"{d}/old.jsonl"))}
for k in new:
    print(f"{k:16s} old {old[k]['mmpt_us']:9.1f} us {old[k]['mmpt_tflops']:7.1f} TF/s   new {new[k]['mmpt_us']:9.1f} us {new[k]['mmpt_tflops']:7.1f} TF/s  x{old[k]['mmpt_us'] / new[k]['mmpt_us']:.3f}")
PY
