#!/bin/bash
# Pipelined fast epilogue vs the first fast epilogue (lib/diag/libmmpt_fastv1.so): GEMM
# kernel tests on the shipped library, then the shape timings of both (same box).
set -euo pipefail
TAG=${1:-a}
OUT=gpurun_out/r04_g4f2_${TAG}; mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or gelu or 2gib" -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
S=${2:-qkv_fwd,fc1_fwd_plain,fc1_fwd_gelu,fc2_dx_dgelu_cs,lm_head_fwd,dense_fwd,sq8192,vit_fc1_fwd_big}
ARGS="--tokens 180992 --iters 10 --no-ref --bias --only $S"
for r in 1 2; do
MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_fastv1.so timeout -k 10 240 python -u scripts/bench_gemm.py $ARGS > "$OUT/v1_$r.jsonl" 2> "$OUT/v1.err"
timeout -k 10 240 python -u scripts/bench_gemm.py $ARGS > "$OUT/v2_$r.jsonl" 2> "$OUT/v2.err"
done
python3 - "$OUT" <<'PY'
import json, sys
d = sys.argv[1]
names = ["v1_1", "v2_1", "v1_2", "v2_2"]
runs = [{r["shape"]: r for r in map(json.loads, open(f"{d}/{n}.jsonl"))} for n in names]
print(f"{'shape':18s} " + " ".join(f"{n:>18s}" for n in names) + "  (us, TF/s)")
for k in runs[0]:
    print(f"{k:18s} " + " ".join(f"{r[k]['mmpt_us']:9.1f} {r[k]['mmpt_tflops']:7.1f}" for r in runs))
PY
