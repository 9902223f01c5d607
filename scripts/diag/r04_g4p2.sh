#!/bin/bash
# gemm4p correctness (kernel tests, default switches) + model-shape timing, then the
# round-end style validation (full -m gpu suite, smoke, default bench, kernel trace).
set -euo pipefail
TAG=${1:-a}
OUT=gpurun_out/r04_g4p_${TAG}; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or gelu or 2gib" -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
S=sq8192,qkv_fwd,dense_fwd,fc1_fwd_plain,fc2_fwd_resid,fc2_fwd_plain,lm_head_fwd,qkv_dw,dense_dw,fc1_dw,fc2_dw,lm_head_dw,sq8192_dw
timeout -k 10 300 python -u scripts/bench_gemm.py --tokens 180992 --no-ref --bias --only $S > "$OUT/v.jsonl" 2> "$OUT/v.err" || { tail -20 "$OUT/v.err"; exit 1; }
MMPT_GEMM_4P=0 timeout -k 10 300 python -u scripts/bench_gemm.py --tokens 180992 --no-ref --bias --only $S > "$OUT/v0.jsonl" 2> "$OUT/v0.err" || { tail -20 "$OUT/v0.err"; exit 1; }
paste <(python3 -c "import json;[print(json.loads(l)['shape'],json.loads(l)['mmpt_us']) for l in open('$OUT/v0.jsonl')]") <(python3 -c "import json;[print(json.loads(l)['mmpt_us']) for l in open('$OUT/v.jsonl')]")
bash scripts/diag/r04_full.sh "$TAG"
