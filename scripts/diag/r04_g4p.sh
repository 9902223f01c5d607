#!/bin/bash
# gemm4p (4-wave pipelined GEMM) on one box: correctness through the kernel tests with
# MMPT_GEMM_4P=1, then the model shapes at T = 180992 with MMPT_GEMM_4P=0 / 1.
set -euo pipefail
OUT=gpurun_out/r04_g4p_${1:-a}; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_state_gpu.py tests/test_kernels_gpu.py -k "state or 2gib or segments" -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/state.log" 2>&1 || { tail -30 "$OUT/state.log"; exit 1; }
tail -1 "$OUT/state.log"
MMPT_GEMM_4P=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or gelu" -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/tests4p.log" 2>&1 || { tail -30 "$OUT/tests4p.log"; exit 1; }
tail -1 "$OUT/tests4p.log"
S=sq8192,qkv_fwd,dense_fwd,fc1_fwd_gelu,fc1_fwd_plain,fc2_fwd_resid,fc2_fwd_plain,lm_head_fwd,fc2_dx_dgelu_cs,fc1_dw_both
for v in 0 1 0 1; do
  MMPT_GEMM_4P=$v timeout -k 10 300 python -u scripts/bench_gemm.py --tokens 180992 --no-ref --bias --only $S > "$OUT/v${v}.jsonl.tmp" 2> "$OUT/v$v.err" || { tail -20 "$OUT/v$v.err"; exit 1; }
  cat "$OUT/v${v}.jsonl.tmp" >> "$OUT/v${v}.jsonl"
done
paste <(python3 -c "import json,sys;[print(json.loads(l)['shape'],json.loads(l)['mmpt_us']) for l in open('$OUT/v0.jsonl')]") <(python3 -c "import json,sys;[print(json.loads(l)['mmpt_us']) for l in open('$OUT/v1.jsonl')]")
