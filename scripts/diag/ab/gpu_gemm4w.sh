#!/bin/bash
# 4-wave GEMM (MMPT_GEMM_4W=1) vs the 8-wave gemm256 on the plain ROWS_K x ROWS_K shapes, after
# the GEMM kernel tests run through it; then the forward K-ring A/B (variant libraries).
set -euo pipefail
O=gpurun_out/g4w_${1:-a}; mkdir -p $O
MMPT_GEMM_4W=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--tokens 180992 --iters 5 --no-ref --bias --only qkv_fwd,dense_fwd,fc1_fwd_plain,fc2_fwd_plain,sq8192,sq4096"
for v in 0 1 0 1; do
  MMPT_GEMM_4W=$v timeout -k 10 240 python -u scripts/bench_gemm.py $A > $O/v$v.jsonl 2> $O/v$v.err
  python -c "import sys,json; print('4w=$v', ' '.join(f\"{r['shape']}={r['mmpt_us']}/{r['mmpt_tflops']}\" for r in map(json.loads, open('$O/v$v.jsonl'))))"
done
