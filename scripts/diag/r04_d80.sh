#!/bin/bash
# head_dim 80 computed natively (MMPT_ATTN_NATIVE80): bitwise A/B test + attention kernel tests,
# attention microbench (D = 80 native vs padded), and the lm_head weight-gradient split A/B.
set -euo pipefail
OUT=gpurun_out/d80_r04
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > "$OUT/tests.log" 2>&1
timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/bench_attn.json" 2> "$OUT/bench_attn.err"
for sp in 0 1 2 3 4; do
  if [ "$sp" = 0 ]; then unset MMPT_GEMM_SPLITS; else export MMPT_GEMM_SPLITS=$sp; fi
  timeout -k 10 180 python -u scripts/bench_gemm.py --no-ref --iters 5 --tokens 130816 --only lm_head_dw,fc1_dw > "$OUT/dw_split$sp.txt" 2>&1
done
echo d80 done
