#!/bin/bash
# gemm4p fast epilogues (epilogue4f): GEMM kernel tests with every epilogue on gemm4p
# (MMPT_GEMM_4P=2) and with the defaults, then the epilogue-cost A/B (r04_epi_diag.sh).
set -euo pipefail
TAG=${1:-a}
OUT=gpurun_out/r04_g4f_${TAG}; mkdir -p "$OUT"
K="gemm or gelu or 2gib"
MMPT_GEMM_4P=2 timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -k "$K" -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/tests_4p2.log" 2>&1 || { tail -30 "$OUT/tests_4p2.log"; exit 1; }
tail -1 "$OUT/tests_4p2.log"
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -k "$K" -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/tests_default.log" 2>&1 || { tail -30 "$OUT/tests_default.log"; exit 1; }
tail -1 "$OUT/tests_default.log"
bash scripts/diag/r04_epi_diag.sh "$TAG" qkv_fwd,fc1_fwd_plain,fc1_fwd_gelu,fc2_dx_dgelu_cs,lm_head_fwd,dense_fwd,fc2_fwd_resid,sq8192,vit_fc1_fwd_big,vit_qkv_fwd
