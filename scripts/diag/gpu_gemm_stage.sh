#!/bin/bash
# LDS-staged GEMM epilogue stores: GEMM kernel tests, then the A/B against the per-lane
# store build (lib/diag/libmmpt_nostg.so, scripts/diag/build_variants.sh).
set -euo pipefail
mkdir -p gpurun_out/stage
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "gemm or gelu or swiglu" > gpurun_out/stage/tests.txt 2>&1
tail -3 gpurun_out/stage/tests.txt
bash scripts/diag/gemm_variants_ab.sh stage "${1:-fc1_fwd_gelu,fc2_dx_dgelu_cs,qkv_fwd,fc1_fwd_plain,fc1_dx,lm_head_fwd,fc2_fwd_resid}" nostg
