#!/bin/bash
# ViT (D = 64) attention with 2 query tiles per wave (lib/diag/libmmpt_qt2.so) vs 1 (default):
# the attention tests on the variant, then the attention microbench alternated.
set -euo pipefail
OUT=gpurun_out/qt64_r04; mkdir -p "$OUT"
V=multimodal_llm_pretraining_amd/lib/diag/libmmpt_qt2.so
MMPT_LIB=$V timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > "$OUT/tests_qt2.log" 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/bench_qt1_$i.json" 2> "$OUT/bench_qt1_$i.err"
  MMPT_LIB=$V timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/bench_qt2_$i.json" 2> "$OUT/bench_qt2_$i.err"
done
echo qt64 done
