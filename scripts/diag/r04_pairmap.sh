#!/bin/bash
# dK/dV pair kernel: pairs (p, p+4) sharing a SIMD (default build) vs (2p, 2p+1) (lib/diag/libmmpt_pm0.so):
# bitwise pair-vs-ring tests on the new placement, then the attention microbench alternated.
set -euo pipefail
OUT=gpurun_out/pairmap_r04
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > "$OUT/tests.log" 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/bench_pm1_$i.json" 2> "$OUT/bench_pm1_$i.err"
  MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_pm0.so timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/bench_pm0_$i.json" 2> "$OUT/bench_pm0_$i.err"
done
echo pairmap done
