#!/bin/bash
# SADDR-form LDS-DMA with integer LDS addresses (default) vs per-lane 64-bit addresses (sa0)
# attention tests, then the attention microbench alternated.
set -euo pipefail
OUT=gpurun_out/saddr_r04
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > "$OUT/tests.log" 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/bench_sa1_$i.json" 2> "$OUT/bench_sa1_$i.err"
  MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_sa0.so timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/bench_sa0_$i.json" 2> "$OUT/bench_sa0_$i.err"
done
echo pairmap done
