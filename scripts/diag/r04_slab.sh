#!/bin/bash
# D = 256 slab images (default) vs the row-major swizzled images (preslab: the commit before)
# attention tests, then the attention microbench alternated.
set -euo pipefail
OUT=gpurun_out/slab_r04
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > "$OUT/tests.log" 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/bench_slab_$i.json" 2> "$OUT/bench_slab_$i.err"
  MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_preslab.so timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 > "$OUT/bench_preslab_$i.json" 2> "$OUT/bench_preslab_$i.err"
done
echo pairmap done
