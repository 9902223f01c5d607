#!/bin/bash
# GEMM epilogue A/B: the GEMM kernel tests, then shape timings (with the model's forward bias)
# for the shipped library and a variant (MMPT_LIB) on the same box.
set -euo pipefail
O=gpurun_out/epi_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemm or gelu" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--tokens 180992 --iters 5 --no-ref --bias --only ${ONLY:-qkv_fwd,dense_fwd,fc1_fwd_gelu,fc2_fwd_resid,qkv_dx,fc1_dx,fc2_dx_dgelu,lm_head_fwd,lm_head_dx,fc1_dw}"
for v in ${VARIANTS:-new p0 new}; do
  if [ "$v" = new ]; then L=""; else L=multimodal_llm_pretraining_amd/lib/diag/libmmpt_$v.so; fi
  MMPT_LIB=$L timeout -k 10 240 python -u scripts/bench_gemm.py $A > $O/$v.jsonl 2> $O/$v.err
  python -c "import sys,json; print('$v', ' '.join(f\"{r['shape']}={r['mmpt_us']}\" for r in map(json.loads, open('$O/$v.jsonl'))))"
done
