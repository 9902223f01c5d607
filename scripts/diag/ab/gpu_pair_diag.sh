#!/bin/bash
# Wave-pair dK/dV diagnostics: each MMPT_ATTN_PDIAG variant library (scripts/diag/build_variants.sh)
# on the attention microbench, then PMC passes over the shipped kernel.
set -euo pipefail
OUT=gpurun_out/pdiag_${1:-a}; mkdir -p "$OUT"
for v in pd0 pd1 pd2 pd3 pd4 pd5 pd6 pd7 pd8 pd0; do
  MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_$v.so timeout -k 10 120 python -u scripts/bench_attn.py \
      | grep pythia_bench | sed "s/^/$v /" >> "$OUT/diag.txt"
done
cat "$OUT/diag.txt"
bash scripts/diag/attn_pmc.sh pdiag_${1:-a}
cat gpurun_out/pmc_pdiag_${1:-a}/summary.txt | head -80
