#!/bin/bash
# Attention microbench over variant libraries (scripts/diag/build_variants.sh), interleaved twice.
set -euo pipefail
OUT=gpurun_out/av_${1:-a}; mkdir -p "$OUT"; shift
for rep in 1 2; do
  for v in "$@"; do
    MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_$v.so timeout -k 10 120 python -u scripts/bench_attn.py \
        | grep pythia_bench | sed "s/^/$v /" >> "$OUT/ab.txt"
  done
done
cat "$OUT/ab.txt"
