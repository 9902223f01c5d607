#!/bin/bash
# Where the gemm256 mainloop spends its time: the shape timings with the shipped kernel and
# the diagnostic builds (1 = no vmcnt waits, 2 = no LDS-DMA, 3 = no fragment reads), built with
# bash scripts/diag/build_variants.sh d1:gemm:-DMMPT_GEMM_DIAG=1 d2:gemm:-DMMPT_GEMM_DIAG=2 d3:gemm:-DMMPT_GEMM_DIAG=3
set -euo pipefail
OUT=gpurun_out/diag_${1:-x}
ONLY=${2:-qkv_fwd,fc1_fwd_plain,fc2_fwd_plain,fc1_dx,qkv_dw,sq8192}
mkdir -p "$OUT"
ARGS="--tokens 180992 --iters 5 --no-ref --only $ONLY"
timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/d0.jsonl" 2> "$OUT/d0.err"
for d in 1 2 3; do
  MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_d$d.so timeout -k 10 200 \
      python -u scripts/bench_gemm.py $ARGS > "$OUT/d$d.jsonl" 2> "$OUT/d$d.err"
done
python - "$OUT" <<'PY'
import json, sys
d = sys.argv[1]
runs = [{r["shape"]: r for r in map(json.loads, open(f"{d}/d{i}.jsonl"))} for i in range(4)]
print(f"{'shape':16s} {'shipped':>16s} {'no-wait':>16s} {'no-dma':>16s} {'no-ds_read':>16s}  (us, TF/s)")
for k in runs[0]:
    print(f"{k:16s} " + " ".join(f"{r[k]['mmpt_us']:8.1f} {r[k]['mmpt_tflops']:7.1f}" for r in runs))
PY
