#!/bin/bash
# What the epilogue costs per kernel at the K = 2048 model shapes: gemm256 vs gemm4p, each
# with the shipped epilogue and with the diagnostic no-epilogue build (MMPT_GEMM_DIAG=4,
# wrong results), built by: bash scripts/diag/build_variants.sh d4:gemm:-DMMPT_GEMM_DIAG=4
set -euo pipefail
OUT=gpurun_out/epi_diag_${1:-x}
mkdir -p "$OUT"
S=${2:-qkv_fwd,fc1_fwd_plain,fc1_fwd_gelu,fc2_dx_dgelu_cs,lm_head_fwd,dense_fwd,sq8192}
ARGS="--tokens 180992 --iters 10 --no-ref --bias --only $S"
D4=multimodal_llm_pretraining_amd/lib/diag/libmmpt_d4.so
MMPT_GEMM_4P=0 timeout -k 10 240 python -u scripts/bench_gemm.py $ARGS > "$OUT/g256.jsonl" 2> "$OUT/g256.err"
MMPT_GEMM_4P=2 timeout -k 10 240 python -u scripts/bench_gemm.py $ARGS > "$OUT/g4p.jsonl" 2> "$OUT/g4p.err"
MMPT_LIB=$D4 MMPT_GEMM_4P=0 timeout -k 10 240 python -u scripts/bench_gemm.py $ARGS > "$OUT/g256_noepi.jsonl" 2> "$OUT/g256_noepi.err"
MMPT_LIB=$D4 MMPT_GEMM_4P=2 timeout -k 10 240 python -u scripts/bench_gemm.py $ARGS > "$OUT/g4p_noepi.jsonl" 2> "$OUT/g4p_noepi.err"
python3 - "$OUT" <<'PY'
import json, sys
d = sys.argv[1]
names = ["g256", "g4p", "g256_noepi", "g4p_noepi"]
runs = [{r["shape"]: r for r in map(json.loads, open(f"{d}/{n}.jsonl"))} for n in names]
print(f"{'shape':18s} " + " ".join(f"{n:>18s}" for n in names) + "  (us, TF/s)")
for k in runs[0]:
    print(f"{k:18s} " + " ".join(f"{r[k]['mmpt_us']:9.1f} {r[k]['mmpt_tflops']:7.1f}" for r in runs))
PY
