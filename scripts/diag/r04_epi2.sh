#!/bin/bash
# What the fast epilogue's global stores cost (lib/diag/libmmpt_d5.so: everything but the
# stores, wrong results) and nontemporal stores for the plain / dGELU outputs too
# (libmmpt_nt.so), against the shipped library; then the GEMM PMC passes.
set -euo pipefail
TAG=${1:-a}
OUT=gpurun_out/r04_epi2_${TAG}; mkdir -p "$OUT"
S=qkv_fwd,fc1_fwd_gelu,fc2_dx_dgelu_cs,lm_head_fwd,dense_fwd,sq8192
ARGS="--tokens 180992 --iters 10 --no-ref --bias --only $S"
D=multimodal_llm_pretraining_amd/lib/diag
timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/ship.jsonl" 2> "$OUT/ship.err"
MMPT_LIB=$D/libmmpt_d5.so timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/nostore.jsonl" 2> "$OUT/nostore.err"
MMPT_LIB=$D/libmmpt_nt.so timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/nt.jsonl" 2> "$OUT/nt.err"
timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/ship2.jsonl" 2> "$OUT/ship2.err"
python3 - "$OUT" <<'PY'
import json, sys
d = sys.argv[1]
names = ["ship", "nostore", "nt", "ship2"]
runs = [{r["shape"]: r for r in map(json.loads, open(f"{d}/{n}.jsonl"))} for n in names]
print(f"{'shape':18s} " + " ".join(f"{n:>18s}" for n in names) + "  (us, TF/s)")
for k in runs[0]:
    print(f"{k:18s} " + " ".join(f"{r[k]['mmpt_us']:9.1f} {r[k]['mmpt_tflops']:7.1f}" for r in runs))
PY
bash scripts/diag/r04_pmc_gemm.sh "$TAG"
