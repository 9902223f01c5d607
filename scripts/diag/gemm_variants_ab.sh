#!/bin/bash
# A/B of GEMM variant libraries (scripts/diag/build_variants.sh) against the shipped
# libmmpt.so on the bench-size shapes, two interleaved rounds each.
# Usage: bash scripts/diag/gemm_variants_ab.sh <tag> "<shape,list>" name1 [name2 ...]
set -euo pipefail
TAG=$1; ONLY=$2; shift 2
OUT=gpurun_out/var_${TAG}
mkdir -p "$OUT"
ARGS="--tokens 180992 --iters 5 --no-ref --only $ONLY"
for round in 1 2; do
  timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/base_$round.jsonl" 2> "$OUT/base_$round.err"
  for v in "$@"; do
    MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_$v.so timeout -k 10 200 \
        python -u scripts/bench_gemm.py $ARGS > "$OUT/${v}_$round.jsonl" 2> "$OUT/${v}_$round.err"
  done
done
python - "$OUT" base "$@" <<'PY'
import json, sys
d, names = sys.argv[1], sys.argv[2:]
best = {}
for n in names:
    for r in (1, 2):
        for rec in map(json.loads, open(f"{d}/{n}_{r}.jsonl")):
            k = (n, rec["shape"])
            best[k] = min(best.get(k, 1e30), rec["mmpt_us"])
shapes = sorted({s for _, s in best}, key=lambda s: s)
print(f"{'shape':16s} " + " ".join(f"{n:>14s}" for n in names) + "   (best-of-2 us; ratio vs base)")
for s in shapes:
    b = best[("base", s)]
    print(f"{s:16s} " + " ".join(f"{best[(n, s)]:8.1f} x{b / best[(n, s)]:.3f}" for n in names))
PY
