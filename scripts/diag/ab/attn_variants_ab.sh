#!/bin/bash
# A/B of attention variant libraries (scripts/diag/build_variants.sh) against the shipped
# libmmpt.so: the attention GPU tests on each variant, then scripts/bench_attn.py, two
# interleaved rounds.  Usage: bash scripts/attn_variants_ab.sh <tag> name1 [name2 ...]
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/attn_${TAG}
mkdir -p "$OUT"
for v in "$@"; do
  [ -n "${NOTEST:-}" ] && break  # diagnostic builds compute wrong results by design
  MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_$v.so timeout -k 10 300 \
      python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "attention or gqa" > "$OUT/pytest_$v.log" 2>&1 || { tail -20 "$OUT/pytest_$v.log"; exit 1; }
  echo "$v: $(tail -1 "$OUT/pytest_$v.log")"
done
for round in 1 2; do
  timeout -k 10 200 python -u scripts/bench_attn.py --iters 10 ${LONG:+--long} > "$OUT/base_$round.jsonl" 2> /dev/null
  for v in "$@"; do
    MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_$v.so timeout -k 10 200 \
        python -u scripts/bench_attn.py --iters 10 ${LONG:+--long} > "$OUT/${v}_$round.jsonl" 2> /dev/null
  done
done
python - "$OUT" base "$@" <<'PY'
import json, sys
d, names = sys.argv[1], sys.argv[2:]
best = {}
for n in names:
    for r in (1, 2):
        for rec in map(json.loads, open(f"{d}/{n}_{r}.jsonl")):
            for k in ("fwd_us", "bwd_us"):
                key = (n, rec["case"], k)
                best[key] = min(best.get(key, 1e30), rec[k])
for case in sorted({c for _, c, _ in best}):
    for k in ("fwd_us", "bwd_us"):
        b = best[("base", case, k)]
        print(f"{case:8s} {k:7s} " + " ".join(f"{n}={best[(n, case, k)]:8.1f} (x{b / best[(n, case, k)]:.3f})" for n in names))
PY
