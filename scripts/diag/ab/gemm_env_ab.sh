#!/bin/bash
# A/B of one environment knob on the shipped library: shape timings with and without it.
# Usage: bash scripts/gemm_env_ab.sh <tag> "<shape,list>" "VAR=value"
set -euo pipefail
TAG=$1; ONLY=$2; ENVSET=$3
OUT=gpurun_out/env_${TAG}
mkdir -p "$OUT"
ARGS="--tokens 180992 --iters 5 --no-ref --only $ONLY"
for round in 1 2; do
  timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/base_$round.jsonl" 2> /dev/null
  env $ENVSET timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/var_$round.jsonl" 2> /dev/null
done
python - "$OUT" <<'PY'
import json, sys
d = sys.argv[1]
best = {}
for n in ("base", "var"):
    for r in (1, 2):
        for rec in map(json.loads, open(f"{d}/{n}_{r}.jsonl")):
            k = (n, rec["shape"])
            best[k] = min(best.get(k, 1e30), rec["mmpt_us"])
for s in sorted({s for _, s in best}):
    print(f"{s:18s} base {best[('base', s)]:9.1f} us   var {best[('var', s)]:9.1f} us   x{best[('base', s)] / best[('var', s)]:.3f}")
PY
