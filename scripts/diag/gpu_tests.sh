#!/bin/bash
# Run selected -m gpu test files on the GPU box (each under its own time limit), then
# optional bench lines.  Usage: bash scripts/diag/gpu_tests.sh <tag> "<test files>" ["<bench args>" ...]
set -euo pipefail
TAG=$1; FILES=$2; shift 2
OUT=gpurun_out/t_${TAG}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -v --timeout 200 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
i=0
for B in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $B > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" \
      || { tail -20 "$OUT/bench_$i.err"; exit 1; }
  cat "$OUT/bench_$i.json"
done
