#!/bin/bash
# GPU-box check (run via gpurun from the repo root): the -m gpu suite, smoke(), then the
# default bench line (with cpu_baseline).  Each GPU step has its own time limit; steps
# are chained so the first failure ends the call.
# Usage: bash scripts/gpu_check.sh <tag> [pytest -k expr]
set -euo pipefail
TAG=${1:-check}
K=${2:-}
OUT=gpurun_out/check_${TAG}
mkdir -p "$OUT"
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    "${KARG[@]}" > "$OUT/pytest.log" 2>&1
echo "pytest ok"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke ok"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
