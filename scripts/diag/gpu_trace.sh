#!/bin/bash
# Kernel tests + default bench + a rocprofv3 kernel-trace of the bench (per-kernel
# averages -> scripts/trace_summary.py).  Usage: bash scripts/diag/gpu_trace.sh <tag> [pytest -k expr]
set -euo pipefail
TAG=$1; K=${2:-gemm}
OUT=gpurun_out/tr_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --steps 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
echo traced
