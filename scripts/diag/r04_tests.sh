#!/bin/bash
# The whole -m gpu suite on one box (verbose, to a file), no -x: every failure is listed.
set -uo pipefail
TAG=${1:-x}
OUT=gpurun_out/r04_${TAG}; mkdir -p "$OUT"
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -25 "$OUT/gpu_tests.log" | grep -E "FAILED|ERROR|passed|failed" || true
exit $rc
