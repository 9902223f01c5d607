#!/bin/bash
# One GPU-box profiling session for the headline bench (run via gpurun from the repo root):
#   1. kernel-trace + stats of `bench.py` (per-kernel average durations),
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE — they cannot share a pass on gfx950)
#      restricted to the GEMM kernels, for HBM bytes per launch.
# Every GPU step has its own time limit and the steps are chained with &&.
# Usage: bash scripts/diag/gpu_profile.sh <tag> [extra bench args]
set -euo pipefail
TAG=${1:-r01}
shift || true
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-yardstick $*"

timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run \
    -- python3 bench.py $BENCH_ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm -f csv \
    -d "$OUT/fetch" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-yardstick \
    > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gemm -f csv \
    -d "$OUT/write" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-yardstick \
    > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"
echo "profile ${TAG} done"
