#!/bin/bash
# L2->fabric bytes per launch of the bench line's GEMM kernels (gemm4p now dominant):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over the default bench command
# (they cannot share a pass on gfx950), summarised by scripts/pmc_traffic.py.
set -euo pipefail
OUT=gpurun_out/traffic_r04
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm -f csv \
    -d "$OUT/fetch" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-yardstick \
    > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gemm -f csv \
    -d "$OUT/write" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-yardstick \
    > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"
echo traffic done
