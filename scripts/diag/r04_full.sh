#!/bin/bash
# Round-4 validation on one box: the whole -m gpu suite (verbose, to a file), smoke(), the
# default bench line, then a kernel-trace profile of the bench (no yardstick launches).
# Usage: bash scripts/diag/r04_full.sh <tag> [skip-tests]
set -euo pipefail
TAG=${1:-x}
OUT=gpurun_out/r04_${TAG}; mkdir -p "$OUT"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
      > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -2 "$OUT/gpu_tests.log"
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
cat "$OUT/bench_default.json"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run \
    -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-yardstick \
    > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || { tail -20 "$OUT/trace_bench.err"; exit 1; }
python3 scripts/diag/prof_vs_line.py "$OUT/trace_bench.json" "$OUT/trace/run_kernel_stats.csv" "$OUT/prof_check.json" > /dev/null
echo "r04 ${TAG} done"
