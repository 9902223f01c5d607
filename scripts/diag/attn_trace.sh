#!/bin/bash
# Kernel-trace stats of the attention microbench (per-kernel average durations).
set -euo pipefail
TAG=${1:-attn}
OUT=gpurun_out/atr_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- python3 scripts/bench_attn.py --iters 5 > "$OUT/bench.log" 2>&1
python3 - "$OUT/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("mmpt::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    print(f"{n:48s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
