#!/bin/bash
# D = 256 dK/dV: wave-pair kernel vs the ring kernel — attention tests, microbench A/B, trace.
set -euo pipefail
OUT=gpurun_out/pair_${1:-a}; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "attention or gqa" -x -v --timeout 120 \
    --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
MMPT_ATTN_PAIR=1 timeout -k 10 180 python -u scripts/bench_attn.py > "$OUT/pair.jsonl"
MMPT_ATTN_PAIR=0 timeout -k 10 180 python -u scripts/bench_attn.py > "$OUT/ring.jsonl"
MMPT_ATTN_PAIR=1 timeout -k 10 180 python -u scripts/bench_attn.py > "$OUT/pair2.jsonl"
cat "$OUT"/*.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 scripts/bench_attn.py --iters 5 > "$OUT/trace.log" 2>&1
python3 - "$OUT/trace/run_kernel_stats.csv" <<'PY'
import csv, sys, glob
f = sys.argv[1]
if not glob.glob(f): f = glob.glob(f.rsplit('/', 1)[0] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("mmpt::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    print(f"{n:52s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
