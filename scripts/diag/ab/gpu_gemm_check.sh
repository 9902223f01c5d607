#!/bin/bash
# GEMM change check: element-wise GEMM tests, shape timings vs hipBLASLt, then the bench.
set -euo pipefail
TAG=$1
OUT=gpurun_out/gc_${TAG}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k gemm > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u scripts/diag/probe_hipblaslt.py > "$OUT/probe.log" 2>&1
grep mmpt "$OUT/probe.log"
timeout -k 10 300 python -u bench.py --steps 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['gemm_all_variants_tflops'])"
