#!/bin/bash
# Full-size parity run on one box: test_fullsize_gpu + the full-size loss tests, deltas to
# gpurun_out/parity/parity_deltas.jsonl (tests/parity_record.py).
set -euo pipefail
OUT=gpurun_out/parity; mkdir -p $OUT
rm -f $OUT/parity_deltas.jsonl
timeout -k 10 1000 python -u -m pytest tests/test_fullsize_gpu.py "tests/test_parity_gpu.py::test_full_size_loss" -m gpu -v -s --timeout 500 --timeout-method thread > $OUT/fullsize.log 2>&1 || { grep -E "ok$|FAIL|passed|failed|Error" $OUT/fullsize.log | tail -40; exit 1; }
grep -E "passed|failed" $OUT/fullsize.log | tail -2
