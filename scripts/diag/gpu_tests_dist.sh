#!/bin/bash
# Distributed / sharding / offload GPU tests (two gloo ranks on cuda:0, forced RCCL at world 1).
set -euo pipefail
OUT=gpurun_out/dist_${1:-x}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_memory_gpu.py tests/test_distributed_gpu.py tests/test_sharding_gpu.py tests/test_dp_oracle_gpu.py tests/test_rccl_gpu.py tests/test_dropin_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -3
