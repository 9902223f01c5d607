set -euo pipefail
mkdir -p gpurun_out/combo1
timeout -k 10 600 python -u -m pytest tests/test_rccl_gpu.py -m gpu -x -v -s --timeout 500 --timeout-method thread > gpurun_out/combo1/rccl.log 2>&1 || { tail -30 gpurun_out/combo1/rccl.log; exit 1; }
grep -E "passed|failed" gpurun_out/combo1/rccl.log | tail -2
bash scripts/gpu_attn_ab.sh ds4 MMPT_ATTN_DS=0
