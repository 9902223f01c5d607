#!/bin/bash
# 256x256 persistent vs 128x128 (2 workgroups per CU) kernel on the bench shapes
set -euo pipefail
O=gpurun_out/tile_ab; mkdir -p $O
A="--tokens 180992 --iters 5 --no-ref --bias --only ${ONLY:-qkv_fwd,dense_fwd,fc1_fwd_gelu,fc1_fwd_plain,fc2_fwd_resid,fc2_dx_dgelu,lm_head_fwd}"
for t in 256 128; do
  MMPT_GEMM_TILE=$t timeout -k 10 240 python -u scripts/bench_gemm.py $A > $O/t$t.jsonl 2> $O/t$t.err
  python -c "import sys,json; print('$t', ' '.join(f\"{r['shape']}={r['mmpt_us']}/{r['mmpt_tflops']}\" for r in map(json.loads, open('$O/t$t.jsonl'))))"
done
