#!/bin/bash
# A/B of the persistent gemm256 staggered start (MMPT_GEMM_STAGGER = percent of the modelled
# quarter-tile delay) on the bench's activation-GEMM shapes.
set -euo pipefail
O=gpurun_out/stagger; mkdir -p $O
A="--tokens 180992 --iters 5 --no-ref --only ${ONLY:-qkv_fwd,fc1_fwd_gelu,fc1_fwd_plain,fc2_fwd_resid,fc1_dx,fc2_dx_dgelu,lm_head_fwd}"
for s in ${LEVELS:-0 100 200 0 100}; do
  MMPT_GEMM_STAGGER=$s timeout -k 10 240 python -u scripts/bench_gemm.py $A > $O/s$s.jsonl 2> $O/s$s.err
  cat $O/s$s.jsonl | python -c "import sys,json; print('$s', ' '.join(f\"{r['shape']}={r['mmpt_us']}\" for r in map(json.loads, sys.stdin)))"
done
