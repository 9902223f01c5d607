#!/bin/bash
# one-GPU preview of the strong-scaling curve + BASELINE C2 / C4 lines.
#   * ViT-B/16 + Pythia-1B at global batch 128 / 64 / 32 (the per-rank work at N = 2 / 4 / 8 of
#     the 256-sample headline batch) for ddp, zero_2 and zero_3, every collective of the mode
#     executed on a world-1 RCCL group (MMPT_FORCE_COLLECTIVES=1) -> comm.busy_ms per step
#   * C2: pythia-1b ZeRO-1, micro-batch 16 (GA 64 at the model class's batch 1024)
#   * C4 per GPU: pythia-1b ZeRO-3 + activation checkpointing, 128 samples (1024 / 8 ranks)
# Usage: bash scripts/diag/r04_scale.sh <tag>
set -euo pipefail
TAG=${1:-a}
OUT=gpurun_out/r04_scale_${TAG}; mkdir -p "$OUT"
run() {  # <name> <timeout> <bench args...>
  local name=$1 to=$2; shift 2
  MMPT_FORCE_COLLECTIVES=1 timeout -k 10 "$to" python -u bench.py --no-cpu-baseline --no-yardstick "$@" \
      > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d.get('comm') or {}; print(sys.argv[2], d['value'], d['ms_per_step'], c.get('busy_ms'), c.get('exposed_ms'))" "$OUT/$name.json" "$name"
}
for gb in 128 64 32; do
  for mode in ddp zero_2 zero_3; do
    sh=$mode; [ "$mode" = ddp ] && sh=""
    run "vitp1b_gb${gb}_${mode}" 300 --global-batch "$gb" ${sh:+--sharding $sh} --steps 4 --warmup 2
  done
done
run c2_pythia1b_zero1_mbs16 600 --model pythia-1b --sharding zero_1 --micro-batch 16 --steps 2 --warmup 1
run c4_pythia1b_zero3_ac_gb128 400 --model pythia-1b --sharding zero_3 --activation-checkpointing --global-batch 128 --steps 3 --warmup 1
echo "r04 scale ${TAG} done"
