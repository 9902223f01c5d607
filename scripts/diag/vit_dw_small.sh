# ViT qkv / fc weight gradients at 6,304 tokens (per-rank 32): the planner's 128^2 split vs 256^2
set -e
OUT=gpurun_out/vitdw; mkdir -p $OUT
S=vit_qkv_dw,vit_qkv_dw_cs,vit_fc1_dw
for r in 1 2; do
  timeout -k 10 200 python scripts/bench_gemm.py --no-ref --iters 20 --vit-tokens 6304 --only $S > $OUT/plan_$r.jsonl
  for sp in 4 6; do
    MMPT_GEMM_SPLITS=$sp timeout -k 10 200 python scripts/bench_gemm.py --no-ref --iters 20 --vit-tokens 6304 --only $S > $OUT/sp${sp}_$r.jsonl
  done
done
