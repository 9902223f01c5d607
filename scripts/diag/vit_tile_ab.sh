# ViT-B/16's short-K GEMMs (K = 768 / 3072 at 50,432 tokens) on 256^2 (gemm4p) vs 128^2 tiles
set -e
OUT=gpurun_out/vit_tile; mkdir -p $OUT
S=vit_qkv_fwd,vit_o_fwd,vit_fc1_fwd_big,vit_fc2_fwd,vit_fc2_dx,vit_fc1_dx,vit_qkv_dx
for r in 1 2; do
  timeout -k 10 200 python scripts/bench_gemm.py --no-ref --bias --iters 20 --only $S > $OUT/t256_$r.jsonl
  MMPT_GEMM_TILE=128 timeout -k 10 200 python scripts/bench_gemm.py --no-ref --bias --iters 20 --only $S > $OUT/t128_$r.jsonl
done
