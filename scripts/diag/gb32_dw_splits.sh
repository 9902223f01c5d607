# weight-gradient GEMMs at the 8-GPU work's 22,624 tokens: planner vs forced K-split counts
set -e
OUT=gpurun_out/gb32dw; mkdir -p $OUT
S=qkv_dw,qkv_dw_cs,dense_dw,vit_qkv_dw_cs,vit_fc1_dw
for r in 1 2; do for sp in 0 1 2 3 4 6; do
  if [ $sp = 0 ]; then E=""; else E="MMPT_GEMM_SPLITS=$sp"; fi
  env $E timeout -k 10 200 python scripts/bench_gemm.py --no-ref --iters 20 --tokens 22624 --vit-tokens 6304 --only $S > $OUT/sp${sp}_$r.jsonl
done; done
