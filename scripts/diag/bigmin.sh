set -e
S=vit_qkv_fwd,vit_o_fwd,vit_fc1_fwd_big,vit_fc2_fwd,vit_qkv_dx,vit_fc1_dx,vit_fc2_dx,vit_qkv_dw_cs
mkdir -p gpurun_out/bigmin
for V in 6304 12608; do
 timeout -k 10 120 python scripts/bench_gemm.py --no-ref --bias --vit-tokens $V --only $S > gpurun_out/bigmin/def_$V.jsonl
 MMPT_GEMM_BIG_MIN=32 timeout -k 10 120 python scripts/bench_gemm.py --no-ref --bias --vit-tokens $V --only $S > gpurun_out/bigmin/b32_$V.jsonl
done
