# gemm4p tile-walk group size (MMPT_GEMM_GROUP) at the bench shapes, alternating
set -e
OUT=gpurun_out/group_ab; mkdir -p $OUT
S=qkv_fwd,qkv_dxt,fc1_dxt,dense_fwd,fc1_fwd_gelu,fc2_dx_dgelu_cs,lm_head_fwd,fc1_dw,qkv_dw_cs
for r in 1 2; do for g in 0 2 4 8 16; do
  if [ $g = 0 ]; then E=""; else E="MMPT_GEMM_GROUP=$g"; fi
  env $E timeout -k 10 300 python scripts/bench_gemm.py --no-ref --bias --iters 10 --only $S > $OUT/g${g}_$r.jsonl
done; done
