set -e
O=gpurun_out/d4; mkdir -p $O
A="--tokens 180992 --iters 5 --no-ref --only qkv_fwd,fc1_fwd_gelu,fc1_fwd_plain,fc2_fwd_resid,fc2_fwd_plain,fc1_dx,fc2_dx_dgelu,qkv_dw,fc1_dw,lm_head_fwd"
timeout -k 10 240 python -u scripts/bench_gemm.py $A > $O/d0.jsonl 2> $O/d0.err
MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_d4.so timeout -k 10 240 python -u scripts/bench_gemm.py $A > $O/d4.jsonl 2> $O/d4.err
