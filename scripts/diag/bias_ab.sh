# forward (bias) vs input-gradient (no bias) GEMMs of one shape: does the bias cost?
set -e
OUT=gpurun_out/bias_ab; mkdir -p $OUT
S=dense_fwd,dense_dxt,qkv_fwd,fc2_fwd_plain,fc1_dxt
for r in 1 2; do
  timeout -k 10 120 python scripts/bench_gemm.py --no-ref --iters 30 --only $S > $OUT/nobias_$r.jsonl
  timeout -k 10 120 python scripts/bench_gemm.py --no-ref --iters 30 --bias --only $S > $OUT/bias_$r.jsonl
done
