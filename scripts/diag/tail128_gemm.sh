set -e
OUT=gpurun_out/tail128g; mkdir -p $OUT
S=dense_fwd,fc2_fwd_resid,qkv_dxt,dense_dxt,fc1_dxt
for r in 1 2; do for t in 0 1; do
  MMPT_GEMM_TAIL128=$t timeout -k 10 120 python scripts/bench_gemm.py --no-ref --bias --tokens 32784 --iters 50 --only $S > $OUT/t${t}_$r.jsonl
done; done
