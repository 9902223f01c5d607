# C5's weight-gradient GEMMs (Pythia-2.8B, T = 69,568) at forced K-split counts vs the planner
set -e
OUT=gpurun_out/p28dw; mkdir -p $OUT
S=p28_fc1_dw,p28_fc2_dw,p28_qkv_dw,p28_dense_dw
timeout -k 10 200 python scripts/bench_gemm.py --no-ref --iters 10 --tokens 69568 --only $S > $OUT/plan.jsonl
for sp in 1 2 3 4 5 6 8; do
  MMPT_GEMM_SPLITS=$sp timeout -k 10 200 python scripts/bench_gemm.py --no-ref --iters 10 --tokens 69568 --only $S > $OUT/sp$sp.jsonl
done
