# weight-gradient tail split: GEMM tests, then C5's Pythia-2.8B weight gradients with it off / on
set -e
OUT=gpurun_out/wtail; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -k "gemm" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
S=p28_fc1_dw,p28_fc2_dw,p28_qkv_dw,p28_qkv_dw_cs,p28_dense_dw,lm_head_dw,fc1_dw,qkv_dw
for r in 1 2; do for w in 0 1; do
  MMPT_GEMM_WTAIL=$w timeout -k 10 200 python scripts/bench_gemm.py --no-ref --iters 10 --tokens 69568 --only $S > $OUT/w${w}_$r.jsonl
done; done
