# forward tail split generalised (+ the erf-GELU tail epilogue): GEMM tests, then the fc1 / qkv
# forward GEMMs at the bench's 180,992 and the 8-GPU work's 22,624 tokens with it off / on
set -e
OUT=gpurun_out/tailgelu; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -k "gemm" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
S=fc1_fwd_gelu,qkv_fwd,dense_fwd,fc2_fwd_resid
for T in 180992 22624; do for r in 1 2; do for t in 0 1; do
  MMPT_GEMM_TAIL=$t timeout -k 10 200 python scripts/bench_gemm.py --no-ref --bias --iters 20 --tokens $T --only $S > $OUT/T${T}_t${t}_$r.jsonl
done; done; done
