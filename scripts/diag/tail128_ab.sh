# gemm tests, then A/B of the 128-row tail (MMPT_GEMM_TAIL128) on the C2 shape (T = 16 x 2049)
set -e
OUT=gpurun_out/tail128; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -k "gemm" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for t in 0 1; do
    n=c2_t${t}_$r
    MMPT_GEMM_TAIL128=$t MMPT_FORCE_COLLECTIVES=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline \
        --no-yardstick --model pythia-1b --sharding zero_1 --micro-batch 16 --global-batch 256 \
        --steps 3 --warmup 1 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], (d.get('clock') or {}).get('median_mhz'))" $OUT/$n.json $n
  done
done
