# A/B of the big-tile threshold (MMPT_GEMM_BIG_MIN) at per-rank 32 / 64 (forced world-1 RCCL)
set -e
OUT=gpurun_out/bigmin_ab; mkdir -p $OUT
for r in 1 2; do
  for gb in 32 64; do
    for bm in 256 128; do
      n=gb${gb}_bm${bm}_$r
      MMPT_GEMM_BIG_MIN=$bm MMPT_FORCE_COLLECTIVES=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline \
          --no-yardstick --global-batch $gb --steps 6 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err \
          || { tail -20 $OUT/$n.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('clock_mhz'))" $OUT/$n.json $n
    done
  done
done
