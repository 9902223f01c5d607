# weight-gradient tail split on / off on one box: default bench line and C5
set -e
OUT=gpurun_out/wtail_bench; mkdir -p $OUT
for w in 0 1 0 1; do
  n=c3_w$w_$RANDOM
  MMPT_GEMM_WTAIL=$w timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-yardstick --steps 6 --warmup 2 \
      > $OUT/c3_w${w}.json.tmp 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('c3 wtail', sys.argv[2], d['value'], d['ms_per_step'], d['clock']['median_mhz'])" $OUT/c3_w${w}.json.tmp $w
done
for w in 0 1; do
  MMPT_GEMM_WTAIL=$w timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-yardstick --model clip-l14-336-pythia-2.8b \
      --sharding zero_3 --offload --micro-batch 64 --steps 3 --warmup 1 > $OUT/c5_w$w.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('c5 wtail', sys.argv[2], d['value'], d['ms_per_step'], d['step_ms'], d['clock']['median_mhz'])" $OUT/c5_w$w.json $w
done
