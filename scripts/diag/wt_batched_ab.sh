# W^T refresh in one launch vs one per weight: tests, then per-rank 32 / 256 bench A/B
set -e
OUT=gpurun_out/wtb; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_adam_overlap_gpu.py tests/test_sharding_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -k "transpose or adam or zero or shard" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do for b in 0 1; do
  MMPT_WT_BATCHED=$b MMPT_FORCE_COLLECTIVES=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-yardstick \
      --global-batch 32 --steps 8 --warmup 2 > $OUT/gb32_b${b}_$r.json 2> $OUT/gb32.err || { tail -20 $OUT/gb32.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['clock']['median_mhz'])" $OUT/gb32_b${b}_$r.json
done; done
