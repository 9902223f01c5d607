set -euo pipefail
OUT=gpurun_out/r3a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_fullsize_gpu.py tests/test_parity_gpu.py -m gpu -x -v -s --timeout 400 --timeout-method thread > $OUT/fullsize.log 2>&1 || { tail -40 $OUT/fullsize.log; exit 1; }
tail -3 $OUT/fullsize.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
