set -euo pipefail
OUT=gpurun_out/r3b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "segments or staged or non_finite or gelu or embed" > $OUT/k.log 2>&1 || { tail -40 $OUT/k.log; exit 1; }
tail -3 $OUT/k.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench_staged.json 2> $OUT/bench_staged.err || { tail -20 $OUT/bench_staged.err; exit 1; }
cat $OUT/bench_staged.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline --resident-inputs > $OUT/bench_resident.json 2> $OUT/bench_resident.err || { tail -20 $OUT/bench_resident.err; exit 1; }
cat $OUT/bench_resident.json
