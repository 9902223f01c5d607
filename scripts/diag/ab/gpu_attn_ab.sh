#!/bin/bash
# Attention change check on one box: the attention / GQA kernel tests, the attention
# microbench with the shipped default and with an environment switch off (A/B), a
# rocprofv3 kernel-trace of the microbench, then the default bench line.
# Usage: bash scripts/gpu_attn_ab.sh <tag> <ENV=VALUE for the B arm>
set -euo pipefail
TAG=$1; BARM=$2
OUT=gpurun_out/attn_${TAG}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "attention or gqa" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u scripts/bench_attn.py > $OUT/attn_a.jsonl 2> $OUT/attn_a.err || { tail -20 $OUT/attn_a.err; exit 1; }
cat $OUT/attn_a.jsonl
timeout -k 10 300 env $BARM python -u scripts/bench_attn.py > $OUT/attn_b.jsonl 2> $OUT/attn_b.err || { tail -20 $OUT/attn_b.err; exit 1; }
cat $OUT/attn_b.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 scripts/bench_attn.py --iters 5 > $OUT/trace.jsonl 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
