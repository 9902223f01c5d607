# C5 and llava-pretrain bench lines on the final tree (after `gpu.sh <tag> scale`)
set -e
OUT=gpurun_out/final_lines; mkdir -p $OUT
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-yardstick --model clip-l14-336-pythia-2.8b \
    --sharding zero_3 --offload --micro-batch 64 --steps 3 --warmup 1 > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('c5', d['value'], d['ms_per_step'], d['clock']['median_mhz'])" $OUT/c5.json
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-yardstick --model llava-pretrain \
    --steps 3 --warmup 1 > $OUT/llava.json 2> $OUT/llava.err || { tail -20 $OUT/llava.err; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('llava', d['value'], d['ms_per_step'], d['clock']['median_mhz'])" $OUT/llava.json
