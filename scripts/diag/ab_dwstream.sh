set -euo pipefail
mkdir -p gpurun_out/ab
MMPT_DW_STREAM=0 timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline --no-probe > gpurun_out/ab/off.json 2>gpurun_out/ab/off.err
MMPT_DW_STREAM=1 timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline --no-probe > gpurun_out/ab/on.json 2>gpurun_out/ab/on.err
MMPT_DW_STREAM=1 timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline > gpurun_out/ab/on_probe.json 2>gpurun_out/ab/on_probe.err
for f in off on on_probe; do python -c "import json;d=json.load(open('gpurun_out/ab/$f.json'));print('$f',d['value'],d['ms_per_step'],d['max_memory_reserved_gb'])"; done
