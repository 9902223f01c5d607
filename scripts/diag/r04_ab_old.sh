#!/bin/bash
# Same-box A/B of the default bench line: the current library vs the one built from the
# pre-attention-work commit 76dbe3e (lib/diag/libmmpt_old.so), alternated.
set -euo pipefail
OUT=gpurun_out/r04_abold; mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$OUT/new_1.json" 2> "$OUT/new_1.err"
MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_old.so timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$OUT/old_1.json" 2> "$OUT/old_1.err"
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$OUT/new_2.json" 2> "$OUT/new_2.err"
MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_old.so timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$OUT/old_2.json" 2> "$OUT/old_2.err"
echo ab done
