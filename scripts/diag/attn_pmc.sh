#!/bin/bash
# PMC passes over the attention microbench (one counter group per pass).
set -euo pipefail
TAG=${1:-attn}
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
CMD="python3 scripts/bench_attn.py --iters 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
    --kernel-include-regex attn -f csv -d "$OUT/sq" -o run -- $CMD > "$OUT/sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM \
    --kernel-include-regex attn -f csv -d "$OUT/lds" -o run -- $CMD > "$OUT/lds.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT \
    --kernel-include-regex attn -f csv -d "$OUT/tcc" -o run -- $CMD > "$OUT/tcc.log" 2>&1
python3 scripts/pmc_summary.py $(find "$OUT" -name "*counter_collection.csv") > "$OUT/summary.txt"
echo done
