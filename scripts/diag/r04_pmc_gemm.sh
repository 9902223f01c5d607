#!/bin/bash
# LDS activity per MFMA, gemm4p vs gemm256, on the 8192^3 yardstick and the
# qkv forward shape (one counter group per rocprofv3 pass, gfx950 slot limits), then the
# L2->fabric bytes of the bench line's dominant kernel (FETCH_SIZE / WRITE_SIZE passes over
# the default bench command, for profiles/pmc_traffic.json).
set -euo pipefail
TAG=${1:-a}
OUT=gpurun_out/pmc_r04_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for g4 in 0 1; do
  CMD="python3 scripts/bench_gemm.py --no-ref --iters 3 --bias --tokens 180992 --only sq8192,qkv_fwd,fc1_fwd_gelu"
  MMPT_GEMM_4P=$g4 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT \
      --kernel-include-regex gemm -f csv -d "$OUT/lds_g4p$g4" -o run -- $CMD > "$OUT/lds_g4p$g4.log" 2>&1
done
python3 scripts/pmc_summary.py $(find "$OUT" -name "*counter_collection.csv") > "$OUT/summary.txt" || true
echo pmc gemm done
