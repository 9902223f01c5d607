#!/bin/bash
# dGELU output rounding streamlined (one v_cvt_pk per product pair): GEMM kernel tests, then
# the dGELU shapes against the previous library (lib/diag/libmmpt_prev.so), alternating.
set -euo pipefail
OUT=gpurun_out/r04_dg_${1:-a}; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or gelu" -m gpu -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
ARGS="--tokens 180992 --iters 10 --no-ref --bias --only fc2_dx_dgelu_cs,fc1_fwd_gelu,qkv_fwd"
for r in 1 2; do
  MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_prev.so timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/p$r.jsonl" 2> "$OUT/p.err"
  timeout -k 10 200 python -u scripts/bench_gemm.py $ARGS > "$OUT/n$r.jsonl" 2> "$OUT/n.err"
done
python3 - "$OUT" <<'PY'
import json, sys
d = sys.argv[1]
names = ["p1", "n1", "p2", "n2"]
runs = [{r["shape"]: r for r in map(json.loads, open(f"{d}/{n}.jsonl"))} for n in names]
print(f"{'shape':18s} " + " ".join(f"{n:>18s}" for n in names) + "  (us, TF/s)")
for k in runs[0]:
    print(f"{k:18s} " + " ".join(f"{r[k]['mmpt_us']:9.1f} {r[k]['mmpt_tflops']:7.1f}" for r in runs))
PY
