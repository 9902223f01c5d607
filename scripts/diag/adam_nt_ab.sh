# AdamW kernel: normal vs non-temporal stores (lib/diag/libmmpt_adamnt.so), and its tests on both
set -e
OUT=gpurun_out/adamnt; mkdir -p $OUT
V=multimodal_llm_pretraining_amd/lib/diag/libmmpt_adamnt.so
MMPT_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_adam_overlap_gpu.py -m gpu -q -x \
    --timeout 200 --timeout-method thread -k "adam" > $OUT/tests_nt.log 2>&1 || { tail -20 $OUT/tests_nt.log; exit 1; }
tail -1 $OUT/tests_nt.log
for r in 1 2; do
  timeout -k 10 300 python scripts/diag/misc_bench.py | grep adam > $OUT/ship_$r.jsonl
  MMPT_LIB=$V timeout -k 10 300 python scripts/diag/misc_bench.py | grep adam > $OUT/nt_$r.jsonl
done
cat $OUT/*.jsonl
