# dQ-from-dS kernel: K^T ring depth variants and component diagnostics (lib/diag/libmmpt_*.so)
# under the attention trace (diagnostic builds give wrong results: timing only)
set -e
bash scripts/diag/attn_trace.sh ship > gpurun_out/kd_ship.txt
for v in kd2 kd5 dqd1 dqd2 dqd3 dqd4; do
  MMPT_LIB=multimodal_llm_pretraining_amd/lib/diag/libmmpt_$v.so bash scripts/diag/attn_trace.sh $v > gpurun_out/kd_$v.txt
done
