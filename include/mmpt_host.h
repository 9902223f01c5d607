/*
 * mmpt_host.h — C-ABI of the host-side (CPU) part of the step: the optimizer that
 * runs when optimizer state is offloaded to host memory (libmmpt_host.so).
 *
 * Replaces DeepSpeed's CPU Adam (`DeepSpeedCPUAdam`, csrc/adam/cpu_adam_impl.cpp in
 * deepspeed 0.16.2) that the reference selects with
 * `zero_optimization.offload_optimizer.device = "cpu"` (src/train.py:182-194, driven by
 * TrainingConfig.offloading, experiments/config.py:68-74), and the FSDP
 * `CPUOffload(offload_params=True)` optimizer step (src/train.py:204-213).
 * Same conventions as mmpt.h: plain pointers, int status, mmpt_host_last_error().
 */
#ifndef MMPT_HOST_H_
#define MMPT_HOST_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMPT_HOST_ABI_VERSION 1

int mmpt_host_abi_version(void);
const char* mmpt_host_last_error(void);

/* Adam / AdamW over n fp32 elements in host memory, torch.optim single-tensor math
 * (the same operation order as mmpt_adam_step on the device):
 *   g' = g * grad_scale (grad_scale may be NULL → 1)
 *   AdamW: p *= 1 - lr*wd;   Adam: g' += wd*p
 *   m += (1-b1)(g' - m);  v = v*b2 + (1-b2) g'^2
 *   p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
 * and, if param_bf16 != NULL, writes bf16(p) (round-to-nearest-even) for the H2D copy.
 * `threads` ≤ 0 → all OpenMP threads. */
int mmpt_host_adam_step(int64_t n, float* param, const float* grad, float* exp_avg,
                        float* exp_avg_sq, uint16_t* param_bf16, float lr, float beta1,
                        float beta2, float eps, float weight_decay, int adamw, int64_t step,
                        const float* grad_scale, int threads);

/* Floats per vector of the Adam update clone this host runs (16: AVX-512, 8: AVX2). */
int mmpt_host_simd_width(void);

/* Σ x² over n host fp32 values (double accumulation), for clipping offloaded shards. */
int mmpt_host_sumsq(int64_t n, const float* x, double* out, int threads);

#ifdef __cplusplus
}
#endif
#endif
