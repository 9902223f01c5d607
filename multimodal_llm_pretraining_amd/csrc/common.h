// Shared device helpers for the mmpt HIP library (gfx950 / CDNA4 only).
//
// Numerics follow torch.autocast(bfloat16) as used by the reference's HF
// Trainer with `bf16=True` (src/train.py:113): bf16 GEMM operands, fp32
// accumulation, fp32 LayerNorm / softmax / cross-entropy, fp32 master weights.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mmpt.h"

typedef uint16_t bf16_t;
typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace mmpt {

// ---- bf16 <-> f32 -------------------------------------------------------
__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// Round-to-nearest-even; a plain cast lowers to v_cvt_pk_bf16_f32 on gfx950
// (keeps NaN a NaN, MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

// ---- wave (64-lane) reductions -----------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- erf-GELU (tf:activations.py GELUActivation, approximate="none") ----
__device__ __forceinline__ float gelu_f(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

}  // namespace mmpt

// ---- error plumbing shared by every C-ABI entry point -------------------
namespace mmpt {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
}  // namespace mmpt

#define MMPT_REQUIRE(cond, ...)                 \
  do {                                          \
    if (!(cond)) {                              \
      ::mmpt::set_error(__VA_ARGS__);           \
      return MMPT_ERR_ARG;                      \
    }                                           \
  } while (0)
