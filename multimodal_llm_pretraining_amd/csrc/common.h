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

// Rotary pair (dims i, i + half) of one row: q·cos + rotate_half(q)·sin, or its transpose
// (the backward).  One fused multiply-add per output with the other product rounded first —
// written out so every kernel that rotates (rope8 / rope, the attention backward's dQ / dK
// epilogues) rounds identically, whatever contraction hipcc would otherwise pick.
__device__ __forceinline__ void rope_rot(float x1, float x2, float c1, float c2, float s1, float s2,
                                         bool inverse, float& o1, float& o2) {
  if (!inverse) {
    o1 = __builtin_fmaf(x1, c1, -(x2 * s1));
    o2 = __builtin_fmaf(x2, c2, x1 * s2);
  } else {
    o1 = __builtin_fmaf(x1, c1, x2 * s2);
    o2 = __builtin_fmaf(x2, c2, -(x1 * s1));
  }
}

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
// Φ(x) via erfc(z) = t·exp(-z² + P(t)), t = 1/(1 + z/2) (Numerical Recipes "erfcc",
// fractional error < 1.2e-7 everywhere): ~16 VALU incl. one rcp and one exp, no
// branches — vs the library erff's two divergent polynomial paths.  Checked on every
// finite bf16 input |x| < 20: GELU rounded to bf16 is bitwise equal to the exact
// erf-GELU rounded to bf16 (max fp32 rel. error 1e-5, dGELU abs. error 2e-7).
__device__ __forceinline__ float erfc_half_phi(float ax, float* e_half_x2) {
  // returns erfc(|x|/sqrt2); *e_half_x2 = exp(-x^2/2)
  const float z = ax * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.5f * z);
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float e = __expf(-z * z);  // = exp(-x^2/2)
  *e_half_x2 = e;
  return t * e * __expf(p);
}
__device__ __forceinline__ float phi_f(float x, float* e_half_x2) {
  const float r = erfc_half_phi(fabsf(x), e_half_x2);
  return x >= 0.f ? 1.0f - 0.5f * r : 0.5f * r;
}
__device__ __forceinline__ float gelu_f(float x) {
  float e;
  return x * phi_f(x, &e);
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  float e;
  const float cdf = phi_f(x, &e);
  return cdf + x * (0.3989422804014327f * e);
}

// ---- quick-GELU (tf:activations.py QuickGELUActivation: x * sigmoid(1.702 x), CLIP's
// hidden_act) with the bf16 roundings autocast applies between its three ops:
// t = bf16(1.702 x), s = bf16(sigmoid(t)), y = bf16(x s).
__device__ __forceinline__ float qgelu_sig(float x) {
  const float t = round_bf(1.702f * x);
  return round_bf(__builtin_amdgcn_rcpf(1.0f + __expf(-t)));
}
__device__ __forceinline__ float qgelu_f(float x) { return x * qgelu_sig(x); }
// d/dx through autograd's bf16 graph: mul -> g·s and (g·x) -> sigmoid_backward ->
// ·1.702, the two input-gradient contributions summed in bf16.  g is the bf16 grad of y.
// (s = qgelu_sig(x) given: the gemm4p epilogue takes it from a table)
__device__ __forceinline__ float dqgelu_s(float g, float x, float s) {
  const float a = round_bf(g * s);
  const float gs = round_bf(g * x);
  const float gt = round_bf(gs * (1.0f - s) * s);
  return round_bf(a + round_bf(gt * 1.702f));
}
__device__ __forceinline__ float dqgelu_f(float g, float x) { return dqgelu_s(g, x, qgelu_sig(x)); }

// ---- LDS-DMA ---------------------------------------------------------------
// One LDS-DMA piece (global_load_lds_dwordx4: 64 lanes x 16 B to the wave-uniform LDS
// address `lds`).  Issued from inline asm (cdna_hip_programming.md §5.7 recipe, M0
// written and restored in the same statement) so hipcc does not see a pending LDS
// write: with the builtin it drains every DMA in flight (vmcnt(0)) before each
// ds_read_b64_tr_b16 it cannot disambiguate.  Completion is counted by the kernels'
// own s_waitcnt vmcnt(N).
__device__ __forceinline__ void glds16(const void* gsrc, char* lds) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)LDS_PTR(char, lds));
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(dst)
      : "memory");
}

// LDS byte address of an LDS pointer (wave-uniform)
__device__ __forceinline__ uint32_t lds_addr(const char* lds) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(char, lds));
}
// glds16 in the instruction's SADDR form: global address = the wave-uniform base `sbase` (an
// SGPR pair) + the per-lane 32-bit byte offset `voff` — no per-lane 64-bit address math — into
// the wave-uniform LDS byte address `m0v` (+ 16 B per lane).  m0 is neither saved nor restored:
// it is a reserved register hipcc does not allocate, and nothing else in these kernels reads it
// (gfx9 DS instructions take no m0; the only m0 writes in the disassembly are these helpers').
__device__ __forceinline__ void glds16_so(const void* sbase, uint32_t voff, uint32_t m0v) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :
               : "v"(voff), "s"(sbase), "s"(m0v)
               : "memory");
}

}  // namespace mmpt

// ---- error plumbing shared by every C-ABI entry point -------------------
namespace mmpt {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
int* gemm_switch(const char* name, int* prev);  // gemm.hip: mmpt_set_switch's GEMM slots
int* misc_switch(const char* name, int* prev);  // misc.hip: MMPT_CE_REG
}  // namespace mmpt

#define MMPT_REQUIRE(cond, ...)                 \
  do {                                          \
    if (!(cond)) {                              \
      ::mmpt::set_error(__VA_ARGS__);           \
      return MMPT_ERR_ARG;                      \
    }                                           \
  } while (0)
