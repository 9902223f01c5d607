// K1: bf16 MFMA GEMM with fused epilogues (replaces aten::addmm / mm launched by
// nn.Linear under autocast).
//
// Two kernels:
//   gemm4p_kernel: 256x256x64 tile, 256 threads = 4 waves of 128x128, 1 workgroup per CU,
//     persistent, 128 KiB LDS, one straight-line K-tile of 128 MFMA slots (see the comment
//     above it) — every big activation / weight-gradient GEMM (round 4; the 8-wave gemm256
//     kernel of rounds 1-3 was retired in round 5);
//   gemm128_kernel: 128x128x64, 256 threads = 4 waves (2x2, 64x64 per wave), 64 KiB
//     LDS, 2 per CU — small problems (ViT, projector) where 256^2 tiles cannot fill
//     256 CUs, and the big ones gemm4p does not take (mixed layouts, unaligned operands).
// MFMA v_mfma_f32_16x16x32_bf16.  Operands are staged HBM -> LDS with
// global_load_lds_dwordx4 (no VGPR round trip); a K tail is zero-filled by pointing
// the DMA source of out-of-range chunks at a zero page.
//
// LDS images (lane-linear for the DMA; swizzle on the SOURCE address, mirrored on
// the read — cdna_hip_programming.md rule 21):
//   ROWS_K operand: [R rows][64 k], 128-B rows, chunk' = chunk ^ (row & 7)
//       -> fragments by ds_read_b128 (conflict-free for the b128 lane groups);
//   K_ROWS operand: [64 k][R rows], 2R-byte rows, chunk' = chunk ^ s(k),
//       s(k) = 2*((k&3) | ((k>>3)&1)<<2) -> fragments by ds_read_b64_tr_b16
//       (hardware transpose; the 8 k-rows of a 32-lane half land on 8 distinct
//       32-B chunk pairs of the bank row: conflict-free).
// The MFMA is issued as D = Bfrag·Afrag so the accumulator holds C^T: lane l owns
// C[m = l&15][n = 4(l>>4) + i] -> 8-B (bf16) / 16-B (f32) vector stores.
//
// Split-K (weight gradients, K = tokens >> M, N): blockIdx.y selects a K range;
// partial fp32 tiles go to a workspace slab per split and a second kernel sums
// the slabs in fixed order (bitwise reproducible, no atomics), rounds to bf16
// (autocast grad dtype) and accumulates into the fp32 gradient.
#include <math.h>
#include <stdio.h>
#include <algorithm>
#include <cmath>
#include <type_traits>
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace mmpt {
namespace {

constexpr int BK = 64;

struct GemmParams {
  const bf16_t* A;
  const bf16_t* B;
  int M, N, K;
  long lda, ldb;
  void* C;
  long ldc;
  const bf16_t* bias;
  const bf16_t* aux;
  long ld_aux;
  void* C2;
  long ldc2;
  int tiles_m, tiles_n;
  int splits, kchunk;  // split-K: K range [s*kchunk, min(K, (s+1)*kchunk))
  float* slab;         // splits x M x N fp32 (split mode only)
  int wide;            // 16-B aligned rows everywhere: 8-column epilogue
  int group;           // tile rows walked together (coord_of; MMPT_GEMM_GROUP, default 8)
  int krev;            // gemm4p: odd tiles of a workgroup walk K last-to-first (MMPT_GEMM_KREV)
};

// ---- erf-GELU tables (the GELU / dGELU epilogues) ------------------------------------------
// The epilogue's GELU input is a bf16 value (the rounded pre-activation), so GELU and GELU'
// are functions of 16 bits.  For |x| in [2^-16, 32) — 21 binades x 128 mantissas x 2 signs =
// 5376 inputs — the tables hold bf16(GELU(x)) and fp32(GELU'(x)) computed on the host in
// double from erfc (no cancellation for x << 0), i.e. correctly rounded; below 2^-16 the
// two-term series (relative error < 2^-33) and above 32 the limits (x / -0, 1 / 0) are exact
// at these precisions.  32 KiB beside the 128-KiB staging area in LDS replace the ~25 VALU +
// 3 transcendental erfc evaluation per element with a 2-/4-byte LDS read.
constexpr int LUT_E0 = 127 - 16, LUT_NE = 21, LUT_N = 2 * LUT_NE * 128;
constexpr int LUT_BYTES = LUT_N * 2 + LUT_N * 4;  // bf16 GELU | fp32 GELU'
__device__ __attribute__((aligned(16))) char g_gelu_lut[LUT_BYTES];
// Round 5: the same two-part tables for the gemm4p quick-GELU and SwiGLU epilogues (same slots,
// same out-of-table fixup through the general code), correctly rounded from double on the host:
//   quick-GELU (CLIP): bf16(x · s(x)) | fp32 s(x), s(x) = bf16(sigmoid(bf16(1.702f · x)));
//   SiLU (Llama SwiGLU): bf16(silu(x)) | fp32 sigmoid(x).
__device__ __attribute__((aligned(16))) char g_qgelu_lut[LUT_BYTES];
__device__ __attribute__((aligned(16))) char g_silu_lut[LUT_BYTES];

// Branch-free table lookups for 8 values at once: the 8 slot computations, then the 8 LDS
// reads back to back, then the 8 selects.  (A per-element helper with early returns compiled
// to exec-masked branches with an lgkmcnt(0) wait after every single 2-byte LDS read: the
// LDS latency paid 128 times per row block.)  Slot of a bf16-valued x: the table index for
// |x| in [2^-16, 32); below that the two-term series, above (and inf / nan) the limits.
struct LutSlots {
  int idx[8];
  bool tab[8], tiny[8];
};
__device__ __forceinline__ LutSlots lut_slots8(const float* x) {
  LutSlots s;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t b = __float_as_uint(x[e]) >> 16;
    const int ei = (int)((b >> 7) & 0xff) - LUT_E0;
    const int k = (int)(((b >> 15) * LUT_NE + ei) * 128 + (b & 0x7f));
    s.tab[e] = (unsigned)ei < (unsigned)LUT_NE;
    s.tiny[e] = ei < 0;
    s.idx[e] = s.tab[e] ? k : 0;
  }
  return s;
}
__device__ __forceinline__ void gelu_lut8(const char* lut, const float* x, float* y) {
  const LutSlots s = lut_slots8(x);
  uint32_t t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = *(const bf16_t*)(lut + 2 * s.idx[e]);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    // |x| >= 32: x or -0 (copysign(max(x, 0), x): no branch), +inf -> +inf; -inf and nan ->
    // nan, as x * 0.5 * (1 + erf(x / sqrt 2)) gives them (the formula of the reference's
    // GPU GELU and of gelu_f; fmaxf alone would turn a nan into 0)
    const float lim = __builtin_copysignf(fmaxf(x[e], 0.f), x[e]);
    const float big = x[e] >= -3.4028235e38f ? lim : __builtin_nanf("");
    const float out = s.tiny[e] ? x[e] * fmaf(0.3989422804014327f, x[e], 0.5f) : big;
    y[e] = s.tab[e] ? bf2f((bf16_t)t[e]) : out;
  }
}
__device__ __forceinline__ void gelu_grad_lut8(const char* lut, const float* x, float* y) {
  const LutSlots s = lut_slots8(x);
  float t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = *(const float*)(lut + 2 * LUT_N + 4 * s.idx[e]);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    // |x| >= 32: 1 or 0; +-inf / nan: nan (cdf + x * pdf has inf * 0, as in gelu_grad_f)
    const float big = __builtin_fabsf(x[e]) <= 3.4028235e38f ? (float)(x[e] > 0.f)
                                                             : __builtin_nanf("");
    const float out = s.tiny[e] ? fmaf(0.7978845608028654f, x[e], 0.5f) : big;
    y[e] = s.tab[e] ? t[e] : out;
  }
}
// single-value forms (4-column edge epilogue)
__device__ __forceinline__ float gelu_lut(const char* lut, float x) {
  float xs[8] = {x, x, x, x, x, x, x, x}, y[8];
  gelu_lut8(lut, xs, y);
  return y[0];
}
__device__ __forceinline__ float gelu_grad_lut(const char* lut, float x) {
  float xs[8] = {x, x, x, x, x, x, x, x}, y[8];
  gelu_grad_lut8(lut, xs, y);
  return y[0];
}

// ---- packed fast-row epilogues (whole tiles) ------------------------------------------------
// The epilogue is VALU-bound (all 8 waves at once, MFMA idle): ~250 instructions per 8-column
// row for GELU through the generic per-element code.  These forms work on bf16 PAIRS: the
// table slot of two bf16 values comes from 16-bit packed integer ops on the packed word the
// rounding already produced (|x| & 0x7fff - E0·128 is the in-table offset, + 2688 for x < 0);
// a slot outside the table (|x| < 2^-16 or >= 32, or inf / nan) clamps into it and a
// wave-uniform fixup recomputes that row with the general code (rare: P ~ 1e-5 per value).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
constexpr unsigned short LUT_OFF0 = (unsigned short)(LUT_E0 << 7), LUT_HALF = LUT_NE * 128;
// in-table slots of the two bf16 values of `pk`; `bad` accumulates nonzero for any outside
__device__ __forceinline__ u16x2 lut_slots2(uint32_t pk, uint32_t& bad) {
  const u16x2 mag = __builtin_bit_cast(u16x2, pk & 0x7fff7fffu);
  const u16x2 d = mag - (u16x2){LUT_OFF0, LUT_OFF0};  // wraps high for |x| < 2^-16
  bad |= __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(d, (u16x2){LUT_HALF - 1, LUT_HALF - 1}));
  const u16x2 dc = __builtin_elementwise_min(d, (u16x2){LUT_HALF - 1, LUT_HALF - 1});
  const u16x2 neg = __builtin_bit_cast(u16x2, pk) >> (u16x2){15, 15};
  return neg * (u16x2){LUT_HALF, LUT_HALF} + dc;
}
__device__ __forceinline__ uint32_t pack_pair(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}
// GELU of 4 packed bf16 pairs -> 4 packed bf16 pairs (table values; `bad` as above)
__device__ __forceinline__ void gelu_pk8(const char* lut, const uint32_t* pre, uint32_t* act,
                                         uint32_t& bad) {
  u16x2 sl[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) sl[q] = lut_slots2(pre[q], bad);
  bf16_t t[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    t[2 * q] = *(const bf16_t*)(lut + 2 * (uint32_t)sl[q].x);
    t[2 * q + 1] = *(const bf16_t*)(lut + 2 * (uint32_t)sl[q].y);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) act[q] = (uint32_t)t[2 * q] | ((uint32_t)t[2 * q + 1] << 16);
}
// GELU'(x) (fp32) of 4 packed bf16 pairs of x
__device__ __forceinline__ void gelu_grad_pk8(const char* lut, const uint32_t* x, float* gd,
                                              uint32_t& bad) {
  u16x2 sl[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) sl[q] = lut_slots2(x[q], bad);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    gd[2 * q] = *(const float*)(lut + 2 * LUT_N + 4 * (uint32_t)sl[q].x);
    gd[2 * q + 1] = *(const float*)(lut + 2 * LUT_N + 4 * (uint32_t)sl[q].y);
  }
}

// The quick-GELU epilogues (CLIP) are their own instantiations: EPI_ = 7/8/9 runs the
// code of its base epilogue (1/2/6) with the activation chosen at compile time (a runtime
// switch inlined both activations and spilled the 2-waves/SIMD register budget).
// Internal epilogues: split-K fp32 slabs (EPI_SPLIT), and (round 5) the split-K form of
// F32_ACC_COLSUM (EPI_SPLIT_CS: slabs + per-split row sums of op(A), see csa()).
constexpr int EPI_SPLIT = 100, EPI_SPLIT_CS = 102;
template <int E>
constexpr int epi_base() {
  return E == MMPT_EPI_BF16_QGELU            ? MMPT_EPI_BF16_GELU
         : E == MMPT_EPI_BF16_DQGELU         ? MMPT_EPI_BF16_DGELU
         : E == MMPT_EPI_BF16_DQGELU_COLSUM  ? MMPT_EPI_BF16_DGELU_COLSUM
         : E == MMPT_EPI_F32_ACC_COLSUM      ? MMPT_EPI_F32_ACC
         : E == EPI_SPLIT_CS                 ? EPI_SPLIT
                                             : E;
}
// CSA: the weight-gradient GEMM also sums its A operand (dY) over K, row by row — the bias
// gradient, from the fragments the MFMAs already read (gemm4p only)
template <int E>
constexpr bool csa() {
  return E == MMPT_EPI_F32_ACC_COLSUM || E == EPI_SPLIT_CS;
}
template <int E>
constexpr bool epi_quick() {
  return E == MMPT_EPI_BF16_QGELU || E == MMPT_EPI_BF16_DQGELU ||
         E == MMPT_EPI_BF16_DQGELU_COLSUM;
}
template <bool QK>
__device__ __forceinline__ float act_f(float x) {
  if constexpr (QK) return qgelu_f(x);
  else return gelu_f(x);
}
// bf16(d act / d pre) applied to the bf16-rounded incoming gradient g
template <bool QK>
__device__ __forceinline__ float dact_f(float g, float x) {
  if constexpr (QK) return dqgelu_f(g, x);
  else return round_bf(g * gelu_grad_f(x));
}

// SwiGLU pieces with autocast's bf16 roundings (torch's CPU silu / silu_backward on bf16
// tensors compute in fp32 and round once): s = bf16(silu(g)), act = bf16(s * u).
__device__ __forceinline__ float silu_bf(float g) { return round_bf(g / (1.0f + __expf(-g))); }
// (dg, du) from the act gradient d and the forward's bf16 gate/up values
// (s = silu_bf(g), sig = sigmoid(g) given: the gemm4p epilogue takes them from a table)
__device__ __forceinline__ void dswiglu_s(float d, float g, float u, float s, float sig, float& dg,
                                          float& du) {
  du = round_bf(d * s);
  const float ds = round_bf(d * u);
  dg = round_bf(ds * sig * (1.0f + g * (1.0f - sig)));
}
__device__ __forceinline__ void dswiglu(float d, float g, float u, float& dg, float& du) {
  dswiglu_s(d, g, u, silu_bf(g), 1.0f / (1.0f + __expf(-g)), dg, du);
}
// blocked gate|up column of feature column n (128-column blocks; up = gate + 128)
__device__ __forceinline__ long swiglu_gcol(int n) { return (long)(n >> 7) * 256 + (n & 127); }

__device__ __forceinline__ int swz_kr(int kr) {
  return 2 * ((kr & 3) | (((kr >> 3) & 1) << 2));
}

// 16 zero bytes in global memory: the DMA source of every chunk past the K limit, so a
// K tail is zero-filled by the staging itself (no LDS writes, no extra barrier).
__device__ __attribute__((aligned(16))) bf16_t g_zero16[8];

// Branch-free per-lane choice between the operand chunk and the zero page: the
// opaque asm keeps hipcc from splitting the DMA into two divergent branches.
__device__ __forceinline__ const bf16_t* select_src(bool valid, const bf16_t* p) {
  uintptr_t a = valid ? (uintptr_t)p : (uintptr_t)g_zero16;
  asm volatile("" : "+v"(a));
  return (const bf16_t*)a;
}

// --- HBM -> LDS staging of an R-row operand image ---------------------------
// Issues NP 1-KiB DMA pieces (global_load_lds_dwordx4, 64 lanes x 16 B) starting at
// piece q0 of the image.  Rows past Rlim are clamped (their results are discarded);
// k >= klim reads the zero page.
template <int LAYOUT, int R, int NP, bool ASM>
__device__ __forceinline__ void stage_pieces(const bf16_t* __restrict__ src, long ld, int Rlim,
                                             int klim, int r0, int k0, char* img, int q0,
                                             int lane) {
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int q = q0 + i;
    const bf16_t* g;
    if constexpr (LAYOUT == MMPT_ROWS_K) {
      const int r = q * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (r & 7);
      const int gr = min(r0 + r, Rlim - 1);
      const int gk = k0 + lc * 8;
      g = select_src(gk < klim, src + (long)gr * ld + gk);
    } else {
      constexpr int CPR = R / 8;        // 16-B chunks per k-row
      constexpr int RPP = 64 / CPR;     // k-rows per piece
      const int kr = q * RPP + lane / CPR;
      const int lc = (lane % CPR) ^ swz_kr(kr);
      const int gk = k0 + kr;
      const int gr = min(r0 + lc * 8, Rlim - 8);
      g = select_src(gk < klim, src + (long)gk * ld + gr);
    }
    if constexpr (ASM)
      glds16(g, img + q * 1024);
    else
      __builtin_amdgcn_global_load_lds((const void*)g, LDS_PTR(void, img + q * 1024), 16, 0, 0);
  }
}

// whole R x 64 image, pieces split evenly over NW waves
template <int LAYOUT, int R, int NW>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ src, long ld, int Rlim, int klim,
                                      int r0, int k0, char* img, int wave, int lane) {
  constexpr int PIECES = R * BK * 2 / 1024;
  static_assert(PIECES % NW == 0, "pieces must split evenly over waves");
  stage_pieces<LAYOUT, R, PIECES / NW, false>(src, ld, Rlim, klim, r0, k0, img, wave * (PIECES / NW), lane);
}

// op[row = rbase + (lane&15)][k = kk*32 + 8*(lane>>4) + j], j = 0..7
template <int LAYOUT, int R>
__device__ __forceinline__ v8s frag(const char* img, int rbase, int kk, int lane) {
  if constexpr (LAYOUT == MMPT_ROWS_K) {
    const int r = rbase + (lane & 15);
    const int lc = kk * 4 + (lane >> 4);
    return *(const v8s*)(img + r * 128 + ((lc ^ (r & 7)) * 16));
  } else {
    constexpr int RB = R * 2;
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int col = rbase + 4 * p;
    const int lc = col >> 3, half = p & 1;
    const int kr = kk * 32 + 8 * g + q;
    const char* a = img + kr * RB + ((lc ^ swz_kr(kr)) * 16) + half * 8;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a + 4 * RB));
    return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

// c + w.x * v[2E] + w.y * v[2E + 1] (CSA row sums; w = bf16 (1, 1), or (0, 0)): one
// v_dot2c_f32_bf16.  (Pairs are taken with shufflevector: bit-casting elements of a bit-cast
// uint4 made hipcc sum the first pair four times.)
#ifndef MMPT_CSA_MODE
#define MMPT_CSA_MODE 0  // A/B builds only: 1 = shift / mask + two v_add_f32, 9 = no sums (wrong)
#endif
template <int E>
__device__ __forceinline__ float frag_pair_sum(v8s v, float c, uint32_t w) {
  typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
  typedef short v2s_ __attribute__((ext_vector_type(2)));
  const v2s_ pr = __builtin_shufflevector(v, v, 2 * E, 2 * E + 1);
  if constexpr (MMPT_CSA_MODE == 9) {
    return c;
  } else if constexpr (MMPT_CSA_MODE == 1) {
    const uint32_t d = __builtin_bit_cast(uint32_t, pr);
    if (w == 0u) return c;
    return (c + __builtin_bit_cast(float, d << 16)) + __builtin_bit_cast(float, d & 0xffff0000u);
  } else {
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(v2bf, pr), __builtin_bit_cast(v2bf, w),
                                           c, false);
  }
}

__device__ __forceinline__ void store_bf16x4(bf16_t* p, float a, float b, float c, float d) {
  uint2 v;
  v.x = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
  v.y = (uint32_t)f2bf(c) | ((uint32_t)f2bf(d) << 16);
  *(uint2*)p = v;
}
__device__ __forceinline__ void load_bf16x4(const bf16_t* p, float* o) {
  const uint2 v = *(const uint2*)p;
  o[0] = bf2f(v.x & 0xffff);
  o[1] = bf2f(v.x >> 16);
  o[2] = bf2f(v.y & 0xffff);
  o[3] = bf2f(v.y >> 16);
}

// the big-tile kernel evaluates the erf-GELU epilogues from the LDS tables (see LUT_E0)
#ifndef MMPT_GEMM_LUT
#define MMPT_GEMM_LUT 1  // 0: evaluate erfc per element (A/B builds only)
#endif
template <int EPI_>
constexpr bool gelu_uses_lut() {
  constexpr int E = epi_base<EPI_>();
  return MMPT_GEMM_LUT && !epi_quick<EPI_>() &&
         (E == MMPT_EPI_BF16_GELU || E == MMPT_EPI_BF16_DGELU || E == MMPT_EPI_BF16_DGELU_COLSUM);
}

template <int EPI_, bool LUT = false>  // LUT: erf-GELU from the LDS tables `lut`
__device__ __forceinline__ void epilogue4(const GemmParams& p, int m, int n, const float* v,
                                          const float* bias, int split, float* cs = nullptr,
                                          const char* lut = nullptr) {
  constexpr int EPI = epi_base<EPI_>();
  constexpr bool QK = epi_quick<EPI_>();
  if constexpr (EPI == MMPT_EPI_BF16) {
    store_bf16x4((bf16_t*)p.C + (long)m * p.ldc + n, v[0] + bias[0], v[1] + bias[1],
                 v[2] + bias[2], v[3] + bias[3]);
  } else if constexpr (EPI == MMPT_EPI_BF16_GELU) {
    float pre[4], act[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pre[e] = round_bf(v[e] + bias[e]);
      act[e] = LUT ? gelu_lut(lut, pre[e]) : act_f<QK>(pre[e]);
    }
    store_bf16x4((bf16_t*)p.C + (long)m * p.ldc + n, pre[0], pre[1], pre[2], pre[3]);
    store_bf16x4((bf16_t*)p.C2 + (long)m * p.ldc2 + n, act[0], act[1], act[2], act[3]);
  } else if constexpr (EPI == MMPT_EPI_BF16_DGELU || EPI == MMPT_EPI_BF16_DGELU_COLSUM) {
    float x[4], o[4];
    load_bf16x4(p.aux + (long)m * p.ld_aux + n, x);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = LUT ? round_bf(round_bf(v[e]) * gelu_grad_lut(lut, x[e]))
                                       : dact_f<QK>(round_bf(v[e]), x[e]);
    store_bf16x4((bf16_t*)p.C + (long)m * p.ldc + n, o[0], o[1], o[2], o[3]);
    if constexpr (EPI == MMPT_EPI_BF16_DGELU_COLSUM) {
#pragma unroll
      for (int e = 0; e < 4; ++e) cs[e] += o[e];
    }
  } else if constexpr (EPI == MMPT_EPI_F32_ACC || EPI == MMPT_EPI_F32_STORE) {
    float4* c = (float4*)((float*)p.C + (long)m * p.ldc + n);
    float4 o = make_float4(round_bf(v[0]), round_bf(v[1]), round_bf(v[2]), round_bf(v[3]));
    if constexpr (EPI == MMPT_EPI_F32_ACC) {
      const float4 old = *c;
      o.x += old.x;
      o.y += old.y;
      o.z += old.z;
      o.w += old.w;
    }
    *c = o;
  } else if constexpr (EPI == MMPT_EPI_BF16_DSWIGLU) {
    const long gc = swiglu_gcol(n);
    float g[4], u[4], dg[4], du[4];
    load_bf16x4(p.aux + (long)m * p.ld_aux + gc, g);
    load_bf16x4(p.aux + (long)m * p.ld_aux + gc + 128, u);
#pragma unroll
    for (int e = 0; e < 4; ++e) dswiglu(round_bf(v[e]), g[e], u[e], dg[e], du[e]);
    store_bf16x4((bf16_t*)p.C + (long)m * p.ldc + gc, dg[0], dg[1], dg[2], dg[3]);
    store_bf16x4((bf16_t*)p.C + (long)m * p.ldc + gc + 128, du[0], du[1], du[2], du[3]);
  } else if constexpr (EPI == MMPT_EPI_BF16_SWIGLU) {
    // gemm4p's fast epilogue only (it pairs the gate and up columns); never launched here
  } else if constexpr (EPI == MMPT_EPI_F32_RESID) {
    float r[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = round_bf(v[e] + bias[e]);
    if (p.aux != nullptr) {
      float x[4];
      load_bf16x4(p.aux + (long)m * p.ld_aux + n, x);
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = round_bf(r[e] + x[e]);
    }
    const float4 res = *(const float4*)((const float*)p.C2 + (long)m * p.ldc2 + n);
    *(float4*)((float*)p.C + (long)m * p.ldc + n) =
        make_float4(res.x + r[0], res.y + r[1], res.z + r[2], res.w + r[3]);
  } else {  // split-K partial: raw fp32 into this split's slab
    *(float4*)(p.slab + ((long)split * p.M + m) * p.N + n) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Column-sum partials (EPI_BF16_DGELU_COLSUM): sum a lane's NC column accumulators over
// the 16 lanes that hold the same columns (lane & 15 = row), then one lane stores them to
// partial row `prow` of C2 ([rows][N] fp32).  All lanes must call (shuffles).
template <int NC>
__device__ __forceinline__ void colsum_store(const GemmParams& p, float* cs, int prow, int n,
                                             int lane) {
#pragma unroll
  for (int e = 0; e < NC; ++e) {
    float v = cs[e];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    cs[e] = v;
  }
  if ((lane & 15) == 0 && n < p.N) {
    float* dst = (float*)p.C2 + (long)prow * p.N + n;
    if (NC == 8 && n + 8 <= p.N) {
      ((float4*)dst)[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
      ((float4*)dst)[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
    } else {
      *(float4*)dst = make_float4(cs[0], cs[1], cs[2], cs[3]);
    }
  }
}

// Epilogue output stores (16 B per lane): default cache policy, or nontemporal (NT; the GELU
// forward's two outputs).  Write-through (sc1) and sc0 sc1 nt forms were measured mixed and
// dropped (profiles/r02/epilogue/gemm_store_policy_ab_rejected.txt).
#ifndef MMPT_GEMM_GELU_NT
#define MMPT_GEMM_GELU_NT 1  // nontemporal stores for the GELU forward epilogue (-2% at the bench shape)
#endif
template <bool NT = false>
__device__ __forceinline__ void st_out(void* ptr, uint4 v) {
  if constexpr (NT) {
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(u4v{v.x, v.y, v.z, v.w}, (u4v*)ptr);
  } else {
    *(uint4*)ptr = v;
  }
}
__device__ __forceinline__ void st_out(void* ptr, float4 v) {
  st_out(ptr, uint4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                    __float_as_uint(v.w)});
}

__device__ __forceinline__ uint4 pack_bf16x8(const float* v) {
  uint4 o;
  o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
  o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
  return o;
}
__device__ __forceinline__ void unpack_bf16x8(uint4 u, float* o) {
  o[0] = bf2f(u.x & 0xffff); o[1] = bf2f(u.x >> 16);
  o[2] = bf2f(u.y & 0xffff); o[3] = bf2f(u.y >> 16);
  o[4] = bf2f(u.z & 0xffff); o[5] = bf2f(u.z >> 16);
  o[6] = bf2f(u.w & 0xffff); o[7] = bf2f(u.w >> 16);
}

// 8 consecutive columns n..n+7 of row m (n % 8 == 0, n + 8 <= N, p.wide): one 16-B
// store per bf16 output row segment, two per fp32 one (T21: store-issue-bound tails).
// Epilogues that read global memory (aux = GELU pre-activation / attention output,
// residual stream, accumulated gradient) take those operands PREFETCHED by the caller:
// the loads of a whole 128-column half of the tile are issued together before any
// store, instead of one dependent load -> math -> store chain per row (the compiler
// cannot hoist a load above the previous row's store: C may alias C2).
template <int EPI>
constexpr bool epi_loads_aux() {
  return EPI == MMPT_EPI_BF16_DGELU || EPI == MMPT_EPI_BF16_DGELU_COLSUM ||
         EPI == MMPT_EPI_F32_RESID;
}
template <int EPI>
constexpr bool epi_loads_c() {
  return EPI == MMPT_EPI_F32_ACC || EPI == MMPT_EPI_F32_RESID;
}

template <int EPI_, bool LUT = false>  // LUT: erf-GELU from the LDS tables `lut`
__device__ __forceinline__ void epilogue8(const GemmParams& p, int m, int n, const float* v,
                                          int split, float* cs, const uint4& qa,
                                          const float4& qc0, const float4& qc1, const uint4& qb,
                                          const char* lut = nullptr) {
  // qb: the 8 bias values of columns n..n+7 (zeros without bias), loaded by the caller once
  // per column group — a load here, after the previous row's store, would make the wave wait
  // for that store (vmcnt counts loads and stores in one in-order counter)
  constexpr int EPI = epi_base<EPI_>();
  constexpr bool QK = epi_quick<EPI_>();
  float bias[8];
  unpack_bf16x8(qb, bias);
  if constexpr (EPI == MMPT_EPI_BF16) {
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = v[e] + bias[e];
    st_out((bf16_t*)p.C + (long)m * p.ldc + n, pack_bf16x8(o));
  } else if constexpr (EPI == MMPT_EPI_BF16_GELU) {
    float pre[8], act[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) pre[e] = round_bf(v[e] + bias[e]);
    if constexpr (LUT) {
      gelu_lut8(lut, pre, act);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) act[e] = act_f<QK>(pre[e]);
    }
    st_out((bf16_t*)p.C + (long)m * p.ldc + n, pack_bf16x8(pre));
    st_out((bf16_t*)p.C2 + (long)m * p.ldc2 + n, pack_bf16x8(act));
  } else if constexpr (EPI == MMPT_EPI_BF16_DGELU || EPI == MMPT_EPI_BF16_DGELU_COLSUM) {
    float x[8], o[8];
    unpack_bf16x8(qa, x);
    if constexpr (LUT) {
      float gd[8];
      gelu_grad_lut8(lut, x, gd);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = round_bf(round_bf(v[e]) * gd[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = dact_f<QK>(round_bf(v[e]), x[e]);
    }
    st_out((bf16_t*)p.C + (long)m * p.ldc + n, pack_bf16x8(o));
    if constexpr (EPI == MMPT_EPI_BF16_DGELU_COLSUM) {
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += o[e];
    }
  } else if constexpr (EPI == MMPT_EPI_F32_ACC || EPI == MMPT_EPI_F32_STORE) {
    float4* c = (float4*)((float*)p.C + (long)m * p.ldc + n);
    float4 o0 = make_float4(round_bf(v[0]), round_bf(v[1]), round_bf(v[2]), round_bf(v[3]));
    float4 o1 = make_float4(round_bf(v[4]), round_bf(v[5]), round_bf(v[6]), round_bf(v[7]));
    if constexpr (EPI == MMPT_EPI_F32_ACC) {
      const float4 a0 = qc0, a1 = qc1;
      o0.x += a0.x; o0.y += a0.y; o0.z += a0.z; o0.w += a0.w;
      o1.x += a1.x; o1.y += a1.y; o1.z += a1.z; o1.w += a1.w;
    }
    st_out(c, o0);
    st_out(c + 1, o1);
  } else if constexpr (EPI == MMPT_EPI_BF16_DSWIGLU) {
    const long gc = swiglu_gcol(n);
    const bf16_t* a = p.aux + (long)m * p.ld_aux + gc;
    float g[8], u[8], dg[8], du[8];
    unpack_bf16x8(*(const uint4*)a, g);
    unpack_bf16x8(*(const uint4*)(a + 128), u);
#pragma unroll
    for (int e = 0; e < 8; ++e) dswiglu(round_bf(v[e]), g[e], u[e], dg[e], du[e]);
    bf16_t* c = (bf16_t*)p.C + (long)m * p.ldc + gc;
    *(uint4*)c = pack_bf16x8(dg);
    *(uint4*)(c + 128) = pack_bf16x8(du);
  } else if constexpr (EPI == MMPT_EPI_F32_RESID) {
    float r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = round_bf(v[e] + bias[e]);
    if (p.aux != nullptr) {
      float x[8];
      unpack_bf16x8(qa, x);
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = round_bf(r[e] + x[e]);
    }
    const float4 r0 = qc0, r1 = qc1;
    float4* c = (float4*)((float*)p.C + (long)m * p.ldc + n);
    st_out(c, make_float4(r0.x + r[0], r0.y + r[1], r0.z + r[2], r0.w + r[3]));
    st_out(c + 1, make_float4(r1.x + r[4], r1.y + r[5], r1.z + r[6], r1.w + r[7]));
  } else {
    float4* c = (float4*)(p.slab + ((long)split * p.M + m) * p.N + n);
    st_out(c, make_float4(v[0], v[1], v[2], v[3]));
    st_out(c + 1, make_float4(v[4], v[5], v[6], v[7]));
  }
}


// Tile coordinates of this workgroup: XCD-aware bijective remap (blocks b and b+8 share
// an XCD, so an XCD gets a contiguous run of tile ids), then grouped order (GROUP tile
// rows walk the N tiles together so their A panels stay L2-resident).  blockIdx.y is
// the split index (split-K), folded into the remap so a tile's splits share an XCD.
struct TileCoord {
  int m0, n0, split;
};
// work id (tile-major over splits) -> tile coordinates, grouped order
__device__ __forceinline__ TileCoord coord_of(const GemmParams& p, int wid0, int BM, int BN) {
  const int ntiles = p.tiles_m * p.tiles_n;
  const int wid = wid0 % ntiles;
  const int GROUP = p.group;
  const int per_group = GROUP * p.tiles_n;
  const int first_m = (wid / per_group) * GROUP;
  const int gsize = min(p.tiles_m - first_m, GROUP);
  const int tm = first_m + (wid % per_group) % gsize;
  const int tn = (wid % per_group) / gsize;
  return {tm * BM, tn * BN, wid0 / ntiles};
}
// first work id of XCD x's contiguous run (nwg ids over 8 XCDs, the first r8 runs one longer)
__device__ __forceinline__ int xcd_run_start(int nwg, int x) {
  const int q8 = nwg >> 3, r8 = nwg & 7;
  return x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;
}
__device__ __forceinline__ TileCoord tile_coord(const GemmParams& p, int BM, int BN) {
  const int nwg = p.tiles_m * p.tiles_n * gridDim.y;
  const int bid = blockIdx.y * gridDim.x + blockIdx.x;
  return coord_of(p, xcd_run_start(nwg, bid & 7) + (bid >> 3), BM, BN);
}
// Persistent launch (gemm4p): a 1-D grid of G workgroups (G % 8 == 0, one per CU), WG b
// on XCD b & 7 walks its XCD's contiguous run of work ids with stride G / 8 — at any time
// the XCD's 32 CUs hold 32 consecutive ids (8 tile rows x 4 tile columns: shared A/B
// panels in that XCD's L2), the same placement as the one-tile-per-WG remap above.
// Returns the k-th work id of this WG, or -1.  G >= nwg: one tile per WG (the remap above).
__device__ __forceinline__ int work_id(int nwg, int k) {
  const int G = gridDim.x, b = blockIdx.x;
  if (G >= nwg) return k == 0 && b < nwg ? xcd_run_start(nwg, b & 7) + (b >> 3) : -1;
  const int x = b & 7, j = (b >> 3) + k * (G >> 3);
  const int size = (nwg >> 3) + (x < (nwg & 7) ? 1 : 0);
  return j < size ? xcd_run_start(nwg, x) + j : -1;
}

// =============================================================================
// 128x128x64 tile, 4 waves (2x2, 64x64 per wave), 2 workgroups per CU: the small
// problems (ViT, projector, short K).  2-slot LDS double buffer, one barrier per
// K-tile (block-level overlap at 2 WG/CU hides the DMA).
// =============================================================================
template <int LA, int LB, int EPI_>
__global__ __launch_bounds__(256, 2) void gemm128_kernel(GemmParams p) {
  constexpr int EPI = epi_base<EPI_>();
  constexpr int BM = 128, BN = 128, WGN = 2, NW = 4;
  constexpr int TM = 4, TN = 4;
  constexpr int IMGA = BM * BK * 2, IMGB = BN * BK * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * (IMGA + IMGB)];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const TileCoord tc = tile_coord(p, BM, BN);
  const int m0 = tc.m0, n0 = tc.n0, split = tc.split;
  int kbeg = 0, kend = p.K;
  if constexpr (EPI == EPI_SPLIT) {
    kbeg = split * p.kchunk;
    kend = min(p.K, kbeg + p.kchunk);
  }

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BK - 1) / BK;
  stage<LA, BM, NW>(p.A, p.lda, p.M, kend, m0, kbeg, smem, wave, lane);
  stage<LB, BN, NW>(p.B, p.ldb, p.N, kend, n0, kbeg, smem + IMGA, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * (IMGA + IMGB);
    if (t + 1 < nk) {
      char* nxt = smem + ((t + 1) & 1) * (IMGA + IMGB);
      stage<LA, BM, NW>(p.A, p.lda, p.M, kend, m0, kbeg + (t + 1) * BK, nxt, wave, lane);
      stage<LB, BN, NW>(p.B, p.ldb, p.N, kend, n0, kbeg + (t + 1) * BK, nxt + IMGA, wave, lane);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v8s a[TM], b[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = frag<LB, BN>(cur + IMGA, wn * (BN / WGN) + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = frag<LA, BM>(cur, wm * (BM / 2) + i * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((v8bf)b[j], (v8bf)a[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane owns C[m][n..n+3]
  const int mrow = m0 + wm * (BM / 2) + (lane & 15);
  const int ncol = n0 + wn * (BN / WGN) + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = ncol + j * 16;
    float cs[4] = {0.f, 0.f, 0.f, 0.f};
    if (n < p.N) {
      float bias[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == MMPT_EPI_BF16 || EPI == MMPT_EPI_BF16_GELU || EPI == MMPT_EPI_F32_RESID) {
        if (p.bias != nullptr) load_bf16x4(p.bias + n, bias);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = mrow + i * 16;
        if (m >= p.M) continue;
        const v4f a = acc[i][j];
        const float v[4] = {a[0], a[1], a[2], a[3]};
        epilogue4<EPI_>(p, m, n, v, bias, split, cs);
      }
    }
    if constexpr (EPI == MMPT_EPI_BF16_DGELU_COLSUM)
      colsum_store<4>(p, cs, (m0 / BM) * 2 + wm, n, lane);
  }
}

// =============================================================================
// Buffer-resource LDS-DMA (gemm4p): the per-lane byte offset (row·ld + chunk·8)·2 is
// loop-invariant (computed once per tile), the K-tile advance is the SCALAR base of the
// resource, so a steady-state piece costs no VALU; an offset at or past num_records reads
// zeros (the K-tail form).
// =============================================================================
constexpr uint32_t BUF_OOB = 0x7ffffff0u;  // num_records: every valid offset is below
typedef int v4i_t __attribute__((ext_vector_type(4)));
// the same resource as 4 SGPRs for the inline-asm form
__device__ __forceinline__ v4i_t buf_rsrc4(const bf16_t* base) {
  const uintptr_t b = (uintptr_t)base;
  v4i_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
  r[2] = (int)BUF_OOB;
  r[3] = 0x00020000;
  return r;
}
// per-lane byte offsets of the wave's 2 pieces of a 128-row half image (rows r0..), relative
// to the K-tile base (ROWS_K: src + r0*ld + k0; K_ROWS: src + k0*ld) - the same source chunks
// as stage_pieces, with the row clamps folded in.  ROWS_K offsets are relative to the half's
// first row, so they stay below the resource's 2-GiB range for any operand size (an absolute
// row offset overflows past 2 GiB: the fc2 / lm_head operands at 180,992 tokens are 3-13 GB);
// the base row is clamped like the rows (min(r0, Rlim - 1)), so every read stays in bounds.
template <int LAYOUT>
__device__ __forceinline__ void buf_offsets(long ld, int Rlim, int r0, int wave, int lane,
                                            uint32_t* voff) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wave * 2 + i;
    if constexpr (LAYOUT == MMPT_ROWS_K) {
      const int r = q * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (r & 7);
      const int gr = min(r0 + r, Rlim - 1) - min(r0, Rlim - 1);
      voff[i] = (uint32_t)(((long)gr * ld + lc * 8) * 2);
    } else {
      constexpr int CPR = 16, RPP = 4;  // 128 rows: 16 chunks per k-row, 4 k-rows per piece
      const int kr = q * RPP + lane / CPR;
      const int lc = (lane % CPR) ^ swz_kr(kr);
      const int gr = min(r0 + lc * 8, Rlim - 8);
      voff[i] = (uint32_t)(((long)kr * ld + gr) * 2);
    }
  }
}

#ifndef MMPT_GEMM_DIAG
#define MMPT_GEMM_DIAG 0
#endif
// Diagnostic 7 (never shipped; scripts/diag/gemm_clock.py): the in-kernel clock of
// MI355X_MICROARCH.md 'DVFS give-back' item 6 — each workgroup of gemm4p stamps
// s_memtime (shader cycles) and s_memrealtime (100 MHz) at its start and end into a buffer of
// its own that nothing else reads (g_gemm_clock, copied out by mmpt_gemm_diag_clock).
#if MMPT_GEMM_DIAG == 7
__device__ unsigned long long g_gemm_clock[1024 * 4];
struct ClockStamp {
  unsigned long long c0, r0;
  __device__ ClockStamp() : c0(__builtin_amdgcn_s_memtime()), r0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ ~ClockStamp() {
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
      unsigned long long* d = g_gemm_clock + 4 * (blockIdx.x & 1023);
      d[0] = c0;
      d[1] = c1;
      d[2] = r0;
      d[3] = r1;
    }
  }
};
#define MMPT_GEMM_CLOCK ClockStamp clock_stamp_;
#else
#define MMPT_GEMM_CLOCK
#endif

template <bool ACC>
__global__ __launch_bounds__(256) void splitk_reduce(int M, int N, int splits, const float* slab,
                                                     float* C, long ldc) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;  // float4 index
  const long n4 = (long)M * (N / 4);
  if (idx >= n4) return;
  const int m = (int)(idx / (N / 4)), n = (int)(idx % (N / 4)) * 4;
  float4 s = *(const float4*)(slab + (long)m * N + n);
  for (int k = 1; k < splits; ++k) {
    const float4 v = *(const float4*)(slab + ((long)k * M + m) * N + n);
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  float4 o = make_float4(round_bf(s.x), round_bf(s.y), round_bf(s.z), round_bf(s.w));
  float4* c = (float4*)(C + (long)m * ldc + n);
  if (ACC) {
    const float4 old = *c;
    o.x += old.x;
    o.y += old.y;
    o.z += old.z;
    o.w += old.w;
  }
  *c = o;
}


// The tail rows of a tail-split GEMM (round 5, mmpt_gemm_bf16: the last few tile rows that
// would otherwise run as a partial last round on a few CUs): acc = the splits' fp32 partials in
// split order, then the formula of the fast epilogue (epilogue4f) — plain: C = bf16(acc + bias);
// residual: v = bf16(acc + bias), v = bf16(v + aux) when aux is given, C = C2 + v (fp32).
// Bias absent = +0 added, as the fast epilogue does.  8 columns per thread.
template <bool RES>
__global__ __launch_bounds__(256) void tail_epi_kernel(int M, int N, int splits, const float* slab,
                                                       const bf16_t* bias, const bf16_t* aux,
                                                       long ld_aux, void* C, long ldc,
                                                       const float* C2, long ldc2) {
  const int n8 = N / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)M * n8) return;
  const int m = (int)(idx / n8), n = (int)(idx % n8) * 8;
  float a[8];
  {
    const float4* q = (const float4*)(slab + (long)m * N + n);
    const float4 x0 = q[0], x1 = q[1];
    a[0] = x0.x; a[1] = x0.y; a[2] = x0.z; a[3] = x0.w;
    a[4] = x1.x; a[5] = x1.y; a[6] = x1.z; a[7] = x1.w;
  }
  for (int k = 1; k < splits; ++k) {
    const float4* q = (const float4*)(slab + ((long)k * M + m) * N + n);
    const float4 x0 = q[0], x1 = q[1];
    a[0] += x0.x; a[1] += x0.y; a[2] += x0.z; a[3] += x0.w;
    a[4] += x1.x; a[5] += x1.y; a[6] += x1.z; a[7] += x1.w;
  }
  float b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (bias != nullptr) unpack_bf16x8(*(const uint4*)(bias + n), b);
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = round_bf(a[e] + b[e]);
  if constexpr (RES) {
    if (aux != nullptr) {
      float x[8];
      unpack_bf16x8(*(const uint4*)(aux + (long)m * ld_aux + n), x);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = round_bf(v[e] + x[e]);
    }
    const float4* r = (const float4*)(C2 + (long)m * ldc2 + n);
    const float4 r0 = r[0], r1 = r[1];
    float4* c = (float4*)((float*)C + (long)m * ldc + n);
    c[0] = make_float4(r0.x + v[0], r0.y + v[1], r0.z + v[2], r0.w + v[3]);
    c[1] = make_float4(r1.x + v[4], r1.y + v[5], r1.z + v[6], r1.w + v[7]);
  } else {
    uint4 o;
    o.x = pack_pair(v[0], v[1]);
    o.y = pack_pair(v[2], v[3]);
    o.z = pack_pair(v[4], v[5]);
    o.w = pack_pair(v[6], v[7]);
    *(uint4*)((bf16_t*)C + (long)m * ldc + n) = o;
  }
}

// =============================================================================
// 4-wave 256x256x64 GEMM with a hand-ordered software pipeline (round 4, MMPT_GEMM_4P=1,
// ROWS_K x ROWS_K, K % 64 == 0, no split-K / SwiGLU): one wave per SIMD, 128x128 wave tiles,
// 256 fp32 accumulators pinned in AGPRs by inline-asm MFMAs.  The order of one K-tile follows
// the installed hipBLASLt MT256x256x64_MI16x16 kernels (disassembled for study):
// 128 MFMAs per wave with every other instruction slotted between them, LDS-DMA two K-tiles
// ahead into the buffer just released, four barriers per K-tile, counted vmcnt waits (no
// drain).  Per K-tile t (buffer X = t & 1 holds tile t, Y = X ^ 1 tile t + 1):
//   MFMA  0..19  k-half 0 of t; reads b[1] <- B(t, k-half 1) from X       | lgkmcnt(0), barrier 1
//   MFMA 20..51  ...; DMA B(t+2) -> X (8 pieces); reads a[1] <- A(t, kh 1) | lgkmcnt(0), barrier 2
//   MFMA 52..67  ...; DMA A(t+2) -> X (pieces 0-3)        | vmcnt: B(t+1) landed, barrier 3
//   MFMA 68..103 k-half 1 of t; reads b[0] <- B(t+1, kh 0) from Y; DMA A(t+2) pieces 4-7
//                                                         | vmcnt: A(t+1) landed, barrier 4
//   MFMA 104..127 ...; reads a[0] <- A(t+1, kh 0) from Y
// Per CU and K-tile: 128 KiB of fragment reads (4 waves x (128 + 128) rows x 128 B) against the
// 8-wave kernel's 192 KiB, the same 64 KiB of LDS-DMA, 4 barriers instead of 8.
// =============================================================================


// one accumulator element AGPR -> VGPR at this point of the program (a plain read lets hipcc
// copy all 256 accumulators out right after the last MFMA: 256 live VGPRs, spills)
__device__ __forceinline__ float acc_read(float a) {
  float v;
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(a));
  return v;
}
// Epilogue of the 4-wave kernel: the wave's 128x128 block (8 row groups i x 8 column groups j)
// through the per-8-column bodies (epilogue8 / epilogue4):
// v_permlane16_swap of (2y, 2y+1) gives lane group g 8 consecutive columns of the 32-column
// group y; a column group's aux / C operands are loaded for all 8 row groups ahead of its rows.
template <int EPI_>
__device__ __forceinline__ void epilogue4w(const GemmParams& p, v4f (&acc)[8][8], int m0, int n0,
                                           int split, int lane, int wm, int wn, const char* lut) {
  constexpr int EPI = epi_base<EPI_>();
  static_assert(EPI != MMPT_EPI_BF16_SWIGLU, "4-wave SwiGLU forward: the fast epilogue only");
  if constexpr (MMPT_GEMM_DIAG == 4) {  // diagnostic: no epilogue (opaque runtime test)
    if (p.ldc != -7) return;
  }
  constexpr bool CS = EPI == MMPT_EPI_BF16_DGELU_COLSUM;
  constexpr bool LT = gelu_uses_lut<EPI_>();
  constexpr bool LDA = epi_loads_aux<EPI>(), LDC = epi_loads_c<EPI>();
  constexpr bool BIAS = EPI == MMPT_EPI_BF16 || EPI == MMPT_EPI_BF16_GELU || EPI == MMPT_EPI_F32_RESID;
  const int g = lane >> 4;
  const int cwl = (g & 1) * 16 + (g >> 1) * 8;
  const int prow = (m0 / 256) * 2 + wm;  // column-sum partial row: this wave's 128-row half
  const int mb = m0 + wm * 128 + (lane & 15);
  // one column group per iteration (not unrolled: four copies of the GELU bodies made hipcc
  // keep the accumulators in scratch); its 16 accumulator tiles are taken out by a switch
#pragma nounroll
  for (int y = 0; y < 4; ++y) {
    v4f cg[8][2];
    switch (y) {
#define MMPT_TAKE(Y)                                                             \
  case Y:                                                                        \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {                              \
      cg[i][0] = acc[i][2 * (Y)];                                                \
      cg[i][1] = acc[i][2 * (Y) + 1];                                            \
    }                                                                            \
    break;
      MMPT_TAKE(0)
      MMPT_TAKE(1)
      MMPT_TAKE(2)
      default: MMPT_TAKE(3)
#undef MMPT_TAKE
    }
    const int n = n0 + wn * 128 + y * 32 + cwl;
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float csj[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const bool w8 = p.wide && n + 8 <= p.N;
    uint4 qb = {0u, 0u, 0u, 0u};
    if constexpr (BIAS) {
      if (p.bias != nullptr && w8) qb = *(const uint4*)(p.bias + n);
    }
    uint4 qa[8];
    float4 qc[8][2];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      qa[i] = uint4{0u, 0u, 0u, 0u};
      qc[i][0] = qc[i][1] = float4{0.f, 0.f, 0.f, 0.f};
    }
    if (w8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = min(mb + i * 16, p.M - 1);
        if constexpr (LDA) {
          if (p.aux != nullptr) qa[i] = *(const uint4*)(p.aux + (long)m * p.ld_aux + n);
        }
        if constexpr (LDC) {
          const float4* src = EPI == MMPT_EPI_F32_ACC
                                  ? (const float4*)((const float*)p.C + (long)m * p.ldc + n)
                                  : (const float4*)((const float*)p.C2 + (long)m * p.ldc2 + n);
          qc[i][0] = src[0];
          qc[i][1] = src[1];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      v4f c0 = cg[i][0], c1 = cg[i][1];
      const int m = mb + i * 16;
      if (p.wide) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(c0[e]),
                                                          __float_as_uint(c1[e]), false, false);
          c0[e] = __uint_as_float(r[0]);
          c1[e] = __uint_as_float(r[1]);
        }
        if (m >= p.M || n >= p.N) continue;
        const float v[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
        if (n + 8 <= p.N) {
          epilogue8<EPI_, LT>(p, m, n, v, split, cs, qa[i], qc[i][0], qc[i][1], qb, lut);
        } else {
          float bias[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (BIAS) {
            if (p.bias != nullptr) load_bf16x4(p.bias + n, bias);
          }
          epilogue4<EPI_, LT>(p, m, n, v, bias, split, cs, lut);
        }
      } else {
        if (m >= p.M) continue;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int n4 = n0 + wn * 128 + y * 32 + jj * 16 + 4 * g;
          if (n4 >= p.N) continue;
          float bias[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (BIAS) {
            if (p.bias != nullptr) load_bf16x4(p.bias + n4, bias);
          }
          const v4f c = jj == 0 ? c0 : c1;
          const float v[4] = {c[0], c[1], c[2], c[3]};
          epilogue4<EPI_, LT>(p, m, n4, v, bias, split, csj[jj], lut);
        }
      }
    }
    if constexpr (CS) {
      if (p.wide) {
        colsum_store<8>(p, cs, prow, n, lane);
      } else {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          colsum_store<4>(p, csj[jj], prow, n0 + wn * 128 + y * 32 + jj * 16 + 4 * g, lane);
      }
    }
  }
}

// Fast whole-tile epilogue of the 4-wave kernel (bf16 outputs: plain + bias, erf-GELU from the
// LDS table, erf-dGELU (+ column sums)).  Row group i (rows m0 + wm*128 + 16i + lane&15) at a
// time: its four 32-column groups y leave the accumulators through v_permlane16_swap as 8
// consecutive columns per lane, packed in pairs (the fast rows), and go through a
// wave-private 4-KiB LDS staging image (row r16 = lane & 15 at 16-B chunk (4y + cwl/8) ^ r16),
// read back as 4 rows x 256 B per instruction — whole 128-B lines per store instead of 16 rows
// x 64 B.  The image is wave-private, so no barrier: a wave's LDS operations run in order.
// The operands the epilogue reads come from registers: the bias (qb) and the dGELU
// pre-activations of row groups 0 and 1 (qa) were loaded by the caller before the tile's last
// K-tile; row group i + 2's pre-activations are loaded while row group i is processed, behind
// only this epilogue's own stores (no LDS-DMA of the next tile is issued in between: the
// compiler's vmcnt for them is exact).  Edge tiles run the same code with masked stores (the
// launch requires 16-B aligned outputs and N % 8 == 0 for these epilogues).
#ifndef MMPT_GEMM_4P_FAST
#define MMPT_GEMM_4P_FAST 1
#endif
// STG (round 5, measured and NOT kept: 1-2.5% slower on every plain shape and -0.3% on the
// step, profiles/r05/stg_rejected/): the plain fast epilogue staged in the 32 KiB of LDS left
// beside the K-tile buffers so the next tile's K-tile-1 A pieces go out before its stores and
// the first K-tile's waits leave the stores in flight.  Kept buildable (-DMMPT_GEMM_STG=1).
#ifndef MMPT_GEMM_STG
#define MMPT_GEMM_STG 0
#endif
#ifndef MMPT_GEMM_STG_RELAX  // (diagnostic) bit 0: loop-top wait, bit 1: first K-tile waits
#define MMPT_GEMM_STG_RELAX 3
#endif
#ifndef MMPT_GEMM_4P_NT
#define MMPT_GEMM_4P_NT 1  // nontemporal stores for the plain / dGELU outputs too: lm_head fwd +3%,
                           // qkv fwd +1.6%, 8192^3 +3% (profiles/r04/epi2/); 0 for A/B builds
#endif
// gemm4p's table (LDS) epilogues: the erf-GELU forms (g_gelu_lut), and since round 5 the
// quick-GELU forward (g_qgelu_lut) and the SwiGLU forward (g_silu_lut) — forward activations
// are functions of one bf16 value.  Their backward forms (dQGELU: four roundings around
// s(x); dSwiGLU: two operands per output) run the general per-element code (epilogue4w).
template <int EPI_>
constexpr bool lut4() {
  return gelu_uses_lut<EPI_>() ||
         (MMPT_GEMM_LUT && (EPI_ == MMPT_EPI_BF16_QGELU || EPI_ == MMPT_EPI_BF16_SWIGLU ||
                            EPI_ == MMPT_EPI_BF16_DSWIGLU));
}
template <int EPI_>
constexpr bool epi4_fast() {
  constexpr int E = epi_base<EPI_>();
  return MMPT_GEMM_4P_FAST &&
         (E == MMPT_EPI_BF16 || E == MMPT_EPI_F32_RESID ||
          (lut4<EPI_>() && (E == MMPT_EPI_BF16_GELU || E == MMPT_EPI_BF16_DGELU ||
                            E == MMPT_EPI_BF16_DGELU_COLSUM || E == MMPT_EPI_BF16_SWIGLU ||
                            E == MMPT_EPI_BF16_DSWIGLU)));
}
// VM instructions a fast epilogue issues at least (the next tile's first wait leaves them,
// and the K-tile-1 A pieces issued after them, in flight)
template <int EPI_>
constexpr int epi4_aux_pd() {
  return epi_base<EPI_>() == MMPT_EPI_BF16_DGELU_COLSUM || EPI_ == MMPT_EPI_BF16_DSWIGLU ? 1 : 2;
}
template <int EPI_>
constexpr int epi4_fast_vm() {
  constexpr int E = epi_base<EPI_>();
  return E == MMPT_EPI_BF16 ? 32
         : E == MMPT_EPI_BF16_SWIGLU ? 48  // 32 gate|up row stores + 16 activation row stores
         : E == MMPT_EPI_BF16_DSWIGLU ? 64  // 32 d gate + 32 d up row stores (+ the aux loads)
         : E == MMPT_EPI_BF16_GELU || E == MMPT_EPI_F32_RESID ? 64
                                                              : 32 + 4 * (8 - epi4_aux_pd<EPI_>());
}
// SwiGLU forward on gemm4p: wave wn takes B column tiles {wn·64 + 16j} (j < 4, gate) and
// {128 + wn·64 + 16(j − 4)} (j >= 4, up) instead of wn·128 + 16j, so each lane holds the gate
// AND up value of its features (blocked gate|up weight: 128 gate rows, then their 128 up rows)
template <int EPI_>
constexpr bool swiglu_map() {
  return EPI_ == MMPT_EPI_BF16_SWIGLU;
}
// Residual epilogue operands of rows m + 4q (q = 0..3), columns n..n+7, in the row layout of
// the staged rows: the attention output (aux, bf16) and the residual stream (C2, fp32)
__device__ __forceinline__ void res_load(const GemmParams& p, long m, int n, uint4 (&ra)[4],
                                         float4 (&rc)[4][2]) {
  const int nn = min(n, p.N - 8);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long mm = min(m + 4 * q, (long)p.M - 1);
    if (p.aux != nullptr) ra[q] = *(const uint4*)(p.aux + mm * p.ld_aux + nn);
    const float4* c2 = (const float4*)((const float*)p.C2 + mm * p.ldc2 + nn);
    rc[q][0] = c2[0];
    rc[q][1] = c2[1];
  }
}
template <int EPI_>
__device__ __forceinline__ void epilogue4f(const GemmParams& p, v4f (&acc)[8][8], int m0, int n0,
                                           int lane, int wm, int wn, const char* lut, char* stg,
                                           const uint4 (&qb)[4], uint4 (&qa)[3][4],
                                           uint4 (&qu)[3][4], uint4 (&ra)[2][4],
                                           float4 (&rc)[2][4][2]) {
  constexpr int EPI = epi_base<EPI_>();
  constexpr bool GELU = EPI == MMPT_EPI_BF16_GELU;  // erf or quick (QK)
  constexpr bool QK = epi_quick<EPI_>();
  constexpr bool SW = EPI == MMPT_EPI_BF16_SWIGLU;
  constexpr bool DSW = EPI == MMPT_EPI_BF16_DSWIGLU;  // (d gate, d up) from d act, tables
  constexpr bool RES = EPI == MMPT_EPI_F32_RESID;
  constexpr bool DG = EPI == MMPT_EPI_BF16_DGELU || EPI == MMPT_EPI_BF16_DGELU_COLSUM;
  constexpr bool CS = EPI == MMPT_EPI_BF16_DGELU_COLSUM;
  constexpr int PD = epi4_aux_pd<EPI_>();  // pre-activation prefetch distance (row groups)
  static_assert(!(QK && DG), "fast epilogue: the dQGELU forms run epilogue4w");
  if constexpr (MMPT_GEMM_DIAG == 4) {
    if (p.ldc != -7) return;
  }
  const int g = lane >> 4, r16 = lane & 15;
  const int cwl = (g & 1) * 16 + (g >> 1) * 8;
  const long mw = m0 + wm * 128;
  const int nw = n0 + wn * 128;
  float bf[4][8];
  if constexpr (!DG && !SW && !DSW) {
#pragma unroll
    for (int y = 0; y < 4; ++y) unpack_bf16x8(qb[y], bf[y]);
  }
  // the wave's staged 16-B chunk r16 of a row lands at output column ccol (SwiGLU: chunks 0-7
  // are the gate columns wn·64.., 8-15 the up columns 128 + wn·64..)
  const int ccol = SW ? n0 + wn * 64 + (r16 & 7) * 8 + (r16 >> 3) * 128 : nw + r16 * 8;
  // dSwiGLU: the wave's 128 features are one 128-column block of the blocked [M][2N] gate|up
  // layout: d gate at block column gb, d up at gb + 128 (gbc: clamped for the aux loads)
  const int gb = (nw >> 7) * 256, gbc = (min(nw, p.N - 128) >> 7) * 256;
  bf16_t* const crow = RES ? nullptr : (bf16_t*)p.C + (mw + g) * p.ldc + (DSW ? gb + r16 * 8 : ccol);
  bf16_t* const c2row = GELU  ? (bf16_t*)p.C2 + (mw + g) * p.ldc2 + nw + r16 * 8
                        : DSW ? crow + 128
                              : nullptr;
  // SwiGLU activation rows: features n0/2 + wn·64 + 8·(lane & 7), rows 8q + lane/8 of a group
  bf16_t* const arow = SW ? (bf16_t*)p.C2 + (mw + (lane >> 3)) * p.ldc2 + (n0 >> 1) + wn * 64 +
                                (lane & 7) * 8
                          : nullptr;
  // pre-activation of row group i, column group y (rows / columns past the end clamped: their
  // outputs are never stored)
  auto aux_at = [&](int i, int y) -> const uint4* {
    const long m = min(mw + r16 + 16 * i, (long)p.M - 1);
    return (const uint4*)(p.aux + m * p.ld_aux + min(nw + cwl + 32 * y, p.N - 8));
  };
  // dSwiGLU operands (forward gate / up values) of row group i, column group y
  auto dsw_at = [&](int i, int y, int up) -> const uint4* {
    const long m = min(mw + r16 + 16 * i, (long)p.M - 1);
    return (const uint4*)(p.aux + m * p.ld_aux + gbc + 128 * up + cwl + 32 * y);
  };
  char* const wst = stg + r16 * 256;  // writer row
  float cs[4][8];
#pragma unroll
  for (int y = 0; y < 4; ++y)
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[y][e] = 0.f;
  // Two-stage software pipeline over the 8 row groups (one wave per SIMD: nothing else hides
  // the epilogue's latencies).  front(i): the row group's accumulators out (v_accvgpr_read +
  // v_permlane16_swap), packed, and its 32 GELU / GELU' table reads issued.  back(i): the rare
  // fixup, the outputs into the staging image, the staging reads, the stores.  Program order
  // per step: back-1(i) [staging writes + reads issued] -> front(i+1) [its table reads in
  // flight under ...] -> back-2(i) [the stores of row group i].
  struct FE {
    uint32_t pk[4][4];  // plain / GELU: bf16(v + bias) pairs;  dGELU: bf16(v) pairs
    uint32_t o[4][4];   // GELU: table outputs
    float gd[4][8];     // dGELU: GELU'(pre-activation)
    uint4 xa[4];        // dGELU: the pre-activations (fixup input)
    uint32_t bad;
  };
  FE fe[2];
  auto front = [&](auto ic, FE& f) {
    constexpr int i = decltype(ic)::value;
    if constexpr (DG) {
      if constexpr (i + PD < 8) {
#pragma unroll
        for (int y = 0; y < 4; ++y) qa[(i + PD) % (PD + 1)][y] = *aux_at(i + PD, y);
      }
    }
    if constexpr (DSW) {
      if constexpr (i + PD < 8) {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          qa[(i + PD) % (PD + 1)][y] = *dsw_at(i + PD, y, 0);
          qu[(i + PD) % (PD + 1)][y] = *dsw_at(i + PD, y, 1);
        }
      }
    }
    if constexpr (RES) {
      if constexpr (i > 0) res_load(p, mw + 16 * i + g, nw + r16 * 8, ra[i & 1], rc[i & 1]);
    }
    f.bad = 0;
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      float c0[4], c1[4], v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        c0[e] = acc_read(acc[i][2 * y][e]);
        c1[e] = acc_read(acc[i][2 * y + 1][e]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(c0[e]),
                                                         __float_as_uint(c1[e]), false, false);
        v[e] = __uint_as_float(sw[0]);
        v[4 + e] = __uint_as_float(sw[1]);
      }
      if constexpr (!DG && !SW && !DSW) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          f.pk[y][q] = pack_pair(v[2 * q] + bf[y][2 * q], v[2 * q + 1] + bf[y][2 * q + 1]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) f.pk[y][q] = pack_pair(v[2 * q], v[2 * q + 1]);
      }
    }
    if constexpr (GELU) {  // erf- or quick-GELU table values
#pragma unroll
      for (int y = 0; y < 4; ++y) gelu_pk8(lut, f.pk[y], f.o[y], f.bad);
    }
    if constexpr (SW) {  // bf16(silu(gate)) table values (gate: column groups 0, 1)
#pragma unroll
      for (int y = 0; y < 2; ++y) gelu_pk8(lut, f.pk[y], f.o[y], f.bad);
    }
    if constexpr (DG) {
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        f.xa[y] = qa[i % (PD + 1)][y];
        const uint32_t x4[4] = {f.xa[y].x, f.xa[y].y, f.xa[y].z, f.xa[y].w};
        gelu_grad_pk8(lut, x4, f.gd[y], f.bad);
      }
    }
    if constexpr (DSW) {
      // bf16(silu(g)) and fp32 sigmoid(g) of the forward's gate values from the table, one
      // column group ahead of the math, then (dg, du) = dswiglu_s: pk <- dg, o <- du
      bf16_t st[2][8];
      float sg[2][8];
      uint32_t bady[2];
      auto lookup = [&](int y, int b) {
        const uint4 gq = qa[i % (PD + 1)][y];
        const uint32_t g4[4] = {gq.x, gq.y, gq.z, gq.w};
        bady[b] = 0;
        u16x2 s2[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) s2[q] = lut_slots2(g4[q], bady[b]);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t k = (e & 1) ? (uint32_t)s2[e >> 1].y : (uint32_t)s2[e >> 1].x;
          st[b][e] = *(const bf16_t*)(lut + 2 * k);
          sg[b][e] = *(const float*)(lut + 2 * LUT_N + 4 * k);
        }
      };
      lookup(0, 0);
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int b = y & 1;
        if (y + 1 < 4) lookup(y + 1, b ^ 1);
        float d[8], gv[8], uv[8], dg[8], du[8];
        unpack_bf16x8(qa[i % (PD + 1)][y], gv);
        if (__builtin_amdgcn_ballot_w64(bady[b] != 0) != 0) {  // rare: general code
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            st[b][e] = f2bf(silu_bf(gv[e]));
            sg[b][e] = 1.0f / (1.0f + __expf(-gv[e]));
          }
        }
        unpack_bf16x8(uint4{f.pk[y][0], f.pk[y][1], f.pk[y][2], f.pk[y][3]}, d);
        unpack_bf16x8(qu[i % (PD + 1)][y], uv);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          dswiglu_s(d[e], gv[e], uv[e], bf2f(st[b][e]), sg[b][e], dg[e], du[e]);
        // straight into the staging image (back1 of the previous row group has issued its
        // staging reads: a wave's LDS operations run in order), not through registers
        char* const w = wst + (((4 * y + (cwl >> 3)) ^ r16) << 4);
        *(uint4*)w = pack_bf16x8(dg);
        *(uint4*)(w + 4096) = pack_bf16x8(du);
      }
    }
  };
  uint4 st0[4], st1[4];  // row group i's staged rows, read back
  auto back1 = [&](auto ic, FE& f) {
    constexpr int i = decltype(ic)::value;
    if constexpr (GELU) {
      if (__builtin_amdgcn_ballot_w64(f.bad != 0) != 0) {  // rare: general code
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          float pre[8], act[8];
          unpack_bf16x8(uint4{f.pk[y][0], f.pk[y][1], f.pk[y][2], f.pk[y][3]}, pre);
          if constexpr (QK) {
#pragma unroll
            for (int e = 0; e < 8; ++e) act[e] = qgelu_f(pre[e]);
          } else {
            gelu_lut8(lut, pre, act);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) f.o[y][q] = pack_pair(act[2 * q], act[2 * q + 1]);
        }
      }
    }
    if constexpr (SW) {
      if (__builtin_amdgcn_ballot_w64(f.bad != 0) != 0) {  // rare: general code
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          float gt[8], s[8];
          unpack_bf16x8(uint4{f.pk[y][0], f.pk[y][1], f.pk[y][2], f.pk[y][3]}, gt);
#pragma unroll
          for (int e = 0; e < 8; ++e) s[e] = silu_bf(gt[e]);
#pragma unroll
          for (int q = 0; q < 4; ++q) f.o[y][q] = pack_pair(s[2 * q], s[2 * q + 1]);
        }
      }
      // act = bf16(bf16(silu(gate)) · up): the up values are column groups y + 2
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        float s[8], u[8];
        unpack_bf16x8(uint4{f.o[y][0], f.o[y][1], f.o[y][2], f.o[y][3]}, s);
        unpack_bf16x8(uint4{f.pk[y + 2][0], f.pk[y + 2][1], f.pk[y + 2][2], f.pk[y + 2][3]}, u);
#pragma unroll
        for (int q = 0; q < 4; ++q) f.o[y][q] = pack_pair(s[2 * q] * u[2 * q], s[2 * q + 1] * u[2 * q + 1]);
        *(uint4*)(wst + 4096 + (((4 * y + (cwl >> 3)) ^ r16) << 4)) =
            uint4{f.o[y][0], f.o[y][1], f.o[y][2], f.o[y][3]};
      }
    }
    if constexpr (DG) {
      if (__builtin_amdgcn_ballot_w64(f.bad != 0) != 0) {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          float x[8];
          unpack_bf16x8(f.xa[y], x);
          gelu_grad_lut8(lut, x, f.gd[y]);
        }
      }
    }
#pragma unroll
    for (int y = 0; y < 4 && !DSW; ++y) {  // (dSwiGLU: staged by front)
      char* const w = wst + (((4 * y + (cwl >> 3)) ^ r16) << 4);
      if constexpr (!DG) {
        *(uint4*)w = uint4{f.pk[y][0], f.pk[y][1], f.pk[y][2], f.pk[y][3]};
        if constexpr (GELU || DSW) *(uint4*)(w + 4096) = uint4{f.o[y][0], f.o[y][1], f.o[y][2], f.o[y][3]};
      } else {  // o = bf16(bf16(v) · GELU'(pre-activation)): one v_cvt_pk per product pair
        float vb[8];
        unpack_bf16x8(uint4{f.pk[y][0], f.pk[y][1], f.pk[y][2], f.pk[y][3]}, vb);
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[q] = pack_pair(vb[2 * q] * f.gd[y][2 * q], vb[2 * q + 1] * f.gd[y][2 * q + 1]);
        if constexpr (CS) {  // the column sums add the rounded outputs
          if (mw + 16 * i + r16 < p.M) {
            float ov[8];
            unpack_bf16x8(uint4{o[0], o[1], o[2], o[3]}, ov);
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[y][e] += ov[e];
          }
        }
        *(uint4*)w = uint4{o[0], o[1], o[2], o[3]};
      }
    }
    // the row group's 16 rows x 256 B back as 4 rows per instruction (row 4q + g, chunk r16)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 4 * q + g;
      const int roff = row * 256 + ((r16 ^ row) << 4);
      st0[q] = *(const uint4*)(stg + roff);
      if constexpr (GELU || DSW) st1[q] = *(const uint4*)(stg + 4096 + roff);
    }
    if constexpr (SW) {  // the activation rows: 8 rows x 128 B per instruction
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int row = 8 * q + (lane >> 3), c = lane & 7;
        st1[q] = *(const uint4*)(stg + 4096 + row * 256 + ((c ^ row) << 4));
      }
    }
  };
  auto back2 = [&](auto ic) {
    constexpr int i = decltype(ic)::value;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int krow = 16 * i + 4 * q;  // wave-uniform row offset (SALU)
      asm volatile("" : "+s"(krow));
      // diagnostic 5 (never shipped): everything but the global stores
      if (mw + krow + g < p.M && ccol < p.N && (MMPT_GEMM_DIAG != 5 || p.ldc == -7)) {
        if constexpr (RES) {
          // C = C2 + bf16(bf16(acc + bias) + aux) in the row layout of the staged rows
          float r[8];
          unpack_bf16x8(st0[q], r);
          if (p.aux != nullptr) {
            float x[8];
            unpack_bf16x8(ra[i & 1][q], x);
#pragma unroll
            for (int e = 0; e < 8; ++e) r[e] = round_bf(r[e] + x[e]);
          }
          const float4 c0 = rc[i & 1][q][0], c1 = rc[i & 1][q][1];
          float4* c = (float4*)((float*)p.C + (mw + krow + g) * p.ldc + nw + r16 * 8);
          st_out(c, make_float4(c0.x + r[0], c0.y + r[1], c0.z + r[2], c0.w + r[3]));
          st_out(c + 1, make_float4(c1.x + r[4], c1.y + r[5], c1.z + r[6], c1.w + r[7]));
        } else {
          st_out<(GELU && MMPT_GEMM_GELU_NT) || MMPT_GEMM_4P_NT>(crow + (long)krow * p.ldc, st0[q]);
          if constexpr (GELU) st_out<MMPT_GEMM_GELU_NT>(c2row + (long)krow * p.ldc2, st1[q]);
          if constexpr (DSW) st_out<MMPT_GEMM_4P_NT>(c2row + (long)krow * p.ldc, st1[q]);
        }
      }
    }
    if constexpr (SW) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        int krow = 16 * i + 8 * q;
        asm volatile("" : "+s"(krow));
        if (mw + krow + (lane >> 3) < p.M) st_out<MMPT_GEMM_4P_NT>(arow + (long)krow * p.ldc2, st1[q]);
      }
    }
  };
  using I_ = std::integral_constant<int, 0>;
  front(I_{}, fe[0]);
#define MMPT_E4_STEP(I)                                                       \
  {                                                                          \
    back1(std::integral_constant<int, I>{}, fe[(I)&1]);                      \
    __builtin_amdgcn_sched_barrier(0);                                       \
    if constexpr ((I) + 1 < 8) front(std::integral_constant<int, (I) + 1>{}, fe[((I) + 1) & 1]); \
    __builtin_amdgcn_sched_barrier(0);                                       \
    back2(std::integral_constant<int, I>{});                                 \
    __builtin_amdgcn_sched_barrier(0);                                       \
  }
  MMPT_E4_STEP(0) MMPT_E4_STEP(1) MMPT_E4_STEP(2) MMPT_E4_STEP(3)
  MMPT_E4_STEP(4) MMPT_E4_STEP(5) MMPT_E4_STEP(6) MMPT_E4_STEP(7)
#undef MMPT_E4_STEP
  if constexpr (CS) {
    const int prow = (m0 / 256) * 2 + wm;
#pragma unroll
    for (int y = 0; y < 4; ++y) colsum_store<8>(p, cs[y], prow, nw + 32 * y + cwl, lane);
  }
}

#define MFMA4(acc, bf, af)                                                                 \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(bf), "v"(af) \
               : "memory")
#define MFMA4Z(acc, bf, af)                                                                \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(bf), "v"(af) \
               : "memory")
// one LDS-DMA piece (64 lanes x 16 B) to LDS byte address `m0` (wave-uniform).  M0 is not
// restored: in gemm4p every M0 reader is this statement, which sets it first.
__device__ __forceinline__ void dma_m0(v4i_t srd, uint32_t voff, uint32_t m0) {
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :: "v"(voff), "s"(srd), "s"(m0) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// KT (round 5): K % 64 != 0 — the last K-tile's DMA pieces past K read an out-of-range buffer
// offset (zeros), so the K tail contributes nothing; instantiated only for the forms that meet
// odd K in practice (weight gradients at token counts that are not a multiple of 64, the CLIP
// patch embedding's K = 588), with the forward K order
template <int LA, int LB, int EPI_, bool KT>
__device__ __forceinline__ void gemm4p_body(const GemmParams& p) {
  MMPT_GEMM_CLOCK
  constexpr int EPI = epi_base<EPI_>();
  constexpr int IMG = 256 * BK * 2;  // 32 KiB: one operand's K-tile image (two 128-row halves)
  constexpr bool USE_LUT = lut4<EPI_>();
  // STG (round 5): the fast plain epilogue stages its output
  // rows in the LDS left free beside the two K-tile buffers (4 waves x 8 KiB), not in buffer 1,
  // so the next tile's K-tile-1 A pieces go out BEFORE the epilogue's stores and its first
  // K-tile's waits may leave the stores in flight: the tile round's store burst drains under
  // ~1.5 K-tiles of MFMAs instead of ~0.5
  // (plain only: the residual instantiation, at 512 VGPRs already, spilled with it)
  constexpr bool STG = MMPT_GEMM_STG && epi4_fast<EPI_>() && !USE_LUT && EPI_ == MMPT_EPI_BF16;
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG + (USE_LUT ? LUT_BYTES : STG ? 32768 : 0)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = p.tiles_m * p.tiles_n * p.splits;
  int w = work_id(nwg, 0);  // persistent: one workgroup per CU walks its XCD's run of tiles
  if (w < 0) return;
  const char* lut = nullptr;
  if constexpr (USE_LUT) {
    constexpr bool FWD = epi_base<EPI_>() == MMPT_EPI_BF16_GELU || EPI == MMPT_EPI_BF16_SWIGLU;
    constexpr bool BOTH = EPI == MMPT_EPI_BF16_DSWIGLU;  // silu and sigmoid
    constexpr int lo = FWD || BOTH ? 0 : 2 * LUT_N, hi = FWD ? 2 * LUT_N : LUT_BYTES;
    const char* src = EPI == MMPT_EPI_BF16_SWIGLU || BOTH ? g_silu_lut
                      : epi_quick<EPI_>()          ? g_qgelu_lut
                                                   : g_gelu_lut;
    for (int i = lo / 16 + tid; i < hi / 16; i += 256)
      ((uint4*)(smem + 4 * IMG))[i] = ((const uint4*)src)[i];
    lut = smem + 4 * IMG;
  }
  TileCoord tc = coord_of(p, w, 256, 256);
  int kbeg = 0, nk = (p.K + (KT ? BK - 1 : 0)) / BK;
  // K order of the current tile: with p.krev, a workgroup's odd tiles (ordinal 1, 3, ...) walk
  // their K-tiles last-to-first, so the A K-slices a tile round loaded last — the ones still in
  // the XCD's L2 when the next round starts on the same row band — are the first it reads
  int kdir = 1;
  // this wave's 8 DMA pieces per operand and K-tile (loop-invariant per-lane byte offsets,
  // the K advance in the resource base):
  //   ROWS_K: the 256-row XOR image (128-B rows, chunk ^ row&7), rows 64*wave + 8q + lane/8,
  //           offsets relative to the tile's first row (rows past the end clamped);
  //   K_ROWS: two 128-row half images in the K_ROWS format ([64 k][128 rows], chunk ^
  //           s(k)), pieces 4*wave .. 4*wave+3 of each half (buf_offsets, absolute columns).
  uint32_t va[8], vb[8];
  const bf16_t *Ab, *Bb;
  auto op_offsets = [&](auto lay_c, long ld, int R, int r0, uint32_t* v) {
    constexpr int L = decltype(lay_c)::value;
    if constexpr (L == MMPT_ROWS_K) {
      const int lr = lane >> 3, lc = (lane & 7) ^ lr;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = 64 * wave + 8 * q + lr;
        v[q] = (uint32_t)(((long)min(r0 + r, R - 1) - r0) * ld * 2 + lc * 16);
      }
    } else {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        buf_offsets<MMPT_K_ROWS>(ld, R, r0 + hh * 128, 2 * wave, lane, v + 4 * hh);
        buf_offsets<MMPT_K_ROWS>(ld, R, r0 + hh * 128, 2 * wave + 1, lane, v + 4 * hh + 2);
      }
    }
  };
  // k offset within a K-tile of this lane's chunk in DMA piece q (op_offsets' layouts), and
  // (KT) per-lane bit q of ktA / ktB = piece q of the tile's last K-tile lies past K (set per
  // tile by `offsets`: one register per operand instead of 16 hoisted k offsets)
  auto kk_of = [&](auto lay_c, int q) -> int {
    constexpr int L = decltype(lay_c)::value;
    if constexpr (L == MMPT_ROWS_K) return ((lane & 7) ^ (lane >> 3)) * 8;
    else return (4 * wave + (q & 3)) * 4 + (lane >> 4);
  };
  uint32_t ktA = 0, ktB = 0;
  auto offsets = [&](const TileCoord& c, int ord) {
    if constexpr (EPI == EPI_SPLIT) {
      kbeg = c.split * p.kchunk;
      nk = (min(p.K, kbeg + p.kchunk) - kbeg + (KT ? BK - 1 : 0)) / BK;
    }
    op_offsets(std::integral_constant<int, LA>{}, p.lda, p.M, c.m0, va);
    op_offsets(std::integral_constant<int, LB>{}, p.ldb, p.N, c.n0, vb);
    if constexpr (KT) {
      const int rem = p.K - (kbeg + (nk - 1) * BK);  // valid k of the last K-tile, 8..56
      ktA = ktB = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        ktA |= (kk_of(std::integral_constant<int, LA>{}, q) >= rem ? 1u : 0u) << q;
        ktB |= (kk_of(std::integral_constant<int, LB>{}, q) >= rem ? 1u : 0u) << q;
      }
    }
    kdir = (!KT && p.krev && (ord & 1)) ? -1 : 1;
    const int k0 = kbeg + (kdir < 0 ? (nk - 1) * BK : 0);  // the first K-tile walked
    Ab = LA == MMPT_ROWS_K ? p.A + (long)c.m0 * p.lda + k0 : p.A + (long)k0 * p.lda;
    Bb = LB == MMPT_ROWS_K ? p.B + (long)c.n0 * p.ldb + k0 : p.B + (long)k0 * p.ldb;
  };
  char* const imgA0 = smem;            // buffer b: A at smem + 2b*IMG, B at smem + (2b+1)*IMG
  // LDS byte address of the image base (M0 of the DMA), as a 32-bit scalar: the per-piece M0
  // is then one scalar add (a generic LDS pointer costs a 64-bit add + null test)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(char, smem));
  // LDS offset of piece q of this wave within an operand image
  auto piece_lds = [&](auto lay_c, int q) -> uint32_t {
    constexpr int L = decltype(lay_c)::value;
    if constexpr (L == MMPT_ROWS_K) return (uint32_t)((8 * wave + q) * 1024);
    else return (uint32_t)((q >> 2) * 16384 + (4 * wave + (q & 3)) * 1024);
  };
  // KT: piece q of the tile's LAST K-tile lies past K -> an out-of-range offset (zeros)
  auto kt_off = [&](uint32_t m, int t, int q, uint32_t v) -> uint32_t {
    if constexpr (KT) {
      if (t == nk - 1 && ((m >> q) & 1u)) return BUF_OOB;
    }
    return v;
  };
  auto dmaA = [&](int buf, int t, int q) {
    const uint32_t vo = kt_off(ktA, t, q, va[q]);
    t *= kdir;
    const bf16_t* base = LA == MMPT_ROWS_K ? Ab + t * BK : Ab + (long)t * BK * p.lda;
    dma_m0(buf_rsrc4(base), vo,
           lds0 + (uint32_t)((2 * buf) * IMG) + piece_lds(std::integral_constant<int, LA>{}, q));
  };
  auto dmaB = [&](int buf, int t, int q) {
    const uint32_t vo = kt_off(ktB, t, q, vb[q]);
    t *= kdir;
    const bf16_t* base = LB == MMPT_ROWS_K ? Bb + t * BK : Bb + (long)t * BK * p.ldb;
    dma_m0(buf_rsrc4(base), vo,
           lds0 + (uint32_t)((2 * buf + 1) * IMG) + piece_lds(std::integral_constant<int, LB>{}, q));
  };
  // prologue DMA of a tile: K-tiles 0 and 1 (B pieces first, as in the loop)
  auto prologue = [&]() {
#pragma unroll
    for (int q = 0; q < 8; ++q) dmaB(0, 0, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dmaA(0, 0, q);
    if (nk > 1) {
#pragma unroll
      for (int q = 0; q < 8; ++q) dmaB(1, 1, q);
#pragma unroll
      for (int q = 0; q < 8; ++q) dmaA(1, 1, q);
    }
  };
  // fragments: rows 16i + (lane & 15) of the wave's 128-row half, k-half s (frag)
  auto rdA = [&](int buf, int s, int i) -> v8s {
    return frag<LA, 128>(imgA0 + (2 * buf) * IMG + wm * 16384, 16 * i, s, lane);
  };
  auto rdB = [&](int buf, int s, int j) -> v8s {
    if constexpr (swiglu_map<EPI_>())  // gate tiles j < 4, their up tiles j >= 4 (see swiglu_map)
      return frag<LB, 128>(imgA0 + (2 * buf + 1) * IMG + (j >> 2) * 16384, wn * 64 + 16 * (j & 3),
                           s, lane);
    return frag<LB, 128>(imgA0 + (2 * buf + 1) * IMG + wn * 16384, 16 * j, s, lane);
  };
  v8s a[2][8], b[2][8];
  v4f acc[8][8];
  // CSA: this lane's running Σ_k of A rows 16i + (lane & 15) over its k quarter (lane >> 4);
  // one pair per even MFMA slot of the fragment's 8 uses (a chain of 4 dependent adds in one
  // slot stalled the in-order issue: the split-K weight gradient ran 27% slower)
  constexpr bool CSA = csa<EPI_>();
  float cs[8];
  int cs_lo = 0, cs_hi = 0;  // (see C1 / C2 below)
  uint32_t cs_w = 0u;
  // one K-tile, straight-line: 128 MFMA slots with the other instructions placed by slot
  // index at compile time (DMA: tile t+2 is staged; NXT: tile t+1 exists and is read ahead)
  // XS: epilogue stores of the previous tile issued between this K-tile's t+1 pieces and its
  // t+2 pieces (STG, first K-tile after a whole tile): the two waits may leave them in flight
  // Z: the tile's first K-tile — its k-half-0 MFMAs (the first use of every accumulator) take
  // srcC = 0 instead of reading the accumulators
  // CS (CSA kernels): 0 = no row sums in this K-tile; 1 = sum every A fragment; 2 = the same
  // with the runtime weight cs_w (1 or 0: one instance for the tile's last two K-tiles)
  auto ktile = [&](int t, auto dma_c, auto nxt_c, auto xs_c, auto z_c, auto cs_c) {
    constexpr bool DMA = decltype(dma_c)::value, NXT = decltype(nxt_c)::value;
    constexpr int CS = decltype(cs_c)::value;
    constexpr int XS = decltype(xs_c)::value;
    constexpr bool Z = decltype(z_c)::value;
    const int X = t & 1, Y = X ^ 1;
#define G4_STEP(U)                                                                            \
  {                                                                                           \
    constexpr int s_ = (U) >> 6, i_ = ((U)&63) >> 3, j_ = (U)&7;                              \
    if constexpr (Z && s_ == 0) MFMA4Z(acc[i_][j_], b[s_][j_], a[s_][i_]);                   \
    else MFMA4(acc[i_][j_], b[s_][j_], a[s_][i_]);                                            \
    if constexpr (CS != 0 && (j_ & 1) == 0)                                                   \
      cs[i_] = frag_pair_sum<j_ / 2>(a[s_][i_], cs[i_], CS == 1 ? 0x3f803f80u : cs_w);         \
    if constexpr ((U) < 16 && ((U)&1)) b[1][(U) >> 1] = rdB(X, 1, (U) >> 1);                  \
    if constexpr ((U) == 19 && DMA) {                                                         \
      lgkm_wait0();                                                                           \
      __builtin_amdgcn_s_barrier();                                                           \
    }                                                                                         \
    if constexpr (DMA && (U) >= 21 && (U) < 53 && (((U)-21) & 3) == 0) dmaB(X, t + 2, ((U)-21) >> 2); \
    if constexpr ((U) >= 22 && (U) < 54 && (((U)-22) & 3) == 0) a[1][((U)-22) >> 2] = rdA(X, 1, ((U)-22) >> 2); \
    if constexpr ((U) == 55 && DMA) {                                                         \
      lgkm_wait0();                                                                           \
      __builtin_amdgcn_s_barrier();                                                           \
    }                                                                                         \
    if constexpr (DMA && (U) >= 56 && (U) < 72 && (((U)-56) & 3) == 0) dmaA(X, t + 2, ((U)-56) >> 2); \
    if constexpr ((U) == 71 && NXT) { /* B(t+1) landed */                                     \
      vm_wait_n<((DMA ? 20 : 8) + XS < 63 ? (DMA ? 20 : 8) + XS : 63)>();                   \
      __builtin_amdgcn_s_barrier();                                                           \
    }                                                                                         \
    if constexpr (NXT && (U) >= 72 && (U) < 104 && (((U)-72) & 3) == 1) b[0][((U)-72) >> 2] = rdB(Y, 0, ((U)-72) >> 2); \
    if constexpr (DMA && (U) >= 74 && (U) < 106 && (((U)-74) & 7) == 0) dmaA(X, t + 2, 4 + (((U)-74) >> 3)); \
    if constexpr ((U) == 107 && NXT) { /* A(t+1) landed */                                    \
      vm_wait_n<((DMA ? 16 : 0) + XS < 63 ? (DMA ? 16 : 0) + XS : 63)>();                   \
      __builtin_amdgcn_s_barrier();                                                           \
    }                                                                                         \
    if constexpr (NXT && (U) >= 108 && (U) < 124 && (((U)-108) & 1) == 0) a[0][((U)-108) >> 1] = rdA(Y, 0, ((U)-108) >> 1); \
  }
#define G4_S4(U) G4_STEP(U) G4_STEP((U) + 1) G4_STEP((U) + 2) G4_STEP((U) + 3)
#define G4_S16(U) G4_S4(U) G4_S4((U) + 4) G4_S4((U) + 8) G4_S4((U) + 12)
    G4_S16(0) G4_S16(16) G4_S16(32) G4_S16(48) G4_S16(64) G4_S16(80) G4_S16(96) G4_S16(112)
#undef G4_S16
#undef G4_S4
#undef G4_STEP
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using C0 = std::integral_constant<int, 0>;
  // CSA: tile column c of a tile row sums the A rows over its share [cs_lo, cs_hi) of the main
  // loop's K-tiles, and the last column the final two K-tiles (weight cs_w) — the row-sum VALU
  // spread over the tile columns (every tile summing every fragment slowed the split-K weight
  // gradient 12%: VALU issue is not hidden under the MFMAs).  Each range runs as its own loop:
  // choosing the K-tile instance by a branch per K-tile spilled ~1200 VGPRs.
  using C1 = std::integral_constant<int, CSA ? 1 : 0>;
  using C2 = std::integral_constant<int, CSA ? 2 : 0>;
  offsets(tc, 0);
  prologue();
  // VM instructions the previous tile's epilogue issued AFTER this tile's prologue DMA, at
  // least (whole tiles: 32 row stores per wave): the first wait may leave them in flight
  constexpr int EPI_VM = EPI == MMPT_EPI_BF16 || EPI == MMPT_EPI_F32_RESID ||
                                 EPI == MMPT_EPI_F32_STORE || EPI == MMPT_EPI_F32_ACC ||
                                 EPI == EPI_SPLIT
                             ? 32
                             : 0;
  // fast epilogue (epilogue4f): K-tile 1's A pieces of the next tile are issued after it (its
  // LDS image is the staging area), so the next tile's first wait may leave in flight: K-tile
  // 1's B pieces (8), at least epi4_fast_vm stores / loads, K-tile 1's A pieces (8)
  constexpr bool FAST = epi4_fast<EPI_>();
  constexpr int FAST_VM = 16 + epi4_fast_vm<EPI_>() < 63 ? 16 + epi4_fast_vm<EPI_>() : 63;
  constexpr bool DG = EPI == MMPT_EPI_BF16_DGELU || EPI == MMPT_EPI_BF16_DGELU_COLSUM;
  bool relax = false;
  for (int it = 1;; ++it) {
    // K-tile 0 of this tile landed (K-tile 1's 16 pieces, and the epilogue stores of the
    // previous tile when `relax`, may stay in flight)
    if (nk > 1) {
      if constexpr (STG) {  // K-tile 1's B and A pieces (16) are older than the stores
        if (relax && (MMPT_GEMM_STG_RELAX & 1)) vm_wait_n<FAST_VM>();
        else vm_wait_n<16>();
      } else if constexpr (FAST) {
        if (relax) vm_wait_n<FAST_VM>();
        else vm_wait_n<8>();
      } else {
        if (EPI_VM > 0 && relax) vm_wait_n<16 + EPI_VM>();
        else vm_wait_n<16>();
      }
    } else {
      vm_wait_n<0>();
    }
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) a[0][i] = rdA(0, 0, i);
#pragma unroll
    for (int j = 0; j < 8; ++j) b[0][j] = rdB(0, 0, j);
    if constexpr (CSA) {
#pragma unroll
      for (int i = 0; i < 8; ++i) cs[i] = 0.f;
      const int col = tc.n0 / 256, nm = nk - 2 > 0 ? nk - 2 : 0;  // main-loop K-tiles
      cs_lo = (int)((long)nm * col / p.tiles_n);
      cs_hi = (int)((long)nm * (col + 1) / p.tiles_n);
      cs_w = col == p.tiles_n - 1 ? 0x3f803f80u : 0u;
    }
    using X0 = std::integral_constant<int, 0>;
    using XE = std::integral_constant<int, epi4_fast_vm<EPI_>()>;
    int t0 = 0;
    if constexpr (STG) {
      // No accumulator zeroing here: the tile's first K-tile runs its k-half-0 MFMAs with srcC
      // = 0.  (A C++ zeroing that hipcc sank next to an MFMA in the peeled first K-tile lacked
      // the VALU-write -> MFMA-srcC wait states — the MFMAs are inline asm, invisible to its
      // hazard recognizer — and gave wrong tiles.)
      if ((MMPT_GEMM_STG_RELAX & 2) && relax && nk > 2) {  // the previous stores in flight
        ktile(0, T_{}, T_{}, XE{}, T_{}, C0{});
      } else if ((MMPT_GEMM_STG_RELAX & 2) && relax && nk == 2) {
        ktile(0, F_{}, T_{}, XE{}, T_{}, C0{});
      } else if (nk > 2) {
        ktile(0, T_{}, T_{}, X0{}, T_{}, C0{});
      } else if (nk == 2) {
        ktile(0, F_{}, T_{}, X0{}, T_{}, C0{});
      }
      t0 = nk >= 2 ? 1 : 0;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (CSA) {
      int t = t0;
      for (; t < cs_lo; ++t) ktile(t, T_{}, T_{}, X0{}, F_{}, C0{});
      for (; t < cs_hi; ++t) ktile(t, T_{}, T_{}, X0{}, F_{}, C1{});
      for (; t + 2 < nk; ++t) ktile(t, T_{}, T_{}, X0{}, F_{}, C0{});
    } else {
      for (int t = t0; t + 2 < nk; ++t) ktile(t, T_{}, T_{}, X0{}, F_{}, C0{});
    }
    if (nk >= 2 && nk - 2 >= t0) ktile(nk - 2, F_{}, T_{}, X0{}, F_{}, C2{});
    // the fast epilogue's operands load under the last K-tile (no LDS-DMA is in flight there)
    const bool fast = FAST;  // (the launch guarantees its alignment / N % 8 conditions)
    uint4 qb[4], qa[3][4], qu[3][4], qra[2][4];
    float4 qrc[2][4][2];
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      qb[y] = uint4{0u, 0u, 0u, 0u};
      qa[0][y] = qa[1][y] = qa[2][y] = uint4{0u, 0u, 0u, 0u};
      qu[0][y] = qu[1][y] = qu[2][y] = uint4{0u, 0u, 0u, 0u};
      qra[0][y] = qra[1][y] = uint4{0u, 0u, 0u, 0u};
      qrc[0][y][0] = qrc[0][y][1] = qrc[1][y][0] = qrc[1][y][1] = float4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (FAST) {
      if (fast) {
        const int nq = tc.n0 + wn * 128 + ((lane >> 4) & 1) * 16 + (lane >> 5) * 8;
        if constexpr (EPI == MMPT_EPI_BF16_DSWIGLU) {  // row group 0's gate / up values
          const long m = min(tc.m0 + wm * 128 + (lane & 15), p.M - 1);
          const int gbc = (min(tc.n0 + wn * 128, p.N - 128) >> 7) * 256;
          const int cl = ((lane >> 4) & 1) * 16 + (lane >> 5) * 8;
#pragma unroll
          for (int y = 0; y < 4; ++y) {
            qa[0][y] = *(const uint4*)(p.aux + m * p.ld_aux + gbc + cl + 32 * y);
            qu[0][y] = *(const uint4*)(p.aux + m * p.ld_aux + gbc + 128 + cl + 32 * y);
          }
        } else if constexpr (!DG) {
          if (p.bias != nullptr) {
#pragma unroll
            for (int y = 0; y < 4; ++y) qb[y] = *(const uint4*)(p.bias + min(nq + 32 * y, p.N - 8));
          }
          if constexpr (EPI == MMPT_EPI_F32_RESID)
            res_load(p, tc.m0 + wm * 128 + (lane >> 4), tc.n0 + wn * 128 + (lane & 15) * 8, qra[0], qrc[0]);
        } else {
#pragma unroll
          for (int r = 0; r < epi4_aux_pd<EPI_>(); ++r) {
            const long m = min(tc.m0 + wm * 128 + (lane & 15) + 16 * r, p.M - 1);
#pragma unroll
            for (int y = 0; y < 4; ++y)
              qa[r][y] = *(const uint4*)(p.aux + m * p.ld_aux + min(nq + 32 * y, p.N - 8));
          }
        }
      }
    }
    if (STG && nk == 1) ktile(0, F_{}, F_{}, X0{}, std::integral_constant<bool, STG>{}, C0{});
    else ktile(nk - 1, F_{}, F_{}, X0{}, F_{}, C2{});
    if constexpr (FAST) {
      // wait for those loads HERE, before the next tile's DMA: hipcc does not see the asm
      // LDS-DMA, and its wait at their first use would drain the DMA as well
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        asm volatile("" ::"v"(qb[y].x), "v"(qb[y].y), "v"(qb[y].z), "v"(qb[y].w));
        asm volatile("" ::"v"(qa[0][y].x), "v"(qa[0][y].y), "v"(qa[0][y].z), "v"(qa[0][y].w));
        asm volatile("" ::"v"(qa[1][y].x), "v"(qa[1][y].y), "v"(qa[1][y].z), "v"(qa[1][y].w));
        asm volatile("" ::"v"(qu[0][y].x), "v"(qu[0][y].y), "v"(qu[0][y].z), "v"(qu[0][y].w));
        asm volatile("" ::"v"(qra[0][y].x), "v"(qra[0][y].y), "v"(qra[0][y].z), "v"(qra[0][y].w));
        asm volatile("" ::"v"(qrc[0][y][0].x), "v"(qrc[0][y][0].y), "v"(qrc[0][y][0].z), "v"(qrc[0][y][0].w));
        asm volatile("" ::"v"(qrc[0][y][1].x), "v"(qrc[0][y][1].y), "v"(qrc[0][y][1].z), "v"(qrc[0][y][1].w));
      }
    }
    if constexpr (CSA) {
      // the four lane groups hold k quarters of the same rows: fixed-order butterfly, then the
      // first 16 lanes of the wn = 0 waves store the partial row (split, tile column)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        cs[i] += __shfl_xor(cs[i], 16);
        cs[i] += __shfl_xor(cs[i], 32);
      }
      if (wn == 0 && lane < 16) {
        float* dst = (float*)p.C2 + (long)(tc.split * p.tiles_n + tc.n0 / 256) * p.ldc2;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = tc.m0 + wm * 128 + 16 * i + lane;
          if (m < p.M) dst[m] = cs[i];
        }
      }
    }
    // every wave is past its last fragment read: the next tile's prologue DMA runs under this
    // tile's epilogue
    const TileCoord cur = tc;
    w = work_id(nwg, it);
    if constexpr (FAST) {
      lgkm_wait0();
      __builtin_amdgcn_s_barrier();  // buffer 1 (the staging area) is free
      if (w >= 0) {
        tc = coord_of(p, w, 256, 256);
        offsets(tc, it);
#pragma unroll
        for (int q = 0; q < 8; ++q) dmaB(0, 0, q);
#pragma unroll
        for (int q = 0; q < 8; ++q) dmaA(0, 0, q);
        if (nk > 1) {
#pragma unroll
          for (int q = 0; q < 8; ++q) dmaB(1, 1, q);
          if constexpr (STG) {
#pragma unroll
            for (int q = 0; q < 8; ++q) dmaA(1, 1, q);
          }
        }
      }
      epilogue4f<EPI_>(p, acc, cur.m0, cur.n0, lane, wm, wn, lut,
                       smem + (STG ? 4 : 2) * IMG + wave * 8192, qb, qa, qu, qra, qrc);
      if (w < 0) break;
      if constexpr (!STG) {
        if (nk > 1) {
          lgkm_wait0();
          __builtin_amdgcn_s_barrier();  // every wave's staging reads are done
#pragma unroll
          for (int q = 0; q < 8; ++q) dmaA(1, 1, q);
        }
      }
      // whole tiles issue every store (the count the next wait leaves in flight); an edge tile
      // may skip some, so its successor waits for everything but K-tile 1's A pieces
      relax = cur.m0 + 256 <= p.M && cur.n0 + 256 <= p.N;
    } else {
      if (w >= 0) {
        tc = coord_of(p, w, 256, 256);
        offsets(tc, it);
        lgkm_wait0();
        __builtin_amdgcn_s_barrier();
        prologue();
      }
      epilogue4w<EPI_>(p, acc, cur.m0, cur.n0, cur.split, lane, wm, wn, lut);
      if (w < 0) break;
      relax = p.wide && cur.m0 + 256 <= p.M && cur.n0 + 256 <= p.N;
    }
  }
}
// the two entry points (rocprofv3 names them gemm4p_kernel<LA, LB, EPI> / gemm4p_kt_kernel<...>)
template <int LA, int LB, int EPI_>
__global__ __launch_bounds__(256, 1) void gemm4p_kernel(GemmParams p) {
  gemm4p_body<LA, LB, EPI_, false>(p);
}
template <int LA, int LB, int EPI_>
__global__ __launch_bounds__(256, 1) void gemm4p_kt_kernel(GemmParams p) {
  gemm4p_body<LA, LB, EPI_, true>(p);
}
#undef MFMA4
#undef MFMA4Z

int persistent_slots();  // (below) workgroups of a persistent launch

// big-tile kernel switch, read once: MMPT_GEMM_4P=1 (default, see uses_4p), 0 = gemm128 for
// every problem (A/B only; the 8-wave gemm256 kernel of rounds 1-3, this switch's 0 arm until
// round 5, is retired)
int g_gemm_4p = -1;
int gemm_4p() {
  if (g_gemm_4p < 0) {
    const char* e = getenv("MMPT_GEMM_4P");
    g_gemm_4p = e == nullptr ? 1 : atoi(e);
  }
  return g_gemm_4p;
}
// The persistent walk (round 5).  At any time an XCD's 32 CUs hold 32 consecutive work ids:
// GROUP tile rows x 32/GROUP tile columns, whose A / B K-slices they share through the XCD's
// L2; over the launch, A is fetched from beyond L2 once per column block and B once per row
// block.  A (the activations, up to GBs) streams from HBM; B (a weight, <= 200 MB) mostly
// stays in the Infinity Cache.  Measured at T = 180,992 (profiles/r05/walk/): N <= 2048
// (8 tile columns: the dX GEMMs, the N = 2048 forwards, the weight gradients) run best with
// GROUP = 2 (the block spans every column, A is read once) — +6..8% over round 4's GROUP = 8;
// wider N with GROUP = 4 (+0.5..1.5%).  KREV: a workgroup's odd tiles walk K last-to-first,
// so the A K-slices the previous tile round left in L2 are read first (qkv forward: -16%
// L2->fabric bytes), measured +0..0.8% on the wide-N shapes and -2..4% on lm_head dX; NOT the
// default: it changes each odd tile's fp32 summation order, hence the step's rounding (the C5
// ZeRO-3 + offload gradient norm moved by 2.4 sigma of its bf16 noise, past its parity bar),
// while GROUP only changes which CU computes a tile — bitwise the round-4 results.
// Overrides (A/B): MMPT_GEMM_GROUP=<rows>, MMPT_GEMM_KREV=0/1; read once.
int g_gemm_group = -1, g_gemm_krev = -1;  // 0 = automatic (group), 2 = automatic (krev)
int gemm_group_env() {
  if (g_gemm_group < 0) {
    const char* e = getenv("MMPT_GEMM_GROUP");
    const int v = e == nullptr ? 0 : atoi(e);
    g_gemm_group = v >= 1 && v <= 64 ? v : 0;
  }
  return g_gemm_group;
}
int gemm_krev() {
  if (g_gemm_krev < 0) {
    const char* e = getenv("MMPT_GEMM_KREV");
    g_gemm_krev = e == nullptr ? 2 : (e[0] == '1' ? 1 : 0);
  }
  return g_gemm_krev;
}
int walk_group(int tiles_n) {
  const int g = gemm_group_env();
  return g > 0 ? g : (tiles_n <= 8 ? 2 : 4);
}
int walk_krev(int tiles_n) {
  const int k = gemm_krev();
  (void)tiles_n;
  return k < 2 ? k : 0;
}
// the forms gemm4p runs by default whatever the fast path: plain, residual, the fp32 ones and,
// since round 5, the dQGELU (CLIP) and dSwiGLU (Llama) backward forms (general epilogue)
constexpr bool epi_4p_default(int e) {
  return e == MMPT_EPI_BF16 || e == MMPT_EPI_F32_RESID || e == MMPT_EPI_F32_ACC ||
         e == MMPT_EPI_F32_STORE || e == MMPT_EPI_BF16_DQGELU ||
         e == MMPT_EPI_BF16_DQGELU_COLSUM || e == MMPT_EPI_BF16_DSWIGLU;
}
// gemm4p runs a big-tile problem when the operands are both K-contiguous or both
// row-contiguous (the weight-gradient form, split-K included) and K is a whole number of
// K-tiles (every split too: kchunk is a multiple of 64).  epi = the launch epilogue
// (quick-GELU forms included, EPI_SPLIT for split-K slabs).  Default (1): every epilogue with
// the fast whole-tile path (plain, erf-GELU, erf-dGELU (+ column sums), and since round 5 the
// quick-GELU and SwiGLU forwards from their tables) and the general-path ones above (fp32
// residual / accumulate / store, split-K slabs, dQGELU, dSwiGLU): +5..10% over round 4's
// 8-wave kernel at the model shapes (profiles/r04/gemm4p_ab/fast_epilogue_T180992.txt,
// profiles/r05/act4p/).  Everything else runs gemm128.
// The epilogues with the fast whole-tile path (epilogue4f) need 16-B aligned outputs and
// operands (`aligned` = GemmParams::wide) and N % 8 == 0.
constexpr bool epi_4p_fast(int e) {
  return MMPT_GEMM_4P_FAST && (e == MMPT_EPI_BF16 || e == MMPT_EPI_F32_RESID ||
                               (MMPT_GEMM_LUT && (e == MMPT_EPI_BF16_GELU || e == MMPT_EPI_BF16_DGELU ||
                                                  e == MMPT_EPI_BF16_DGELU_COLSUM ||
                                                  e == MMPT_EPI_BF16_QGELU ||
                                                  e == MMPT_EPI_BF16_SWIGLU ||
                                                  e == MMPT_EPI_BF16_DSWIGLU)));
}
// the forms with a K-tail (KT) instantiation: weight gradients (K_ROWS x K_ROWS, fp32 accumulate /
// store / split-K slabs) and the plain forward (the CLIP patch embedding, K = 3 x 14 x 14)
bool kt_form(int la, int epi) {
  return la == MMPT_K_ROWS ? (epi == MMPT_EPI_F32_ACC || epi == MMPT_EPI_F32_STORE || epi == EPI_SPLIT ||
                              epi == MMPT_EPI_F32_ACC_COLSUM || epi == EPI_SPLIT_CS)
                           : epi == MMPT_EPI_BF16;
}
bool uses_4p(bool big, int la, int lb, int epi, int splits, int64_t N, int64_t K, bool aligned) {
  const int g4 = gemm_4p();
  (void)splits;
  if (epi == MMPT_EPI_F32_ACC_COLSUM || epi == EPI_SPLIT_CS)  // (K-tail form since round 6)
    return g4 != 0 && big && la == MMPT_K_ROWS && lb == MMPT_K_ROWS;
  if (!big || la != lb || (K % BK != 0 && !kt_form(la, epi))) return false;
  if (epi_4p_fast(epi) && !(aligned && N % 8 == 0)) return false;
  if (epi == MMPT_EPI_BF16_SWIGLU && !epi_4p_fast(epi)) return false;  // no general-path form
  if ((epi == MMPT_EPI_BF16_SWIGLU || epi == MMPT_EPI_BF16_DSWIGLU) && la != MMPT_ROWS_K)
    return false;  // built for the model's K-contiguous operands only
  return g4 != 0 && (epi_4p_default(epi) || epi_4p_fast(epi) || epi == EPI_SPLIT);
}

// The kernel the calling thread's last mmpt_gemm_bf16 launched (mmpt_gemm_last_kernel_name):
// the choice depends on the operands' alignment, which a shape-only query cannot see.
thread_local char g_last_kernel[64] = "";

// G4: the big-tile kernel gemm4p (the caller checked uses_4p), else gemm128 (small problems, and
// the big ones gemm4p does not take: mixed layouts, unaligned operands, K tails outside kt_form)
template <bool G4, int LA, int LB>
int launch_epi(int epi, const GemmParams& p, dim3 grid, hipStream_t s) {
  if constexpr (G4) {
    if constexpr (LA == LB) {
      snprintf(g_last_kernel, sizeof g_last_kernel, "gemm4p_kernel<%d, %d, %d>", LA, LB, epi);
      const int nwg = p.tiles_m * p.tiles_n * p.splits, slots = persistent_slots();
      const dim3 grid4(slots > 0 && nwg > slots ? slots : nwg);  // persistent: one WG per CU
      if (p.K % BK != 0) {  // K tail (kt_form)
        snprintf(g_last_kernel, sizeof g_last_kernel, "gemm4p_kt_kernel<%d, %d, %d>", LA, LB, epi);
        if constexpr (LA == MMPT_K_ROWS) {
          switch (epi) {
            case MMPT_EPI_F32_ACC:
              gemm4p_kt_kernel<LA, LB, MMPT_EPI_F32_ACC><<<grid4, 256, 0, s>>>(p);
              return check_launch("gemm4p");
            case MMPT_EPI_F32_STORE:
              gemm4p_kt_kernel<LA, LB, MMPT_EPI_F32_STORE><<<grid4, 256, 0, s>>>(p);
              return check_launch("gemm4p");
            case EPI_SPLIT:
              gemm4p_kt_kernel<LA, LB, EPI_SPLIT><<<grid4, 256, 0, s>>>(p);
              return check_launch("gemm4p");
            // the fused bias-gradient row sums at token counts K % 64 != 0 (round 6): the last
            // K-tile's pieces past K read zeros, which add nothing to the sums
            case MMPT_EPI_F32_ACC_COLSUM:
              gemm4p_kt_kernel<LA, LB, MMPT_EPI_F32_ACC_COLSUM><<<grid4, 256, 0, s>>>(p);
              return check_launch("gemm4p");
            case EPI_SPLIT_CS:
              gemm4p_kt_kernel<LA, LB, EPI_SPLIT_CS><<<grid4, 256, 0, s>>>(p);
              return check_launch("gemm4p");
            default: break;
          }
        } else if (epi == MMPT_EPI_BF16) {
          gemm4p_kt_kernel<LA, LB, MMPT_EPI_BF16><<<grid4, 256, 0, s>>>(p);
          return check_launch("gemm4p");
        }
        set_error("gemm: no K-tail form of epilogue %d", epi);
        return MMPT_ERR_ARG;
      }
      switch (epi) {
#define MMPT_CASE4(E) \
  case E: gemm4p_kernel<LA, LB, E><<<grid4, 256, 0, s>>>(p); return check_launch("gemm4p");
        MMPT_CASE4(MMPT_EPI_BF16)
        MMPT_CASE4(MMPT_EPI_BF16_GELU)
        MMPT_CASE4(MMPT_EPI_BF16_DGELU)
        MMPT_CASE4(MMPT_EPI_BF16_DGELU_COLSUM)
        MMPT_CASE4(MMPT_EPI_BF16_QGELU)
        MMPT_CASE4(MMPT_EPI_BF16_DQGELU)
        MMPT_CASE4(MMPT_EPI_BF16_DQGELU_COLSUM)
        MMPT_CASE4(MMPT_EPI_F32_ACC)
        MMPT_CASE4(MMPT_EPI_F32_STORE)
        MMPT_CASE4(MMPT_EPI_F32_RESID)
        MMPT_CASE4(EPI_SPLIT)
#undef MMPT_CASE4
        case MMPT_EPI_BF16_SWIGLU:  // (the model's layout only: x · W^T, both K-contiguous)
          if constexpr (LA == MMPT_ROWS_K) {
            gemm4p_kernel<LA, LB, MMPT_EPI_BF16_SWIGLU><<<grid4, 256, 0, s>>>(p);
            return check_launch("gemm4p");
          }
          break;
        case MMPT_EPI_BF16_DSWIGLU:
          if constexpr (LA == MMPT_ROWS_K) {
            gemm4p_kernel<LA, LB, MMPT_EPI_BF16_DSWIGLU><<<grid4, 256, 0, s>>>(p);
            return check_launch("gemm4p");
          }
          break;
        case MMPT_EPI_F32_ACC_COLSUM:  // (weight gradients: both operands [tokens][features])
          if constexpr (LA == MMPT_K_ROWS) {
            gemm4p_kernel<LA, LB, MMPT_EPI_F32_ACC_COLSUM><<<grid4, 256, 0, s>>>(p);
            return check_launch("gemm4p");
          }
          break;
        case EPI_SPLIT_CS:
          if constexpr (LA == MMPT_K_ROWS) {
            gemm4p_kernel<LA, LB, EPI_SPLIT_CS><<<grid4, 256, 0, s>>>(p);
            return check_launch("gemm4p");
          }
          break;
        default: break;
      }
    }
    set_error("gemm: no gemm4p form of epilogue %d at layouts %d / %d", epi, LA, LB);
    return MMPT_ERR_ARG;
  } else {
    snprintf(g_last_kernel, sizeof g_last_kernel, "gemm128_kernel<%d, %d, %d>", LA, LB, epi);
    switch (epi) {
#define MMPT_CASE(E) \
  case E: gemm128_kernel<LA, LB, E><<<grid, 256, 0, s>>>(p); break;
      MMPT_CASE(MMPT_EPI_BF16)
      MMPT_CASE(MMPT_EPI_BF16_GELU)
      MMPT_CASE(MMPT_EPI_BF16_DGELU)
      MMPT_CASE(MMPT_EPI_BF16_DGELU_COLSUM)
      MMPT_CASE(MMPT_EPI_BF16_QGELU)
      MMPT_CASE(MMPT_EPI_BF16_DQGELU)
      MMPT_CASE(MMPT_EPI_BF16_DQGELU_COLSUM)
      MMPT_CASE(MMPT_EPI_F32_ACC)
      MMPT_CASE(MMPT_EPI_F32_STORE)
      MMPT_CASE(MMPT_EPI_F32_RESID)
      MMPT_CASE(MMPT_EPI_BF16_DSWIGLU)
      MMPT_CASE(EPI_SPLIT)
#undef MMPT_CASE
      case MMPT_EPI_BF16_SWIGLU:
        set_error("gemm: the SWIGLU epilogue runs on gemm4p only (K %% 64 == 0, K-contiguous "
                  "operands, 16-B aligned rows)");
        return MMPT_ERR_ARG;
      case MMPT_EPI_F32_ACC_COLSUM:
      case EPI_SPLIT_CS:
        set_error("gemm: F32_ACC_COLSUM runs on gemm4p only (mmpt_gemm_acc_colsum_rows)");
        return MMPT_ERR_UNSUPPORTED;
      default: set_error("gemm: unknown epilogue %d", epi); return MMPT_ERR_ARG;
    }
    return check_launch("gemm");
  }
}

template <bool G4>
int launch_layouts(int la, int lb, int epi, const GemmParams& p, dim3 grid, hipStream_t s) {
  if (la == MMPT_ROWS_K && lb == MMPT_ROWS_K) return launch_epi<G4, MMPT_ROWS_K, MMPT_ROWS_K>(epi, p, grid, s);
  if (la == MMPT_ROWS_K && lb == MMPT_K_ROWS) return launch_epi<G4, MMPT_ROWS_K, MMPT_K_ROWS>(epi, p, grid, s);
  if (la == MMPT_K_ROWS && lb == MMPT_K_ROWS) return launch_epi<G4, MMPT_K_ROWS, MMPT_K_ROWS>(epi, p, grid, s);
  return launch_epi<G4, MMPT_K_ROWS, MMPT_ROWS_K>(epi, p, grid, s);
}

constexpr int NUM_CUS = 256;

// MMPT_GEMM_TILE=128: every GEMM on the 128x128 kernel (A/B measurements only)
bool force_tile128() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MMPT_GEMM_TILE");
    v = e != nullptr && atoi(e) == 128;
  }
  return v == 1;
}

// MMPT_GEMM_SPLITS=s: weight-gradient GEMMs on 256^2 tiles in s K-splits (A/B measurements only)
int force_splits() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MMPT_GEMM_SPLITS");
    v = e != nullptr ? atoi(e) : 0;
    if (v < 0 || v > 16) v = 0;
  }
  return v;
}

// Non-split problems run 256^2 tiles from 128 of them on (half the CUs, one wave): at 150-225
// tiles gemm4p beats the two 128^2 waves (ViT qkv 6304x2304x768 25.5 vs 36.9 us, fc2
// 12608x768x3072 73.7 vs 107.7 us), at 75 it loses (19.2 -> 21.5 us); per-rank 32 / 64 steps
// +0.2% / +0.45% (profiles/r06/bigmin/).  MMPT_GEMM_BIG_MIN=t overrides (A/B measurements only).
int64_t big_min_tiles() {
  static int64_t v = -1;
  if (v < 0) {
    const char* e = getenv("MMPT_GEMM_BIG_MIN");
    v = e != nullptr && atoi(e) > 0 ? atoi(e) : 128;
  }
  return v;
}

struct Plan {
  bool big;   // 256x256 tile
  int splits;
  int kchunk;
};

Plan plan(int64_t M, int64_t N, int64_t K, int epi) {
  Plan pl{};
  const int64_t t256 = ((M + 255) / 256) * ((N + 255) / 256);
  const int64_t t128 = ((M + 127) / 128) * ((N + 127) / 128);
  pl.big = t256 >= big_min_tiles() || epi == MMPT_EPI_BF16_SWIGLU;  // SWIGLU pairs 128-col quadrants
  if (force_tile128() && epi != MMPT_EPI_BF16_SWIGLU) pl.big = false;  // A/B only
  pl.splits = 1;
  pl.kchunk = (int)K;
  const bool splittable = epi == MMPT_EPI_F32_ACC || epi == MMPT_EPI_F32_STORE ||
                          epi == MMPT_EPI_F32_ACC_COLSUM;  // (the same plan as F32_ACC)
  if (splittable) {
    // weight gradients: K = tokens. Pick (tile, splits) minimising the padded wave
    // count ceil(blocks / slots) / blocks-work, slots = 256 (256^2, 1 per CU) or
    // 512 (128^2, 2 per CU); keep >= 1024 k per split and <= 16 splits (<= 2 from 512 tiles).
    // Model: a CU fully busy with one 256^2 block retires 4 128^2-tile units in 4 time
    // units; with two 128^2 blocks it retires 2 units in 2.67 (128^2 runs at ~0.75x the
    // 256^2 rate).  Slab write+read adds sp*8 B per output element vs 2K flops per
    // element: factor (1 + sp*800/K) at ~5 TB/s : ~1 PF/s.
    double best = 1e30;
    for (int big = 1; big >= 0; --big) {
      const int64_t tiles = big ? t256 : t128;
      const int64_t slots = big ? NUM_CUS : 2 * NUM_CUS;
      const double wave_cost = big ? 4.0 : 2.67;
      // (many tiles: up to 4 splits, which evens out the last wave — lm_head's weight
      // gradient, 1576 tiles = 6.2 rounds of 256, runs 25 rounds of a quarter of the K:
      // 1108 / 1141 / 1149 / 1165 TF/s at 1 / 2 / 3 / 4 splits, profiles/r04/d80/)
      const int64_t max_sp = tiles < 2 * slots ? 16 : 4;
      for (int64_t sp = 1; sp <= max_sp && (sp == 1 || K / sp >= 1024); ++sp) {
        const int64_t blocks = tiles * sp;
        const double waves = (double)((blocks + slots - 1) / slots);
        const double cost = waves * wave_cost / (double)sp *
                            (sp > 1 ? 1.0 + (double)sp * 800.0 / (double)K : 1.0);
        if (cost < best - 1e-9) {
          best = cost;
          pl.big = big;
          pl.splits = (int)sp;
        }
      }
    }
    if (force_splits() > 0) {
      pl.big = true;
      pl.splits = force_splits();
    }
    if (pl.splits > 1) {
      int64_t kc = (K + pl.splits - 1) / pl.splits;
      kc = (kc + BK - 1) / BK * BK;
      pl.splits = (int)((K + kc - 1) / kc);
      pl.kchunk = (int)kc;
    }
  }
  return pl;
}

// Tail split (round 5).  A persistent launch runs ceil(tiles / 256) rounds; the N = 2048 GEMMs
// of the step have 707 x 8 = 5656 tiles = 22 rounds + 24 tiles, so one CU in ten works through a
// 23rd tile (up to ~0.2 ms at K = 8192) while the rest wait.  Instead the bottom `rows` tile rows
// — the fewest that leave a whole number of rounds above them — run as a split-K GEMM over
// ~all CUs (fp32 slabs in the caller's workspace) and tail_epi_kernel applies the epilogue.
// Only for the fast plain / residual epilogues on gemm4p shapes with K >= 2048; the tail rows'
// fp32 sums run in split order (the other rows are bitwise unchanged).  MMPT_GEMM_TAIL=0: off.
struct TailPlan {
  int rows = 0;    // tail tile rows (0: no tail split)
  int splits = 0;  // K splits of the tail
  int kchunk = 0;
};
int g_gemm_tail = -1;
int gemm_tail() {
  if (g_gemm_tail < 0) {
    const char* e = getenv("MMPT_GEMM_TAIL");
    g_gemm_tail = e != nullptr && e[0] == '0' ? 0 : 1;
  }
  return g_gemm_tail;
}
int g_gemm_tail128 = -1;
bool gemm_tail128() {
  if (g_gemm_tail128 < 0) {
    const char* e = getenv("MMPT_GEMM_TAIL128");
    g_gemm_tail128 = e != nullptr && e[0] == '0' ? 0 : 1;
  }
  return g_gemm_tail128 == 1;
}
int persistent_slots();
TailPlan tail_plan(int la, int lb, int epi, int64_t M, int64_t N, int64_t K) {
  TailPlan t;
  if (!gemm_tail() || la != MMPT_ROWS_K || lb != MMPT_ROWS_K) return t;
  if (epi != MMPT_EPI_BF16 && epi != MMPT_EPI_F32_RESID) return t;
  if (K % BK != 0 || K < 2048 || N % 8 != 0) return t;
  const Plan pl = plan(M, N, K, epi);
  if (!pl.big || pl.splits != 1) return t;
  const int64_t slots = persistent_slots();
  if (slots <= 0) return t;
  const int64_t tm = (M + 255) / 256, tn = (N + 255) / 256;
  int64_t g = slots, b = tn;  // q = slots / gcd(tn, slots) tile rows make whole rounds
  while (b) {
    const int64_t r = g % b;
    g = b;
    b = r;
  }
  const int64_t q = slots / g;
  const int64_t rt = tm % q;
  if (rt == 0 || tm - rt < q) return t;
  // a tail of <= 128 rows runs on 128-row tiles (gemm128, see the launch) in up to 16 splits of
  // >= 2 K-tiles: its few rows make the slabs small (16 x 16 x 2048 fp32 = 2 MiB at C2's shape)
  const bool small = M - (tm - rt) * 256 <= 128 && gemm_tail128();
  const int64_t tail_tiles = small ? (N + 127) / 128 : rt * tn;
  int64_t sp = slots / tail_tiles;
  sp = std::min<int64_t>(sp, 16);
  sp = std::min<int64_t>(sp, K / BK / (small ? 2 : 8));  // >= 8 (2) K-tiles per split
  if (sp < 2) return t;
  int64_t kc = (K / sp + BK - 1) / BK * BK;
  t.rows = (int)rt;
  t.splits = (int)((K + kc - 1) / kc);
  t.kchunk = (int)kc;
  return t;
}
// Weight-gradient tail split (round 6).  The planner splits a weight-gradient GEMM's K over all
// of its tiles when they make a partial round (C5's fc1 dW: 400 tiles = 1.56 rounds, 5 splits),
// so every tile pays the fp32 slab write + reduce — measured ~4% of the GEMM per split at K =
// 69,568 (scripts/diag/p28_dw_splits.sh), 3x the planner's slab term.  Instead the whole rounds'
// tile rows (or columns) run unsplit, straight into C, and only the rest is split: fc1 dW 1.91
// -> ~1.69 full-K rounds.  F32_ACC / F32_STORE / F32_ACC_COLSUM on 256^2 tiles (the fused row
// sums: a row tail's rows get one partial row per split there, the unsplit rows one; a column
// tail leaves the sums to the unsplit columns, which cover all of K).  The main part's fp32
// sums run in one pass, the tail's in split order (as before).
// MMPT_GEMM_WTAIL=0: off; 2: tail tile columns only (tests).
struct WTail {
  int dim = 0;     // 0: none, 1: tail tile rows (M), 2: tail tile columns (N)
  int lines = 0;   // whole tile rows / columns of the unsplit part
  int splits = 0;
  int kchunk = 0;
};
int g_gemm_wtail = -1;
int gemm_wtail() {
  if (g_gemm_wtail < 0) {
    const char* e = getenv("MMPT_GEMM_WTAIL");
    g_gemm_wtail = e != nullptr && e[0] == '0' ? 0 : e != nullptr && e[0] == '2' ? 2 : 1;
  }
  return g_gemm_wtail;
}
constexpr double SLAB_K = 2000.0;  // measured slab cost per split, in K units (p28 dW sweep)
WTail wtail_plan(int epi, int64_t M, int64_t N, int64_t K) {
  WTail w;
  if (!gemm_wtail() || (epi != MMPT_EPI_F32_ACC && epi != MMPT_EPI_F32_STORE &&
                        epi != MMPT_EPI_F32_ACC_COLSUM))
    return w;
  const Plan pl = plan(M, N, K, epi);
  if (!pl.big || pl.splits < 2 || force_splits() > 0) return w;
  const int64_t slots = 256, tm = (M + 255) / 256, tn = (N + 255) / 256, tiles = tm * tn;
  const int64_t rounds = tiles / slots;
  if (rounds < 1) return w;
  auto split_cost = [&](int64_t t, int64_t sp) {
    return (double)((t * sp + slots - 1) / slots) / (double)sp * (1.0 + (double)sp * SLAB_K / (double)K);
  };
  double best = split_cost(tiles, pl.splits) * 0.97;  // the planner's split, 3% margin
  for (int dim = gemm_wtail() == 2 ? 2 : 1; dim <= 2; ++dim) {
    const int64_t nl = dim == 1 ? tm : tn, other = dim == 1 ? tn : tm;
    const int64_t lines = rounds * slots / other;
    if (lines < 1 || lines >= nl) continue;
    const int64_t tt = (nl - lines) * other;
    for (int64_t sp = 2; sp <= 16 && K / sp >= 1024; ++sp) {
      const double c = (double)((lines * other + slots - 1) / slots) + split_cost(tt, sp);
      if (c < best - 1e-9) {
        best = c;
        w.dim = dim;
        w.lines = (int)lines;
        w.splits = (int)sp;
      }
    }
  }
  if (w.dim != 0) {
    int64_t kc = (K + w.splits - 1) / w.splits;
    kc = (kc + BK - 1) / BK * BK;
    w.splits = (int)((K + kc - 1) / kc);
    w.kchunk = (int)kc;
  }
  return w;
}
int64_t wtail_slab_bytes(int64_t M, int64_t N, const WTail& w) {
  if (w.dim == 0) return 0;
  const int64_t rows = w.dim == 1 ? M - (int64_t)w.lines * 256 : M;
  const int64_t cols = w.dim == 2 ? N - (int64_t)w.lines * 256 : N;
  return (int64_t)w.splits * rows * cols * (int64_t)sizeof(float);
}

int64_t tail_rows_of(int64_t M, const TailPlan& t) {  // matrix rows in the tail
  return M - (((M + 255) / 256) - t.rows) * 256;
}

thread_local hipEvent_t g_probe_event = nullptr;
thread_local int64_t g_last_tail_rows = 0;

// float -> bf16 round-to-nearest-even (finite values)
bf16_t host_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (bf16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
float host_bf16_f(float f) {
  const uint32_t u = (uint32_t)host_bf16(f) << 16;
  float r;
  memcpy(&r, &u, 4);
  return r;
}
// double -> bf16, correctly rounded: to float by round-to-odd (truncate, sticky bit into the
// last place), then float -> bf16 RNE — no double rounding
bf16_t host_bf16_d(double d) {
  float f = (float)d;
  if ((double)f != d) {
    if (std::fabs((double)f) > std::fabs(d)) f = std::nextafter(f, 0.0f);
    uint32_t u;
    memcpy(&u, &f, 4);
    u |= 1u;
    memcpy(&f, &u, 4);
  }
  return host_bf16(f);
}

// GELU / GELU' tables (see LUT_E0) and the quick-GELU / SiLU tables (round 5): built in double
// on the host, uploaded once per process and device (ordered on the first table-epilogue
// launch's stream)
int ensure_gelu_lut(hipStream_t s) {
  static bool uploaded[64] = {};  // per device (a `__device__` array exists once per device)
  static char host[3][LUT_BYTES];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    set_error("gemm: GELU table upload: no current device");
    return MMPT_ERR_UNSUPPORTED;
  }
  if (uploaded[dev]) return MMPT_OK;
  for (int sgn = 0; sgn < 2; ++sgn)
    for (int ei = 0; ei < LUT_NE; ++ei)
      for (int mnt = 0; mnt < 128; ++mnt) {
        const int k = (sgn * LUT_NE + ei) * 128 + mnt;
        const uint32_t bits = ((uint32_t)sgn << 15) | ((uint32_t)(ei + LUT_E0) << 7) | (uint32_t)mnt;
        float xf;
        const uint32_t xb = bits << 16;
        memcpy(&xf, &xb, 4);
        const double x = xf;
        // erf-GELU: bf16(x Φ(x)) (through float, as before) | fp32 Φ(x) + x φ(x)
        const double phi = 0.5 * erfc(-x / 1.4142135623730951);
        ((bf16_t*)host[0])[k] = host_bf16((float)(x * phi));
        ((float*)(host[0] + 2 * LUT_N))[k] = (float)(phi + x * exp(-0.5 * x * x) * 0.3989422804014327);
        // quick-GELU with autocast's roundings: t = bf16(1.702f x), s = bf16(sigmoid(t)),
        // y = bf16(x s) (x s is exact in float: two 8-bit significands)
        const float t = host_bf16_f(1.702f * xf);
        const bf16_t sb = host_bf16_d(1.0 / (1.0 + exp(-(double)t)));
        float sf;
        const uint32_t su = (uint32_t)sb << 16;
        memcpy(&sf, &su, 4);
        ((bf16_t*)host[1])[k] = host_bf16(xf * sf);
        ((float*)(host[1] + 2 * LUT_N))[k] = sf;
        // SiLU: bf16(x sigmoid(x)) | fp32 sigmoid(x)
        const double sig = 1.0 / (1.0 + exp(-x));
        ((bf16_t*)host[2])[k] = host_bf16_d(x * sig);
        ((float*)(host[2] + 2 * LUT_N))[k] = (float)sig;
      }
  const void* syms[3] = {HIP_SYMBOL(g_gelu_lut), HIP_SYMBOL(g_qgelu_lut), HIP_SYMBOL(g_silu_lut)};
  for (int i = 0; i < 3; ++i) {
    const hipError_t e = hipMemcpyToSymbolAsync(syms[i], host[i], LUT_BYTES, 0,
                                                hipMemcpyHostToDevice, s);
    if (e != hipSuccess) {
      set_error("gemm: GELU table upload: %s", hipGetErrorString(e));
      return (int)e;
    }
  }
  (void)hipStreamSynchronize(s);  // pageable source: complete before `host` is reused
  uploaded[dev] = true;
  return MMPT_OK;
}

// workgroups of a persistent gemm4p launch: the device's CU count rounded down to a
// multiple of 8 (whole XCDs); MMPT_GEMM_PERSIST=0 -> 0 (one workgroup per tile)
int persistent_slots() {
  static int slots = -1;
  if (slots < 0) {
    const char* e = getenv("MMPT_GEMM_PERSIST");
    int dev = 0, cus = NUM_CUS;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = NUM_CUS;
    slots = (e != nullptr && e[0] == '0') ? 0 : (cus / 8) * 8;
  }
  return slots;
}

}  // namespace
}  // namespace mmpt

using namespace mmpt;

extern "C" int64_t mmpt_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K, int epilogue) {
  const Plan pl = plan(M, N, K, epilogue);
  if (pl.splits > 1)  // (the weight-gradient tail split needs no more than the full split)
    return std::max((int64_t)pl.splits * M * N * (int64_t)sizeof(float),
                    wtail_slab_bytes(M, N, wtail_plan(epilogue, M, N, K)));
  // the tail split's slabs (ROWS_K x ROWS_K: the only layout the step's forward / dX GEMMs use)
  const TailPlan t = tail_plan(MMPT_ROWS_K, MMPT_ROWS_K, epilogue, M, N, K);
  return t.rows > 0 ? (int64_t)t.splits * tail_rows_of(M, t) * N * (int64_t)sizeof(float) : 0;
}

extern "C" int64_t mmpt_gemm_last_tail_rows(void) { return g_last_tail_rows; }

extern "C" int mmpt_gemm_plan(int64_t M, int64_t N, int64_t K, int epilogue, int64_t workspace_bytes,
                              int* tile, int* splits) {
  MMPT_REQUIRE(M > 0 && N > 0 && K > 0 && tile && splits, "gemm_plan: bad arguments");
  Plan pl = plan(M, N, K, epilogue);
  if (pl.splits > 1 && workspace_bytes < (int64_t)pl.splits * M * N * (int64_t)sizeof(float))
    pl.splits = 1;
  *tile = pl.big ? 256 : 128;
  *splits = pl.splits;
  return MMPT_OK;
}

extern "C" int mmpt_gemm_kernel_name(int layout_a, int layout_b, int epilogue, int64_t M,
                                     int64_t N, int64_t K, int64_t workspace_bytes, char* buf,
                                     int len) {
  MMPT_REQUIRE(M > 0 && N > 0 && K > 0 && buf && len > 0, "gemm_kernel_name: bad arguments");
  int tile = 0, splits = 0;
  const int rc = mmpt_gemm_plan(M, N, K, epilogue, workspace_bytes, &tile, &splits);
  if (rc) return rc;
  const int epi = splits > 1 ? (epilogue == MMPT_EPI_F32_ACC_COLSUM ? EPI_SPLIT_CS : EPI_SPLIT)
                             : epilogue;
  // (assumes 16-B aligned operands; mmpt_gemm_last_kernel_name reports the launch's own choice)
  if (uses_4p(tile == 256, layout_a, layout_b, epi, splits, N, K, true))
    snprintf(buf, (size_t)len, "gemm4p_kernel<%d, %d, %d>", layout_a, layout_b, epi);
  else
    snprintf(buf, (size_t)len, "gemm128_kernel<%d, %d, %d>", layout_a, layout_b, epi);
  return MMPT_OK;
}

namespace mmpt {
// mmpt_set_switch's GEMM slots (attention.hip): the switch's storage and its current value
int* gemm_switch(const char* name, int* prev) {
  if (strcmp(name, "MMPT_GEMM_KREV") == 0) {
    *prev = gemm_krev();
    return &g_gemm_krev;
  }
  if (strcmp(name, "MMPT_GEMM_TAIL") == 0) {
    *prev = gemm_tail();
    return &g_gemm_tail;
  }
  if (strcmp(name, "MMPT_GEMM_WTAIL") == 0) {
    *prev = gemm_wtail();
    return &g_gemm_wtail;
  }
  if (strcmp(name, "MMPT_GEMM_TAIL128") == 0) {
    *prev = gemm_tail128();
    return &g_gemm_tail128;
  }
  return nullptr;
}
}  // namespace mmpt

extern "C" int mmpt_gemm_last_kernel_name(char* buf, int len) {
  MMPT_REQUIRE(buf && len > 0, "gemm_last_kernel_name: bad arguments");
  snprintf(buf, (size_t)len, "%s", g_last_kernel);
  return MMPT_OK;
}

namespace mmpt {
namespace {
// column-sum partial rows: one per 128-row half tile of the kernel that runs (gemm4p: 256-row
// tiles; gemm128: 128-row).  The query answers for BOTH column-sum epilogues with 16-B aligned
// operands, K-contiguous: the larger count when the erf and quick forms would take different
// kernels (N % 8 != 0: the fast erf form needs it, the general quick form does not).
int64_t colsum_rows_written(int64_t M, int64_t N, int64_t K, int epi, bool aligned) {
  const Plan pl = plan(M, N, K, epi);
  const bool g4 = pl.big && uses_4p(true, MMPT_ROWS_K, MMPT_ROWS_K, epi, 1, N, K, aligned);
  const int64_t bm = g4 ? 256 : 128;
  return 2 * ((M + bm - 1) / bm);
}
int64_t colsum_rows_query(int64_t M, int64_t N, int64_t K) {
  return std::max(colsum_rows_written(M, N, K, MMPT_EPI_BF16_DGELU_COLSUM, true),
                  colsum_rows_written(M, N, K, MMPT_EPI_BF16_DQGELU_COLSUM, true));
}
}  // namespace
}  // namespace mmpt

extern "C" int64_t mmpt_gemm_colsum_rows(int64_t M, int64_t N, int64_t K) {
  return colsum_rows_query(M, N, K);
}

extern "C" int64_t mmpt_gemm_acc_colsum_rows(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const Plan pl = plan(M, N, K, MMPT_EPI_F32_ACC_COLSUM);
  const int e = pl.splits > 1 ? EPI_SPLIT_CS : MMPT_EPI_F32_ACC_COLSUM;
  // one partial row per (K split, 256-column tile): see gemm4p_body's CSA; the weight-gradient
  // tail split's row tail may run more splits than the plan
  const WTail w = pl.splits > 1 ? wtail_plan(MMPT_EPI_F32_ACC_COLSUM, M, N, K) : WTail{};
  const int64_t sp = std::max<int64_t>(pl.splits, w.dim == 1 ? w.splits : 1);
  return uses_4p(pl.big, MMPT_K_ROWS, MMPT_K_ROWS, e, pl.splits, N, K, true)
             ? sp * ((N + 255) / 256)
             : 0;
}

extern "C" void mmpt_gemm_probe_event(void* hip_event) { g_probe_event = (hipEvent_t)hip_event; }

extern "C" int mmpt_gemm_bf16(int layout_a, int layout_b, int epilogue, int64_t M, int64_t N,
                              int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb,
                              void* C, int64_t ldc, const void* bias_bf16, const void* aux_bf16,
                              int64_t ld_aux, void* C2, int64_t ldc2, void* workspace,
                              int64_t workspace_bytes, void* stream) {
  MMPT_REQUIRE(M > 0 && N > 0 && K > 0, "gemm: empty problem M=%lld N=%lld K=%lld",
               (long long)M, (long long)N, (long long)K);
  // quick-GELU variants are validated as their erf-GELU bases (same operands)
  const int launch_epilogue = epilogue;
  if (epilogue == MMPT_EPI_BF16_QGELU) epilogue = MMPT_EPI_BF16_GELU;
  else if (epilogue == MMPT_EPI_BF16_DQGELU) epilogue = MMPT_EPI_BF16_DGELU;
  else if (epilogue == MMPT_EPI_BF16_DQGELU_COLSUM) epilogue = MMPT_EPI_BF16_DGELU_COLSUM;
  // F32_ACC_COLSUM: F32_ACC's operands and plan, plus the row-sum partials in C2
  const bool acc_cs = epilogue == MMPT_EPI_F32_ACC_COLSUM;
  if (acc_cs) {
    MMPT_REQUIRE(layout_a == MMPT_K_ROWS && layout_b == MMPT_K_ROWS,
                 "gemm: F32_ACC_COLSUM needs K_ROWS operands");
    MMPT_REQUIRE(C2 != nullptr && ((uintptr_t)C2 & 15) == 0 && ldc2 >= M && ldc2 % 8 == 0,
                 "gemm: F32_ACC_COLSUM needs a 16-B aligned partial buffer C2 [rows][ldc2 >= M]");
    epilogue = MMPT_EPI_F32_ACC;
  }
  MMPT_REQUIRE(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "gemm: dims too large");
  MMPT_REQUIRE(A && B && C, "gemm: null operand");
  MMPT_REQUIRE(layout_a == MMPT_ROWS_K || layout_a == MMPT_K_ROWS, "gemm: bad layout_a");
  MMPT_REQUIRE(layout_b == MMPT_ROWS_K || layout_b == MMPT_K_ROWS, "gemm: bad layout_b");
  // 16-byte DMA pieces: the contiguous dim of every operand must be a multiple of 8 bf16
  MMPT_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0, "gemm: A/B not 16-B aligned");
  MMPT_REQUIRE(lda % 8 == 0 && ldb % 8 == 0, "gemm: lda/ldb must be multiples of 8");
  MMPT_REQUIRE(layout_a == MMPT_ROWS_K ? (K % 8 == 0 && lda >= K) : (M % 8 == 0 && lda >= M),
               "gemm: A contiguous dim must be a multiple of 8 (and lda >= it)");
  MMPT_REQUIRE(layout_b == MMPT_ROWS_K ? (K % 8 == 0 && ldb >= K) : (N % 8 == 0 && ldb >= N),
               "gemm: B contiguous dim must be a multiple of 8 (and ldb >= it)");
  MMPT_REQUIRE(N % 4 == 0 && ldc % 4 == 0 && ldc >= N, "gemm: N and ldc must be multiples of 4");
  if (epilogue == MMPT_EPI_BF16_GELU)
    MMPT_REQUIRE(C2 != nullptr && ldc2 % 4 == 0, "gemm: GELU epilogue needs C2");
  if (epilogue == MMPT_EPI_BF16_DGELU || epilogue == MMPT_EPI_BF16_DGELU_COLSUM)
    MMPT_REQUIRE(aux_bf16 != nullptr && ld_aux % 4 == 0, "gemm: DGELU epilogue needs aux");
  if (epilogue == MMPT_EPI_BF16_DGELU_COLSUM)
    MMPT_REQUIRE(C2 != nullptr && ((uintptr_t)C2 & 15) == 0,
                 "gemm: DGELU_COLSUM needs a 16-B aligned partial buffer C2");
  if (epilogue == MMPT_EPI_F32_RESID)
    MMPT_REQUIRE(C2 != nullptr && ldc2 % 4 == 0 && (aux_bf16 == nullptr || ld_aux % 4 == 0),
                 "gemm: RESID epilogue needs C2 (residual input)");
  if (epilogue == MMPT_EPI_BF16_SWIGLU)
    MMPT_REQUIRE(N % 256 == 0 && C2 != nullptr && bias_bf16 == nullptr && ldc2 >= N / 2 &&
                     ldc % 8 == 0 && ldc2 % 8 == 0 && ((uintptr_t)C & 15) == 0 &&
                     ((uintptr_t)C2 & 15) == 0,
                 "gemm: SWIGLU needs N %% 256 == 0 (blocked gate|up), C2 [M][N/2], no bias, "
                 "16-B aligned rows");
  if (epilogue == MMPT_EPI_BF16_DSWIGLU)
    MMPT_REQUIRE(N % 128 == 0 && aux_bf16 != nullptr && ldc >= 2 * N && ld_aux >= 2 * N &&
                     ldc % 8 == 0 && ld_aux % 8 == 0 && ((uintptr_t)C & 15) == 0 &&
                     ((uintptr_t)aux_bf16 & 15) == 0 && bias_bf16 == nullptr,
                 "gemm: DSWIGLU needs N %% 128 == 0, aux/C [M][2N] blocked, 16-B aligned rows");
  MMPT_REQUIRE((epilogue >= MMPT_EPI_BF16 && epilogue <= MMPT_EPI_BF16_DGELU_COLSUM) ||
                   epilogue == MMPT_EPI_BF16_SWIGLU || epilogue == MMPT_EPI_BF16_DSWIGLU,
               "gemm: bad epilogue");

  Plan pl = plan(M, N, K, epilogue);
  if (pl.splits > 1 && (workspace == nullptr ||
                        workspace_bytes < (int64_t)pl.splits * M * N * (int64_t)sizeof(float))) {
    pl.splits = 1;  // no workspace: single pass (same numerics, less parallelism)
    pl.kchunk = (int)K;
  }
  GemmParams p;
  p.A = (const bf16_t*)A;
  p.B = (const bf16_t*)B;
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.lda = lda;
  p.ldb = ldb;
  p.C = C;
  p.ldc = ldc;
  p.bias = (const bf16_t*)bias_bf16;
  p.aux = (const bf16_t*)aux_bf16;
  p.ld_aux = ld_aux;
  p.C2 = C2;
  p.ldc2 = ldc2;
  p.splits = pl.splits;
  p.kchunk = pl.kchunk;
  p.slab = (float*)workspace;
  {
    // 8-column epilogue needs 16-B aligned row segments in every epilogue operand
    const int ob = (epilogue == MMPT_EPI_BF16 || epilogue == MMPT_EPI_BF16_GELU ||
                    epilogue == MMPT_EPI_BF16_DGELU || epilogue == MMPT_EPI_BF16_DGELU_COLSUM ||
                    epilogue == MMPT_EPI_BF16_SWIGLU || epilogue == MMPT_EPI_BF16_DSWIGLU) ? 2 : 4;
    auto al = [](const void* q, int64_t ld, int eb) {
      return q == nullptr || (((uintptr_t)q & 15) == 0 && (ld * eb) % 16 == 0);
    };
    p.wide = al(C, ldc, ob) && al(bias_bf16, 0, 2) && al(aux_bf16, ld_aux, 2) &&
             (epilogue == MMPT_EPI_BF16_DGELU_COLSUM ? N % 4 == 0
                                                    : al(C2, ldc2, epilogue == MMPT_EPI_F32_RESID ? 4 : 2)) &&
             (pl.splits == 1 || (N % 8 == 0 && ((uintptr_t)workspace & 15) == 0));
  }
  hipStream_t s = (hipStream_t)stream;
  if (epilogue == MMPT_EPI_BF16_DGELU_COLSUM) {  // (the quick form too)
    // C2 holds mmpt_gemm_colsum_rows rows; the kernel that runs writes one per 128-row half tile
    // (gemm4p) or per 64-row half (gemm128); rows it leaves are zeroed for the fixed-order reduce
    const bool g4 = pl.big && uses_4p(true, layout_a, layout_b, launch_epilogue, pl.splits, N, K,
                                      p.wide);
    const int64_t bm = g4 ? 256 : 128, written = 2 * ((M + bm - 1) / bm);
    const int64_t have = colsum_rows_query(M, N, K);
    MMPT_REQUIRE(written <= have,
                 "gemm: %lld column-sum partial rows needed, mmpt_gemm_colsum_rows gave %lld (it "
                 "assumes 16-B aligned, K-contiguous operands)", (long long)written, (long long)have);
    if (written < have) {
      const hipError_t e = hipMemsetAsync((float*)C2 + written * N, 0,
                                          (size_t)((have - written) * N) * sizeof(float), s);
      if (e != hipSuccess) {
        set_error("gemm: colsum partial rows: %s", hipGetErrorString(e));
        return (int)e;
      }
    }
  }
  const WTail wt = pl.splits > 1 ? wtail_plan(acc_cs ? MMPT_EPI_F32_ACC_COLSUM : epilogue, M, N, K)
                                 : WTail{};
  if (acc_cs) {
    // C2 holds mmpt_gemm_acc_colsum_rows rows (the planned K splits x the 256-column tiles);
    // with less workspace this call runs fewer splits, and the rows it leaves are zeroed for the
    // fixed-order reduce
    const int64_t have = mmpt_gemm_acc_colsum_rows(M, N, K);
    MMPT_REQUIRE(have > 0 && uses_4p(pl.big, layout_a, layout_b,
                                     pl.splits > 1 ? EPI_SPLIT_CS : MMPT_EPI_F32_ACC_COLSUM,
                                     pl.splits, N, K, true),
                 "gemm: F32_ACC_COLSUM does not take M=%lld N=%lld K=%lld (see "
                 "mmpt_gemm_acc_colsum_rows)", (long long)M, (long long)N, (long long)K);
    // (under the weight-gradient tail split every row is zeroed: its parts write subsets)
    const int64_t written = wt.dim != 0 ? 0 : pl.splits * ((N + 255) / 256);
    if (written < have) {
      const hipError_t e = hipMemsetAsync((float*)C2 + written * ldc2, 0,
                                          (size_t)((have - written) * ldc2) * sizeof(float), s);
      if (e != hipSuccess) {
        set_error("gemm: acc colsum partial rows: %s", hipGetErrorString(e));
        return (int)e;
      }
    }
  }
  const int epi = pl.splits > 1 ? (acc_cs ? EPI_SPLIT_CS : EPI_SPLIT) : launch_epilogue;
  if (MMPT_GEMM_LUT && pl.big &&
      (epi == MMPT_EPI_BF16_GELU || epi == MMPT_EPI_BF16_DGELU ||
       epi == MMPT_EPI_BF16_DGELU_COLSUM || epi == MMPT_EPI_BF16_QGELU ||
       epi == MMPT_EPI_BF16_DQGELU || epi == MMPT_EPI_BF16_DQGELU_COLSUM ||
       epi == MMPT_EPI_BF16_SWIGLU || epi == MMPT_EPI_BF16_DSWIGLU)) {
    const int rc = ensure_gelu_lut(s);
    if (rc) return rc;
  }
  // one launch over rows [.., p.M) of p (splits / kchunk / epilogue as given)
  auto launch = [&](GemmParams& q, int e, bool small = false) -> int {
    // gemm4p for the big problems it takes (uses_4p), gemm128 for everything else
    const bool g4 = !small && uses_4p(pl.big, layout_a, layout_b, e, q.splits, q.N, q.K, q.wide);
    const int bm = g4 ? 256 : 128;
    q.tiles_m = (q.M + bm - 1) / bm;
    q.tiles_n = (q.N + bm - 1) / bm;
    dim3 grid(q.tiles_m * q.tiles_n, q.splits);
    if (g4) {  // persistent: one workgroup per CU walks its XCD's run of tiles
      const int nwg = q.tiles_m * q.tiles_n * q.splits;
      const int slots = persistent_slots();
      grid = dim3(slots > 0 && nwg > slots ? slots : nwg, 1);
      q.group = walk_group(q.tiles_n);  // the walk measured for gemm4p
      // (never with the fused row sums: their K-tile shares are split by loop index, so the
      // columns of one tile row must walk K in the same direction)
      const bool cs = e == MMPT_EPI_F32_ACC_COLSUM || e == EPI_SPLIT_CS;
      q.krev = q.K % BK == 0 && !cs ? walk_krev(q.tiles_n) : 0;
    } else {  // gemm128: one workgroup per tile, round 4's GROUP = 8, forward K order
      q.group = gemm_group_env() > 0 ? gemm_group_env() : 8;
      q.krev = 0;
    }
    return g4 ? launch_layouts<true>(layout_a, layout_b, e, q, grid, s)
              : launch_layouts<false>(layout_a, layout_b, e, q, grid, s);
  };
  g_last_tail_rows = 0;
  const TailPlan tp = pl.splits == 1 ? tail_plan(layout_a, layout_b, launch_epilogue, M, N, K)
                                     : TailPlan{};
  const int64_t mt = tp.rows > 0 ? tail_rows_of(M, tp) : 0;
  if (tp.rows > 0 && p.wide && workspace != nullptr && ((uintptr_t)workspace & 15) == 0 &&
      workspace_bytes >= (int64_t)tp.splits * mt * N * (int64_t)sizeof(float) &&
      uses_4p(true, layout_a, layout_b, launch_epilogue, 1, N, K, true)) {
    // rows [0, M - mt): whole rounds; rows [M - mt, M): split-K slabs + tail_epi_kernel
    const int64_t m0 = M - mt;
    GemmParams q = p;
    q.M = (int)m0;
    int rc = launch(q, launch_epilogue);
    if (g_probe_event != nullptr) {  // bench.py: end of the main kernel (the tail is probed apart)
      (void)hipEventRecord(g_probe_event, s);
      g_probe_event = nullptr;
    }
    if (rc) return rc;
    const char* main_name = g_last_kernel;
    char keep[64];
    snprintf(keep, sizeof keep, "%s", main_name);
    const int eb = launch_epilogue == MMPT_EPI_F32_RESID ? 4 : 2;
    GemmParams t = p;
    t.M = (int)mt;
    t.A = p.A + m0 * lda;  // ROWS_K
    t.C = (char*)C + m0 * ldc * eb;
    t.splits = tp.splits;
    t.kchunk = tp.kchunk;
    t.slab = (float*)workspace;
    // a tail of <= 128 rows (T = 16 * 2049 = 32,784: 16 rows) on 128-row tiles: a 256-row tile
    // would run 16x the MFMAs its rows need (MMPT_GEMM_TAIL128=0: gemm4p, A/B only)
    rc = launch(t, EPI_SPLIT, mt <= 128 && gemm_tail128());  // (tail_plan's `small`)
    snprintf(g_last_kernel, sizeof g_last_kernel, "%s", keep);  // the probe names the main launch
    if (rc) return rc;
    const long n8 = mt * (N / 8);
    const unsigned blocks = (unsigned)((n8 + 255) / 256);
    const bf16_t* aux_t = aux_bf16 ? (const bf16_t*)aux_bf16 + m0 * ld_aux : nullptr;
    if (launch_epilogue == MMPT_EPI_F32_RESID)
      tail_epi_kernel<true><<<blocks, 256, 0, s>>>((int)mt, (int)N, tp.splits, t.slab, p.bias, aux_t,
                                                   ld_aux, t.C, ldc, (const float*)C2 + m0 * ldc2,
                                                   ldc2);
    else
      tail_epi_kernel<false><<<blocks, 256, 0, s>>>((int)mt, (int)N, tp.splits, t.slab, p.bias,
                                                    nullptr, 0, t.C, ldc, nullptr, 0);
    g_last_tail_rows = mt;
    return check_launch("gemm_tail_epilogue");
  }
  if (wt.dim != 0 && pl.big && p.wide && workspace != nullptr &&
      ((uintptr_t)workspace & 15) == 0 && workspace_bytes >= wtail_slab_bytes(M, N, wt)) {
    // whole rounds unsplit into C, the rest split-K through slabs + splitk_reduce
    const int64_t l0 = (int64_t)wt.lines * 256;
    GemmParams q = p;
    q.splits = 1;
    q.kchunk = (int)K;
    if (wt.dim == 1) q.M = (int)l0;
    else q.N = (int)l0;
    int rc = launch(q, acc_cs ? MMPT_EPI_F32_ACC_COLSUM : epilogue);
    if (rc) return rc;
    char keep[64];
    snprintf(keep, sizeof keep, "%s", g_last_kernel);
    GemmParams t = p;
    t.splits = wt.splits;
    t.kchunk = wt.kchunk;
    t.slab = (float*)workspace;
    if (wt.dim == 1) {
      t.M = (int)(M - l0);
      t.A = p.A + (layout_a == MMPT_K_ROWS ? l0 : l0 * lda);
      t.C = (float*)C + l0 * ldc;
      if (acc_cs) t.C2 = (float*)C2 + l0;  // the tail rows' partial sums, one row per split
    } else {
      t.N = (int)(N - l0);
      t.B = p.B + (layout_b == MMPT_K_ROWS ? l0 : l0 * ldb);
      t.C = (float*)C + l0;
    }
    rc = launch(t, acc_cs && wt.dim == 1 ? EPI_SPLIT_CS : EPI_SPLIT);
    if (g_probe_event != nullptr) {  // bench.py: end of the GEMM launches (before the reduce)
      (void)hipEventRecord(g_probe_event, s);
      g_probe_event = nullptr;
    }
    snprintf(g_last_kernel, sizeof g_last_kernel, "%s", keep);  // the probe names the main launch
    if (rc) return rc;
    const long n4 = (long)t.M * (t.N / 4);
    const unsigned blocks = (unsigned)((n4 + 255) / 256);
    if (epilogue == MMPT_EPI_F32_ACC)
      splitk_reduce<true><<<blocks, 256, 0, s>>>(t.M, t.N, t.splits, t.slab, (float*)t.C, ldc);
    else
      splitk_reduce<false><<<blocks, 256, 0, s>>>(t.M, t.N, t.splits, t.slab, (float*)t.C, ldc);
    return check_launch("gemm_wtail_reduce");
  }
  int rc = launch(p, epi);
  if (g_probe_event != nullptr) {  // bench.py: end of the main kernel (before the reduce)
    (void)hipEventRecord(g_probe_event, s);
    g_probe_event = nullptr;
  }
  if (rc || pl.splits == 1) return rc;
  const long n4 = M * (N / 4);
  const unsigned blocks = (unsigned)((n4 + 255) / 256);
  if (epilogue == MMPT_EPI_F32_ACC)
    splitk_reduce<true><<<blocks, 256, 0, s>>>((int)M, (int)N, pl.splits, p.slab, (float*)C, ldc);
  else
    splitk_reduce<false><<<blocks, 256, 0, s>>>((int)M, (int)N, pl.splits, p.slab, (float*)C, ldc);
  return check_launch("gemm_splitk_reduce");
}

#if MMPT_GEMM_DIAG == 7
// diagnostic 7 only (not in include/mmpt.h): the last launch's per-workgroup clock stamps,
// 4 x u64 per workgroup (s_memtime start / end, s_memrealtime start / end), n workgroups
extern "C" int mmpt_gemm_diag_clock(unsigned long long* host, int n) {
  MMPT_REQUIRE(host && n > 0 && n <= 1024, "gemm_diag_clock: bad arguments");
  const hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_clock),
                                           (size_t)n * 4 * sizeof(unsigned long long), 0,
                                           hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    set_error("gemm_diag_clock: %s", hipGetErrorString(e));
    return (int)e;
  }
  return MMPT_OK;
}
#endif
