// Host-side Adam(W) for optimizer-state offload (include/mmpt_host.h).
//
// One pass over the shard: the compiler vectorises the plain loop of adam_range (no
// intrinsics), cloned for AVX-512 (16 floats per iteration) and the AVX2 baseline with
// runtime dispatch; OpenMP static split over contiguous chunks so each thread streams its
// own part of p/g/m/v (28 B/param, host-DRAM bound).
// fp-contract is off: every product/sum rounds as written, matching the device kernel's
// sequence of float operations up to its own FMA contraction (tests: ≤ 2 ulp).
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

#include <string>

#include "mmpt_host.h"

namespace {
thread_local std::string g_err;

int fail(const char* msg) {
  g_err = msg;
  return -1;
}

// round-to-nearest-even, NaN kept quiet; branch-free so the update loop vectorises
inline uint16_t bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint32_t r = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
  const uint32_t q = (u >> 16) | 0x40u;
  return (uint16_t)((u & 0x7fffffffu) > 0x7f800000u ? q : r);
}
}  // namespace

extern "C" int mmpt_host_abi_version(void) { return MMPT_HOST_ABI_VERSION; }
extern "C" const char* mmpt_host_last_error(void) { return g_err.c_str(); }

namespace {
// One contiguous range [i0, i1), the loop unswitched on (AdamW, L2 decay, bf16 shadow) so
// it has no control flow and vectorises; fp-contract off and exact sqrt/div keep every
// element's operations the device kernel's.
template <bool ADAMW, bool L2, bool PB>
__attribute__((always_inline)) inline void adam_loop(int64_t i0, int64_t i1, float* __restrict__ p,
                                                     const float* __restrict__ g,
                                                     float* __restrict__ m, float* __restrict__ v,
                                                     uint16_t* __restrict__ pb, float step_size,
                                                     float bc2_sqrt, float sc, float decay,
                                                     float omb1, float b2, float omb2, float eps,
                                                     float wd) {
  for (int64_t i = i0; i < i1; ++i) {
    float gr = g[i] * sc;
    float pi = p[i];
    if constexpr (ADAMW) pi *= decay;
    if constexpr (L2) gr += wd * pi;
    float mi = m[i];
    mi += omb1 * (gr - mi);
    const float vi = v[i] * b2 + omb2 * gr * gr;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi -= step_size * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if constexpr (PB) pb[i] = bf16_rne(pi);
  }
}
// cloned for AVX-512 (the GPU boxes' EPYC hosts: 16 floats per iteration) and the -mavx2
// baseline (8), picked at load time (GCC target_clones / ifunc); the update is bitwise the
// same whichever clone runs
__attribute__((target_clones("avx512f", "default"))) void adam_range(
    int64_t i0, int64_t i1, float* __restrict__ p, const float* __restrict__ g,
    float* __restrict__ m, float* __restrict__ v, uint16_t* __restrict__ pb, float step_size,
    float bc2_sqrt, float sc, float decay, float omb1, float b2, float omb2, float eps, float wd,
    int adamw) {
#define MMPT_ADAM(A, L, P) \
  adam_loop<A, L, P>(i0, i1, p, g, m, v, pb, step_size, bc2_sqrt, sc, decay, omb1, b2, omb2, eps, wd)
  const bool l2 = !adamw && wd != 0.f;
  if (adamw) {
    if (pb) MMPT_ADAM(true, false, true); else MMPT_ADAM(true, false, false);
  } else if (l2) {
    if (pb) MMPT_ADAM(false, true, true); else MMPT_ADAM(false, true, false);
  } else {
    if (pb) MMPT_ADAM(false, false, true); else MMPT_ADAM(false, false, false);
  }
#undef MMPT_ADAM
}
}  // namespace

extern "C" int mmpt_host_adam_step(int64_t n, float* p, const float* g, float* m, float* v,
                                   uint16_t* pb, float lr, float b1, float b2, float eps,
                                   float wd, int adamw, int64_t step, const float* gscale,
                                   int threads) {
  if (n < 0 || !p || !g || !m || !v || step < 1) return fail("host_adam_step: bad args");
  const double bc1 = 1.0 - pow((double)b1, (double)step);
  const double bc2 = 1.0 - pow((double)b2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float sc = gscale ? gscale[0] : 1.0f;
  const float decay = 1.0f - lr * wd;
  const float omb1 = 1.0f - b1, omb2 = 1.0f - b2;
  const int nt = threads > 0 ? threads : omp_get_max_threads();
  // static split into contiguous per-thread ranges (each thread streams its own part)
#pragma omp parallel num_threads(nt)
  {
    const int64_t T = omp_get_num_threads(), t = omp_get_thread_num();
    const int64_t per = (n + T - 1) / T;
    const int64_t i0 = t * per, i1 = i0 + per < n ? i0 + per : n;
    if (i0 < i1)
      adam_range(i0, i1, p, g, m, v, pb, step_size, bc2_sqrt, sc, decay, omb1, b2, omb2, eps, wd,
                 adamw);
  }
  return 0;
}

extern "C" int mmpt_host_simd_width(void) {
  // floats per vector of the adam_range clone this host runs
  return __builtin_cpu_supports("avx512f") ? 16 : 8;
}

extern "C" int mmpt_host_sumsq(int64_t n, const float* x, double* out, int threads) {
  if (n < 0 || !x || !out) return fail("host_sumsq: bad args");
  const int nt = threads > 0 ? threads : omp_get_max_threads();
  double acc = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : acc) num_threads(nt)
  for (int64_t i = 0; i < n; ++i) acc += (double)x[i] * (double)x[i];
  *out = acc;
  return 0;
}
