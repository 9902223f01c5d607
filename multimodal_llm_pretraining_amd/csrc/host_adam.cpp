// Host-side Adam(W) for optimizer-state offload (include/mmpt_host.h).
//
// One pass over the shard: 16 floats per AVX-512/AVX2 iteration as the compiler
// vectorises the plain loop below (-O3 -mavx2 -mfma; no intrinsics so the same source
// serves every x86-64 host of the pool), OpenMP static split over contiguous chunks so
// each thread streams its own part of p/g/m/v (28 B/param, host-DRAM bound).
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

inline uint16_t bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
}  // namespace

extern "C" int mmpt_host_abi_version(void) { return MMPT_HOST_ABI_VERSION; }
extern "C" const char* mmpt_host_last_error(void) { return g_err.c_str(); }

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
#pragma omp parallel for schedule(static) num_threads(nt)
  for (int64_t i = 0; i < n; ++i) {
    float gr = g[i] * sc;
    float pi = p[i];
    if (adamw) {
      pi *= decay;
    } else if (wd != 0.f) {
      gr += wd * pi;
    }
    float mi = m[i];
    mi += omb1 * (gr - mi);
    float vi = v[i] * b2 + omb2 * gr * gr;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi -= step_size * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if (pb) pb[i] = bf16_rne(pi);
  }
  return 0;
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
