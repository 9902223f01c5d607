// K4: LayerNorm forward / backward (fp32 statistics, as autocast runs
// aten::layer_norm in fp32).  One wave per row, float4 loads; GPTNeoX's two
// LayerNorms over the same residual (input_layernorm / post_attention_layernorm,
// tf:models/gpt_neox/modeling_gpt_neox.py:245-246, 263-269) share one read of x
// and one set of statistics.  The backward fuses the residual-gradient add and
// both LN input-gradients into one pass; dγ/dβ use a fixed-shape two-stage
// reduction (per-block partial rows, then a column sum) so results are
// bitwise reproducible.
#include "common.h"

namespace mmpt {
namespace {

constexpr int LN_WAVES = 4;
constexpr int LN_BWD_BLOCKS = 512;

// RMS = true: LlamaRMSNorm (tf:models/llama/modeling_llama.py LlamaRMSNorm.forward, fp32
// under autocast): rstd = rsqrt(mean(x²) + eps), y = bf16(w · (x · rstd)) — no mean, no
// bias (b1 / mean_out unused).
template <int MAXJ, bool RMS = false>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int rows, int h, float eps,
                                                     const float* __restrict__ x, long ldx,
                                                     const float* __restrict__ w1,
                                                     const float* __restrict__ b1, bf16_t* y1,
                                                     const float* __restrict__ w2,
                                                     const float* __restrict__ b2, bf16_t* y2,
                                                     float* mean_out, float* rstd_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * LN_WAVES + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = h >> 2;
  const float4* xr = (const float4*)(x + (long)row * ldx);
  float4 v[MAXJ];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int i = j * 64 + lane;
    v[j] = i < nv ? xr[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  }
  const float mean = RMS ? 0.f : wave_sum(s) / (float)h;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int i = j * 64 + lane;
    if (i < nv) {
      const float a = v[j].x - mean, b = v[j].y - mean, c = v[j].z - mean, d = v[j].w - mean;
      ss += (a * a + b * b) + (c * c + d * d);
    }
  }
  const float var = wave_sum(ss) / (float)h;
  const float rstd = 1.0f / sqrtf(var + eps);
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int i = j * 64 + lane;
    if (i >= nv) continue;
    const float xh[4] = {(v[j].x - mean) * rstd, (v[j].y - mean) * rstd, (v[j].z - mean) * rstd,
                         (v[j].w - mean) * rstd};
    const float4 g = ((const float4*)w1)[i];
    const float4 bb = RMS ? make_float4(0.f, 0.f, 0.f, 0.f) : ((const float4*)b1)[i];
    uint2 o;
    o.x = (uint32_t)f2bf(xh[0] * g.x + bb.x) | ((uint32_t)f2bf(xh[1] * g.y + bb.y) << 16);
    o.y = (uint32_t)f2bf(xh[2] * g.z + bb.z) | ((uint32_t)f2bf(xh[3] * g.w + bb.w) << 16);
    ((uint2*)(y1 + (long)row * h))[i] = o;
    if (y2 != nullptr) {
      const float4 g2 = ((const float4*)w2)[i], c2 = ((const float4*)b2)[i];
      o.x = (uint32_t)f2bf(xh[0] * g2.x + c2.x) | ((uint32_t)f2bf(xh[1] * g2.y + c2.y) << 16);
      o.y = (uint32_t)f2bf(xh[2] * g2.z + c2.z) | ((uint32_t)f2bf(xh[3] * g2.w + c2.w) << 16);
      ((uint2*)(y2 + (long)row * h))[i] = o;
    }
  }
}

// The same forward with the workgroups persistent (a grid of MMPT_LN_FWD_BLOCKS) and γ / β of
// both LayerNorms staged once per workgroup in LDS ([4][h/4] float4): the per-row kernel above
// re-reads 4 × h floats of weights per row through the vector-memory path (32 of its 56 VMEM
// instructions per row at h = 2048).  Bitwise the same arithmetic.
#ifndef MMPT_LN_FWD_PERSIST
#define MMPT_LN_FWD_PERSIST 1  // round 5: Pythia's dual LN 623 -> 551 us (profiles/r05/ln_prefetch/)
#endif
#ifndef MMPT_LN_FWD_BLOCKS
#define MMPT_LN_FWD_BLOCKS 1024
#endif
template <int MAXJ>
__global__ __launch_bounds__(256) void ln_fwd_persist_kernel(int rows, int h, float eps,
                                                             const float* __restrict__ x, long ldx,
                                                             const float* __restrict__ w1,
                                                             const float* __restrict__ b1, bf16_t* y1,
                                                             const float* __restrict__ w2,
                                                             const float* __restrict__ b2, bf16_t* y2,
                                                             float* mean_out, float* rstd_out) {
  extern __shared__ float4 wl[];  // [q][nv]: γ1, β1, γ2, β2
  const int lane = threadIdx.x & 63, nv = h >> 2;
  const int nq = y2 != nullptr ? 4 : 2;
  for (int e = threadIdx.x; e < nq * nv; e += 256) {
    const int q = e / nv, i = e - q * nv;
    const float* src = q == 0 ? w1 : q == 1 ? b1 : q == 2 ? w2 : b2;
    wl[e] = ((const float4*)src)[i];
  }
  __syncthreads();
  for (int row = blockIdx.x * LN_WAVES + (threadIdx.x >> 6); row < rows; row += gridDim.x * LN_WAVES) {
    const float4* xr = (const float4*)(x + (long)row * ldx);
    float4 v[MAXJ];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int i = j * 64 + lane;
      v[j] = i < nv ? xr[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    }
    const float mean = wave_sum(s) / (float)h;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int i = j * 64 + lane;
      if (i < nv) {
        const float a = v[j].x - mean, b = v[j].y - mean, c = v[j].z - mean, d = v[j].w - mean;
        ss += (a * a + b * b) + (c * c + d * d);
      }
    }
    const float var = wave_sum(ss) / (float)h;
    const float rstd = 1.0f / sqrtf(var + eps);
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int i = j * 64 + lane;
      if (i >= nv) continue;
      const float xh[4] = {(v[j].x - mean) * rstd, (v[j].y - mean) * rstd, (v[j].z - mean) * rstd,
                           (v[j].w - mean) * rstd};
      const float4 g = wl[i], bb = wl[nv + i];
      uint2 o;
      o.x = (uint32_t)f2bf(xh[0] * g.x + bb.x) | ((uint32_t)f2bf(xh[1] * g.y + bb.y) << 16);
      o.y = (uint32_t)f2bf(xh[2] * g.z + bb.z) | ((uint32_t)f2bf(xh[3] * g.w + bb.w) << 16);
      ((uint2*)(y1 + (long)row * h))[i] = o;
      if (y2 != nullptr) {
        const float4 g2 = wl[2 * nv + i], c2 = wl[3 * nv + i];
        o.x = (uint32_t)f2bf(xh[0] * g2.x + c2.x) | ((uint32_t)f2bf(xh[1] * g2.y + c2.y) << 16);
        o.y = (uint32_t)f2bf(xh[2] * g2.z + c2.z) | ((uint32_t)f2bf(xh[3] * g2.w + c2.w) << 16);
        ((uint2*)(y2 + (long)row * h))[i] = o;
      }
    }
  }
}

// fp32-output LayerNorm (CLIP's pre_layrnorm: its output IS the fp32 residual stream,
// tf:models/clip/modeling_clip.py CLIPVisionTransformer.forward), one wave per row.
template <int MAXJ>
__global__ __launch_bounds__(256) void ln_fwd32_kernel(int rows, int h, float eps,
                                                       const float* __restrict__ x,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ b, float* y,
                                                       float* mean_out, float* rstd_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * LN_WAVES + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = h >> 2;
  const float4* xr = (const float4*)(x + (long)row * h);
  float4 v[MAXJ];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int i = j * 64 + lane;
    v[j] = i < nv ? xr[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  }
  const float mean = wave_sum(s) / (float)h;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int i = j * 64 + lane;
    if (i < nv) {
      const float a = v[j].x - mean, bb = v[j].y - mean, c = v[j].z - mean, d = v[j].w - mean;
      ss += (a * a + bb * bb) + (c * c + d * d);
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)h + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int i = j * 64 + lane;
    if (i >= nv) continue;
    const float4 g = ((const float4*)w)[i], bb = ((const float4*)b)[i];
    ((float4*)(y + (long)row * h))[i] =
        make_float4((v[j].x - mean) * rstd * g.x + bb.x, (v[j].y - mean) * rstd * g.y + bb.y,
                    (v[j].z - mean) * rstd * g.z + bb.z, (v[j].w - mean) * rstd * g.w + bb.w);
  }
}

__device__ __forceinline__ float4 ld_bf16x4(const bf16_t* p) {
  const uint2 u = *(const uint2*)p;
  return make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
}

// partials layout: [block][4][h] = dw1, db1, dw2, db2
// DY32: dy1 is fp32 (the fp32-output LayerNorm above); otherwise bf16 (GEMM operand)
template <int MAXJ, bool DY32 = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    int rows, int h, const float* __restrict__ x, long ldx, const float* __restrict__ mean,
    const float* __restrict__ rstd, const bf16_t* __restrict__ dy1, const float* __restrict__ w1,
    const bf16_t* __restrict__ dy2, const float* __restrict__ w2, const float* dresid, float* dx,
    float* __restrict__ partials) {
  __shared__ float red[LN_WAVES][256 * 4];  // staging for the cross-wave dγ/dβ sum
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nv = h >> 2;
  const bool two = dy2 != nullptr;
  float4 aw1[MAXJ], ab1[MAXJ], aw2[MAXJ], ab2[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    aw1[j] = ab1[j] = aw2[j] = ab2[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int row = blockIdx.x * LN_WAVES + wave; row < rows; row += gridDim.x * LN_WAVES) {
    const float mu = mean[row], rs = rstd[row];
    const float4* xr = (const float4*)(x + (long)row * ldx);
    float4 xh[MAXJ], g1[MAXJ], g2[MAXJ];
    float s1a = 0.f, s1b = 0.f, s2a = 0.f, s2b = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int i = j * 64 + lane;
      xh[j] = g1[j] = g2[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i >= nv) continue;
      const float4 xv = xr[i];
      xh[j] = make_float4((xv.x - mu) * rs, (xv.y - mu) * rs, (xv.z - mu) * rs, (xv.w - mu) * rs);
      const float4 d1 = DY32 ? ((const float4*)((const float*)(const void*)dy1 + (long)row * h))[i]
                             : ld_bf16x4(dy1 + (long)row * h + i * 4);
      const float4 ww1 = ((const float4*)w1)[i];
      g1[j] = make_float4(d1.x * ww1.x, d1.y * ww1.y, d1.z * ww1.z, d1.w * ww1.w);
      s1a += (g1[j].x * xh[j].x + g1[j].y * xh[j].y) + (g1[j].z * xh[j].z + g1[j].w * xh[j].w);
      s1b += (g1[j].x + g1[j].y) + (g1[j].z + g1[j].w);
      aw1[j].x += d1.x * xh[j].x; aw1[j].y += d1.y * xh[j].y;
      aw1[j].z += d1.z * xh[j].z; aw1[j].w += d1.w * xh[j].w;
      ab1[j].x += d1.x; ab1[j].y += d1.y; ab1[j].z += d1.z; ab1[j].w += d1.w;
      if (two) {
        const float4 d2 = ld_bf16x4(dy2 + (long)row * h + i * 4);
        const float4 ww2 = ((const float4*)w2)[i];
        g2[j] = make_float4(d2.x * ww2.x, d2.y * ww2.y, d2.z * ww2.z, d2.w * ww2.w);
        s2a += (g2[j].x * xh[j].x + g2[j].y * xh[j].y) + (g2[j].z * xh[j].z + g2[j].w * xh[j].w);
        s2b += (g2[j].x + g2[j].y) + (g2[j].z + g2[j].w);
        aw2[j].x += d2.x * xh[j].x; aw2[j].y += d2.y * xh[j].y;
        aw2[j].z += d2.z * xh[j].z; aw2[j].w += d2.w * xh[j].w;
        ab2[j].x += d2.x; ab2[j].y += d2.y; ab2[j].z += d2.z; ab2[j].w += d2.w;
      }
    }
    const float inv_h = 1.0f / (float)h;
    const float c1a = wave_sum(s1a) * inv_h, c1b = wave_sum(s1b) * inv_h;
    float c2a = 0.f, c2b = 0.f;
    if (two) {
      c2a = wave_sum(s2a) * inv_h;
      c2b = wave_sum(s2b) * inv_h;
    }
    float4* dxr = (float4*)(dx + (long)row * h);
    const float4* drr = dresid ? (const float4*)(dresid + (long)row * h) : nullptr;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int i = j * 64 + lane;
      if (i >= nv) continue;
      float4 o = drr ? drr[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      o.x += rs * (g1[j].x - xh[j].x * c1a - c1b);
      o.y += rs * (g1[j].y - xh[j].y * c1a - c1b);
      o.z += rs * (g1[j].z - xh[j].z * c1a - c1b);
      o.w += rs * (g1[j].w - xh[j].w * c1a - c1b);
      if (two) {
        o.x += rs * (g2[j].x - xh[j].x * c2a - c2b);
        o.y += rs * (g2[j].y - xh[j].y * c2a - c2b);
        o.z += rs * (g2[j].z - xh[j].z * c2a - c2b);
        o.w += rs * (g2[j].w - xh[j].w * c2a - c2b);
      }
      dxr[i] = o;
    }
  }
  // cross-wave reduction of the per-lane dγ/dβ accumulators, one quantity at a time
  // (fully unrolled: every accumulator index is a compile-time constant, no scratch)
  float* out = partials + (long)blockIdx.x * 4 * h;
#pragma unroll
  for (int qn = 0; qn < 4; ++qn) {
    if (qn >= 2 && !two) break;
#pragma unroll
    for (int j0 = 0; j0 < MAXJ; j0 += 4) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int j = j0 + jj;
        if (j < MAXJ) {
          const float4 val = qn == 0 ? aw1[j] : qn == 1 ? ab1[j] : qn == 2 ? aw2[j] : ab2[j];
          *(float4*)&red[wave][(jj * 64 + lane) * 4] = val;
        }
      }
      __syncthreads();
      for (int e = threadIdx.x; e < 1024; e += 256) {
        const int jj = e >> 8, rem = e & 255;  // rem = lane*4 + comp
        const int j = j0 + jj;
        const int col = (j * 64 + (rem >> 2)) * 4 + (rem & 3);
        if (j < MAXJ && col < h)
          out[qn * h + col] = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
      }
      __syncthreads();
    }
  }
}

// Backward, one WORKGROUP per row (256 threads, PT float4 per thread): ~70 VGPRs, so
// 8 waves/SIMD keep enough loads in flight to stream at HBM rate (the wave-per-row
// kernel above holds every row's 4 accumulator sets in one wave: ~240 VGPRs, 2 waves/
// SIMD, latency-bound at ~2.3 TB/s).  Row sums: wave_sum + a 4-wave LDS exchange
// (double-buffered by row parity: one barrier per row).  Optional fused outputs:
// dx_bf16 = bf16(dx) (the next GEMMs' operand) and Σ_rows bf16(dx) (a bias gradient
// that autocast's addmm backward would compute from that bf16 tensor) as quantity 4.
// partials layout: [block][5][h] = dw1, db1, dw2, db2, Σ bf16(dx)
#ifndef MMPT_LN_BLOCKS
#define MMPT_LN_BLOCKS 1024
#endif
#ifndef MMPT_LN_PREFETCH
#define MMPT_LN_PREFETCH 1  // the residual-gradient row loads before the row-sum barrier (round 5: -0.9%); 0 = after it
#endif
constexpr int LNR_BLOCKS = MMPT_LN_BLOCKS;
// RMS = true: the RMSNorm backward (μ = 0, no dβ): dx = rstd·(g − x̂·mean(g·x̂)), g = dy·w.
template <int PT, bool RMS = false>
__global__ __launch_bounds__(256) void ln_bwd_rows_kernel(
    int rows, int h, const float* __restrict__ x, long ldx, const float* __restrict__ mean,
    const float* __restrict__ rstd, const bf16_t* __restrict__ dy1, const float* __restrict__ w1,
    const bf16_t* __restrict__ dy2, const float* __restrict__ w2, const float* dresid, float* dx,
    bf16_t* __restrict__ dxb, int want_dsum, float* __restrict__ partials) {
  __shared__ float red[2][4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nv = h >> 2;
  const bool two = dy2 != nullptr;
  float4 aw1[PT], ab1[PT], aw2[PT], ab2[PT], as[PT];
  float4 ww1[PT], ww2[PT];
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    aw1[j] = ab1[j] = aw2[j] = ab2[j] = as[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int i = j * 256 + tid;
    ww1[j] = i < nv ? ((const float4*)w1)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    ww2[j] = (two && i < nv) ? ((const float4*)w2)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  int par = 0;
  for (int row = blockIdx.x; row < rows; row += gridDim.x, par ^= 1) {
    const float mu = RMS ? 0.f : mean[row], rs = rstd[row];
    const float4* xr = (const float4*)(x + (long)row * ldx);
    float4 xh[PT], g1[PT], g2[PT], dr[PT];
    float s1a = 0.f, s1b = 0.f, s2a = 0.f, s2b = 0.f;
    const float4* drr = dresid ? (const float4*)(dresid + (long)row * h) : nullptr;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = j * 256 + tid;
      xh[j] = g1[j] = g2[j] = dr[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i >= nv) continue;
      if (MMPT_LN_PREFETCH && drr) dr[j] = drr[i];
      const float4 xv = xr[i];
      xh[j] = make_float4((xv.x - mu) * rs, (xv.y - mu) * rs, (xv.z - mu) * rs, (xv.w - mu) * rs);
      const float4 d1 = ld_bf16x4(dy1 + (long)row * h + i * 4);
      g1[j] = make_float4(d1.x * ww1[j].x, d1.y * ww1[j].y, d1.z * ww1[j].z, d1.w * ww1[j].w);
      s1a += (g1[j].x * xh[j].x + g1[j].y * xh[j].y) + (g1[j].z * xh[j].z + g1[j].w * xh[j].w);
      s1b += (g1[j].x + g1[j].y) + (g1[j].z + g1[j].w);
      aw1[j].x += d1.x * xh[j].x; aw1[j].y += d1.y * xh[j].y;
      aw1[j].z += d1.z * xh[j].z; aw1[j].w += d1.w * xh[j].w;
      ab1[j].x += d1.x; ab1[j].y += d1.y; ab1[j].z += d1.z; ab1[j].w += d1.w;
      if (two) {
        const float4 d2 = ld_bf16x4(dy2 + (long)row * h + i * 4);
        g2[j] = make_float4(d2.x * ww2[j].x, d2.y * ww2[j].y, d2.z * ww2[j].z, d2.w * ww2[j].w);
        s2a += (g2[j].x * xh[j].x + g2[j].y * xh[j].y) + (g2[j].z * xh[j].z + g2[j].w * xh[j].w);
        s2b += (g2[j].x + g2[j].y) + (g2[j].z + g2[j].w);
        aw2[j].x += d2.x * xh[j].x; aw2[j].y += d2.y * xh[j].y;
        aw2[j].z += d2.z * xh[j].z; aw2[j].w += d2.w * xh[j].w;
        ab2[j].x += d2.x; ab2[j].y += d2.y; ab2[j].z += d2.z; ab2[j].w += d2.w;
      }
    }
    s1a = wave_sum(s1a);
    s1b = wave_sum(s1b);
    if (two) {
      s2a = wave_sum(s2a);
      s2b = wave_sum(s2b);
    }
    if (lane == 0) {
      red[par][wave][0] = s1a;
      red[par][wave][1] = s1b;
      red[par][wave][2] = s2a;
      red[par][wave][3] = s2b;
    }
    __syncthreads();
    const float inv_h = 1.0f / (float)h;
    const float c1a = ((red[par][0][0] + red[par][1][0]) + (red[par][2][0] + red[par][3][0])) * inv_h;
    const float c1b = RMS ? 0.f : ((red[par][0][1] + red[par][1][1]) + (red[par][2][1] + red[par][3][1])) * inv_h;
    const float c2a = ((red[par][0][2] + red[par][1][2]) + (red[par][2][2] + red[par][3][2])) * inv_h;
    const float c2b = ((red[par][0][3] + red[par][1][3]) + (red[par][2][3] + red[par][3][3])) * inv_h;
    float4* dxr = (float4*)(dx + (long)row * h);
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = j * 256 + tid;
      if (i >= nv) continue;
      float4 o = MMPT_LN_PREFETCH ? dr[j] : drr ? drr[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      o.x += rs * (g1[j].x - xh[j].x * c1a - c1b);
      o.y += rs * (g1[j].y - xh[j].y * c1a - c1b);
      o.z += rs * (g1[j].z - xh[j].z * c1a - c1b);
      o.w += rs * (g1[j].w - xh[j].w * c1a - c1b);
      if (two) {
        o.x += rs * (g2[j].x - xh[j].x * c2a - c2b);
        o.y += rs * (g2[j].y - xh[j].y * c2a - c2b);
        o.z += rs * (g2[j].z - xh[j].z * c2a - c2b);
        o.w += rs * (g2[j].w - xh[j].w * c2a - c2b);
      }
      dxr[i] = o;
      if (dxb != nullptr) {
        uint2 u;
        u.x = (uint32_t)f2bf(o.x) | ((uint32_t)f2bf(o.y) << 16);
        u.y = (uint32_t)f2bf(o.z) | ((uint32_t)f2bf(o.w) << 16);
        ((uint2*)(dxb + (long)row * h))[i] = u;
        if (want_dsum) {
          as[j].x += round_bf(o.x); as[j].y += round_bf(o.y);
          as[j].z += round_bf(o.z); as[j].w += round_bf(o.w);
        }
      }
    }
  }
  float4* out = (float4*)(partials + (long)blockIdx.x * 5 * h);
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    const int i = j * 256 + tid;
    if (i >= nv) continue;
    out[i] = aw1[j];
    if (!RMS) out[nv + i] = ab1[j];
    if (two) {
      out[2 * nv + i] = aw2[j];
      out[3 * nv + i] = ab2[j];
    }
    if (want_dsum) out[4 * nv + i] = as[j];
  }
}

// Σ over blocks of partials[b][q][c] (QS quantities per block) -> param grads (+=); the
// bias-gradient quantity (q == 4) is rounded to bf16 first (autocast grad dtype).
__global__ __launch_bounds__(256) void ln_rows_reduce(int nblk, int h, const float* __restrict__ partials,
                                                      float* dw1, float* db1, float* dw2, float* db2,
                                                      float* ds1, float* ds2) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.y, c = blockIdx.x * 64 + lane;
  float* dst = q == 0 ? dw1 : q == 1 ? db1 : q == 2 ? dw2 : q == 3 ? db2 : ds1;
  if (dst == nullptr) return;  // uniform per workgroup
  float s = 0.f;
  if (c < h)
#pragma unroll 8
    for (int b = wave; b < nblk; b += 4) s += partials[((long)b * 5 + q) * h + c];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && c < h) {
    float v = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    if (q == 4) {
      v = round_bf(v);
      if (ds2 != nullptr) ds2[c] += v;
    }
    dst[c] += v;
  }
}

// Σ over blocks of partials[b][q][c] -> param grads (+=): one workgroup per
// (64 columns, quantity); its 4 waves split the blocks, LDS combine (fixed order).
__global__ __launch_bounds__(256) void ln_bwd_reduce(int nblk, int h, const float* __restrict__ partials,
                                                     float* dw1, float* db1, float* dw2,
                                                     float* db2) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.y, c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < h)
    for (int b = wave; b < nblk; b += 4) s += partials[((long)b * 4 + q) * h + c];
  red[wave][lane] = s;
  __syncthreads();
  float* dst = q == 0 ? dw1 : q == 1 ? db1 : q == 2 ? dw2 : db2;
  if (wave == 0 && c < h && dst) dst[c] += (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

template <int MAXJ>
void launch_fwd(int rows, int h, float eps, const float* x, long ldx, const float* w1,
                const float* b1, bf16_t* y1, const float* w2, const float* b2, bf16_t* y2,
                float* mean, float* rstd, hipStream_t s) {
  const int nblk = (rows + LN_WAVES - 1) / LN_WAVES;
  if (MMPT_LN_FWD_PERSIST && nblk > MMPT_LN_FWD_BLOCKS) {
    const size_t lds = (size_t)(y2 != nullptr ? 4 : 2) * h * sizeof(float);
    ln_fwd_persist_kernel<MAXJ><<<MMPT_LN_FWD_BLOCKS, 256, lds, s>>>(rows, h, eps, x, ldx, w1, b1,
                                                                     y1, w2, b2, y2, mean, rstd);
    return;
  }
  ln_fwd_kernel<MAXJ><<<nblk, 256, 0, s>>>(rows, h, eps, x, ldx, w1, b1, y1, w2, b2, y2, mean, rstd);
}

template <int MAXJ, bool DY32 = false>
void launch_bwd(int nblk, int rows, int h, const float* x, long ldx, const float* mean,
                const float* rstd, const bf16_t* dy1, const float* w1, const bf16_t* dy2,
                const float* w2, const float* dresid, float* dx, float* partials,
                hipStream_t s) {
  ln_bwd_kernel<MAXJ, DY32><<<nblk, 256, 0, s>>>(rows, h, x, ldx, mean, rstd, dy1, w1, dy2, w2,
                                                 dresid, dx, partials);
}

int pick_maxj(int64_t h) {
  const int64_t per = (h / 4 + 63) / 64;
  if (per <= 1) return 1;
  if (per <= 2) return 2;
  if (per <= 4) return 4;
  if (per <= 8) return 8;
  if (per <= 12) return 12;
  if (per <= 16) return 16;
  return -1;
}

}  // namespace
}  // namespace mmpt

using namespace mmpt;

extern "C" int mmpt_layernorm_fwd(int64_t rows, int64_t h, float eps, const float* x,
                                  int64_t ldx, const float* w1, const float* b1, void* y1,
                                  const float* w2, const float* b2, void* y2, float* mean,
                                  float* rstd, void* stream) {
  MMPT_REQUIRE(rows > 0 && h > 0 && h % 4 == 0 && ldx % 4 == 0, "layernorm_fwd: bad shape");
  MMPT_REQUIRE(x && w1 && b1 && y1 && mean && rstd, "layernorm_fwd: null pointer");
  MMPT_REQUIRE(y2 == nullptr || (w2 && b2), "layernorm_fwd: y2 needs w2/b2");
  const int mj = pick_maxj(h);
  MMPT_REQUIRE(mj > 0, "layernorm_fwd: h=%lld too large", (long long)h);
  hipStream_t s = (hipStream_t)stream;
  bf16_t *o1 = (bf16_t*)y1, *o2 = (bf16_t*)y2;
  switch (mj) {
    case 1: launch_fwd<1>(rows, h, eps, x, ldx, w1, b1, o1, w2, b2, o2, mean, rstd, s); break;
    case 2: launch_fwd<2>(rows, h, eps, x, ldx, w1, b1, o1, w2, b2, o2, mean, rstd, s); break;
    case 4: launch_fwd<4>(rows, h, eps, x, ldx, w1, b1, o1, w2, b2, o2, mean, rstd, s); break;
    case 8: launch_fwd<8>(rows, h, eps, x, ldx, w1, b1, o1, w2, b2, o2, mean, rstd, s); break;
    case 12: launch_fwd<12>(rows, h, eps, x, ldx, w1, b1, o1, w2, b2, o2, mean, rstd, s); break;
    default: launch_fwd<16>(rows, h, eps, x, ldx, w1, b1, o1, w2, b2, o2, mean, rstd, s); break;
  }
  return check_launch("layernorm_fwd");
}

extern "C" int64_t mmpt_layernorm_bwd_workspace_bytes(int64_t rows, int64_t h) {
  const int64_t nblk = std::min<int64_t>(LN_BWD_BLOCKS, (rows + LN_WAVES - 1) / LN_WAVES);
  return nblk * 4 * h * (int64_t)sizeof(float);
}

extern "C" int mmpt_layernorm_bwd(int64_t rows, int64_t h, const float* x, int64_t ldx,
                                  const float* mean, const float* rstd, const void* dy1,
                                  const float* w1, const void* dy2, const float* w2,
                                  const float* dresid, float* dx, float* dw1, float* db1,
                                  float* dw2, float* db2, void* workspace, void* stream) {
  MMPT_REQUIRE(rows > 0 && h > 0 && h % 4 == 0 && ldx % 4 == 0, "layernorm_bwd: bad shape");
  MMPT_REQUIRE(x && mean && rstd && dy1 && w1 && dx && workspace, "layernorm_bwd: null pointer");
  MMPT_REQUIRE(dy2 == nullptr || w2, "layernorm_bwd: dy2 needs w2");
  const int mj = pick_maxj(h);
  MMPT_REQUIRE(mj > 0, "layernorm_bwd: h=%lld too large", (long long)h);
  const int nblk = (int)std::min<int64_t>(LN_BWD_BLOCKS, (rows + LN_WAVES - 1) / LN_WAVES);
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const bf16_t *d1 = (const bf16_t*)dy1, *d2 = (const bf16_t*)dy2;
  switch (mj) {
    case 1: launch_bwd<1>(nblk, rows, h, x, ldx, mean, rstd, d1, w1, d2, w2, dresid, dx, part, s); break;
    case 2: launch_bwd<2>(nblk, rows, h, x, ldx, mean, rstd, d1, w1, d2, w2, dresid, dx, part, s); break;
    case 4: launch_bwd<4>(nblk, rows, h, x, ldx, mean, rstd, d1, w1, d2, w2, dresid, dx, part, s); break;
    case 8: launch_bwd<8>(nblk, rows, h, x, ldx, mean, rstd, d1, w1, d2, w2, dresid, dx, part, s); break;
    case 12: launch_bwd<12>(nblk, rows, h, x, ldx, mean, rstd, d1, w1, d2, w2, dresid, dx, part, s); break;
    default: launch_bwd<16>(nblk, rows, h, x, ldx, mean, rstd, d1, w1, d2, w2, dresid, dx, part, s); break;
  }
  int rc = check_launch("layernorm_bwd");
  if (rc) return rc;
  if (dw1 || db1 || dw2 || db2) {
    const int nq = dy2 ? 4 : 2;
    dim3 rg((unsigned)((h + 63) / 64), (unsigned)nq);
    ln_bwd_reduce<<<rg, 256, 0, s>>>(nblk, (int)h, part, dw1, db1, dy2 ? dw2 : nullptr,
                                     dy2 ? db2 : nullptr);
    rc = check_launch("layernorm_bwd_reduce");
  }
  return rc;
}

extern "C" int64_t mmpt_layernorm_bwd_ex_workspace_bytes(int64_t rows, int64_t h) {
  return std::min<int64_t>(LNR_BLOCKS, rows) * 5 * h * (int64_t)sizeof(float);
}

extern "C" int mmpt_layernorm_bwd_ex(int64_t rows, int64_t h, const float* x, int64_t ldx,
                                     const float* mean, const float* rstd, const void* dy1,
                                     const float* w1, const void* dy2, const float* w2,
                                     const float* dresid, float* dx, void* dx_bf16, float* dw1,
                                     float* db1, float* dw2, float* db2, float* dsum,
                                     float* dsum2, void* workspace, void* stream) {
  MMPT_REQUIRE(rows > 0 && h > 0 && h % 4 == 0 && ldx % 4 == 0, "layernorm_bwd_ex: bad shape");
  MMPT_REQUIRE(x && mean && rstd && dy1 && w1 && dx && workspace, "layernorm_bwd_ex: null pointer");
  MMPT_REQUIRE(dy2 == nullptr || w2, "layernorm_bwd_ex: dy2 needs w2");
  MMPT_REQUIRE(dsum == nullptr || dx_bf16, "layernorm_bwd_ex: dsum needs dx_bf16");
  MMPT_REQUIRE(dsum2 == nullptr || dsum, "layernorm_bwd_ex: dsum2 needs dsum");
  const int64_t per = (h / 4 + 255) / 256;
  MMPT_REQUIRE(per <= 4, "layernorm_bwd_ex: h=%lld too large", (long long)h);
  const int nblk = (int)std::min<int64_t>(LNR_BLOCKS, rows);
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const bf16_t *d1 = (const bf16_t*)dy1, *d2 = (const bf16_t*)dy2;
  bf16_t* xb = (bf16_t*)dx_bf16;
  const int ws = dsum != nullptr;
#define MMPT_LNR(PT) \
  ln_bwd_rows_kernel<PT><<<nblk, 256, 0, s>>>((int)rows, (int)h, x, ldx, mean, rstd, d1, w1, d2, w2, \
                                               dresid, dx, xb, ws, part)
  if (per <= 1) MMPT_LNR(1);
  else if (per <= 2) MMPT_LNR(2);
  else MMPT_LNR(4);
#undef MMPT_LNR
  int rc = check_launch("layernorm_bwd_ex");
  if (rc) return rc;
  dim3 rg((unsigned)((h + 63) / 64), 5u);
  ln_rows_reduce<<<rg, 256, 0, s>>>(nblk, (int)h, part, dw1, db1, dy2 ? dw2 : nullptr,
                                    dy2 ? db2 : nullptr, dsum, dsum2);
  return check_launch("layernorm_bwd_ex_reduce");
}

extern "C" int mmpt_layernorm_f32_fwd(int64_t rows, int64_t h, float eps, const float* x,
                                      const float* w, const float* b, float* y, float* mean,
                                      float* rstd, void* stream) {
  MMPT_REQUIRE(rows > 0 && h > 0 && h % 4 == 0, "layernorm_f32_fwd: bad shape");
  MMPT_REQUIRE(x && w && b && y && mean && rstd, "layernorm_f32_fwd: null pointer");
  const int mj = pick_maxj(h);
  MMPT_REQUIRE(mj > 0, "layernorm_f32_fwd: h=%lld too large", (long long)h);
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = (unsigned)((rows + LN_WAVES - 1) / LN_WAVES);
  const int r = (int)rows, hh = (int)h;
  switch (mj) {
    case 1: ln_fwd32_kernel<1><<<g, 256, 0, s>>>(r, hh, eps, x, w, b, y, mean, rstd); break;
    case 2: ln_fwd32_kernel<2><<<g, 256, 0, s>>>(r, hh, eps, x, w, b, y, mean, rstd); break;
    case 4: ln_fwd32_kernel<4><<<g, 256, 0, s>>>(r, hh, eps, x, w, b, y, mean, rstd); break;
    case 8: ln_fwd32_kernel<8><<<g, 256, 0, s>>>(r, hh, eps, x, w, b, y, mean, rstd); break;
    case 12: ln_fwd32_kernel<12><<<g, 256, 0, s>>>(r, hh, eps, x, w, b, y, mean, rstd); break;
    default: ln_fwd32_kernel<16><<<g, 256, 0, s>>>(r, hh, eps, x, w, b, y, mean, rstd); break;
  }
  return check_launch("layernorm_f32_fwd");
}

extern "C" int mmpt_layernorm_f32_bwd(int64_t rows, int64_t h, const float* x, const float* mean,
                                      const float* rstd, const float* dy, const float* w,
                                      float* dx, float* dw, float* db, void* workspace,
                                      void* stream) {
  MMPT_REQUIRE(rows > 0 && h > 0 && h % 4 == 0, "layernorm_f32_bwd: bad shape");
  MMPT_REQUIRE(x && mean && rstd && dy && w && dx && workspace, "layernorm_f32_bwd: null pointer");
  const int mj = pick_maxj(h);
  MMPT_REQUIRE(mj > 0, "layernorm_f32_bwd: h=%lld too large", (long long)h);
  const int nblk = (int)std::min<int64_t>(LN_BWD_BLOCKS, (rows + LN_WAVES - 1) / LN_WAVES);
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const bf16_t* d1 = (const bf16_t*)(const void*)dy;
  const int r = (int)rows, hh = (int)h;
#define MMPT_LN32B(J) launch_bwd<J, true>(nblk, r, hh, x, hh, mean, rstd, d1, w, nullptr, nullptr, nullptr, dx, part, s)
  switch (mj) {
    case 1: MMPT_LN32B(1); break;
    case 2: MMPT_LN32B(2); break;
    case 4: MMPT_LN32B(4); break;
    case 8: MMPT_LN32B(8); break;
    case 12: MMPT_LN32B(12); break;
    default: MMPT_LN32B(16); break;
  }
#undef MMPT_LN32B
  int rc = check_launch("layernorm_f32_bwd");
  if (rc) return rc;
  if (dw || db) {
    dim3 rg((unsigned)((h + 63) / 64), 2u);
    ln_bwd_reduce<<<rg, 256, 0, s>>>(nblk, hh, part, dw, db, nullptr, nullptr);
    rc = check_launch("layernorm_f32_bwd_reduce");
  }
  return rc;
}

// ---- RMSNorm (Llama): forward / backward over the same kernels (RMS instantiation) ----
extern "C" int mmpt_rmsnorm_fwd(int64_t rows, int64_t h, float eps, const float* x, int64_t ldx,
                                const float* w, void* y, float* rstd, void* stream) {
  MMPT_REQUIRE(rows > 0 && h > 0 && h % 4 == 0 && ldx % 4 == 0, "rmsnorm_fwd: bad shape");
  MMPT_REQUIRE(x && w && y && rstd, "rmsnorm_fwd: null pointer");
  const int mj = pick_maxj(h);
  MMPT_REQUIRE(mj > 0, "rmsnorm_fwd: h=%lld too large", (long long)h);
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = (unsigned)((rows + LN_WAVES - 1) / LN_WAVES);
  const int r = (int)rows, hh = (int)h;
  bf16_t* o = (bf16_t*)y;
#define MMPT_RMSF(J) ln_fwd_kernel<J, true><<<g, 256, 0, s>>>(r, hh, eps, x, ldx, w, nullptr, o, \
                                                             nullptr, nullptr, nullptr, nullptr, rstd)
  switch (mj) {
    case 1: MMPT_RMSF(1); break;
    case 2: MMPT_RMSF(2); break;
    case 4: MMPT_RMSF(4); break;
    case 8: MMPT_RMSF(8); break;
    case 12: MMPT_RMSF(12); break;
    default: MMPT_RMSF(16); break;
  }
#undef MMPT_RMSF
  return check_launch("rmsnorm_fwd");
}

extern "C" int64_t mmpt_rmsnorm_bwd_workspace_bytes(int64_t rows, int64_t h) {
  return mmpt_layernorm_bwd_ex_workspace_bytes(rows, h);
}

extern "C" int mmpt_rmsnorm_bwd(int64_t rows, int64_t h, const float* x, int64_t ldx,
                                const float* rstd, const void* dy, const float* w,
                                const float* dresid, float* dx, void* dx_bf16, float* dw,
                                void* workspace, void* stream) {
  MMPT_REQUIRE(rows > 0 && h > 0 && h % 4 == 0 && ldx % 4 == 0, "rmsnorm_bwd: bad shape");
  MMPT_REQUIRE(x && rstd && dy && w && dx && workspace, "rmsnorm_bwd: null pointer");
  const int64_t per = (h / 4 + 255) / 256;
  MMPT_REQUIRE(per <= 4, "rmsnorm_bwd: h=%lld too large", (long long)h);
  const int nblk = (int)std::min<int64_t>(LNR_BLOCKS, rows);
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const bf16_t* d1 = (const bf16_t*)dy;
  bf16_t* xb = (bf16_t*)dx_bf16;
#define MMPT_RMSB(PT) \
  ln_bwd_rows_kernel<PT, true><<<nblk, 256, 0, s>>>((int)rows, (int)h, x, ldx, nullptr, rstd, d1, w, \
                                                     nullptr, nullptr, dresid, dx, xb, 0, part)
  if (per <= 1) MMPT_RMSB(1);
  else if (per <= 2) MMPT_RMSB(2);
  else MMPT_RMSB(4);
#undef MMPT_RMSB
  int rc = check_launch("rmsnorm_bwd");
  if (rc || dw == nullptr) return rc;
  dim3 rg((unsigned)((h + 63) / 64), 1u);
  ln_rows_reduce<<<rg, 256, 0, s>>>(nblk, (int)h, part, dw, nullptr, nullptr, nullptr, nullptr,
                                    nullptr);
  return check_launch("rmsnorm_bwd_reduce");
}
