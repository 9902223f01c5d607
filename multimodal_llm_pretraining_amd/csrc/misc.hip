// HBM-bound kernels of the training step: bias-grad column sums, partial RoPE,
// fused cross-entropy fwd+bwd, deterministic sums, embedding gather / LLaVA
// image merge, ViT patch embedding glue, feature select, fused Adam/AdamW with
// bf16 shadow write, grad-norm and casts.  All loads/stores are 8-16 B per lane
// (cdna_hip_programming.md Guideline 13); reductions are fixed-shape two-stage
// so every result is bitwise reproducible run to run.
#include <math.h>
#include <string.h>

#include "common.h"

namespace mmpt {
namespace {

__device__ __forceinline__ float4 ld4bf(const bf16_t* p) {
  const uint2 u = *(const uint2*)p;
  return make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
}
__device__ __forceinline__ void st4bf(bf16_t* p, float4 v) {
  uint2 u;
  u.x = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
  u.y = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
  *(uint2*)p = u;
}

// ---------------- bias gradient: column sums of a bf16 [rows, cols] -------
// stage 1: one block per (2048-column group, 64-row chunk); 8 columns per thread
// (16-B loads, a row of the group is one contiguous 4-KiB read per block).
// stage 2: one block per 64 columns, the 4 waves split the chunks, LDS combine.
constexpr int CS_ROWS = 128;
__global__ __launch_bounds__(256) void colsum_stage1(int rows, int cols, const bf16_t* dy,
                                                     long ld, float* part) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c0 >= cols) return;
  const int r0 = blockIdx.y * CS_ROWS, r1 = min(rows, r0 + CS_ROWS);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int r = r0; r < r1; ++r) {
    const v8s v = *(const v8s*)(dy + (long)r * ld + c0);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += bf2f((bf16_t)v[e]);
  }
  float4* o = (float4*)(part + (long)blockIdx.y * cols + c0);
  o[0] = make_float4(s[0], s[1], s[2], s[3]);
  o[1] = make_float4(s[4], s[5], s[6], s[7]);
}
__global__ __launch_bounds__(256) void colsum_stage2(int nch, int cols, const float* part,
                                                     float* out, float* out2, int accumulate) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < cols)
#pragma unroll 8
    for (int k = wave; k < nch; k += 4) s += part[(long)k * cols + c];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && c < cols) {
    float t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    t = round_bf(t);  // addmm's grad_bias is produced in bf16 under autocast
    out[c] = accumulate ? out[c] + t : t;
    if (out2) out2[c] = accumulate ? out2[c] + t : t;
  }
}

// ---------------- partial rotary embedding (in place, q and k parts) -------
// 8 consecutive rotary dims per thread (16-B bf16 loads/stores, float4 cos/sin): the
// same per-element arithmetic as rope_kernel; half % 8 == 0.
__global__ __launch_bounds__(256) void rope8_kernel(long total, int seq, int heads, int nparts, int half,
                                                    bf16_t* qkv, long ld, long hs, long ps,
                                                    const float* __restrict__ cosb,
                                                    const float* __restrict__ sinb, int rot,
                                                    int inverse) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int h8 = half >> 3;
  const int i0 = (int)(idx % h8) * 8;
  long rest = idx / h8;
  const int part = (int)(rest % nparts);
  rest /= nparts;
  const int h = (int)(rest % heads);
  const long t = rest / heads;
  const int pos = (int)(t % seq);
  bf16_t* base = qkv + t * ld + h * hs + part * ps;
  const v8s a = *(const v8s*)(base + i0), bv = *(const v8s*)(base + i0 + half);
  const float* cp = cosb + (long)pos * rot + i0;
  const float* sp = sinb + (long)pos * rot + i0;
  float c1[8], c2[8], s1[8], s2[8];
  *(float4*)c1 = *(const float4*)cp;          *(float4*)(c1 + 4) = *(const float4*)(cp + 4);
  *(float4*)c2 = *(const float4*)(cp + half); *(float4*)(c2 + 4) = *(const float4*)(cp + half + 4);
  *(float4*)s1 = *(const float4*)sp;          *(float4*)(s1 + 4) = *(const float4*)(sp + 4);
  *(float4*)s2 = *(const float4*)(sp + half); *(float4*)(s2 + 4) = *(const float4*)(sp + half + 4);
  v8s o1, o2;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x1 = bf2f((bf16_t)a[e]), x2 = bf2f((bf16_t)bv[e]);
    float r1, r2;
    rope_rot(x1, x2, c1[e], c2[e], s1[e], s2[e], inverse != 0, r1, r2);
    o1[e] = (short)f2bf(r1);
    o2[e] = (short)f2bf(r2);
  }
  *(v8s*)(base + i0) = o1;
  *(v8s*)(base + i0 + half) = o2;
}

// One rotary pair (W = 2: two adjacent pairs) per thread, lanes on consecutive pairs of a row (a
// wave covers ~3 heads' q and k rotary dims of one token) and 32-bit index arithmetic — for
// rotary halves that are not a multiple of 8 (Pythia-2.8B: rot 20).  At C5's shape (69,568
// tokens x 32 heads) 286 us per launch (round 6; the round-5 one-row-per-lane kernel, 160 B
// between lanes: 553 us; rope_kernel's 64-bit divisions: 253 us in round 5's model).  The
// touched rotary dims span ~2/3 of the qkv cache lines, read and partially written back.
// Same per-element arithmetic as rope_kernel.
// W = 2: two adjacent pairs per thread (4-B bf16x2 / float2 accesses; half even, 4-B aligned rows)
template <int W>
__global__ __launch_bounds__(256) void rope_pair_kernel(int total, int seq, int heads, int nparts,
                                                        int half, bf16_t* qkv, long ld, long hs,
                                                        long ps, const float* __restrict__ cosb,
                                                        const float* __restrict__ sinb, int rot,
                                                        int inverse) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const unsigned hw = (unsigned)(half / W);
  const unsigned r1 = (unsigned)idx / hw;
  const int i = (idx - (int)(r1 * hw)) * W;
  const unsigned r2 = r1 / (unsigned)nparts;
  const int part = (int)(r1 - r2 * nparts);
  const unsigned t = r2 / (unsigned)heads;
  const int h = (int)(r2 - t * heads);
  const int pos = (int)(t % (unsigned)seq);
  bf16_t* base = qkv + (long)t * ld + h * hs + part * ps;
  const float* cp = cosb + pos * rot + i;
  const float* sp = sinb + pos * rot + i;
  if constexpr (W == 1) {
    const float x1 = bf2f(base[i]), x2 = bf2f(base[i + half]);
    float o1, o2;
    rope_rot(x1, x2, cp[0], cp[half], sp[0], sp[half], inverse != 0, o1, o2);
    base[i] = f2bf(o1);
    base[i + half] = f2bf(o2);
  } else {
    const uint32_t a = *(const uint32_t*)(base + i), bv = *(const uint32_t*)(base + i + half);
    const float2 c1 = *(const float2*)cp, c2 = *(const float2*)(cp + half);
    const float2 s1 = *(const float2*)sp, s2 = *(const float2*)(sp + half);
    float r1a, r2a, r1b, r2b;
    rope_rot(bf2f((bf16_t)(a & 0xffff)), bf2f((bf16_t)(bv & 0xffff)), c1.x, c2.x, s1.x, s2.x,
             inverse != 0, r1a, r2a);
    rope_rot(bf2f((bf16_t)(a >> 16)), bf2f((bf16_t)(bv >> 16)), c1.y, c2.y, s1.y, s2.y,
             inverse != 0, r1b, r2b);
    *(uint32_t*)(base + i) = (uint32_t)f2bf(r1a) | ((uint32_t)f2bf(r1b) << 16);
    *(uint32_t*)(base + i + half) = (uint32_t)f2bf(r2a) | ((uint32_t)f2bf(r2b) << 16);
  }
}

__global__ __launch_bounds__(256) void rope_kernel(long total, int seq, int heads, int nparts, int half,
                                                   bf16_t* qkv, long ld, long hs, long ps,
                                                   const float* __restrict__ cosb,
                                                   const float* __restrict__ sinb, int rot,
                                                   int inverse) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int i = (int)(idx % half);
  long rest = idx / half;
  const int part = (int)(rest % nparts);
  rest /= nparts;
  const int h = (int)(rest % heads);
  const long t = rest / heads;
  const int pos = (int)(t % seq);
  bf16_t* base = qkv + t * ld + h * hs + part * ps;
  const float x1 = bf2f(base[i]), x2 = bf2f(base[i + half]);
  const float c1 = cosb[pos * rot + i], c2 = cosb[pos * rot + i + half];
  const float s1 = sinb[pos * rot + i], s2 = sinb[pos * rot + i + half];
  float o1, o2;  // q*cos + rotate_half(q)*sin, or (inverse) the transpose of the rotation
  rope_rot(x1, x2, c1, c2, s1, s2, inverse != 0, o1, o2);
  base[i] = f2bf(o1);
  base[i + half] = f2bf(o2);
}

// ---------------- cross entropy (one 256-thread block per row) -------------
__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = sh[0];
  for (int k = 1; k < 4; ++k) r = is_max ? fmaxf(r, sh[k]) : r + sh[k];
  return r;
}

// vocab_valid <= vocab: logit columns >= vocab_valid are padding (a vocabulary padded to a
// multiple of 8 for 16-B rows, e.g. Llama-3's 128256 + <image> = 128257 -> 128264): they
// take no part in the softmax and get a zero gradient.
__global__ __launch_bounds__(256) void ce_kernel(int vocab, int vocab_valid, const bf16_t* logits,
                                                 long ld, const int64_t* labels, int64_t ignore,
                                                 float scale, float* loss_rows, bf16_t* dl,
                                                 long ldd) {
  __shared__ float sh[4];
  const int row = blockIdx.x;
  const bf16_t* x = logits + (long)row * ld;
  const int64_t lab = labels[row];
  // a label outside [0, vocab_valid) that is not ignore_index (torch's nll_loss asserts on
  // it): the row's loss is NaN and its gradient zero — never an out-of-range read
  const bool bad = lab != ignore && (lab < 0 || lab >= vocab_valid);
  const bool ign = lab == ignore || bad;
  const int nv = vocab >> 3;  // vocab % 8 == 0 enforced by the host wrapper
  // the label's logit before any thread writes dlogits (which may alias the logits)
  const float xlab = threadIdx.x == 0 && !ign ? bf2f(x[lab]) : 0.f;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < nv; c += 256) {
    const v8s v = *(const v8s*)(x + c * 8);
    float f[8];
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      f[e] = c * 8 + e < vocab_valid ? bf2f((bf16_t)v[e]) : -INFINITY;
      mx = fmaxf(mx, f[e]);
    }
    const float nm = fmaxf(m, mx);
    float acc = s * __expf(m - nm);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += __expf(f[e] - nm);
    s = acc;
    m = nm;
  }
  // combine (m, s) across the block
  const float gm = block_reduce(m, sh, true);
  const float gs = block_reduce(m == -INFINITY ? 0.f : s * __expf(m - gm), sh, false);
  const float lse = gm + logf(gs);
  if (threadIdx.x == 0) loss_rows[row] = bad ? __int_as_float(0x7fc00000) : ign ? 0.f : lse - xlab;
  if (dl == nullptr) return;
  bf16_t* d = dl + (long)row * ldd;
  const float inv = 1.0f / gs;
  for (int c = threadIdx.x; c < nv; c += 256) {
    const v8s v = *(const v8s*)(x + c * 8);
    v8s o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float g = 0.f;
      if (!ign && c * 8 + e < vocab_valid) {
        g = __expf(bf2f((bf16_t)v[e]) - gm) * inv;
        if (c * 8 + e == lab) g -= 1.0f;
        g *= scale;
      }
      o[e] = (short)f2bf(g);
    }
    *(v8s*)(d + c * 8) = o;
  }
}

// The same cross entropy with the row held in registers (round 5): each thread loads its NC
// chunks of 8 logits once (thread t holds chunks t, t + 256, ... — ce_kernel's assignment, so
// the online max / sum and every output are bitwise ce_kernel's) and the gradient pass reads
// them from registers instead of from memory a second time: the logits are read once, 13 GB
// per step less traffic at Pythia's 50,304-column rows (NC = 25: 100 VGPRs of row).
template <int NC>
__global__ __launch_bounds__(256) void ce_reg_kernel(int vocab, int vocab_valid, const bf16_t* logits,
                                                     long ld, const int64_t* labels, int64_t ignore,
                                                     float scale, float* loss_rows, bf16_t* dl,
                                                     long ldd) {
  __shared__ float sh[4];
  const int row = blockIdx.x;
  const bf16_t* x = logits + (long)row * ld;
  const int64_t lab = labels[row];
  const bool bad = lab != ignore && (lab < 0 || lab >= vocab_valid);  // (as ce_kernel)
  const bool ign = lab == ignore || bad;
  const int nv = vocab >> 3;
  v8s buf[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = threadIdx.x + k * 256;
    buf[k] = c < nv ? *(const v8s*)(x + c * 8) : v8s{0, 0, 0, 0, 0, 0, 0, 0};
  }
  float m = -INFINITY, s = 0.f;
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = threadIdx.x + k * 256;
    if (c >= nv) break;
    float f[8];
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      f[e] = c * 8 + e < vocab_valid ? bf2f((bf16_t)buf[k][e]) : -INFINITY;
      mx = fmaxf(mx, f[e]);
    }
    const float nm = fmaxf(m, mx);
    float acc = s * __expf(m - nm);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += __expf(f[e] - nm);
    s = acc;
    m = nm;
  }
  const float gm = block_reduce(m, sh, true);
  const float gs = block_reduce(m == -INFINITY ? 0.f : s * __expf(m - gm), sh, false);
  const float lse = gm + logf(gs);
  // the label's logit from the owner thread's registers (with dlogits written in place, a
  // memory read could see another thread's gradient already)
  if (ign) {
    if (threadIdx.x == 0) loss_rows[row] = bad ? __int_as_float(0x7fc00000) : 0.f;
  } else if ((int)((lab >> 3) & 255) == (int)threadIdx.x) {
    const int kl = (int)((lab >> 3) >> 8), el = (int)(lab & 7);
    float xl = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (k == kl && e == el) xl = bf2f((bf16_t)buf[k][e]);
    loss_rows[row] = lse - xl;
  }
  if (dl == nullptr) return;
  bf16_t* d = dl + (long)row * ldd;
  const float inv = 1.0f / gs;
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = threadIdx.x + k * 256;
    if (c >= nv) break;
    v8s o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float g = 0.f;
      if (!ign && c * 8 + e < vocab_valid) {
        g = __expf(bf2f((bf16_t)buf[k][e]) - gm) * inv;
        if (c * 8 + e == lab) g -= 1.0f;
        g *= scale;
      }
      o[e] = (short)f2bf(g);
    }
    *(v8s*)(d + c * 8) = o;
  }
}

// ---------------- deterministic sums ---------------------------------------
constexpr int SUM_BLOCKS = 256;
template <bool SQUARE>
__global__ __launch_bounds__(256) void sum_stage1(long n, const float* x, float* part) {
  __shared__ float sh[4];
  float s = 0.f;
  const long n4 = n >> 2;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 v = ((const float4*)x)[i];
    s += SQUARE ? (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w) : (v.x + v.y) + (v.z + v.w);
  }
  if (blockIdx.x == 0)
    for (long i = n4 * 4 + threadIdx.x; i < n; i += 256) s += SQUARE ? x[i] * x[i] : x[i];
  s = block_reduce(s, sh, false);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}
__global__ __launch_bounds__(256) void sum_stage2(int nparts, const float* part, float* out) {
  __shared__ float sh[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  s = block_reduce(s, sh, false);
  if (threadIdx.x == 0) out[0] = s;
}

// ---------------- embedding gather + image merge ---------------------------
__global__ __launch_bounds__(256) void embed_fwd_kernel(int rows, int h, const int64_t* ids,
                                                        const float* table, const int32_t* imap,
                                                        const bf16_t* img, float* out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nv = h >> 2;
  float4* o = (float4*)(out + (long)row * h);
  const int im = imap ? imap[row] : -1;
  if (im >= 0) {
    const bf16_t* src = img + (long)im * h;
    for (int i = lane; i < nv; i += 64) o[i] = ld4bf(src + i * 4);
  } else {
    const float4* src = (const float4*)(table + ids[row] * (long)h);
    for (int i = lane; i < nv; i += 64) o[i] = src[i];
  }
}
// Image-token rows of the embedding gradient: dimg[imap[row]] = bf16(dout[row]) (the
// masked_scatter backward); text rows are left to embed_bwd_seg_kernel.
__global__ __launch_bounds__(256) void embed_bwd_img_kernel(int rows, int h, const int32_t* imap,
                                                            const float* dout, bf16_t* dimg) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int im = imap[row];
  if (im < 0) return;
  const int nv = h >> 2;
  const float4* d = (const float4*)(dout + (long)row * h);
  for (int i = lane; i < nv; i += 64) st4bf(dimg + (long)im * h + i * 4, d[i]);
}

// Deterministic embedding_dense_backward (K8): the text rows are pre-sorted by
// token id (stable, so positions stay in order inside a segment; Batch builds the order
// once per micro-batch).  One workgroup per (segment, 2048-column slice): it sums the
// segment's rows in position order in fp32 and adds the sum to its table row — every
// table element has exactly one writer, no atomics, bitwise reproducible under any id
// collisions.  8 columns per thread (two float4 per row read).
__global__ __launch_bounds__(256) void embed_bwd_seg_kernel(int h, const int32_t* __restrict__ seg_id,
                                                            const int32_t* __restrict__ seg_off,
                                                            const int32_t* __restrict__ perm,
                                                            const float* __restrict__ dout,
                                                            float* __restrict__ dtable) {
  const int seg = blockIdx.x;
  const int c = (blockIdx.y * 256 + threadIdx.x) * 8;
  if (c >= h) return;
  const int r0 = seg_off[seg], r1 = seg_off[seg + 1];
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  for (int r = r0; r < r1; ++r) {
    const float4* d = (const float4*)(dout + (long)perm[r] * h + c);
    const float4 x = d[0], y = d[1];
    a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
    b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
  }
  float4* t = (float4*)(dtable + (long)seg_id[seg] * h + c);
  float4 o0 = t[0], o1 = t[1];
  o0.x += a.x; o0.y += a.y; o0.z += a.z; o0.w += a.w;
  o1.x += b.x; o1.y += b.y; o1.z += b.z; o1.w += b.w;
  t[0] = o0;
  t[1] = o1;
}

// The same with the segment count in device memory (mmpt_embed_segments builds the order
// on the device): a grid-stride loop over the segments, so the grid is sized without
// knowing nseg on the host.
__global__ __launch_bounds__(256) void embed_bwd_seg_dev_kernel(
    int h, const int32_t* __restrict__ nseg_p, const int32_t* __restrict__ seg_id,
    const int32_t* __restrict__ seg_off, const int32_t* __restrict__ perm,
    const float* __restrict__ dout, float* __restrict__ dtable) {
  const int c = (blockIdx.y * 256 + threadIdx.x) * 8;
  if (c >= h) return;
  const int nseg = nseg_p[0];
  for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    const int r0 = seg_off[seg], r1 = seg_off[seg + 1];
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    for (int r = r0; r < r1; ++r) {
      const float4* d = (const float4*)(dout + (long)perm[r] * h + c);
      const float4 x = d[0], y = d[1];
      a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
      b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
    }
    float4* t = (float4*)(dtable + (long)seg_id[seg] * h + c);
    float4 o0 = t[0], o1 = t[1];
    o0.x += a.x; o0.y += a.y; o0.z += a.z; o0.w += a.w;
    o1.x += b.x; o1.y += b.y; o1.z += b.z; o1.w += b.w;
    t[0] = o0;
    t[1] = o1;
  }
}

// Round 6: a segment longer than EMB_LONG rows — a padded batch where one id
// covers most rows (the reference's collators pad with one id, src/data/llava_data.py:95) —
// is no longer one workgroup's serial loop.  embed_piece_kernel cuts the sorted rows into
// EMB_CH-row chunks; each chunk sums, in position order, its piece of every long segment it
// overlaps (at most two: the one holding its first row, slot 0, and the one holding its last
// row, slot 1) into a partial row; embed_bwd_split_kernel then adds a long segment's pieces in
// chunk order, and sums every short segment serially exactly as embed_bwd_seg_dev_kernel does
// (bitwise unchanged).  Long segments are the sum of per-chunk partial sums: deterministic,
// one writer per table row, a different fp32 association than one serial loop.
constexpr int EMB_CH = 256, EMB_LONG = 1024;

// sum of rows perm[r0 .. r1) of dout at columns [c, c + 8), in order, 4 rows' loads in flight
__device__ __forceinline__ void emb_rowsum(const int32_t* __restrict__ perm,
                                           const float* __restrict__ dout, int h, int c, int r0,
                                           int r1, float4& a, float4& b) {
  int r = r0;
  for (; r + 4 <= r1; r += 4) {
    float4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4* d = (const float4*)(dout + (long)perm[r + u] * h + c);
      x[u] = d[0];
      y[u] = d[1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a.x += x[u].x; a.y += x[u].y; a.z += x[u].z; a.w += x[u].w;
      b.x += y[u].x; b.y += y[u].y; b.z += y[u].z; b.w += y[u].w;
    }
  }
  for (; r < r1; ++r) {
    const float4* d = (const float4*)(dout + (long)perm[r] * h + c);
    const float4 x = d[0], y = d[1];
    a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
    b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
  }
}

// the segment holding sorted row `row` (seg_off ascending, seg_off[nseg] = text rows)
__device__ __forceinline__ int emb_seg_of(const int32_t* __restrict__ seg_off, int nseg, int row) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (seg_off[mid] <= row) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(256) void embed_piece_kernel(
    int h, const int32_t* __restrict__ nseg_p, const int32_t* __restrict__ seg_off,
    const int32_t* __restrict__ perm, const float* __restrict__ dout, float* __restrict__ part) {
  const int c = (blockIdx.y * 256 + threadIdx.x) * 8;
  if (c >= h) return;
  const int nseg = nseg_p[0];
  if (nseg <= 0) return;
  const int ntext = seg_off[nseg];
  const int ch = blockIdx.x, q0 = ch * EMB_CH;
  if (q0 >= ntext) return;
  const int q1 = min(q0 + EMB_CH, ntext);
  const int sf = emb_seg_of(seg_off, nseg, q0), sl = emb_seg_of(seg_off, nseg, q1 - 1);
  for (int k = 0; k < 2; ++k) {
    const int sg = k == 0 ? sf : sl;
    if (k == 1 && sl == sf) break;
    const int r0 = seg_off[sg], r1 = seg_off[sg + 1];
    if (r1 - r0 <= EMB_LONG) continue;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    emb_rowsum(perm, dout, h, c, max(r0, q0), min(r1, q1), a, b);
    float4* o = (float4*)(part + ((long)ch * 2 + k) * h + c);
    o[0] = a;
    o[1] = b;
  }
}

__global__ __launch_bounds__(256) void embed_bwd_split_kernel(
    int h, const int32_t* __restrict__ nseg_p, const int32_t* __restrict__ seg_id,
    const int32_t* __restrict__ seg_off, const int32_t* __restrict__ perm,
    const float* __restrict__ dout, const float* __restrict__ part, float* __restrict__ dtable) {
  const int c = (blockIdx.y * 256 + threadIdx.x) * 8;
  if (c >= h) return;
  const int nseg = nseg_p[0];
  for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    const int r0 = seg_off[seg], r1 = seg_off[seg + 1];
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (r1 - r0 <= EMB_LONG) {
      emb_rowsum(perm, dout, h, c, r0, r1, a, b);  // (embed_bwd_seg_dev_kernel's order)
    } else {
      const int c0 = r0 / EMB_CH, c1 = (r1 - 1) / EMB_CH;
      for (int ch = c0; ch <= c1; ++ch) {
        // in its first chunk the segment holds that chunk's first row only when it starts on
        // the chunk boundary (slot 0); otherwise it holds the chunk's last row (slot 1)
        const int k = (ch == c0 && r0 != ch * EMB_CH) ? 1 : 0;
        const float4* pp = (const float4*)(part + ((long)ch * 2 + k) * h + c);
        const float4 x = pp[0], y = pp[1];
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
        b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
      }
    }
    float4* t = (float4*)(dtable + (long)seg_id[seg] * h + c);
    float4 o0 = t[0], o1 = t[1];
    o0.x += a.x; o0.y += a.y; o0.z += a.z; o0.w += a.w;
    o1.x += b.x; o1.y += b.y; o1.z += b.z; o1.w += b.w;
    t[0] = o0;
    t[1] = o1;
  }
}

// ---------------- row compaction of the lm_head / loss rows ----------------
// dst[r] = src[idx[r]] (bf16 rows, 16-B chunks; one wave per row)
__global__ __launch_bounds__(256) void gather_rows_kernel(int rows, int h8, const int32_t* idx,
                                                          const bf16_t* src, long lds_,
                                                          bf16_t* dst, long ldd) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const uint4* s = (const uint4*)(src + (long)idx[row] * lds_);
  uint4* d = (uint4*)(dst + (long)row * ldd);
  for (int i = threadIdx.x & 63; i < h8; i += 64) d[i] = s[i];
}
// dst[r] = map[r] >= 0 ? src[map[r]] : 0 (the inverse of the gather, zero-filling the rest)
__global__ __launch_bounds__(256) void expand_rows_kernel(int rows, int h8, const int32_t* map,
                                                          const bf16_t* src, long lds_,
                                                          bf16_t* dst, long ldd) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int j = map[row];
  uint4* d = (uint4*)(dst + (long)row * ldd);
  if (j < 0) {
    for (int i = threadIdx.x & 63; i < h8; i += 64) d[i] = make_uint4(0, 0, 0, 0);
  } else {
    const uint4* s = (const uint4*)(src + (long)j * lds_);
    for (int i = threadIdx.x & 63; i < h8; i += 64) d[i] = s[i];
  }
}

// ---------------- ViT patch embedding glue ---------------------------------
// cols[b*np + py*G + px][c*p*p + ky*p + kx] = bf16(pix[b][c][py*p+ky][px*p+kx])
__global__ __launch_bounds__(256) void im2col_kernel(long total8, int C, int S, int p,
                                                     const float* pix, bf16_t* cols) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;  // one 8-wide kx group
  if (idx >= total8) return;
  const int G = S / p;
  const int kgroups = C * p * p / 8;
  const int kg = (int)(idx % kgroups);
  const long prow = idx / kgroups;
  const int k = kg * 8;
  const int c = k / (p * p), ky = (k / p) % p, kx = k % p;
  const int b = (int)(prow / (G * G)), pi = (int)(prow % (G * G));
  const int py = pi / G, px = pi % G;
  const float* src = pix + (((long)b * C + c) * S + (py * p + ky)) * S + px * p + kx;
  const float4 a = *(const float4*)src, bq = *(const float4*)(src + 4);
  v8s o;
  o[0] = (short)f2bf(a.x); o[1] = (short)f2bf(a.y); o[2] = (short)f2bf(a.z); o[3] = (short)f2bf(a.w);
  o[4] = (short)f2bf(bq.x); o[5] = (short)f2bf(bq.y); o[6] = (short)f2bf(bq.z); o[7] = (short)f2bf(bq.w);
  *(v8s*)(cols + prow * (long)(C * p * p) + k) = o;
}

// Any patch size (CLIP-L/14: p = 14, C·p·p = 588): one thread per output element of a
// [rows][ld] im2col matrix; columns k >= C·p·p (the pad to a 16-B row) are written 0.
__global__ __launch_bounds__(256) void im2col_any_kernel(long total, int C, int S, int p, int ld,
                                                         const float* pix, bf16_t* cols) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int k = (int)(idx % ld);
  const long prow = idx / ld;
  float v = 0.f;
  if (k < C * p * p) {
    const int G = S / p;
    const int c = k / (p * p), ky = (k / p) % p, kx = k % p;
    const int b = (int)(prow / (G * G)), pi = (int)(prow % (G * G));
    const int py = pi / G, px = pi % G;
    v = pix[(((long)b * C + c) * S + (py * p + ky)) * S + px * p + kx];
  }
  cols[idx] = f2bf(v);
}

__global__ __launch_bounds__(256) void vit_embed_fwd_kernel(int batch, int np, int h,
                                                            const bf16_t* patch, const float* cls,
                                                            const float* pos, float* out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;  // float4 index
  const int nv = h >> 2;
  const long total = (long)batch * (np + 1) * nv;
  if (idx >= total) return;
  const int c4 = (int)(idx % nv);
  const long r = idx / nv;
  const int j = (int)(r % (np + 1));
  const int b = (int)(r / (np + 1));
  const float4 pe = ((const float4*)(pos + (long)j * h))[c4];
  float4 v = j == 0 ? ((const float4*)cls)[c4] : ld4bf(patch + ((long)b * np + j - 1) * h + c4 * 4);
  v.x += pe.x; v.y += pe.y; v.z += pe.z; v.w += pe.w;
  ((float4*)(out + r * h))[c4] = v;
}
__global__ __launch_bounds__(256) void vit_embed_bwd_kernel(int batch, int np, int h,
                                                            const float* dout, float* dcls,
                                                            float* dpos, bf16_t* dpatch) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;  // (j, c4)
  const int nv = h >> 2;
  if (idx >= (long)(np + 1) * nv) return;
  const int c4 = (int)(idx % nv);
  const int j = (int)(idx / nv);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b = 0; b < batch; ++b) {
    const float4 v = ((const float4*)(dout + ((long)b * (np + 1) + j) * h))[c4];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    if (j > 0 && dpatch) st4bf(dpatch + ((long)b * np + j - 1) * h + c4 * 4, v);
  }
  if (dpos) {
    float4* dp = (float4*)(dpos + (long)j * h) + c4;
    float4 o = *dp;
    o.x += s.x; o.y += s.y; o.z += s.z; o.w += s.w;
    *dp = o;
  }
  if (j == 0 && dcls) {
    float4* dc = (float4*)dcls + c4;
    float4 o = *dc;
    o.x += s.x; o.y += s.y; o.z += s.z; o.w += s.w;
    *dc = o;
  }
}

__global__ __launch_bounds__(256) void select_fwd_kernel(long total4, int np, int h,
                                                         const float* x, bf16_t* out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total4) return;
  const int nv = h >> 2;
  const int c4 = (int)(idx % nv);
  const long r = idx / nv;  // b*np + i
  const long b = r / np, i = r % np;
  st4bf(out + r * h + c4 * 4, ((const float4*)(x + (b * (np + 1) + 1 + i) * h))[c4]);
}
__global__ __launch_bounds__(256) void select_bwd_kernel(long total4, int np, int h,
                                                         const bf16_t* dout, float* dx, int acc) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;  // over batch*(np+1) rows
  if (idx >= total4) return;
  const int nv = h >> 2;
  const int c4 = (int)(idx % nv);
  const long r = idx / nv;
  const long b = r / (np + 1), j = r % (np + 1);
  float4 v = j == 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : ld4bf(dout + (b * np + j - 1) * h + c4 * 4);
  float4* d = (float4*)(dx + r * h) + c4;
  if (acc) {
    const float4 o = *d;
    v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
  }
  *d = v;
}

// ---------------- optimizer ------------------------------------------------
// torch.optim.Adam / AdamW single-tensor math (torch/optim/adam.py _single_tensor_adam):
//   AdamW: p *= 1 - lr*wd;  Adam: g += wd*p
//   m.lerp_(g, 1-b1); v = v*b2 + (1-b2)*g*g
//   p -= step_size * m / (sqrt(v)/bc2_sqrt + eps)
// One quad of the update.  Contraction is spelled out (fp contract off + explicit fmaf, the
// forms the single-quad kernel of rounds 1-5 compiled to), so every inlined copy rounds the
// same way whichever copy an element lands in (grid size decides that).
__device__ __forceinline__ void adam4(float4& P, float4 G, float4& M, float4& V, float sc, float lr,
                                      float b1, float b2, float eps, float wd, int adamw,
                                      float step_size, float bc2_sqrt) {
#pragma clang fp contract(off)
  float* pp = &P.x;
  float* gg = &G.x;
  float* mm = &M.x;
  float* vv = &V.x;
  const float decay = __builtin_fmaf(-lr, wd, 1.0f);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float gr = gg[e] * sc;
    if (adamw) {
      pp[e] = pp[e] * decay;
    } else if (wd != 0.f) {
      gr = __builtin_fmaf(wd, pp[e], gr);
    }
    mm[e] = __builtin_fmaf(1.0f - b1, gr - mm[e], mm[e]);
    vv[e] = __builtin_fmaf(gr, (1.0f - b2) * gr, vv[e] * b2);
    const float denom = sqrtf(vv[e]) / bc2_sqrt + eps;
    pp[e] = __builtin_fmaf(-step_size, mm[e] / denom, pp[e]);
  }
}

// Two float4 quads per lane per iteration (i and i + stride): eight 16-B loads in flight, so a
// small grid (the overlapped update's one workgroup per CU) still keeps HBM busy.
__global__ __launch_bounds__(256) void adam_kernel(long n, float* __restrict__ p,
                                                   const float* g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16_t* __restrict__ pb, float lr, float b1,
                                                   float b2, float eps, float wd, int adamw,
                                                   float step_size, float bc2_sqrt,
                                                   const float* __restrict__ gscale,
                                                   float* __restrict__ gzero) {
  const float sc = gscale ? gscale[0] : 1.0f;
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += 2 * stride) {
    const long j = i + stride;
    const bool two = j < n4;
    float4 P0 = ((float4*)p)[i], G0 = ((const float4*)g)[i], M0 = ((float4*)m)[i],
           V0 = ((float4*)v)[i];
    float4 P1, G1, M1, V1;
    if (two) {
      P1 = ((float4*)p)[j];
      G1 = ((const float4*)g)[j];
      M1 = ((float4*)m)[j];
      V1 = ((float4*)v)[j];
    }
    // zero_grad fused (gzero == g): the gradient is consumed, the next step accumulates from 0
    if (gzero) {
      ((float4*)gzero)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (two) ((float4*)gzero)[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    adam4(P0, G0, M0, V0, sc, lr, b1, b2, eps, wd, adamw, step_size, bc2_sqrt);
    ((float4*)p)[i] = P0;
    ((float4*)m)[i] = M0;
    ((float4*)v)[i] = V0;
    if (pb) st4bf(pb + i * 4, P0);
    if (two) {
      adam4(P1, G1, M1, V1, sc, lr, b1, b2, eps, wd, adamw, step_size, bc2_sqrt);
      ((float4*)p)[j] = P1;
      ((float4*)m)[j] = M1;
      ((float4*)v)[j] = V1;
      if (pb) st4bf(pb + j * 4, P1);
    }
  }
}

// 64x64 tile transpose through LDS (16-B loads and stores, padded rows)
__global__ __launch_bounds__(256) void transpose_kernel(int rows, int cols, const bf16_t* src,
                                                        long lds_, bf16_t* dst, long ldd) {
  __shared__ __attribute__((aligned(16))) bf16_t t[64][72];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tr = threadIdx.x >> 3, tc = (threadIdx.x & 7) * 8;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int r = tr + pass * 32;
    if (r0 + r < rows && c0 + tc < cols)
      *(v8s*)&t[r][tc] = *(const v8s*)(src + (long)(r0 + r) * lds_ + c0 + tc);
  }
  __syncthreads();
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int c = tr + pass * 32;  // output row = source column
    if (c0 + c < cols && r0 + tc < rows) {
      v8s o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (short)t[tc + e][c];
      *(v8s*)(dst + (long)(c0 + c) * ldd + r0 + tc) = o;
    }
  }
}

// Every W^T of the optimizer step in one launch (round 6): desc[i] = {offset, rows, cols,
// first tile} of weight i (src + offset is [rows][cols], dst + offset receives [cols][rows]);
// a workgroup finds its weight by binary search over the first tiles, then transposes one
// 64x64 tile as transpose_kernel does (bitwise the same copy, one launch instead of one per
// weight: 133 per step for ViT-B/16 + Pythia-1B).
__global__ __launch_bounds__(256) void transpose_batched_kernel(int n, const int64_t* __restrict__ desc,
                                                                const bf16_t* src, bf16_t* dst) {
  __shared__ __attribute__((aligned(16))) bf16_t t[64][72];
  const long tile = blockIdx.x;
  int lo = 0, hi = n - 1;  // the last weight whose first tile <= tile
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[4 * mid + 3] <= tile) lo = mid;
    else hi = mid - 1;
  }
  const long off = desc[4 * lo];
  const int rows = (int)desc[4 * lo + 1], cols = (int)desc[4 * lo + 2];
  const int local = (int)(tile - desc[4 * lo + 3]), tx = (cols + 63) / 64;
  const int r0 = (local / tx) * 64, c0 = (local % tx) * 64;
  const bf16_t* s = src + off;
  bf16_t* d = dst + off;
  const int tr = threadIdx.x >> 3, tc = (threadIdx.x & 7) * 8;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int r = tr + pass * 32;
    if (r0 + r < rows && c0 + tc < cols)
      *(v8s*)&t[r][tc] = *(const v8s*)(s + (long)(r0 + r) * cols + c0 + tc);
  }
  __syncthreads();
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int c = tr + pass * 32;
    if (c0 + c < cols && r0 + tc < rows) {
      v8s o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (short)t[tc + e][c];
      *(v8s*)(d + (long)(c0 + c) * rows + r0 + tc) = o;
    }
  }
}

__global__ void clip_coef_kernel(const float* sumsq, float max_norm, float* coef) {
  const float norm = sqrtf(sumsq[0]);
  coef[0] = fminf(1.0f, max_norm / (norm + 1e-6f));
}

__global__ __launch_bounds__(256) void cast_kernel(long n, const float* src, bf16_t* dst) {
  const long n4 = n >> 2;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
    st4bf(dst + i * 4, ((const float4*)src)[i]);
  if (blockIdx.x == 0)
    for (long i = n4 * 4 + threadIdx.x; i < n; i += 256) dst[i] = f2bf(src[i]);
}

inline unsigned grid_for(long work, long per_block, long cap) {
  long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (unsigned)(g > cap ? cap : g);
}

}  // namespace
}  // namespace mmpt

using namespace mmpt;

extern "C" int64_t mmpt_colsum_workspace_bytes(int64_t rows, int64_t cols) {
  return ((rows + CS_ROWS - 1) / CS_ROWS) * cols * (int64_t)sizeof(float);
}

extern "C" int mmpt_colsum_bf16(int64_t rows, int64_t cols, const void* dy, int64_t ld,
                                float* dbias, float* dbias2, int accumulate, void* workspace,
                                void* stream) {
  MMPT_REQUIRE(rows > 0 && cols > 0 && cols % 8 == 0 && ld % 8 == 0, "colsum: cols/ld %% 8");
  MMPT_REQUIRE(dy && dbias && workspace && ((uintptr_t)dy & 15) == 0, "colsum: bad pointer");
  hipStream_t s = (hipStream_t)stream;
  const int nch = (int)((rows + CS_ROWS - 1) / CS_ROWS);
  dim3 g1((unsigned)((cols / 8 + 255) / 256), nch);
  colsum_stage1<<<g1, 256, 0, s>>>((int)rows, (int)cols, (const bf16_t*)dy, ld, (float*)workspace);
  int rc = check_launch("colsum_stage1");
  if (rc) return rc;
  colsum_stage2<<<(unsigned)((cols + 63) / 64), 256, 0, s>>>(nch, (int)cols, (const float*)workspace,
                                                             dbias, dbias2, accumulate);
  return check_launch("colsum_stage2");
}

extern "C" int mmpt_colsum_f32(int64_t rows, int64_t cols, const float* part, float* dbias,
                               float* dbias2, int accumulate, void* stream) {
  MMPT_REQUIRE(rows > 0 && cols > 0 && part && dbias, "colsum_f32: bad arguments");
  colsum_stage2<<<(unsigned)((cols + 63) / 64), 256, 0, (hipStream_t)stream>>>(
      (int)rows, (int)cols, part, dbias, dbias2, accumulate);
  return check_launch("colsum_f32");
}

extern "C" int mmpt_rope_inplace(int64_t tokens, int64_t seq, int64_t heads, int64_t head_dim,
                                 int64_t rot_dims, void* qkv, int64_t ld, int64_t head_stride,
                                 int64_t part_stride, int64_t parts, const float* cos,
                                 const float* sin, int inverse, void* stream) {
  MMPT_REQUIRE(tokens > 0 && seq > 0 && heads > 0 && rot_dims > 0 && rot_dims % 2 == 0 &&
                   rot_dims <= head_dim && (parts == 1 || parts == 2),
               "rope: bad shape");
  MMPT_REQUIRE(qkv && cos && sin, "rope: null pointer");
  const long half = rot_dims / 2;
  const bool vec = half % 8 == 0 && ld % 8 == 0 && head_stride % 8 == 0 && part_stride % 8 == 0 &&
                   rot_dims % 4 == 0 && ((uintptr_t)qkv & 15) == 0 && ((uintptr_t)cos & 15) == 0 &&
                   ((uintptr_t)sin & 15) == 0;
  if (vec) {
    const long total = tokens * heads * parts * (half / 8);
    rope8_kernel<<<grid_for(total, 256, 1L << 30), 256, 0, (hipStream_t)stream>>>(
        total, (int)seq, (int)heads, (int)parts, (int)half, (bf16_t*)qkv, ld, head_stride, part_stride, cos,
        sin, (int)rot_dims, inverse);
    return check_launch("rope");
  }
  const long npairs = tokens * heads * parts * half;
  const bool w2 = half % 2 == 0 && ld % 2 == 0 && head_stride % 2 == 0 && part_stride % 2 == 0 &&
                  ((uintptr_t)qkv & 3) == 0 && ((uintptr_t)cos & 7) == 0 &&
                  ((uintptr_t)sin & 7) == 0 && rot_dims % 2 == 0;
  if (npairs < (1L << 31) - 256) {
    const long n = w2 ? npairs / 2 : npairs;
    const dim3 grid((unsigned)((n + 255) / 256));
    if (w2)
      rope_pair_kernel<2><<<grid, 256, 0, (hipStream_t)stream>>>(
          (int)n, (int)seq, (int)heads, (int)parts, (int)half, (bf16_t*)qkv, ld, head_stride,
          part_stride, cos, sin, (int)rot_dims, inverse);
    else
      rope_pair_kernel<1><<<grid, 256, 0, (hipStream_t)stream>>>(
          (int)n, (int)seq, (int)heads, (int)parts, (int)half, (bf16_t*)qkv, ld, head_stride,
          part_stride, cos, sin, (int)rot_dims, inverse);
    return check_launch("rope");
  }
  const long total = tokens * heads * parts * half;
  rope_kernel<<<grid_for(total, 256, 1L << 30), 256, 0, (hipStream_t)stream>>>(
      total, (int)seq, (int)heads, (int)parts, (int)half, (bf16_t*)qkv, ld, head_stride, part_stride, cos,
      sin, (int)rot_dims, inverse);
  return check_launch("rope");
}

// MMPT_CE_REG=0: the two-pass cross entropy everywhere (A/B); read once, mmpt_set_switch
static int g_ce_reg = -1;
static int ce_reg() {
  if (g_ce_reg < 0) {
    const char* e = getenv("MMPT_CE_REG");
    g_ce_reg = e != nullptr && e[0] == '0' ? 0 : 1;
  }
  return g_ce_reg;
}
namespace mmpt {
int* misc_switch(const char* name, int* prev) {
  if (strcmp(name, "MMPT_CE_REG") == 0) {
    *prev = ce_reg();
    return &g_ce_reg;
  }
  return nullptr;
}
}  // namespace mmpt

extern "C" int mmpt_cross_entropy(int64_t rows, int64_t vocab, int64_t vocab_valid,
                                  const void* logits, int64_t ld, const int64_t* labels,
                                  int64_t ignore_index, float grad_scale, float* loss_rows,
                                  void* dlogits, int64_t ld_d, void* stream) {
  MMPT_REQUIRE(rows > 0 && vocab > 0 && vocab % 8 == 0 && ld % 8 == 0 && ld_d % 8 == 0,
               "cross_entropy: vocab/ld must be multiples of 8");
  MMPT_REQUIRE(vocab_valid > 0 && vocab_valid <= vocab, "cross_entropy: bad vocab_valid");
  MMPT_REQUIRE(logits && labels && loss_rows, "cross_entropy: null pointer");
  const int64_t nc = (vocab / 8 + 255) / 256;  // chunks of 8 logits per thread
  // the row in registers (one read of the logits) up to 32 chunks per thread (vocab <= 65,536;
  // a Llama-sized row would take 250 VGPRs: the two-pass kernel)
  if (nc > 0 && nc <= 32 && ce_reg()) {
    const unsigned g = (unsigned)rows;
    hipStream_t st = (hipStream_t)stream;
#define MMPT_CE(NCV)                                                                           \
  ce_reg_kernel<NCV><<<g, 256, 0, st>>>((int)vocab, (int)vocab_valid, (const bf16_t*)logits, ld, \
                                        labels, ignore_index, grad_scale, loss_rows,           \
                                        (bf16_t*)dlogits, ld_d)
    if (nc <= 8) MMPT_CE(8);
    else if (nc <= 16) MMPT_CE(16);
    else if (nc <= 25) MMPT_CE(25);
    else MMPT_CE(32);
#undef MMPT_CE
    return check_launch("cross_entropy");
  }
  ce_kernel<<<(unsigned)rows, 256, 0, (hipStream_t)stream>>>(
      (int)vocab, (int)vocab_valid, (const bf16_t*)logits, ld, labels, ignore_index, grad_scale, loss_rows,
      (bf16_t*)dlogits, ld_d);
  return check_launch("cross_entropy");
}

extern "C" int64_t mmpt_sum_workspace_bytes(int64_t n) {
  (void)n;
  return SUM_BLOCKS * (int64_t)sizeof(float);
}
extern "C" int64_t mmpt_l2norm_workspace_bytes(int64_t n) { return mmpt_sum_workspace_bytes(n); }

template <bool SQ>
static int run_sum(int64_t n, const float* x, float* out, void* ws, void* stream) {
  MMPT_REQUIRE(n > 0 && x && out && ws, "sum: bad args");
  MMPT_REQUIRE(((uintptr_t)x & 15) == 0, "sum: x must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  sum_stage1<SQ><<<SUM_BLOCKS, 256, 0, s>>>(n, x, (float*)ws);
  int rc = check_launch("sum_stage1");
  if (rc) return rc;
  sum_stage2<<<1, 256, 0, s>>>(SUM_BLOCKS, (const float*)ws, out);
  return check_launch("sum_stage2");
}
extern "C" int mmpt_sum_f32(int64_t n, const float* x, float* out, void* ws, void* stream) {
  return run_sum<false>(n, x, out, ws, stream);
}
extern "C" int mmpt_sumsq_f32(int64_t n, const float* x, float* out, void* ws, void* stream) {
  return run_sum<true>(n, x, out, ws, stream);
}

extern "C" int mmpt_embed_fwd(int64_t rows, int64_t h, const int64_t* ids, const float* table,
                              const int32_t* img_map, const void* img, float* out, void* stream) {
  MMPT_REQUIRE(rows > 0 && h % 4 == 0 && ids && table && out, "embed_fwd: bad args");
  MMPT_REQUIRE(img_map == nullptr || img != nullptr, "embed_fwd: img_map needs img");
  embed_fwd_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      (int)rows, (int)h, ids, table, img_map, (const bf16_t*)img, out);
  return check_launch("embed_fwd");
}
extern "C" int mmpt_embed_bwd(int64_t rows, int64_t h, int64_t nseg, const int32_t* seg_id,
                              const int32_t* seg_off, const int32_t* perm, const int32_t* img_map,
                              const float* dout, float* dtable, void* dimg, void* stream) {
  MMPT_REQUIRE(rows > 0 && h % 8 == 0 && nseg >= 0 && dout, "embed_bwd: bad args (h %% 8 == 0)");
  MMPT_REQUIRE(dtable == nullptr || nseg == 0 || (seg_id && seg_off && perm),
               "embed_bwd: dtable needs the sorted segments");
  MMPT_REQUIRE(dimg == nullptr || img_map != nullptr, "embed_bwd: dimg needs img_map");
  MMPT_REQUIRE(((uintptr_t)dout & 15) == 0 && (dtable == nullptr || ((uintptr_t)dtable & 15) == 0),
               "embed_bwd: dout/dtable must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  if (dimg != nullptr) {
    embed_bwd_img_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, s>>>((int)rows, (int)h, img_map,
                                                                     dout, (bf16_t*)dimg);
    int rc = check_launch("embed_bwd_img");
    if (rc) return rc;
  }
  if (dtable != nullptr && nseg > 0) {
    dim3 grid((unsigned)nseg, (unsigned)((h / 8 + 255) / 256));
    embed_bwd_seg_kernel<<<grid, 256, 0, s>>>((int)h, seg_id, seg_off, perm, dout, dtable);
    return check_launch("embed_bwd_seg");
  }
  return MMPT_OK;
}

extern "C" int mmpt_embed_bwd_dev(int64_t rows, int64_t h, int64_t max_seg,
                                  const int32_t* nseg, const int32_t* seg_id,
                                  const int32_t* seg_off, const int32_t* perm,
                                  const int32_t* img_map, const float* dout, float* dtable,
                                  void* dimg, void* stream) {
  MMPT_REQUIRE(rows > 0 && h % 8 == 0 && max_seg >= 0 && dout, "embed_bwd_dev: bad args (h %% 8 == 0)");
  MMPT_REQUIRE(dtable == nullptr || max_seg == 0 || (nseg && seg_id && seg_off && perm),
               "embed_bwd_dev: dtable needs the device segments");
  MMPT_REQUIRE(dimg == nullptr || img_map != nullptr, "embed_bwd_dev: dimg needs img_map");
  MMPT_REQUIRE(((uintptr_t)dout & 15) == 0 && (dtable == nullptr || ((uintptr_t)dtable & 15) == 0),
               "embed_bwd_dev: dout/dtable must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  if (dimg != nullptr) {
    embed_bwd_img_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, s>>>((int)rows, (int)h, img_map,
                                                                     dout, (bf16_t*)dimg);
    int rc = check_launch("embed_bwd_img");
    if (rc) return rc;
  }
  if (dtable != nullptr && max_seg > 0) {
    // 8 workgroups per CU of a 256-CU part cover the segments in a few strides
    dim3 grid((unsigned)(max_seg < 2048 ? max_seg : 2048), (unsigned)((h / 8 + 255) / 256));
    embed_bwd_seg_dev_kernel<<<grid, 256, 0, s>>>((int)h, nseg, seg_id, seg_off, perm, dout,
                                                   dtable);
    return check_launch("embed_bwd_seg_dev");
  }
  return MMPT_OK;
}

extern "C" int64_t mmpt_embed_bwd_split_workspace_bytes(int64_t rows, int64_t h) {
  if (rows <= 0 || h <= 0) return -1;
  return ((rows + EMB_CH - 1) / EMB_CH) * 2 * h * (int64_t)sizeof(float);
}

extern "C" int mmpt_embed_bwd_split(int64_t rows, int64_t h, int64_t max_seg, const int32_t* nseg,
                                    const int32_t* seg_id, const int32_t* seg_off,
                                    const int32_t* perm, const int32_t* img_map, const float* dout,
                                    float* dtable, void* dimg, void* workspace, int64_t ws_bytes,
                                    void* stream) {
  MMPT_REQUIRE(rows > 0 && h % 8 == 0 && max_seg >= 0 && max_seg <= rows && dout,
               "embed_bwd_split: bad args (h %% 8 == 0, max_seg <= rows)");
  MMPT_REQUIRE(dtable == nullptr || max_seg == 0 || (nseg && seg_id && seg_off && perm),
               "embed_bwd_split: dtable needs the device segments");
  MMPT_REQUIRE(dimg == nullptr || img_map != nullptr, "embed_bwd_split: dimg needs img_map");
  MMPT_REQUIRE(((uintptr_t)dout & 15) == 0 && (dtable == nullptr || ((uintptr_t)dtable & 15) == 0),
               "embed_bwd_split: dout/dtable must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  if (dimg != nullptr) {
    embed_bwd_img_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, s>>>((int)rows, (int)h, img_map,
                                                                     dout, (bf16_t*)dimg);
    int rc = check_launch("embed_bwd_img");
    if (rc) return rc;
  }
  if (dtable == nullptr || max_seg == 0) return MMPT_OK;
  const int64_t need = mmpt_embed_bwd_split_workspace_bytes(max_seg, h);
  MMPT_REQUIRE(workspace != nullptr && ((uintptr_t)workspace & 15) == 0 && ws_bytes >= need,
               "embed_bwd_split: workspace of %lld bytes needed (16-B aligned)", (long long)need);
  const unsigned ys = (unsigned)((h / 8 + 255) / 256);
  embed_piece_kernel<<<dim3((unsigned)((max_seg + EMB_CH - 1) / EMB_CH), ys), 256, 0, s>>>(
      (int)h, nseg, seg_off, perm, dout, (float*)workspace);
  int rc = check_launch("embed_piece");
  if (rc) return rc;
  dim3 grid((unsigned)(max_seg < 2048 ? max_seg : 2048), ys);
  embed_bwd_split_kernel<<<grid, 256, 0, s>>>((int)h, nseg, seg_id, seg_off, perm, dout,
                                              (const float*)workspace, dtable);
  return check_launch("embed_bwd_split");
}

extern "C" int mmpt_im2col_patches(int64_t batch, int64_t channels, int64_t image, int64_t patch,
                                   const float* pixels, void* cols, void* stream) {
  MMPT_REQUIRE(batch > 0 && channels > 0 && patch > 0 && image % patch == 0 && patch % 8 == 0,
               "im2col: image %% patch == 0 and patch %% 8 == 0 required");
  MMPT_REQUIRE(pixels && cols, "im2col: null pointer");
  const long G = image / patch;
  const long total8 = batch * G * G * channels * patch * patch / 8;
  im2col_kernel<<<grid_for(total8, 256, 1L << 30), 256, 0, (hipStream_t)stream>>>(
      total8, (int)channels, (int)image, (int)patch, pixels, (bf16_t*)cols);
  return check_launch("im2col");
}

extern "C" int mmpt_im2col_patches_ex(int64_t batch, int64_t channels, int64_t image,
                                      int64_t patch, const float* pixels, void* cols,
                                      int64_t ld_cols, void* stream) {
  MMPT_REQUIRE(batch > 0 && channels > 0 && patch > 0 && image % patch == 0 &&
                   ld_cols >= channels * patch * patch,
               "im2col_ex: image %% patch == 0 and ld_cols >= C*p*p required");
  MMPT_REQUIRE(pixels && cols, "im2col_ex: null pointer");
  const long G = image / patch;
  const long total = batch * G * G * ld_cols;
  im2col_any_kernel<<<grid_for(total, 256, 1L << 30), 256, 0, (hipStream_t)stream>>>(
      total, (int)channels, (int)image, (int)patch, (int)ld_cols, pixels, (bf16_t*)cols);
  return check_launch("im2col_ex");
}

extern "C" int mmpt_vit_embed_fwd(int64_t batch, int64_t num_patches, int64_t h,
                                  const void* patch_out, const float* cls, const float* pos,
                                  float* out, void* stream) {
  MMPT_REQUIRE(batch > 0 && num_patches > 0 && h % 4 == 0 && patch_out && cls && pos && out,
               "vit_embed_fwd: bad args");
  const long total = batch * (num_patches + 1) * (h / 4);
  vit_embed_fwd_kernel<<<grid_for(total, 256, 1L << 30), 256, 0, (hipStream_t)stream>>>(
      (int)batch, (int)num_patches, (int)h, (const bf16_t*)patch_out, cls, pos, out);
  return check_launch("vit_embed_fwd");
}
extern "C" int mmpt_vit_embed_bwd(int64_t batch, int64_t num_patches, int64_t h,
                                  const float* dout, float* dcls, float* dpos, void* dpatch,
                                  void* stream) {
  MMPT_REQUIRE(batch > 0 && num_patches > 0 && h % 4 == 0 && dout, "vit_embed_bwd: bad args");
  const long total = (num_patches + 1) * (h / 4);
  vit_embed_bwd_kernel<<<grid_for(total, 256, 1L << 30), 256, 0, (hipStream_t)stream>>>(
      (int)batch, (int)num_patches, (int)h, dout, dcls, dpos, (bf16_t*)dpatch);
  return check_launch("vit_embed_bwd");
}

extern "C" int mmpt_select_patches_fwd(int64_t batch, int64_t num_patches, int64_t h,
                                       const float* x, void* out, void* stream) {
  MMPT_REQUIRE(batch > 0 && num_patches > 0 && h % 4 == 0 && x && out, "select_fwd: bad args");
  const long total = batch * num_patches * (h / 4);
  select_fwd_kernel<<<grid_for(total, 256, 1L << 30), 256, 0, (hipStream_t)stream>>>(
      total, (int)num_patches, (int)h, x, (bf16_t*)out);
  return check_launch("select_patches_fwd");
}
extern "C" int mmpt_select_patches_bwd(int64_t batch, int64_t num_patches, int64_t h,
                                       const void* dout, float* dx, int accumulate, void* stream) {
  MMPT_REQUIRE(batch > 0 && num_patches > 0 && h % 4 == 0 && dout && dx, "select_bwd: bad args");
  const long total = batch * (num_patches + 1) * (h / 4);
  select_bwd_kernel<<<grid_for(total, 256, 1L << 30), 256, 0, (hipStream_t)stream>>>(
      total, (int)num_patches, (int)h, (const bf16_t*)dout, dx, accumulate);
  return check_launch("select_patches_bwd");
}

extern "C" int mmpt_adam_step(int64_t n, float* param, const float* grad, float* exp_avg,
                              float* exp_avg_sq, void* param_bf16, float lr, float beta1,
                              float beta2, float eps, float weight_decay, int adamw, int64_t step,
                              const float* grad_scale_ptr, void* stream) {
  MMPT_REQUIRE(n > 0 && n % 4 == 0 && param && grad && exp_avg && exp_avg_sq && step >= 1,
               "adam_step: bad args (n %% 4 == 0, step >= 1)");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  adam_kernel<<<grid_for(n / 4, 256, 8192), 256, 0, (hipStream_t)stream>>>(
      n, param, grad, exp_avg, exp_avg_sq, (bf16_t*)param_bf16, lr, beta1, beta2, eps,
      weight_decay, adamw, step_size, bc2_sqrt, grad_scale_ptr, nullptr);
  return check_launch("adam_step");
}

extern "C" int mmpt_adam_step_zero_grad(int64_t n, float* param, float* grad, float* exp_avg,
                                        float* exp_avg_sq, void* param_bf16, float lr, float beta1,
                                        float beta2, float eps, float weight_decay, int adamw,
                                        int64_t step, const float* grad_scale_ptr, int max_blocks,
                                        void* stream) {
  MMPT_REQUIRE(n > 0 && n % 4 == 0 && param && grad && exp_avg && exp_avg_sq && step >= 1,
               "adam_step_zero_grad: bad args (n %% 4 == 0, step >= 1)");
  MMPT_REQUIRE(((uintptr_t)param & 15) == 0 && ((uintptr_t)grad & 15) == 0 &&
                   ((uintptr_t)exp_avg & 15) == 0 && ((uintptr_t)exp_avg_sq & 15) == 0 &&
                   ((uintptr_t)param_bf16 & 7) == 0,
               "adam_step_zero_grad: buffers must be 16-B aligned (bf16 shadow 8-B)");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  MMPT_REQUIRE(max_blocks >= 0, "adam_step_zero_grad: max_blocks >= 0");
  adam_kernel<<<grid_for(n / 4, 256, max_blocks > 0 ? max_blocks : 8192), 256, 0,
                (hipStream_t)stream>>>(n, param, grad, exp_avg, exp_avg_sq, (bf16_t*)param_bf16,
                                       lr, beta1, beta2, eps, weight_decay, adamw, step_size,
                                       bc2_sqrt, grad_scale_ptr, grad);
  return check_launch("adam_step_zero_grad");
}

extern "C" int mmpt_clip_coef(const float* sumsq, float max_norm, float* coef, void* stream) {
  MMPT_REQUIRE(sumsq && coef, "clip_coef: null pointer");
  clip_coef_kernel<<<1, 1, 0, (hipStream_t)stream>>>(sumsq, max_norm, coef);
  return check_launch("clip_coef");
}

extern "C" int mmpt_transpose_bf16(int64_t rows, int64_t cols, const void* src, int64_t ld_src,
                                   void* dst, int64_t ld_dst, void* stream) {
  MMPT_REQUIRE(rows > 0 && cols > 0 && rows % 8 == 0 && cols % 8 == 0 && ld_src % 8 == 0 &&
                   ld_dst % 8 == 0 && src && dst,
               "transpose: dims and leading dims must be multiples of 8");
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64));
  transpose_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((int)rows, (int)cols, (const bf16_t*)src,
                                                          ld_src, (bf16_t*)dst, ld_dst);
  return check_launch("transpose_bf16");
}

extern "C" int mmpt_transpose_bf16_batched(int64_t n, const int64_t* desc, int64_t total_tiles,
                                           const void* src, void* dst, void* stream) {
  MMPT_REQUIRE(n > 0 && n < (1LL << 31) && desc && src && dst && total_tiles > 0 &&
                   total_tiles < (1LL << 31) && ((uintptr_t)src & 15) == 0 &&
                   ((uintptr_t)dst & 15) == 0,
               "transpose_bf16_batched: bad arguments (desc on the device, 16-B aligned bases)");
  transpose_batched_kernel<<<(unsigned)total_tiles, 256, 0, (hipStream_t)stream>>>(
      (int)n, desc, (const bf16_t*)src, (bf16_t*)dst);
  return check_launch("transpose_bf16_batched");
}

extern "C" int mmpt_cast_f32_bf16(int64_t n, const float* src, void* dst, void* stream) {
  MMPT_REQUIRE(n > 0 && src && dst, "cast: bad args");
  cast_kernel<<<grid_for(n / 4 + 1, 256, 8192), 256, 0, (hipStream_t)stream>>>(n, src, (bf16_t*)dst);
  return check_launch("cast_f32_bf16");
}

extern "C" int mmpt_gather_rows_bf16(int64_t rows, int64_t h, const int32_t* idx, const void* src,
                                     int64_t ld_src, void* dst, int64_t ld_dst, void* stream) {
  MMPT_REQUIRE(rows >= 0 && h > 0 && h % 8 == 0 && ld_src % 8 == 0 && ld_dst % 8 == 0,
               "gather_rows: h and leading dims must be multiples of 8");
  MMPT_REQUIRE(rows == 0 || (idx && src && dst), "gather_rows: null pointer");
  MMPT_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "gather_rows: alignment");
  if (rows == 0) return MMPT_OK;
  gather_rows_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      (int)rows, (int)(h / 8), idx, (const bf16_t*)src, ld_src, (bf16_t*)dst, ld_dst);
  return check_launch("gather_rows");
}

extern "C" int mmpt_expand_rows_bf16(int64_t rows, int64_t h, const int32_t* map, const void* src,
                                     int64_t ld_src, void* dst, int64_t ld_dst, void* stream) {
  MMPT_REQUIRE(rows > 0 && h > 0 && h % 8 == 0 && ld_src % 8 == 0 && ld_dst % 8 == 0,
               "expand_rows: h and leading dims must be multiples of 8");
  MMPT_REQUIRE(map && src && dst, "expand_rows: null pointer");
  MMPT_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "expand_rows: alignment");
  expand_rows_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      (int)rows, (int)(h / 8), map, (const bf16_t*)src, ld_src, (bf16_t*)dst, ld_dst);
  return check_launch("expand_rows");
}
