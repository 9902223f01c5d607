// K1: bf16 MFMA GEMM with fused epilogues (replaces aten::addmm / mm launched by
// nn.Linear under autocast).
//
// Two tile shapes, same code:
//   256x256x64, 512 threads = 8 waves (2 along M x 4 along N, 128x64 per wave),
//     1 workgroup per CU, 128 KiB LDS double buffer — the big activation GEMMs;
//   128x128x64, 256 threads = 4 waves (2x2, 64x64 per wave), 64 KiB LDS, 2 per CU —
//     small problems (ViT, projector) where 256^2 tiles cannot fill 256 CUs.
// MFMA v_mfma_f32_16x16x32_bf16.  Operands are staged HBM -> LDS with
// global_load_lds_dwordx4 (no VGPR round trip); the load of K-tile t+1 is issued
// before the MFMAs of tile t.
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
#include <stdlib.h>

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
};

__device__ __forceinline__ int swz_kr(int kr) {
  return 2 * ((kr & 3) | (((kr >> 3) & 1) << 2));
}

// --- HBM -> LDS staging of an R-row operand image --------------------------
template <int LAYOUT, int R, int NW>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ src, long ld, int Rlim, int K,
                                      int r0, int k0, char* img, int wave, int lane) {
  constexpr int PIECES = R * BK * 2 / 1024;  // 1-KiB DMA pieces in the image
  static_assert(PIECES % NW == 0, "pieces must split evenly over waves");
#pragma unroll
  for (int i = 0; i < PIECES / NW; ++i) {
    const int q = wave * (PIECES / NW) + i;
    const bf16_t* g;
    if constexpr (LAYOUT == MMPT_ROWS_K) {
      const int r = q * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (r & 7);
      const int gr = min(r0 + r, Rlim - 1);
      const int gk = min(k0 + lc * 8, K - 8);
      g = src + (long)gr * ld + gk;
    } else {
      constexpr int CPR = R / 8;        // 16-B chunks per k-row
      constexpr int RPP = 64 / CPR;     // k-rows per piece
      const int kr = q * RPP + lane / CPR;
      const int lc = (lane % CPR) ^ swz_kr(kr);
      const int gk = min(k0 + kr, K - 1);
      const int gr = min(r0 + lc * 8, Rlim - 8);
      g = src + (long)gk * ld + gr;
    }
    __builtin_amdgcn_global_load_lds((const void*)g, LDS_PTR(void, img + q * 1024), 16, 0, 0);
  }
}

template <int LAYOUT, int R, int NT>
__device__ __forceinline__ void zero_k_tail(char* img, int kval, int tid) {
  // kval = valid k in this tile (0 < kval < 64); K % 8 == 0 so chunks are all-or-nothing
  if constexpr (LAYOUT == MMPT_ROWS_K) {
    for (int c = tid; c < R * 8; c += NT) {
      const int r = c >> 3, pc = c & 7;
      if (((pc ^ (r & 7)) * 8) >= kval) *(v8s*)(img + r * 128 + pc * 16) = v8s{0, 0, 0, 0, 0, 0, 0, 0};
    }
  } else {
    constexpr int CPR = R / 8;
    for (int c = tid; c < 64 * CPR; c += NT)
      if (c / CPR >= kval) *(v8s*)(img + c * 16) = v8s{0, 0, 0, 0, 0, 0, 0, 0};
  }
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

// ===== 4-slot ring variant: BK = 32, three K-tiles of DMA in flight ==========
// ROWS_K image: [R rows][32 k], 64-B rows, chunk' = chunk ^ ((row >> 1) & 3)
//   (conflict-free for the ds_read_b128 lane groups with 4 rows per bank row);
// K_ROWS image: [32 k][R rows], same s(k) swizzle as the BK=64 image.
constexpr int RBK = 32;

template <int LAYOUT, int R, int NW>
__device__ __forceinline__ void stage32(const bf16_t* __restrict__ src, long ld, int Rlim, int K,
                                        int r0, int k0, char* img, int wave, int lane) {
  constexpr int PIECES = R * RBK * 2 / 1024;
  static_assert(PIECES % NW == 0, "pieces must split evenly over waves");
#pragma unroll
  for (int i = 0; i < PIECES / NW; ++i) {
    const int q = wave * (PIECES / NW) + i;
    const bf16_t* g;
    if constexpr (LAYOUT == MMPT_ROWS_K) {
      const int r = q * 16 + (lane >> 2);
      const int lc = (lane & 3) ^ ((r >> 1) & 3);
      const int gr = min(r0 + r, Rlim - 1);
      const int gk = min(k0 + lc * 8, K - 8);
      g = src + (long)gr * ld + gk;
    } else {
      constexpr int CPR = R / 8;
      constexpr int RPP = 64 / CPR;
      const int kr = q * RPP + lane / CPR;
      const int lc = (lane % CPR) ^ swz_kr(kr);
      const int gk = min(k0 + kr, K - 1);
      const int gr = min(r0 + lc * 8, Rlim - 8);
      g = src + (long)gk * ld + gr;
    }
    __builtin_amdgcn_global_load_lds((const void*)g, LDS_PTR(void, img + q * 1024), 16, 0, 0);
  }
}

template <int LAYOUT, int R, int NT>
__device__ __forceinline__ void zero_k_tail32(char* img, int kval, int tid) {
  if constexpr (LAYOUT == MMPT_ROWS_K) {
    for (int c = tid; c < R * 4; c += NT) {
      const int r = c >> 2, pc = c & 3;
      if (((pc ^ ((r >> 1) & 3)) * 8) >= kval) *(v8s*)(img + r * 64 + pc * 16) = v8s{0, 0, 0, 0, 0, 0, 0, 0};
    }
  } else {
    constexpr int CPR = R / 8;
    for (int c = tid; c < RBK * CPR; c += NT)
      if (c / CPR >= kval) *(v8s*)(img + c * 16) = v8s{0, 0, 0, 0, 0, 0, 0, 0};
  }
}

template <int LAYOUT, int R>
__device__ __forceinline__ v8s frag32(const char* img, int rbase, int lane) {
  if constexpr (LAYOUT == MMPT_ROWS_K) {
    const int r = rbase + (lane & 15);
    const int lc = lane >> 4;
    return *(const v8s*)(img + r * 64 + ((lc ^ ((r >> 1) & 3)) * 16));
  } else {
    return frag<MMPT_K_ROWS, R>(img, rbase, 0, lane);
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

template <int EPI>
__device__ __forceinline__ void epilogue4(const GemmParams& p, int m, int n, const float* v,
                                          const float* bias, int split) {
  if constexpr (EPI == MMPT_EPI_BF16) {
    store_bf16x4((bf16_t*)p.C + (long)m * p.ldc + n, v[0] + bias[0], v[1] + bias[1],
                 v[2] + bias[2], v[3] + bias[3]);
  } else if constexpr (EPI == MMPT_EPI_BF16_GELU) {
    float pre[4], act[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pre[e] = round_bf(v[e] + bias[e]);
      act[e] = gelu_f(pre[e]);
    }
    store_bf16x4((bf16_t*)p.C + (long)m * p.ldc + n, pre[0], pre[1], pre[2], pre[3]);
    store_bf16x4((bf16_t*)p.C2 + (long)m * p.ldc2 + n, act[0], act[1], act[2], act[3]);
  } else if constexpr (EPI == MMPT_EPI_BF16_DGELU) {
    float x[4];
    load_bf16x4(p.aux + (long)m * p.ld_aux + n, x);
    store_bf16x4((bf16_t*)p.C + (long)m * p.ldc + n, round_bf(v[0]) * gelu_grad_f(x[0]),
                 round_bf(v[1]) * gelu_grad_f(x[1]), round_bf(v[2]) * gelu_grad_f(x[2]),
                 round_bf(v[3]) * gelu_grad_f(x[3]));
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

constexpr int EPI_SPLIT = 100;

template <int BM, int BN, int WGM, int WGN, int LA, int LB, int EPI, int PIPE>
__global__ __launch_bounds__(WGM* WGN * 64, (WGM * WGN * 64) / 256 > 1 ? (WGM * WGN * 64) / 256 : 2)
void gemm_kernel(GemmParams p) {
  constexpr int NT = WGM * WGN * 64;
  constexpr int NW = WGM * WGN;
  constexpr int TM = BM / WGM / 16;  // 16x16 MFMA tiles per wave along M
  constexpr int TN = BN / WGN / 16;
  constexpr int IMGA = BM * BK * 2, IMGB = BN * BK * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * (IMGA + IMGB)];  // == 4 ring slots
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;

  // XCD-aware bijective remap (blocks b and b+8 share an XCD), then grouped order.
  const int ntiles = p.tiles_m * p.tiles_n;
  const int nwg = ntiles * gridDim.y;
  const int bid = blockIdx.y * gridDim.x + blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wid0 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int wid = wid0 % ntiles;  // tile id; split id is blockIdx.y (the slab index)
  constexpr int GROUP = 8;
  const int per_group = GROUP * p.tiles_n;
  const int first_m = (wid / per_group) * GROUP;
  const int gsize = min(p.tiles_m - first_m, GROUP);
  const int tm = first_m + (wid % per_group) % gsize;
  const int tn = (wid % per_group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;
  int split = 0, kbeg = 0, kend = p.K;
  if constexpr (EPI == EPI_SPLIT) {
    split = wid0 / ntiles;
    kbeg = split * p.kchunk;
    kend = min(p.K, kbeg + p.kchunk);
  }

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  if constexpr (PIPE != 1) {
    const int nk = (kend - kbeg + BK - 1) / BK;
    stage<LA, BM, NW>(p.A, p.lda, p.M, p.K, m0, kbeg, smem, wave, lane);
    stage<LB, BN, NW>(p.B, p.ldb, p.N, p.K, n0, kbeg, smem + IMGA, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int t = 0; t < nk; ++t) {
      char* cur = smem + (t & 1) * (IMGA + IMGB);
      if (PIPE != 4 && t + 1 < nk) {
        char* nxt = smem + ((t + 1) & 1) * (IMGA + IMGB);
        stage<LA, BM, NW>(p.A, p.lda, p.M, p.K, m0, kbeg + (t + 1) * BK, nxt, wave, lane);
        stage<LB, BN, NW>(p.B, p.ldb, p.N, p.K, n0, kbeg + (t + 1) * BK, nxt + IMGA, wave, lane);
      } else if (kbeg + t * BK + BK > p.K) {
        const int kval = p.K - (kbeg + t * BK);
        zero_k_tail<LA, BM, NT>(cur, kval, tid);
        zero_k_tail<LB, BN, NT>(cur + IMGA, kval, tid);
        __syncthreads();
      }
      if constexpr (PIPE == 0 || PIPE >= 4) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          v8s a[TM], b[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j) b[j] = frag<LB, BN>(cur + IMGA, wn * (BN / WGN) + j * 16, kk, lane);
#pragma unroll
          for (int i = 0; i < TM; ++i) a[i] = frag<LA, BM>(cur, wm * (BM / WGM) + i * 16, kk, lane);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((v8bf)b[j], (v8bf)a[i], acc[i][j], 0, 0, 0);
        }
      } else {
        // software-pipelined fragments: A streamed in pairs, the reads of pair p+1
        // (and of the next kk's B) are issued before the MFMAs of pair p.
        const char* ia = cur;
        const char* ib = cur + IMGA;
        const int ra = wm * (BM / WGM), rb = wn * (BN / WGN);
        v8s b[TN], bn[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = frag<LB, BN>(ib, rb + j * 16, 0, lane);
        v8s a0 = frag<LA, BM>(ia, ra, 0, lane), a1 = frag<LA, BM>(ia, ra + 16, 0, lane);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
          for (int pr = 0; pr < TM / 2; ++pr) {
            v8s n0 = a0, n1 = a1;
            if (pr + 1 < TM / 2) {
              n0 = frag<LA, BM>(ia, ra + (2 * pr + 2) * 16, kk, lane);
              n1 = frag<LA, BM>(ia, ra + (2 * pr + 3) * 16, kk, lane);
            } else if (kk == 0) {
              n0 = frag<LA, BM>(ia, ra, 1, lane);
              n1 = frag<LA, BM>(ia, ra + 16, 1, lane);
#pragma unroll
              for (int j = 0; j < TN; ++j) bn[j] = frag<LB, BN>(ib, rb + j * 16, 1, lane);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (PIPE == 3) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              acc[2 * pr][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((v8bf)b[j], (v8bf)a0, acc[2 * pr][j], 0, 0, 0);
              acc[2 * pr + 1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((v8bf)b[j], (v8bf)a1, acc[2 * pr + 1][j], 0, 0, 0);
            }
            if constexpr (PIPE == 3) __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            a0 = n0;
            a1 = n1;
          }
          if (kk == 0) {
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = bn[j];
          }
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (PIPE != 5) __syncthreads();
    }
  } else {
    // 4-slot ring of BK=32 K-tiles; slot = A image (BM x 32) + B image (BN x 32).
    constexpr int SA = BM * RBK * 2, SB = BN * RBK * 2, SLOT = SA + SB;
    const int nk = (kend - kbeg + RBK - 1) / RBK;
#pragma unroll
    for (int s0 = 0; s0 < 3; ++s0) {
      if (s0 < nk) {
        stage32<LA, BM, NW>(p.A, p.lda, p.M, p.K, m0, kbeg + s0 * RBK, smem + s0 * SLOT, wave, lane);
        stage32<LB, BN, NW>(p.B, p.ldb, p.N, p.K, n0, kbeg + s0 * RBK, smem + s0 * SLOT + SA, wave, lane);
      }
    }
    for (int t = 0; t < nk; ++t) {
      // tile t has landed once at most the DMAs of tiles t+1, t+2 are outstanding
      // (4 glds per thread per tile; counted waits, never vmcnt(0) in steady state)
      const int ahead = min(2, nk - 1 - t);
      if (ahead == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_barrier" ::: "memory");  // tile t visible to all; tile t-1 fully consumed
      char* cur = smem + (t & 3) * SLOT;
      if (t + 3 < nk) {
        char* nxt = smem + ((t + 3) & 3) * SLOT;
        stage32<LA, BM, NW>(p.A, p.lda, p.M, p.K, m0, kbeg + (t + 3) * RBK, nxt, wave, lane);
        stage32<LB, BN, NW>(p.B, p.ldb, p.N, p.K, n0, kbeg + (t + 3) * RBK, nxt + SA, wave, lane);
      } else if (t == nk - 1 && kbeg + t * RBK + RBK > p.K) {
        const int kval = p.K - (kbeg + t * RBK);
        zero_k_tail32<LA, BM, NT>(cur, kval, tid);
        zero_k_tail32<LB, BN, NT>(cur + SA, kval, tid);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      v8s a[TM], b[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = frag32<LB, BN>(cur + SA, wn * (BN / WGN) + j * 16, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = frag32<LA, BM>(cur, wm * (BM / WGM) + i * 16, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((v8bf)b[j], (v8bf)a[i], acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue: lane owns C[m][n..n+3] ----
  const int mrow = m0 + wm * (BM / WGM) + (lane & 15);
  const int ncol = n0 + wn * (BN / WGN) + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = ncol + j * 16;
    if (n >= p.N) continue;
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
      epilogue4<EPI>(p, m, n, v, bias, split);
    }
  }
}

// Σ_s slab[s][m][n] in split order -> C (+)= f32(bf16(sum))
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

template <int BM, int BN, int WGM, int WGN, int LA, int LB>
int launch_epi(int epi, const GemmParams& p, dim3 grid, hipStream_t s, int pipe) {
  constexpr int NT = WGM * WGN * 64;
  switch (epi) {
#define MMPT_CASE(E) \
  case E:                                                                          \
    if (pipe == 4) gemm_kernel<BM, BN, WGM, WGN, LA, LB, E, 4><<<grid, NT, 0, s>>>(p); \
    else if (pipe == 5) gemm_kernel<BM, BN, WGM, WGN, LA, LB, E, 5><<<grid, NT, 0, s>>>(p); \
    else if (pipe == 2) gemm_kernel<BM, BN, WGM, WGN, LA, LB, E, 2><<<grid, NT, 0, s>>>(p); \
    else if (pipe == 3) gemm_kernel<BM, BN, WGM, WGN, LA, LB, E, 3><<<grid, NT, 0, s>>>(p); \
    else if (pipe == 1) gemm_kernel<BM, BN, WGM, WGN, LA, LB, E, 1><<<grid, NT, 0, s>>>(p); \
    else gemm_kernel<BM, BN, WGM, WGN, LA, LB, E, 0><<<grid, NT, 0, s>>>(p);      \
    break;
    MMPT_CASE(MMPT_EPI_BF16)
    MMPT_CASE(MMPT_EPI_BF16_GELU)
    MMPT_CASE(MMPT_EPI_BF16_DGELU)
    MMPT_CASE(MMPT_EPI_F32_ACC)
    MMPT_CASE(MMPT_EPI_F32_STORE)
    MMPT_CASE(MMPT_EPI_F32_RESID)
    MMPT_CASE(EPI_SPLIT)
#undef MMPT_CASE
    default: set_error("gemm: unknown epilogue %d", epi); return MMPT_ERR_ARG;
  }
  return check_launch("gemm");
}

template <int BM, int BN, int WGM, int WGN>
int launch_layouts(int la, int lb, int epi, const GemmParams& p, dim3 grid, hipStream_t s, int pipe) {
  if (la == MMPT_ROWS_K && lb == MMPT_ROWS_K)
    return launch_epi<BM, BN, WGM, WGN, MMPT_ROWS_K, MMPT_ROWS_K>(epi, p, grid, s, pipe);
  if (la == MMPT_ROWS_K && lb == MMPT_K_ROWS)
    return launch_epi<BM, BN, WGM, WGN, MMPT_ROWS_K, MMPT_K_ROWS>(epi, p, grid, s, pipe);
  if (la == MMPT_K_ROWS && lb == MMPT_K_ROWS)
    return launch_epi<BM, BN, WGM, WGN, MMPT_K_ROWS, MMPT_K_ROWS>(epi, p, grid, s, pipe);
  return launch_epi<BM, BN, WGM, WGN, MMPT_K_ROWS, MMPT_ROWS_K>(epi, p, grid, s, pipe);
}

// Main-loop selection: 0 = 2-slot BK=64 (default), 1 = 4-slot BK=32 ring (measured slower
// on every model shape: profiles/r01_gemm_pipe_ab.txt), 2/3 = explicitly pipelined
// fragment reads (+setprio) (no gain), 4/5 = DIAGNOSTIC ONLY (wrong results): no
// in-loop DMA / no in-loop barrier, to attribute the stall time.
// MMPT_GEMM_PIPE overrides (A/B experiments, scripts/bench_gemm.py).
int pipe_mode() {
  static int mode = [] {
    const char* e = getenv("MMPT_GEMM_PIPE");
    return e ? atoi(e) : 0;
  }();
  return mode;
}

constexpr int NUM_CUS = 256;

struct Plan {
  bool big;   // 256x256 tile
  int splits;
  int kchunk;
};

Plan plan(int64_t M, int64_t N, int64_t K, int epi) {
  Plan pl{};
  const int64_t t256 = ((M + 255) / 256) * ((N + 255) / 256);
  const int64_t t128 = ((M + 127) / 128) * ((N + 127) / 128);
  pl.big = t256 >= NUM_CUS;
  pl.splits = 1;
  pl.kchunk = (int)K;
  const bool splittable = epi == MMPT_EPI_F32_ACC || epi == MMPT_EPI_F32_STORE;
  if (splittable) {
    // weight gradients: K = tokens. Pick (tile, splits) minimising the padded wave
    // count ceil(blocks / slots) / blocks-work, slots = 256 (256^2, 1 per CU) or
    // 512 (128^2, 2 per CU); keep >= 1024 k per split and <= 16 splits.
    // Model (measured, r01): a CU fully busy with one 256^2 block retires 4 128^2-tile
    // units in 4 time units; with two 128^2 blocks it retires 2 units in 2.67 (128^2 runs
    // at ~0.75x the 256^2 rate).  Slab write+read adds sp*8 B per output element vs
    // 2K flops per element: factor (1 + sp*800/K) at ~5 TB/s : ~1 PF/s.
    double best = 1e30;
    for (int big = 1; big >= 0; --big) {
      const int64_t tiles = big ? t256 : t128;
      const int64_t slots = big ? NUM_CUS : 2 * NUM_CUS;
      const double wave_cost = big ? 4.0 : 2.67;
      // split only when the unsplit grid is under two waves (keeps slabs small)
      const int64_t max_sp = tiles < 2 * slots ? 16 : 1;
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
    if (pl.splits > 1) {
      int64_t kc = (K + pl.splits - 1) / pl.splits;
      kc = (kc + BK - 1) / BK * BK;
      pl.splits = (int)((K + kc - 1) / kc);
      pl.kchunk = (int)kc;
    }
  }
  return pl;
}

}  // namespace
}  // namespace mmpt

using namespace mmpt;

extern "C" int64_t mmpt_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K, int epilogue) {
  const Plan pl = plan(M, N, K, epilogue);
  return pl.splits > 1 ? (int64_t)pl.splits * M * N * (int64_t)sizeof(float) : 0;
}

extern "C" int mmpt_gemm_bf16(int layout_a, int layout_b, int epilogue, int64_t M, int64_t N,
                              int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb,
                              void* C, int64_t ldc, const void* bias_bf16, const void* aux_bf16,
                              int64_t ld_aux, void* C2, int64_t ldc2, void* workspace,
                              int64_t workspace_bytes, void* stream) {
  MMPT_REQUIRE(M > 0 && N > 0 && K > 0, "gemm: empty problem M=%lld N=%lld K=%lld",
               (long long)M, (long long)N, (long long)K);
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
  if (epilogue == MMPT_EPI_BF16_DGELU)
    MMPT_REQUIRE(aux_bf16 != nullptr && ld_aux % 4 == 0, "gemm: DGELU epilogue needs aux");
  if (epilogue == MMPT_EPI_F32_RESID)
    MMPT_REQUIRE(C2 != nullptr && ldc2 % 4 == 0 && (aux_bf16 == nullptr || ld_aux % 4 == 0),
                 "gemm: RESID epilogue needs C2 (residual input)");
  MMPT_REQUIRE(epilogue >= MMPT_EPI_BF16 && epilogue <= MMPT_EPI_F32_RESID, "gemm: bad epilogue");

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
  const int bm = pl.big ? 256 : 128;
  p.tiles_m = (int)((M + bm - 1) / bm);
  p.tiles_n = (int)((N + bm - 1) / bm);
  dim3 grid(p.tiles_m * p.tiles_n, pl.splits);
  hipStream_t s = (hipStream_t)stream;
  const int epi = pl.splits > 1 ? EPI_SPLIT : epilogue;
  const int pipe = pipe_mode();
  int rc = pl.big ? launch_layouts<256, 256, 2, 4>(layout_a, layout_b, epi, p, grid, s, pipe)
                  : launch_layouts<128, 128, 2, 2>(layout_a, layout_b, epi, p, grid, s, pipe);
  if (rc || pl.splits == 1) return rc;
  const long n4 = M * (N / 4);
  const unsigned blocks = (unsigned)((n4 + 255) / 256);
  if (epilogue == MMPT_EPI_F32_ACC)
    splitk_reduce<true><<<blocks, 256, 0, s>>>((int)M, (int)N, pl.splits, p.slab, (float*)C, ldc);
  else
    splitk_reduce<false><<<blocks, 256, 0, s>>>((int)M, (int)N, pl.splits, p.slab, (float*)C, ldc);
  return check_launch("gemm_splitk_reduce");
}
