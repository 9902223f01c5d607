// K1: bf16 MFMA GEMM with fused epilogues (replaces aten::addmm / mm launched by
// nn.Linear under autocast).
//
// Tile 128x128x64, 256 threads = 4 waves in a 2x2 arrangement, each wave owns a
// 64x64 sub-tile computed with v_mfma_f32_16x16x32_bf16 (4x4 accumulators).
// Operands are staged HBM -> LDS with global_load_lds_dwordx4 (no VGPR round
// trip) into two LDS buffers (load of tile k+1 overlaps MFMAs on tile k).
//
// LDS images (both lane-linear for the DMA; swizzle is applied to the SOURCE
// address and mirrored on the read, cdna_hip_programming.md rule 21):
//   ROWS_K operand: [128 rows][64 k] bf16, 128-B rows, chunk' = chunk ^ (row & 7)
//       -> fragments by ds_read_b128 (conflict-free for the b128 lane groups);
//   K_ROWS operand: [64 k][128 rows] bf16, 256-B rows, chunk' = chunk ^ s(k),
//       s(k) = 2*((k&3) | ((k>>3)&1)<<2)  -> fragments by ds_read_b64_tr_b16
//       (hardware transpose; the 8 k-rows of one 32-lane half hit 8 distinct
//       32-B chunk pairs: conflict-free).
// The MFMA is issued as D = Bfrag * Afrag so that the accumulator holds C^T:
// lane l owns C[m = l&15][n = 4*(l>>4) + i], i.e. 4 consecutive n per lane ->
// 8-B (bf16) / 16-B (f32) vector stores in the epilogue.
#include "common.h"

namespace mmpt {
namespace {

constexpr int BM = 128;
constexpr int BN = 128;
constexpr int BK = 64;
constexpr int NT = 256;
constexpr int IMG = 128 * 64 * 2;  // bytes of one operand image (16 KiB)

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
};

__device__ __forceinline__ int swz_kr(int kr) {
  return 2 * ((kr & 3) | (((kr >> 3) & 1) << 2));
}

// --- HBM -> LDS staging ---------------------------------------------------
template <int LAYOUT>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ src, long ld, int R, int K,
                                      int r0, int k0, char* img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wave * 4 + i;  // which 1-KiB piece of the 16-KiB image
    const bf16_t* g;
    if constexpr (LAYOUT == MMPT_ROWS_K) {
      const int r = q * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (r & 7);
      const int gr = min(r0 + r, R - 1);
      const int gk = min(k0 + lc * 8, K - 8);
      g = src + (long)gr * ld + gk;
    } else {
      const int kr = q * 4 + (lane >> 4);
      const int lc = (lane & 15) ^ swz_kr(kr);
      const int gk = min(k0 + kr, K - 1);
      const int gr = min(r0 + lc * 8, R - 8);
      g = src + (long)gk * ld + gr;
    }
    __builtin_amdgcn_global_load_lds((const void*)g, LDS_PTR(void, img + q * 1024), 16, 0, 0);
  }
}

// Zero the k >= K part of an image (last K tile only).
template <int LAYOUT>
__device__ __forceinline__ void zero_k_tail(char* img, int k0, int K, int tid) {
  const int kval = K - k0;  // valid k in this tile, 0 < kval < 64
  if constexpr (LAYOUT == MMPT_ROWS_K) {
    // 128 rows x 8 chunks; a chunk (8 k) is fully valid or fully invalid (K % 8 == 0)
    for (int c = tid; c < 128 * 8; c += NT) {
      const int r = c >> 3, pc = c & 7;
      const int lc = pc ^ (r & 7);
      if (lc * 8 >= kval) *(v8s*)(img + r * 128 + pc * 16) = v8s{0, 0, 0, 0, 0, 0, 0, 0};
    }
  } else {
    for (int c = tid; c < 64 * 16; c += NT) {
      const int kr = c >> 4;
      if (kr >= kval) *(v8s*)(img + c * 16) = v8s{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
}

// --- LDS -> VGPR fragments for v_mfma_f32_16x16x32_bf16 -----------------
// returns op[row = rbase + (lane&15)][k = kk*32 + 8*(lane>>4) + j], j = 0..7
template <int LAYOUT>
__device__ __forceinline__ v8s frag(const char* img, int rbase, int kk, int lane) {
  if constexpr (LAYOUT == MMPT_ROWS_K) {
    const int r = rbase + (lane & 15);
    const int lc = kk * 4 + (lane >> 4);
    const int pc = lc ^ (r & 7);
    return *(const v8s*)(img + r * 128 + pc * 16);
  } else {
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int col = rbase + 4 * p;
    const int lc = col >> 3, half = p & 1;
    const int kr = kk * 32 + 8 * g + q;
    const char* a = img + kr * 256 + ((lc ^ swz_kr(kr)) * 16) + half * 8;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a + 4 * 256));
    return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
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

template <int LA, int LB, int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG];  // [buf][A|B]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap (blocks b and b+8 share an XCD), then grouped order.
  const int nwg = p.tiles_m * p.tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GROUP = 8;
  const int per_group = GROUP * p.tiles_n;
  const int first_m = (wid / per_group) * GROUP;
  const int gsize = min(p.tiles_m - first_m, GROUP);
  const int tm = first_m + (wid % per_group) % gsize;
  const int tn = (wid % per_group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  stage<LA>(p.A, p.lda, p.M, p.K, m0, 0, smem, wave, lane);
  stage<LB>(p.B, p.ldb, p.N, p.K, n0, 0, smem + IMG, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * 2 * IMG;
    if (t + 1 < nk) {
      char* nxt = smem + ((t + 1) & 1) * 2 * IMG;
      stage<LA>(p.A, p.lda, p.M, p.K, m0, (t + 1) * BK, nxt, wave, lane);
      stage<LB>(p.B, p.ldb, p.N, p.K, n0, (t + 1) * BK, nxt + IMG, wave, lane);
    } else if (t * BK + BK > p.K) {
      zero_k_tail<LA>(cur, t * BK, p.K, tid);
      zero_k_tail<LB>(cur + IMG, t * BK, p.K, tid);
      __syncthreads();
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v8s a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag<LA>(cur, wm * 64 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag<LB>(cur + IMG, wn * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((v8bf)b[j], (v8bf)a[i],
                                                              acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: lane owns C[m][n..n+3] ----
  const int mrow = m0 + wm * 64 + (lane & 15);
  const int ncol = n0 + wn * 64 + 4 * (lane >> 4);
  float bias[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = ncol + j * 16;
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[j][e] = 0.f;
    if constexpr (EPI == MMPT_EPI_BF16 || EPI == MMPT_EPI_BF16_GELU || EPI == MMPT_EPI_F32_RESID) {
      if (p.bias != nullptr && n < p.N) load_bf16x4(p.bias + n, bias[j]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mrow + i * 16;
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = ncol + j * 16;
      if (n >= p.N) continue;
      const v4f a = acc[i][j];
      float v[4] = {a[0], a[1], a[2], a[3]};
      if constexpr (EPI == MMPT_EPI_BF16) {
        store_bf16x4((bf16_t*)p.C + (long)m * p.ldc + n, v[0] + bias[j][0], v[1] + bias[j][1],
                     v[2] + bias[j][2], v[3] + bias[j][3]);
      } else if constexpr (EPI == MMPT_EPI_BF16_GELU) {
        float pre[4], act[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pre[e] = round_bf(v[e] + bias[j][e]);
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
        for (int e = 0; e < 4; ++e) r[e] = round_bf(v[e] + bias[j][e]);
        if (p.aux != nullptr) {
          float x[4];
          load_bf16x4(p.aux + (long)m * p.ld_aux + n, x);
#pragma unroll
          for (int e = 0; e < 4; ++e) r[e] = round_bf(r[e] + x[e]);
        }
        const float4 res = *(const float4*)((const float*)p.C2 + (long)m * p.ldc2 + n);
        *(float4*)((float*)p.C + (long)m * p.ldc + n) =
            make_float4(res.x + r[0], res.y + r[1], res.z + r[2], res.w + r[3]);
      }
    }
  }
}

template <int LA, int LB>
int launch_epi(int epi, const GemmParams& p, dim3 grid, hipStream_t s) {
  switch (epi) {
    case MMPT_EPI_BF16: gemm_kernel<LA, LB, MMPT_EPI_BF16><<<grid, NT, 0, s>>>(p); break;
    case MMPT_EPI_BF16_GELU: gemm_kernel<LA, LB, MMPT_EPI_BF16_GELU><<<grid, NT, 0, s>>>(p); break;
    case MMPT_EPI_BF16_DGELU: gemm_kernel<LA, LB, MMPT_EPI_BF16_DGELU><<<grid, NT, 0, s>>>(p); break;
    case MMPT_EPI_F32_ACC: gemm_kernel<LA, LB, MMPT_EPI_F32_ACC><<<grid, NT, 0, s>>>(p); break;
    case MMPT_EPI_F32_STORE: gemm_kernel<LA, LB, MMPT_EPI_F32_STORE><<<grid, NT, 0, s>>>(p); break;
    case MMPT_EPI_F32_RESID: gemm_kernel<LA, LB, MMPT_EPI_F32_RESID><<<grid, NT, 0, s>>>(p); break;
    default: set_error("gemm: unknown epilogue %d", epi); return MMPT_ERR_ARG;
  }
  return check_launch("gemm");
}

}  // namespace
}  // namespace mmpt

using namespace mmpt;

extern "C" int mmpt_gemm_bf16(int layout_a, int layout_b, int epilogue, int64_t M, int64_t N,
                              int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb,
                              void* C, int64_t ldc, const void* bias_bf16, const void* aux_bf16,
                              int64_t ld_aux, void* C2, int64_t ldc2, void* stream) {
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
  p.tiles_m = (int)((M + BM - 1) / BM);
  p.tiles_n = (int)((N + BN - 1) / BN);
  dim3 grid(p.tiles_m * p.tiles_n);
  hipStream_t s = (hipStream_t)stream;
  if (layout_a == MMPT_ROWS_K && layout_b == MMPT_ROWS_K)
    return launch_epi<MMPT_ROWS_K, MMPT_ROWS_K>(epilogue, p, grid, s);
  if (layout_a == MMPT_ROWS_K && layout_b == MMPT_K_ROWS)
    return launch_epi<MMPT_ROWS_K, MMPT_K_ROWS>(epilogue, p, grid, s);
  if (layout_a == MMPT_K_ROWS && layout_b == MMPT_K_ROWS)
    return launch_epi<MMPT_K_ROWS, MMPT_K_ROWS>(epilogue, p, grid, s);
  return launch_epi<MMPT_K_ROWS, MMPT_ROWS_K>(epilogue, p, grid, s);
}
