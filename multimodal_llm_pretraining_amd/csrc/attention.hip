// K2/K3: scaled-dot-product attention forward / backward on MFMA
// (replaces torch SDPA as called by tf:models/gpt_neox/modeling_gpt_neox.py:214-229
// (causal) and tf:models/vit/modeling_vit.py:221-232 (bidirectional)).
//
// q/k/v are read in place from the fused QKV GEMM output (K7: no split/transpose
// copies): element (token t, head h, part p, dim d) = qkv[t*ld + h*hs + p*ps + d].
//
// Forward (flash, online softmax): one workgroup = 4 waves = 64 query rows of
// one (batch, head); each wave owns 16 query rows.  Scores are computed
// transposed, S^T = K·Q^T (v_mfma_f32_16x16x32_bf16, K from LDS by ds_read_b128,
// Q^T fragments resident in VGPRs), so a lane holds 16 keys of ONE query row:
// the softmax row max/sum is lane-local plus two cross-group shuffles, and the
// P accumulator is directly the B operand of O^T += V^T·P^T (V^T fragments by
// ds_read_b64_tr_b16 in the same permuted key order: cdna_hip_programming.md §3
// "An accumulator tile as the next MFMA's operand").  No P round trip via LDS.
//
// Backward: δ = rowsum(dO∘O) pre-pass, then two kernels that recompute P from
// the forward's log-sum-exp: (1) dK,dV with the key on the MFMA lane (one
// workgroup per 64-key block sweeping the query blocks), (2) dQ with the query
// on the lane (one workgroup per 64-query block sweeping the key blocks).  No
// atomics: every gradient element has exactly one writer, results are
// bitwise reproducible.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace mmpt {
namespace {

constexpr int ABLK = 64;  // rows (queries or keys) per block
constexpr float LOG2E = 1.4426950408889634f;

struct AttnParams {
  const bf16_t* qkv;
  long ld, hs, ps;
  // k / v of query head h: qkv[t*ld + koff + (h/G)*khs + d], qkv[t*ld + voff + (h/G)*khs + d]
  // (GPTNeoX / ViT: koff = ps, voff = 2ps, khs = hs, G = 1; Llama GQA: G = H / Hkv)
  long koff, voff, khs;
  int G, Hkv;
  int B, S, H;
  float scale;
  bf16_t* out;
  long ld_out;
  float* lse;
  const bf16_t* o;
  const bf16_t* dout;
  const float* delta;
  bf16_t* dqkv;
  bf16_t* ds;  // D = 256 backward: dS tiles (ds_tile) written by dK/dV, read by dQ
  int dr;  // real head dim (<= D of the kernel: 80/96/112 run the D = 128 kernels with the
           // dims past dr zero-filled on load and never stored — Pythia-2.8B has D = 80)
  // fused rope backward (mmpt_attention_bwd_rope, D = 256 pair + dS-tile path, rot = 64): the
  // dQ / dK epilogues apply the inverse rotation (tables [pos][rot], as rope8_kernel reads them)
  const float* rcos;
  const float* rsin;
  int rot;  // 0: no rotation
};
constexpr int FUSED_ROT = 64;  // the rotary width the fused epilogues handle (Pythia: D / 4)

// The inverse rotary pairs (d, d + 32) of the d-tiles dt = 0, 1 and dt + 2 of an accumulator
// tile set x[dt] (C rows = dims 16dt + 4g + i, already scaled) at sequence position pos:
// rope8_kernel's backward arithmetic on the values as they would be stored (bf16), in place
// (the staging that follows rounds the results).
__device__ __forceinline__ void rope_bwd_tiles(v4f* x, const AttnParams& p, int pos, int g) {
  const float* cp = p.rcos + (long)pos * FUSED_ROT + 4 * g;
  const float* sp = p.rsin + (long)pos * FUSED_ROT + 4 * g;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const float4 c1 = *(const float4*)(cp + 16 * dt), c2 = *(const float4*)(cp + 16 * dt + 32);
    const float4 s1 = *(const float4*)(sp + 16 * dt), s2 = *(const float4*)(sp + 16 * dt + 32);
    const float a1[4] = {c1.x, c1.y, c1.z, c1.w}, a2[4] = {c2.x, c2.y, c2.z, c2.w};
    const float b1[4] = {s1.x, s1.y, s1.z, s1.w}, b2[4] = {s2.x, s2.y, s2.z, s2.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float o1, o2;
      rope_rot(round_bf(x[dt][i]), round_bf(x[dt + 2][i]), a1[i], a2[i], b1[i], b2[i], true, o1, o2);
      x[dt][i] = o1;
      x[dt + 2][i] = o2;
    }
  }
}

// 16 zero bytes: the LDS-DMA source of a padded (d >= dr) chunk
__device__ __attribute__((aligned(16))) bf16_t g_azero[8];

// chunk c (8 dims) of a D-wide head row is real?  Only the D = 128 kernels pad.
template <int D>
__device__ __forceinline__ bool chunk_real(int c, int dr) {
  return D != 128 || c * 8 < dr;
}

// Head dims computed by a kernel built for D with DR real dims (DR < D: Pythia-2.8B's 80 in
// the D = 128 image layout): the QK^T / dO·V^T contractions run ceil(DR/32) k-steps of 32
// (dims DR.. of the last one are the zero-filled chunks of the image), the P·V / dS·K /
// dV / dK products DR/16 d-tiles — 3 of 4 and 5 of 8 at DR = 80 instead of the full D.
template <int D, int DR>
constexpr int dr_ksteps() {
  static_assert(DR % 16 == 0 && DR <= D && (DR == D || D == 128), "DR: real dims of a D = 128 kernel");
  return (DR + 31) / 32;
}

// ---- LDS image of ABLK rows x D bf16 (row = token of the block) -----------
template <int D>
struct Img {
  static constexpr int RB = D * 2;    // bytes per row
  static constexpr int CPR = D / 8;   // 16-B chunks per row
  static constexpr int BYTES = ABLK * RB;
  // chunk swizzle.  D >= 128 (rows span whole 256-B bank rows): f(r) = 2(r & 7) serves
  // BOTH reads of one image (cdna_hip_programming.md T10 "one image for row reads AND
  // transposed reads"): a ds_read_b128 lane group (rows {0-3,12-15} at chunk c, rows
  // {4-11} at chunk c+1, c even) lands on 8 distinct even + 8 distinct odd 16-B slots,
  // and a ds_read_b64_tr_b16 32-lane half (rows 0-7 of an 8-row group x chunks c0,
  // c0+1, c0 even) on 16 distinct slots — both conflict-free.  D = 64 (128-B rows, two
  // per bank row): r & 7.
  __device__ static __forceinline__ int swz(int r) { return D >= 128 ? (r & 7) << 1 : (r & 7); }
  // D = 256 (round 4): SLABS of 32 dims — the image is 8 slabs of ROWS rows x 64 B, chunk lc
  // of row r in slab lc / 4 at 16-B slot (lc & 3) ^ fs(r), fs(r) = 2·((r >> 2) & 1).  A k-step
  // (or a d-tile pair) is then a whole slab: every fragment address is one per-lane base plus a
  // compile-time offset (the ds_read offset field), instead of an XOR of the k-step into the
  // lane's swizzle per fragment (~3 VALU each).  Both reads stay conflict-free (a ds_read_b128
  // 16-lane group: rows r = 0..15 at slots 4(r & 3) + ((g ^ fs(r)) ...) cover 16 distinct 16-B
  // slots; a ds_read_b64_tr_b16 32-lane half: 8 rows x 2 chunks on 32 distinct 8-B slots —
  // brute-force checked over every k-step / d-tile, scripts/diag/slab_swizzle_check.py).
  static constexpr bool SLAB = D == 256;
  __device__ static __forceinline__ int fs(int r) { return (r & 4) >> 1; }
  template <int ROWS = ABLK>
  __device__ static __forceinline__ int off(int r, int lc) {
    if constexpr (SLAB) return (lc >> 2) * (ROWS * 64) + r * 64 + (((lc & 3) ^ fs(r)) << 4);
    return r * RB + ((lc ^ swz(r)) << 4);
  }
  // source row / chunk of lane `lane` in 1-KiB piece q of a ROWS-row image (the LDS-DMA
  // destination is lane-linear: the swizzle goes into the per-lane SOURCE chunk)
  template <int ROWS>
  __device__ static __forceinline__ void piece(int q, int lane, int& r, int& lc) {
    if constexpr (SLAB) {
      constexpr int PPS = ROWS / 16;  // pieces per slab (16 rows x 64 B)
      r = (q % PPS) * 16 + (lane >> 2);
      lc = (q / PPS) * 4 + ((lane & 3) ^ fs(r));
    } else {
      constexpr int RPP = 1024 / RB, LPR = 64 / RPP;
      r = q * RPP + lane / LPR;
      lc = (lane % LPR) ^ swz(r);
    }
  }
  // image filled by LDS-DMA (global_load_lds_dwordx4): the destination is lane-linear,
  // so the swizzle is applied to the per-lane SOURCE chunk.  The NW waves of the block
  // each issue (D/8)/NW pieces of 1 KiB.
  template <int NW = 4>
  __device__ static __forceinline__ void dma(char* img, const bf16_t* base, long ld, long col0,
                                             int S, int b, int row0, int wave, int lane,
                                             int dr = D) {
    constexpr int PPW = (D / 8) / NW;  // pieces per wave (64 rows x 2D bytes / 1 KiB / NW)
    static_assert(PPW * NW == D / 8, "pieces must split evenly over waves");
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;
      int r, lc;
      piece<ABLK>(q, lane, r, lc);
      const long t = (long)b * S + min(row0 + r, S - 1);
      const bf16_t* src = chunk_real<D>(lc, dr) ? base + t * ld + col0 + lc * 8 : g_azero;
      glds16(src, img + q * 1024);  // asm: no hipcc drain before tr reads
    }
  }
  // ROWS-row image by LDS-DMA, split over NW waves
  template <int NW, int ROWS>
  __device__ static __forceinline__ void dma_rows(char* img, const bf16_t* base, long ld, long col0,
                                                  int S, int b, int row0, int wave, int lane,
                                                  int dr = D) {
    constexpr int PIECES = ROWS * RB / 1024;
    constexpr int PPW = PIECES / NW;
    static_assert(PPW * NW == PIECES, "pieces must split evenly over waves");
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;
      int r, lc;
      piece<ROWS>(q, lane, r, lc);
      const long t = (long)b * S + min(row0 + r, S - 1);
      const bf16_t* src = chunk_real<D>(lc, dr) ? base + t * ld + col0 + lc * 8 : g_azero;
      glds16(src, img + q * 1024);
    }
  }
  // dma_rows with a uniform base (batch row 0, column col0 folded in) and 32-bit per-lane byte
  // offsets: a sequence is < 2^31 bytes, so no 64-bit multiply per piece (D = 256 pair kernel)
  template <int NW, int ROWS>
  __device__ static __forceinline__ void dma_rows32(char* img, const char* base, int ldb, int S,
                                                    int row0, int wave, int lane) {
    static_assert(D == 256, "full-width rows only");
    constexpr int PPW = ROWS * RB / 1024 / NW;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave * PPW + i;
      int r, lc;
      piece<ROWS>(q, lane, r, lc);
      glds16(base + (min(row0 + r, S - 1) * ldb + lc * 16), img + q * 1024);
    }
  }
  // A-operand fragment with rows = image rows rb..rb+15, k = d in [32ks, 32ks+32)
  template <int ROWS = ABLK>
  __device__ static __forceinline__ v8s row_frag(const char* img, int rb, int ks, int lane) {
    const int r = rb + (lane & 15);
    return *(const v8s*)(img + off<ROWS>(r, ks * 4 + (lane >> 4)));
  }
  // A-operand fragment with rows = d in [cb, cb+16), k = image rows in the
  // permuted order pi(g,j) = 32s + 4g + j (j<4) | 32s + 16 + 4g + (j-4) (j>=4)
  template <int ROWS = ABLK>
  __device__ static __forceinline__ v8s tr_frag(const char* img, int cb, int s, int lane) {
    const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
    const int lc = (cb >> 3) + (pp >> 1);
    const int r1 = 32 * s + 4 * g + q, r2 = r1 + 16;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, img + off<ROWS>(r1, lc) + (pp & 1) * 8));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, img + off<ROWS>(r2, lc) + (pp & 1) * 8));
    return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
};

// Wait for every vector-memory op incl. the asm LDS-DMA (which hipcc does not count),
// and tell hipcc's waitcnt model (the builtin) so it stops re-waiting in the loop
// for loads it thinks are still pending (guide §5 trap (b)).
__device__ __forceinline__ void vm_wait_all() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15
}

// XCD-aware block order: hardware dispatch sends workgroup `bid` to XCD bid % 8, and
// each XCD has its own L2.  Remap so an XCD runs a contiguous range of logical
// (block, batch-head) ids: the q/k blocks of one (batch, head) then share that XCD's L2
// copy of its K/V (or Q/dO) stream instead of every XCD re-fetching it (bijective for
// any grid size).  Within a (batch, head) the last block (the most causal work) first.
__device__ __forceinline__ void attn_block(int& bx, int& bh) {
  const int nx = gridDim.x, n = gridDim.x * gridDim.y;
  const int bid = blockIdx.y * nx + blockIdx.x;
  const int xcd = bid & 7, q8 = n >> 3, r8 = n & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  bx = nx - 1 - wid % nx;
  bh = wid / nx;
}

// Persistent forward: a 1-D grid of G workgroups (G % 8 == 0, one per CU) where WG b on
// XCD b & 7 walks its XCD's contiguous run of the attn_block order (so the query blocks of
// one (batch, head) still run together on one XCD and share its L2 copy of K/V), taking
// the run's items in rounds of G/8 in boustrophedon order — round r forward, round r+1
// backward — which pairs the heaviest causal items with the lightest ones per WG.  Returns
// the k-th logical item (wid in the attn_block numbering) of this WG, or -1.  G >= n: one
// item per workgroup, exactly attn_block's order.
__device__ __forceinline__ int attn_item(int n, int k) {
  const int G = gridDim.x, bid = blockIdx.x;
  const int q8 = n >> 3, r8 = n & 7;
  auto start = [&](int x) { return x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8; };
  if (G >= n) return k == 0 && bid < n ? start(bid & 7) + (bid >> 3) : -1;
  const int x = bid & 7, j = bid >> 3, W = G >> 3;
  const int local = k * W + ((k & 1) ? W - 1 - j : j);
  return local < q8 + (x < r8 ? 1 : 0) ? start(x) + local : -1;
}

// 4-byte-per-lane LDS-DMA (global_load_lds_dword: 64 lanes x 4 B = 256 B at `lds`).
__device__ __forceinline__ void glds4(const void* gsrc, char* lds) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(char, lds));
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(dst)
      : "memory");
}

// glds4 into the wave-uniform LDS byte address m0v (m0 not restored: see glds16_so)
__device__ __forceinline__ void glds4_a(const void* gsrc, uint32_t m0v) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
               :
               : "v"(gsrc), "s"(m0v)
               : "memory");
}

// s_waitcnt vmcnt(k * PPB) for k = 0, 1, 2 (wave-uniform k): a ring keeps at most two
// later blocks of PPB DMA pieces in flight.
template <int PPB>
__device__ __forceinline__ void wait_blocks(int k) {
  if (k >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPB) : "memory");
  else if (k == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPB) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// B-operand fragment for X^T where X row x = (lane&15) is a token row in global
// memory:  B[k = d][col = x], d = 32ks + 8(lane>>4) + j
__device__ __forceinline__ v8s gfrag(const bf16_t* rowptr, int ks, int lane) {
  return *(const v8s*)(rowptr + ks * 32 + 8 * (lane >> 4));
}
template <int D>
__device__ __forceinline__ v8s gfrag_m(const bf16_t* rowptr, int ks, int lane, int dr) {
  if (!chunk_real<D>(ks * 4 + (lane >> 4), dr)) return v8s{0, 0, 0, 0, 0, 0, 0, 0};
  return gfrag(rowptr, ks, lane);
}

__device__ __forceinline__ v4f mfma(v8s a, v8s b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16((v8bf)a, (v8bf)b, c, 0, 0, 0);
}

// pack two 16-row accumulator tiles (rows 4g+i of tile 2s and 2s+1) into a bf16
// B fragment in the permuted k order pi(g, j)
__device__ __forceinline__ v8s pack_pair(v4f a, v4f b) {
  v8s r;
  r[0] = (short)f2bf(a[0]); r[1] = (short)f2bf(a[1]); r[2] = (short)f2bf(a[2]); r[3] = (short)f2bf(a[3]);
  r[4] = (short)f2bf(b[0]); r[5] = (short)f2bf(b[1]); r[6] = (short)f2bf(b[2]); r[7] = (short)f2bf(b[3]);
  return r;
}

// dS tiles (D = 256 backward): the dK/dV kernel already holds dS = P∘(dP − δ) for its keys
// and query block, so it writes it out once and the dQ product becomes dQ = scale · dS·K over
// those tiles — no second recomputation of S, P and dP (Q, dO, V, lse and δ are not read
// again).  One 2-KiB tile per (batch·query head, 32-query block qb, 32-key block kb), square
// indexing over nq = ceil(S/32); inside it the B-fragment order of dQ^T += K^T·dS^T:
// fragment qt (query rows 16qt..16qt+15) is 1 KiB, lane l = 16g + q holds the 8 keys
// pi(g, j) = 4g + j (j < 4) | 16 + 4g + j − 4 (j >= 4) of query row q — a 16-B load per lane.
__device__ __forceinline__ long ds_tile(int bhq, int nq, int qb, int kb) {
  return (((long)bhq * nq + qb) * nq + kb) * 1024;  // in bf16 elements
}

// 8-B staging write of (row r, 16-B chunk position cpos, half h) as two 4-B writes whose
// order depends on r >> 3: with the rows r and r ^ 8 of a 16-lane group at the same chunk
// position mod 8 (the 16 lanes of one ds_write_b64 group can only cover 64 B of one half),
// the two b32 writes put those rows on different banks — conflict-free, 8 LDS cycles
// instead of 6 + 4 conflict cycles
__device__ __forceinline__ void stage_w8(char* row, int cpos, int h, int r, uint2 u) {
  uint32_t* d = (uint32_t*)(row + (cpos << 4) + h * 8);
  const bool sw = (r >> 3) & 1;
  d[sw ? 1 : 0] = sw ? u.y : u.x;
  d[sw ? 0 : 1] = sw ? u.x : u.y;
}
// dS-tile transpose position of fragment lane L (16-B chunk): the low 2 bits XOR the key
// group L >> 4, so the 2-B writes of one instruction (8 target lanes x 2 dwords per 32-lane
// group) land on 16 distinct banks; the 16-B read groups of ds_read_b128 are unions of
// aligned 4-lane blocks, whose positions this only permutes — conflict-free both ways
__device__ __forceinline__ int dst_pos(int L) { return L ^ ((L >> 4) & 3); }

// Diagnostic builds of the forward (never shipped; scripts/build_variants.sh): 1 = no DMA
// wait in the key loop, 2 = no K/V DMA in the loop either, 3 = no K/V fragment reads.
#ifndef MMPT_ATTN_DIAG
#define MMPT_ATTN_DIAG 0
#endif
#ifndef MMPT_ATTN_SD
#define MMPT_ATTN_SD 2  // K fragments one k-step ahead (r03: -1.5..2.5% with VD 3, profiles/r03/attn_fwd_ring)
#endif
#ifndef MMPT_ATTN_DQ_STAGE
#define MMPT_ATTN_DQ_STAGE 0
#endif
// dK/dV diagnostics (never shipped): 1 = no ring DMA / waits in the loop, 2 = no softmax
// (P = raw scores), 3 = no S/dP phase, 4 = no dV/dK phase, 5 = no per-block barrier,
// 7 = no dK MFMAs, 8 = S/dP reads without MFMAs, 9 = dV/dK reads without MFMAs,
// 10 = no K/V fragment loads, 11 = (almost) no dK/dV stores
#ifndef MMPT_ATTN_EARLYQ
#define MMPT_ATTN_EARLYQ 1  // persistent fwd / dQ: next item's fragment loads before the epilogue
#endif
#ifndef MMPT_ATTN_BPA
#define MMPT_ATTN_BPA 2
#endif
#ifndef MMPT_ATTN_BPB
#define MMPT_ATTN_BPB 2
#endif
#ifndef MMPT_ATTN_BDIAG
#define MMPT_ATTN_BDIAG 0
#endif
#ifndef MMPT_ATTN_VD
#define MMPT_ATTN_VD 3
#endif
#ifndef MMPT_ATTN_KD
#define MMPT_ATTN_KD 3  // dQ-from-dS kernel: K^T fragment ring depth (d-tiles ahead)
#endif
// per-block LDS-DMA of whole K/V (forward) and Q/dO (dK/dV pair kernel) blocks through the SADDR
// form with integer LDS addresses (1), or per-lane 64-bit addresses and LDS pointer casts (0)
#ifndef MMPT_ATTN_SADDR
#define MMPT_ATTN_SADDR 1
#endif
// ============================== forward ====================================
// One workgroup = 4 waves = 64·QT query rows; wave w owns QT 16-row query tiles.
// K/V blocks of 64 keys are double-buffered in LDS by LDS-DMA (128 KiB at D=256):
// the DMA of block j+1 is issued before the MFMAs of block j.
template <int D, bool CAUSAL, int QT, int NW, int DR = D>
__global__ __launch_bounds__(NW * 64, 1) void attn_fwd_kernel(AttnParams p) {
  using I = Img<D>;
  constexpr int KS = dr_ksteps<D, DR>(), DT = DR / 16;
  __shared__ __attribute__((aligned(16))) char smem[4 * I::BYTES];  // [buf][K | V]
  const uint32_t lbase = lds_addr(smem);
  // register pipeline depths (k-steps of 4 K fragments / d-tiles of 2 V^T fragments)
  constexpr int SD = MMPT_ATTN_SD < KS ? MMPT_ATTN_SD : KS;
  constexpr int VD = MMPT_ATTN_VD < DT ? MMPT_ATTN_VD : DT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  constexpr int BQ = NW * 16 * QT;
  const int nx = (p.S + BQ - 1) / BQ;
  const int nitems = nx * p.B * p.H;
  int it = 0;
  int wid = attn_item(nitems, 0);
  if (wid < 0) return;  // (workgroup-uniform)
  const float sl2 = p.scale * LOG2E;
  const int nkb_all = (p.S + ABLK - 1) / ABLK;

  // per-item state: (query block, batch, head), its Q fragments in registers
  int b, h, bh, q0, nkb;
  long kcol, vcol;
  int myq[QT];
  v8s qf[QT][KS];
  auto decode = [&](int w, int& b_, int& h_, int& bh_, int& q0_, long& kc, long& vc) {
    const int bx = nx - 1 - w % nx;  // within a (batch, head): the most causal work first
    bh_ = w / nx;
    b_ = bh_ / p.H;
    h_ = bh_ % p.H;
    kc = p.koff + (long)(h_ / p.G) * p.khs;
    vc = p.voff + (long)(h_ / p.G) * p.khs;
    q0_ = bx * BQ;
  };
  auto load_q = [&]() {
    nkb = CAUSAL ? min(nkb_all, (q0 + BQ - 1) / ABLK + 1) : nkb_all;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      myq[qt] = q0 + wave * 16 * QT + qt * 16 + (lane & 15);
      const bf16_t* qrow = p.qkv + (long)(b * p.S + min(myq[qt], p.S - 1)) * p.ld + h * p.hs;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) qf[qt][ks] = gfrag_m<D>(qrow, ks, lane, p.dr);
    }
  };
  // key block kb of (batch bb, k/v columns kc/vc) into LDS buffer `buf`
  auto stage_kv = [&](int buf, int bb, long kc, long vc, int kb) {
    char* img = smem + buf * 2 * I::BYTES;
    if constexpr (D == 256) {
      // K and V pieces share their per-lane row / chunk offsets (32-bit, from a uniform base
      // at the batch's row 0): ~4 VALU per piece pair instead of ~8 of 64-bit math per piece
      constexpr int PPW = (D / 8) / NW;
      const char* bk = (const char*)(p.qkv + (long)bb * p.S * p.ld + kc);
      const char* bv = bk + (vc - kc) * 2;
      const int ldb = (int)p.ld * 2;
      if (MMPT_ATTN_SADDR && kb * ABLK + ABLK <= p.S) {
        // a whole block: wave-uniform bases at its first key, per-lane 32-bit offsets (SADDR)
        const char* bk0 = bk + kb * ABLK * ldb;
        const char* bv0 = bv + kb * ABLK * ldb;
        const uint32_t ia = lbase + buf * 2 * I::BYTES;
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
          const int q = wave * PPW + i;
          int r, lc;
          I::template piece<ABLK>(q, lane, r, lc);
          const int off = r * ldb + (lc << 4);
          glds16_so(bk0, off, ia + q * 1024);
          glds16_so(bv0, off, ia + I::BYTES + q * 1024);
        }
      } else {
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
          const int q = wave * PPW + i;
          int r, lc;
          I::template piece<ABLK>(q, lane, r, lc);
          const int off = min(kb * ABLK + r, p.S - 1) * ldb + (lc << 4);
          glds16(bk + off, img + q * 1024);
          glds16(bv + off, img + I::BYTES + q * 1024);
        }
      }
    } else {
      I::template dma<NW>(img, p.qkv, p.ld, kc, p.S, bb, kb * ABLK, wave, lane, p.dr);
      I::template dma<NW>(img + I::BYTES, p.qkv, p.ld, vc, p.S, bb, kb * ABLK, wave, lane, p.dr);
    }
  };
  decode(wid, b, h, bh, q0, kcol, vcol);
  load_q();
  stage_kv(0, b, kcol, vcol, 0);
  int par = 0;  // LDS buffer of the item's key block kb: (kb + par) & 1
  v4f o[QT][DT];
  float m[QT], l[QT];
  for (;;) {
  // the next item: its key block 0 goes out during this item's last key block, into the
  // buffer that block leaves free
  const int wid_n = attn_item(nitems, it + 1);
  int nb = 0, nh = 0, nbh = 0, nq0 = 0;
  long nkc = 0, nvc = 0;
  if (wid_n >= 0) decode(wid_n, nb, nh, nbh, nq0, nkc, nvc);
  vm_wait_all();
  __syncthreads();
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
    for (int i = 0; i < DT; ++i) o[qt][i] = v4f{0.f, 0.f, 0.f, 0.f};
    m[qt] = -INFINITY;
    l[qt] = 0.f;
  }
  // causal: this wave's rows see key blocks [0, nkb_w); the workgroup sweeps [0, nkb)
  // (later blocks: this wave only helps with the DMA and the barriers)
  const int nkb_w = CAUSAL ? min(nkb, (q0 + wave * 16 * QT + 16 * QT - 1) / ABLK + 1) : nkb;
  for (int kb = 0; kb < nkb_w; ++kb) {
    const int k0 = kb * ABLK;
    // the lane id by v_mbcnt per block: fragment offsets are recomputed at their use instead
    // of ~25 hoisted per-lane offsets held across the loop (registers for the K ring)
    int fl;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(fl));
    char* kimg = smem + ((kb + par) & 1) * 2 * I::BYTES;
    char* vimg = kimg + I::BYTES;
    if (MMPT_ATTN_DIAG != 2) {
      if (kb + 1 < nkb) stage_kv((kb + 1 + par) & 1, b, kcol, vcol, kb + 1);
      else if (wid_n >= 0) stage_kv((kb + 1 + par) & 1, nb, nkc, nvc, 0);
    }
    v4f s[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) s[qt][kt] = v4f{0.f, 0.f, 0.f, 0.f};
    // K fragments software-pipelined SD k-steps ahead in registers (hipcc's own schedule
    // issues each ds_read one MFMA ahead, so every MFMA waits out the LDS latency)
    v8s kfr[SD][4];
#pragma unroll
    for (int ks = 0; ks < SD - 1; ++ks)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) kfr[ks][kt] = I::row_frag(kimg, kt * 16, ks, fl);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + SD - 1 < KS) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
          kfr[(ks + SD - 1) % SD][kt] = I::row_frag(kimg, kt * 16, ks + SD - 1, fl);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const v8s kf = MMPT_ATTN_DIAG == 3 ? qf[0][(ks + kt) & (KS - 1)] : kfr[ks % SD][kt];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) s[qt][kt] = mfma(kf, qf[qt][ks], s[qt][kt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the first V^T fragments go out before the softmax (V is resident since the barrier)
    v8s vfr[VD][2];
#pragma unroll
    for (int dt = 0; dt < VD - 1; ++dt) {
      vfr[dt][0] = I::tr_frag(vimg, dt * 16, 0, fl);
      vfr[dt][1] = I::tr_frag(vimg, dt * 16, 1, fl);
    }
    // ---- online softmax, deferred max (cdna_hip_programming.md T13) ----
    // Raw scores; the mask only on blocks that touch the diagonal or the sequence end
    // (wave-uniform test against this wave's first query row).
    const bool masked = (k0 + ABLK > p.S) ||
                        (CAUSAL && k0 + ABLK - 1 > q0 + wave * 16 * QT);
    if (masked) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = k0 + kt * 16 + 4 * g + i;
            if (key >= p.S || (CAUSAL && key > myq[qt])) s[qt][kt][i] = -INFINITY;
          }
    }
    // m[qt] is the (lane-uniform per row) reference max in log2 units.  Keep it while
    // every lane's block max stays within THR of it (P <= 2^THR, exact in fp32 and
    // bf16-relative); otherwise rescale all rows of the wave to the new row max, before
    // any P of this block is formed (the previous block's P·V is complete).
#ifndef MMPT_ATTN_THR
#define MMPT_ATTN_THR 0.0f
#endif
    constexpr float THR = MMPT_ATTN_THR;
    float lmx[QT];
    bool grow = false;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      float mx = fmaxf(fmaxf(s[qt][0][0], s[qt][0][1]), fmaxf(s[qt][0][2], s[qt][0][3]));
#pragma unroll
      for (int kt = 1; kt < 4; ++kt)
        mx = fmaxf(mx, fmaxf(fmaxf(s[qt][kt][0], s[qt][kt][1]), fmaxf(s[qt][kt][2], s[qt][kt][3])));
      lmx[qt] = mx * sl2;
      grow |= lmx[qt] > m[qt] + THR;
    }
    if (__builtin_amdgcn_read_exec() & __ballot(grow)) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        float mx = lmx[qt];
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mn = fmaxf(m[qt], mx);
        const float alpha = mn == -INFINITY ? 1.f : __builtin_amdgcn_exp2f(m[qt] - mn);
        l[qt] *= alpha;
#pragma unroll
        for (int i = 0; i < DT; ++i) o[qt][i] *= alpha;
        m[qt] = mn;
      }
    }
    v8s pf[QT][2];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      // fully masked rows keep m = -inf: their P is 0 (exp2(-inf))
      const float nm = m[qt] == -INFINITY ? 0.f : -m[qt];
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __builtin_amdgcn_exp2f(fmaf(s[qt][kt][i], sl2, nm));
          s[qt][kt][i] = e;
          rs += e;
        }
      l[qt] += rs;  // lane-partial row sum (this lane's 16 keys); reduced once at the end
      pf[qt][0] = pack_pair(s[qt][0], s[qt][1]);
      pf[qt][1] = pack_pair(s[qt][2], s[qt][3]);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      if (dt + VD - 1 < DT) {
        vfr[(dt + VD - 1) % VD][0] = I::tr_frag(vimg, (dt + VD - 1) * 16, 0, fl);
        vfr[(dt + VD - 1) % VD][1] = I::tr_frag(vimg, (dt + VD - 1) * 16, 1, fl);
      }
      __builtin_amdgcn_sched_barrier(0);
      const v8s v0 = MMPT_ATTN_DIAG == 3 ? qf[0][dt & (KS - 1)] : vfr[dt % VD][0];
      const v8s v1 = MMPT_ATTN_DIAG == 3 ? qf[0][(dt + 1) & (KS - 1)] : vfr[dt % VD][1];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        o[qt][dt] = mfma(v0, pf[qt][0], o[qt][dt]);
        o[qt][dt] = mfma(v1, pf[qt][1], o[qt][dt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (MMPT_ATTN_DIAG == 0 || MMPT_ATTN_DIAG == 3) vm_wait_all();
    __syncthreads();
  }
  for (int kb = nkb_w; kb < nkb; ++kb) {
    if (kb + 1 < nkb) stage_kv((kb + 1 + par) & 1, b, kcol, vcol, kb + 1);
    else if (wid_n >= 0) stage_kv((kb + 1 + par) & 1, nb, nkc, nvc, 0);
    vm_wait_all();
    __syncthreads();
  }
  // every wave is past the item's last barrier: the LDS buffer of the last key block is
  // free (the next item's block 0 went to the other one) and stages this item's O
  const int cb = b, ch = h, cbh = bh, cq0 = q0 + wave * 16 * QT;
  char* ostage = smem + ((nkb - 1 + par) & 1) * 2 * I::BYTES + wave * (16 * QT * I::RB);
  int cq[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) cq[qt] = myq[qt];
  wid = wid_n;
  ++it;
  if (wid >= 0) {
    par = (nkb + par) & 1;
    b = nb;
    h = nh;
    bh = nbh;
    q0 = nq0;
    kcol = nkc;
    vcol = nvc;
    // the next item's Q (this item's is dead since its last key block): in flight under
    // the O epilogue instead of after it (its key block 0 is in LDS already)
    if (MMPT_ATTN_EARLYQ) load_q();
  }
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    l[qt] += __shfl_xor(l[qt], 16, 64);
    l[qt] += __shfl_xor(l[qt], 32, 64);
  }
  // O through the wave's LDS region (chunk c of row r at c ^ (r mod 16): conflict-free
  // 8-B writes and 16-B reads), then whole 16-B-per-lane row segments to HBM instead of
  // 8-B pieces of 16 rows per store (the store-issue-bound tail, guide T21)
  constexpr int CPR = D / 8, RPI = 64 / CPR, SWM = (CPR < 16 ? CPR : 16) - 1;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const float inv = l[qt] > 0.f ? 1.0f / l[qt] : 0.f;
    const int r = qt * 16 + (lane & 15);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      uint2 u;
      u.x = (uint32_t)f2bf(o[qt][dt][0] * inv) | ((uint32_t)f2bf(o[qt][dt][1] * inv) << 16);
      u.y = (uint32_t)f2bf(o[qt][dt][2] * inv) | ((uint32_t)f2bf(o[qt][dt][3] * inv) << 16);
      const int c = 2 * dt + (g >> 1);
      stage_w8(ostage + r * I::RB, c ^ (r & SWM), g & 1, r, u);
    }
    if (g == 0 && cq[qt] < p.S)
      p.lse[(long)cbh * p.S + cq[qt]] = (m[qt] + log2f(l[qt])) / LOG2E;  // natural log
  }
  {
    const int rr = lane / CPR, c = lane % CPR;
#pragma unroll
    for (int i = 0; i < 16 * QT / RPI; ++i) {
      const int r = i * RPI + rr;
      const uint4 v = *(const uint4*)(ostage + r * I::RB + ((c ^ (r & SWM)) << 4));
      if (cq0 + r < p.S && chunk_real<D>(c, p.dr))
        *(uint4*)(p.out + (long)(cb * p.S + cq0 + r) * p.ld_out + ch * p.dr + c * 8) = v;
    }
  }
  if (wid < 0) break;
  if (!MMPT_ATTN_EARLYQ) load_q();
  }  // items
}

// δ[bh][q] = Σ_d dO·O  (fp32 of bf16 values).  16-B loads: LPR = D/8 lanes per (t, h)
// row, 64/LPR rows per wave, shuffle-reduced within the row's lanes.
template <int D>
__global__ __launch_bounds__(256) void attn_delta_kernel(AttnParams p, float* delta) {
  constexpr int LPR = D / 8, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;  // (t, h)
  const bool ok = row < (long)p.B * p.S * p.H;
  const long r = ok ? row : 0;
  const int h = (int)(r % p.H);
  const long t = r / p.H;
  const int c = (lane % LPR) * 8;
  float s = 0.f;
  if (chunk_real<D>(c / 8, p.dr)) {
    const v8s o = *(const v8s*)(p.o + t * p.ld_out + h * p.dr + c);
    const v8s d = *(const v8s*)(p.dout + t * p.ld_out + h * p.dr + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += bf2f((bf16_t)o[e]) * bf2f((bf16_t)d[e]);
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (ok && lane % LPR == 0) {
    const int b = (int)(t / p.S), q = (int)(t % p.S);
    delta[((long)b * p.H + h) * p.S + q] = s;
  }
}

// ======================= dK, dV (ring-pipelined) ===========================
// One workgroup = 4 waves x KT*16 keys (key on the MFMA lane; K/V fragments in
// registers; KT = 2 at D = 256 so every LDS fragment feeds two MFMAs — with one 16-key
// tile per fragment the LDS read rate alone would equal the MFMA rate).  Query blocks
// of QB = 32 rows stream through an NS = 4 slot LDS ring (Q image | dO image | lse, δ),
// filled by LDS-DMA NS-1 blocks ahead: one barrier per block, counted vmcnt waits.
// Per block and wave: S^T, dP^T (row reads of Q/dO), P and dS in registers,
// dV^T += dO^T·P^T and dK^T += Q^T·dS^T (transposed reads of the same images).
#ifndef MMPT_ATTN_DKDV_NS
#define MMPT_ATTN_DKDV_NS 4  // D = 256 ring slots (2: 66 KiB -> two workgroups per CU)
#endif
template <int D>
constexpr int dkdv_slots() { return D == 256 ? MMPT_ATTN_DKDV_NS : 4; }
// workgroups per CU the ring's LDS allows (2 also halves the register budget: KT = 1 only)
template <int D>
constexpr int dkdv_occ() { return dkdv_slots<D>() * (2 * 32 * D * 2 + 256) <= 80 * 1024 ? 2 : 1; }
template <int D, bool CAUSAL, int KT, int NW, bool DS = false, int DR = D>
__global__ __launch_bounds__(NW * 64, dkdv_occ<D>()) void attn_bwd_dkdv_ring_kernel(AttnParams p) {
  using I = Img<D>;
  constexpr int KS = dr_ksteps<D, DR>(), DT = DR / 16;
  constexpr int QB = 32, NS = dkdv_slots<D>();
  static_assert(!DS || (KT == 2 && QB == 32), "dS tiles: 32 keys per wave, 32-query blocks");
  // register-ring depths of the S/dP phase (row fragments) and the dV/dK phase (transposed)
  constexpr int PA = MMPT_ATTN_BPA, PB = MMPT_ATTN_BPB;
  constexpr int KW = 16 * KT;            // keys per wave
  constexpr int KB = NW * KW;            // keys per workgroup
  constexpr int IMG = QB * I::RB;
  constexpr int SLOT = 2 * IMG + 256;
  constexpr int PPB = 2 * (QB * I::RB / 1024) / NW + 1;  // DMA pieces per wave per block
  // (DS: + one 2-KiB transpose area per wave for the dS tile)
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT + (DS ? NW * 2048 : 0)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  // one workgroup per (key block, batch, kv head); GQA: it sweeps the query blocks of
  // the G query heads sharing that kv head, so dK/dV are summed over the group (repeat_kv's
  // backward) in registers — one writer per element, no atomics
  int bx, bh;
  attn_block(bx, bh);
  const int b = bh / p.Hkv, j = bh % p.Hkv;
  const int k0 = bx * KB;
  const int kw0 = k0 + wave * KW;  // this wave's first key
  const long kcol = p.koff + (long)j * p.khs, vcol = p.voff + (long)j * p.khs;

  v8s kf[KT][KS], vf[KT][KS];
  int mykey[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    mykey[kt] = kw0 + kt * 16 + (lane & 15);
    const long krow_t = (long)(b * p.S + min(mykey[kt], p.S - 1)) * p.ld;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (MMPT_ATTN_BDIAG == 10) {  // no K/V fragment loads
        kf[kt][ks] = vf[kt][ks] = v8s{(short)lane, 0, 0, 0, 0, 0, 0, (short)ks};
        continue;
      }
      kf[kt][ks] = gfrag_m<D>(p.qkv + krow_t + kcol, ks, lane, p.dr);
      vf[kt][ks] = gfrag_m<D>(p.qkv + krow_t + vcol, ks, lane, p.dr);
    }
  }
  v4f dk[KT][DT], dv[KT][DT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int i = 0; i < DT; ++i) dk[kt][i] = dv[kt][i] = v4f{0.f, 0.f, 0.f, 0.f};
  const float sl2 = p.scale * LOG2E;

  const int nqb = (p.S + QB - 1) / QB;
  const int qb0 = CAUSAL ? k0 / QB : 0;
  const int cnt = nqb - qb0;   // query blocks visited per query head
  const int total = p.G * cnt; // ring sequence n = gi * cnt + (nqb - 1 - qb)
  // query blocks LAST to first: the key blocks of one (batch, head) run side by side on one
  // XCD (attn_block) and all start on the same query block, so one HBM fetch of each Q/dO
  // block serves all of them through that XCD's L2 (first-to-last, each started at its own
  // diagonal and they drifted apart: L2 hit rate 35%)
  auto issue = [&](int n) {
    const int gi = n / cnt, qb = nqb - 1 - n % cnt;
    const int hq = j * p.G + gi;
    char* sl = smem + (n % NS) * SLOT;
    I::template dma_rows<NW, QB>(sl, p.qkv, p.ld, (long)hq * p.hs, p.S, b, qb * QB, wave, lane, p.dr);
    I::template dma_rows<NW, QB>(sl + IMG, p.dout, p.ld_out, (long)hq * p.dr, p.S, b, qb * QB, wave,
                                lane, p.dr);
    // stats (every wave writes the same 256 B, keeping the waves' vmcnt counts equal):
    // lanes 0-31 lse[q], lanes 32-63 δ[q]
    const long bhq = (long)b * p.H + hq;
    const int q = min(qb * QB + (lane & 31), p.S - 1);
    const float* src = lane < 32 ? p.lse + bhq * p.S + q : p.delta + bhq * p.S + q;
    glds4(src, sl + 2 * IMG);
  };
  const int npre = min(NS - 1, total);
  for (int n = 0; n < npre; ++n) issue(n);
  // K/V fragments (and the ring prologue) resident before the loop: left to hipcc, the
  // first use of each fragment inside the loop gets an s_waitcnt vmcnt(35 .. 4) that runs
  // on EVERY block — and the hardware count includes the ring's LDS-DMA, so each block
  // would drain the prefetched blocks (measured: 2.7 -> x ms per layer at B = 256)
  vm_wait_all();
  // causal: blocks whose every query precedes this wave's first key contribute nothing —
  // the last `skip` of each head's sequence; the wave only keeps the ring moving through
  // them (separate loop: no loop-carried phi on the accumulators).  Clamped to cnt: a wave
  // whose keys all lie past the sequence end skips every block but still joins every barrier.
  const int skip = CAUSAL ? min(cnt, max(0, kw0 / QB - qb0)) : 0;
  for (int gi = 0; gi < p.G; ++gi) {
  const int nb = gi * cnt;
  for (int n = nb; n < nb + cnt - skip; ++n) {
    // block n landed once at most the later prefetched blocks are outstanding
    if (MMPT_ATTN_BDIAG != 1) wait_blocks<PPB>(min(NS - 2, total - 1 - n));
    if (MMPT_ATTN_BDIAG != 5) __syncthreads();
    if (MMPT_ATTN_BDIAG != 1 && n + NS - 1 < total) issue(n + NS - 1);  // into the slot block n-1 used
    const int qb = nqb - 1 - (n - nb);
    const char* qimg = smem + (n % NS) * SLOT;
    const char* dimg = qimg + IMG;
    const float* stat = (const float*)(qimg + 2 * IMG);
    const int q0 = qb * QB;
    v4f s[KT][2], dp[KT][2];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[kt][qt] = dp[kt][qt] = v4f{0.f, 0.f, 0.f, 0.f};
    // Q / dO row fragments through a PA-deep register ring (step u = qt * D/32 + ks): the
    // reads of step u + PA - 1 are in flight under the MFMAs of step u — hipcc's own order
    // waits out the LDS latency before every step, the only wave on its SIMD idle meanwhile
    constexpr int NSA = 2 * KS;
    v8s qfr[PA], dfr[PA];
#pragma unroll
    for (int u = 0; u < PA - 1; ++u) {
      qfr[u] = I::template row_frag<QB>(qimg, (u / KS) * 16, u % KS, lane);
      dfr[u] = I::template row_frag<QB>(dimg, (u / KS) * 16, u % KS, lane);
    }
#pragma unroll
    for (int u = 0; u < NSA; ++u) {
      if (MMPT_ATTN_BDIAG == 3) break;
      const int qt = u / KS, ks = u % KS;
      if (u + PA - 1 < NSA) {
        const int v = u + PA - 1;
        qfr[v % PA] = I::template row_frag<QB>(qimg, (v / KS) * 16, v % KS, lane);
        dfr[v % PA] = I::template row_frag<QB>(dimg, (v / KS) * 16, v % KS, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        if (MMPT_ATTN_BDIAG == 8) {  // reads kept, MFMAs dropped
          s[kt][qt][0] += (float)(qfr[u % PA][0] ^ kf[kt][ks][1]);
          dp[kt][qt][0] += (float)(dfr[u % PA][0] ^ vf[kt][ks][1]);
          continue;
        }
        s[kt][qt] = mfma(qfr[u % PA], kf[kt][ks], s[kt][qt]);
        dp[kt][qt] = mfma(dfr[u % PA], vf[kt][ks], dp[kt][qt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the first dO^T / Q^T fragments of the dV / dK phase go out under the softmax
    v8s dtr[PB], qtr[PB];
#pragma unroll
    for (int dt = 0; dt < PB - 1; ++dt) {
      dtr[dt] = I::template tr_frag<QB>(dimg, dt * 16, 0, lane);
      qtr[dt] = I::template tr_frag<QB>(qimg, dt * 16, 0, lane);
    }
    const bool masked = (q0 + QB > p.S) || (kw0 + KW > p.S) || (CAUSAL && q0 < kw0 + KW - 1);
    v8s pa[KT], da[KT];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float4 ls = *(const float4*)(stat + qt * 16 + 4 * g);
      const float4 dl = *(const float4*)(stat + 32 + qt * 16 + 4 * g);
      const float nls[4] = {-ls.x * LOG2E, -ls.y * LOG2E, -ls.z * LOG2E, -ls.w * LOG2E};
      const float dlv[4] = {dl.x, dl.y, dl.z, dl.w};
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float pr = __builtin_amdgcn_exp2f(fmaf(s[kt][qt][i], sl2, nls[i]));
          if (MMPT_ATTN_BDIAG == 2) {
            dp[kt][qt][i] -= dlv[i];
            continue;
          }
          if (masked) {
            const int q = q0 + qt * 16 + 4 * g + i;
            if (q >= p.S || mykey[kt] >= p.S || (CAUSAL && mykey[kt] > q)) pr = 0.f;
          }
          s[kt][qt][i] = pr;                                // P
          dp[kt][qt][i] = pr * (dp[kt][qt][i] - dlv[i]);   // dS (unscaled)
        }
    }
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      pa[kt] = pack_pair(s[kt][0], s[kt][1]);
      da[kt] = pack_pair(dp[kt][0], dp[kt][1]);
    }
    if constexpr (DS) {
      // this wave's 32 x 32 dS tile: transposed through its LDS area into the dQ fragment
      // order (element (query 16qt + 4g + i, key kk) of this lane -> fragment qt, lane
      // 16((kk & 15) >> 2) + 4g + i, slot (kk & 3) + 4·kt), then two 16-B stores per lane
      char* tl = smem + NS * SLOT + wave * 2048;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const int kk = kt * 16 + (lane & 15);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            *(short*)(tl + qt * 1024 + ((((kk & 15) >> 2) * 16 + 4 * g + i) * 16) +
                      ((kk & 3) + 4 * kt) * 2) = da[kt][qt * 4 + i];
      }
    }
    // (DS: the transposed tile is read back late in the dV/dK phase and stored after it, so
    // neither the LDS write-read latency nor an lgkmcnt drain of the phase's fragment ring
    // sits on the critical path)
    v8s dst0 = v8s{0, 0, 0, 0, 0, 0, 0, 0}, dst1 = dst0;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      if (MMPT_ATTN_BDIAG == 4) break;
      if constexpr (DS) {
        if (dt == DT - 3) {
          const char* tl = smem + NS * SLOT + wave * 2048;
          dst0 = *(const v8s*)(tl + lane * 16);
          dst1 = *(const v8s*)(tl + 1024 + lane * 16);
        }
      }
      if (dt + PB - 1 < DT) {
        dtr[(dt + PB - 1) % PB] = I::template tr_frag<QB>(dimg, (dt + PB - 1) * 16, 0, lane);
        qtr[(dt + PB - 1) % PB] = I::template tr_frag<QB>(qimg, (dt + PB - 1) * 16, 0, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        if (MMPT_ATTN_BDIAG == 9) {  // reads kept, MFMAs dropped
          dv[kt][dt][0] += (float)(dtr[dt % PB][0] ^ pa[kt][1]);
          dk[kt][dt][0] += (float)(qtr[dt % PB][0] ^ da[kt][1]);
          continue;
        }
        dv[kt][dt] = mfma(dtr[dt % PB], pa[kt], dv[kt][dt]);
        if (MMPT_ATTN_BDIAG == 7) continue;  // dK MFMAs dropped
        dk[kt][dt] = mfma(qtr[dt % PB], da[kt], dk[kt][dt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (DS && kw0 < p.S) {  // (non-causal: a wave whose keys all lie past S has no tile column)
      bf16_t* dst = p.ds + ds_tile(b * p.H + j * p.G + n / cnt, (p.S + 31) / 32, qb, kw0 / 32);
      *(v8s*)(dst + lane * 8) = dst0;
      *(v8s*)(dst + 512 + lane * 8) = dst1;
    }
  }
  for (int n = nb + cnt - skip; n < nb + cnt; ++n) {
    wait_blocks<PPB>(min(NS - 2, total - 1 - n));
    __syncthreads();
    if (n + NS - 1 < total) issue(n + NS - 1);
  }
  }  // query heads of the group
  vm_wait_all();
  // dK, dV through LDS (the ring is free once every wave is past its last block): each wave
  // writes its KW rows of dK then dV (chunk c of row r at c ^ (r mod 16)), then stores whole
  // 16-B-per-lane row segments — 2·KW·D/512 stores per lane instead of KT·D/8 8-B pieces of
  // 16 rows each (the store-issue-bound tail)
  __syncthreads();
  static_assert(NW * 2 * KW * I::RB <= NS * SLOT, "dK/dV staging exceeds the ring");
  char* st = smem + wave * (2 * KW * I::RB);
  constexpr int CPR = D / 8, RPI = 64 / CPR, SWM = (CPR < 16 ? CPR : 16) - 1;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const int r = kt * 16 + (lane & 15);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int c = 2 * dt + (g >> 1);
      uint2 u;
      u.x = (uint32_t)f2bf(dk[kt][dt][0] * p.scale) | ((uint32_t)f2bf(dk[kt][dt][1] * p.scale) << 16);
      u.y = (uint32_t)f2bf(dk[kt][dt][2] * p.scale) | ((uint32_t)f2bf(dk[kt][dt][3] * p.scale) << 16);
      stage_w8(st + r * I::RB, c ^ (r & SWM), g & 1, r, u);
      u.x = (uint32_t)f2bf(dv[kt][dt][0]) | ((uint32_t)f2bf(dv[kt][dt][1]) << 16);
      u.y = (uint32_t)f2bf(dv[kt][dt][2]) | ((uint32_t)f2bf(dv[kt][dt][3]) << 16);
      stage_w8(st + (KW + r) * I::RB, c ^ (r & SWM), g & 1, r, u);
    }
  }
  const int rr = lane / CPR, c = lane % CPR;
#pragma unroll
  for (int i = 0; i < 2 * KW / RPI; ++i) {
    const int rw = i * RPI + rr;          // 0 .. 2KW-1: dK rows, then dV rows
    const int r = rw % KW;
    const uint4 v = *(const uint4*)(st + rw * I::RB + ((c ^ (r & SWM)) << 4));
    if (MMPT_ATTN_BDIAG == 11 && (v.x != 0x7fc07fc0u || i < 2 * KW / RPI - 1)) continue;  // no stores
    if (kw0 + r < p.S && chunk_real<D>(c, p.dr))
      *(uint4*)(p.dqkv + (long)(b * p.S + kw0 + r) * p.ld + (rw < KW ? kcol : vcol) + c * 8) = v;
  }
}

// ============== dK, dV through D-split wave pairs (D = 256, dS tiles) ===============
// 8 waves = 4 pairs x 32 keys of one (batch, kv head) key block of 128.  Wave a (role 0) of a
// pair holds the K fragments of the pair's 32 keys and computes S^T, wave b (role 1) holds
// V and computes dP^T (row reads of the Q / dO images); a forms P, the two exchange P and
// dP through LDS (lane to the same lane: both hold the same keys x queries), both form dS,
// and each accumulates dV^T, dK^T for ITS half of D (transposed reads of that half).  Per
// wave 64 K-or-V + 128 dK/dV accumulator registers instead of 128 + 256: two waves per SIMD,
// so one wave's LDS latency runs under the other's MFMAs (the single-wave-per-SIMD kernel
// above stalls on every fragment read).  Same MFMA work and fragment bytes per CU and block;
// + an exchange (4 KiB written and read per wave) and a second barrier per block.  The dS
// tile (for dQ) is transposed per wave: role r handles query rows 16r..16r+15.
#ifndef MMPT_ATTN_PA2
#define MMPT_ATTN_PA2 3
#endif
#ifndef MMPT_ATTN_PB2
#define MMPT_ATTN_PB2 2
#endif
// pair-kernel diagnostics (never shipped, wrong results; scripts/build_variants.sh): 1 = no
// exchange barrier, 2 = no S/dP MFMAs, 3 = no dV/dK MFMAs, 4 = no row-fragment reads, 5 = no
// transposed-fragment reads, 6 = no exchange LDS traffic, 7 = no dS transpose / store, 8 = no
// ring DMA in the block loop
#ifndef MMPT_ATTN_PDIAG
#define MMPT_ATTN_PDIAG 0
#endif
// pair placement: 1 = pair p is waves (p, p + 4) — the waves of a workgroup go to the SIMDs in a
// cyclic order, so w and w + 4 share a SIMD and every SIMD holds one role-0 wave (P = exp(...),
// the softmax VALU) and one role-1 wave; 0 = waves (2p, 2p + 1), which puts both role-0 waves
// of SIMDs 0 / 1 on the same SIMD and doubles that SIMD's softmax phase
#ifndef MMPT_ATTN_PAIRMAP
#define MMPT_ATTN_PAIRMAP 1
#endif

template <int D, bool CAUSAL>
__global__ __launch_bounds__(512, 1) void attn_bwd_dkdv_pair_kernel(AttnParams p) {
  static_assert(D == 256, "pair kernel: D = 256");
  using I = Img<D>;
  constexpr int QB = 32, NS = 3, KT = 2, KW = 32, NW = 8, NP = NW / 2, KB = NP * KW;
  constexpr int IMG = QB * I::RB;
  constexpr int SLOT = 2 * IMG + 256;
  constexpr int PPB = 2 * (IMG / 1024) / NW + 1;  // DMA pieces per wave per block
  constexpr int XB = KT * 2 * 1024;               // exchange bytes per wave
  constexpr int XOFF = NS * SLOT, TOFF = XOFF + NW * XB;
  constexpr int PA = MMPT_ATTN_PA2, PB = MMPT_ATTN_PB2;
  constexpr int DH = D / 32;  // 16-wide d-tiles per half
  constexpr int PD = MMPT_ATTN_PDIAG;
  constexpr int CPR = D / 8, RPI = 64 / CPR, NST = KW / RPI;  // dK/dV store instructions per wave
  static_assert(NP * 2 * KW * I::RB <= TOFF, "dK/dV staging exceeds ring + exchange");
  __shared__ __attribute__((aligned(16))) char smem[TOFF + NP * 2048];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pr = MMPT_ATTN_PAIRMAP ? wave & (NP - 1) : wave >> 1;
  const int role = MMPT_ATTN_PAIRMAP ? wave / NP : wave & 1;
  // Persistent (round 3): the workgroup walks items (128-key block, batch, kv head) in
  // attn_item order; the next item's K/V fragments load under this item's dK/dV epilogue and
  // its first ring blocks are staged before this item's dK/dV stores go out, so neither the
  // fragment prologue nor the ring prologue nor the store tail is exposed per item (they
  // were ~40% of the one-item-per-workgroup kernel at S = 707, profiles/r02/attn_dkdv_diag*).
  const int nx = (p.S + KB - 1) / KB;
  const int nitems = nx * p.B * p.Hkv;
  int it = 0;
  int wid = attn_item(nitems, 0);
  if (wid < 0) return;  // (workgroup-uniform)
  int b = 0, j = 0, k0 = 0, kw0 = 0;
  long kcol = 0, vcol = 0, mycol = 0;
  auto decode = [&](int w) {
    const int bx = nx - 1 - w % nx, bh = w / nx;
    b = bh / p.Hkv;
    j = bh % p.Hkv;
    k0 = bx * KB;
    kw0 = k0 + pr * KW;  // the pair's first key
    kcol = p.koff + (long)j * p.khs;
    vcol = p.voff + (long)j * p.khs;
    mycol = role ? vcol : kcol;
  };
  v8s kvf[KT][D / 32];  // role 0: K, role 1: V (B operand of S^T / dP^T)
  auto load_kv = [&]() {
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int key = kw0 + kt * 16 + (ln & 15);
      const long krow_t = (long)(b * p.S + min(key, p.S - 1)) * p.ld;
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks) kvf[kt][ks] = gfrag(p.qkv + krow_t + mycol, ks, ln);
    }
  };
  const float sl2 = p.scale * LOG2E;
  const int nqb = (p.S + QB - 1) / QB;
  const int nq = (p.S + 31) / 32;
  int qb0 = 0, cnt = 0, total = 0;
  // the ring is filled in sequence order n = 0, 1, ...: a cursor (query head, block, slot)
  // instead of n / cnt, n % cnt, n % NS (runtime divisions: ~40 SALU per block)
  int cur_gi = 0, cur_r = 0, cur_slot = 0;
  const uint32_t lbase = lds_addr(smem);  // LDS byte address of the ring (once: no per-piece cast)
  // the item's Q / dO bases (batch row 0, its first query head): a block's wave-uniform base is
  // then this + a 32-bit offset (a sequence spans < 2 GiB), no 64-bit multiplies per block
  const char* qbase = nullptr;
  const char* dbase = nullptr;
  const float* lbase_s = nullptr;  // lse / δ of the item's first query head
  const float* dbase_s = nullptr;
  auto setup = [&]() {
    cur_gi = cur_r = cur_slot = 0;
    qb0 = CAUSAL ? k0 / QB : 0;
    cnt = nqb - qb0;
    total = p.G * cnt;
    qbase = (const char*)(p.qkv + (long)b * p.S * p.ld + (long)j * p.G * p.hs);
    dbase = (const char*)(p.dout + (long)b * p.S * p.ld_out + (long)j * p.G * p.dr);
    lbase_s = p.lse + ((long)b * p.H + (long)j * p.G) * p.S;
    dbase_s = p.delta + ((long)b * p.H + (long)j * p.G) * p.S;
  };
  auto issue = [&]() {  // query blocks last to first (L2 sharing, as the ring kernel)
    // every per-lane value from a fresh v_mbcnt: nothing lane-dependent stays live across the
    // loops (hipcc spilled a hoisted 64-bit source address and reloaded it with vmcnt(0) inside
    // the block loop, draining the prefetched ring)
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    const int qb = nqb - 1 - cur_r;
    const int hq = j * p.G + cur_gi;
    char* sl = smem + cur_slot * SLOT;
    const uint32_t sla = lbase + cur_slot * SLOT;
    if (++cur_r == cnt) {
      cur_r = 0;
      ++cur_gi;
    }
    cur_slot = cur_slot == NS - 1 ? 0 : cur_slot + 1;
    const long t0 = (long)b * p.S;
    if (MMPT_ATTN_SADDR && qb * QB + QB <= p.S) {
      // a whole block: wave-uniform bases at its first row, per-lane 32-bit offsets (SADDR form)
      const int gi = hq - j * p.G;
      const char* bq = qbase + (qb * QB * (int)p.ld + gi * (int)p.hs) * 2;
      const char* bd = dbase + (qb * QB * (int)p.ld_out + gi * p.dr) * 2;
      constexpr int PPW = QB * I::RB / 1024 / NW;
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        const int q = wave * PPW + i;
        int r, lc;
        I::template piece<QB>(q, ln, r, lc);
        glds16_so(bq, r * (int)p.ld * 2 + lc * 16, sla + q * 1024);
        glds16_so(bd, r * (int)p.ld_out * 2 + lc * 16, sla + IMG + q * 1024);
      }
    } else {
      I::template dma_rows32<NW, QB>(sl, (const char*)(p.qkv + t0 * p.ld + (long)hq * p.hs),
                                     (int)p.ld * 2, p.S, qb * QB, wave, ln);
      I::template dma_rows32<NW, QB>(sl + IMG, (const char*)(p.dout + t0 * p.ld_out + (long)hq * p.dr),
                                     (int)p.ld_out * 2, p.S, qb * QB, wave, ln);
    }
    const int q = min(qb * QB + (ln & 31), p.S - 1);
    if (MMPT_ATTN_SADDR) {
      const float* src = (ln < 32 ? lbase_s : dbase_s) + ((hq - j * p.G) * p.S + q);
      glds4_a(src, sla + 2 * IMG);
    } else {
      const long bhq = (long)b * p.H + hq;
      glds4((ln < 32 ? p.lse : p.delta) + bhq * p.S + q, sl + 2 * IMG);
    }
  };
  decode(wid);
  setup();
  load_kv();
  for (int n = 0; n < min(NS - 1, total); ++n) issue();
  // exchange: the pair's P (written by role 0) and dP (role 1) at fixed places, both read
  // back by both waves — no role-dependent select per element
  char* xme = smem + XOFF + wave * XB;  // (wave = the role's slot: xp / xd below)
  const char* xp = smem + XOFF + (MMPT_ATTN_PAIRMAP ? pr : 2 * pr) * XB;
  const char* xd = smem + XOFF + (MMPT_ATTN_PAIRMAP ? NP + pr : 2 * pr + 1) * XB;
  char* tl = smem + TOFF + pr * 2048 + role * 1024;  // this wave's half of the dS transpose
  const int d0 = role * DH;
  bool drain_all = true;
  for (;;) {  // items
  // this item's K/V fragments and first ring blocks have landed once at most the previous
  // item's NST / 2 dV stores (the youngest vector-memory ops of every wave) are in flight
  if (drain_all) vm_wait_all();
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST / 2) : "memory");
  int mykey[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) mykey[kt] = kw0 + kt * 16 + (lane & 15);
  v4f dk[KT][DH], dv[KT][DH];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int i = 0; i < DH; ++i) dk[kt][i] = dv[kt][i] = v4f{0.f, 0.f, 0.f, 0.f};
  const int skip = CAUSAL ? min(cnt, max(0, kw0 / QB - qb0)) : 0;
  int use_slot = 0;  // ring slot of the block being consumed (n % NS)
    for (int gi = 0; gi < p.G; ++gi) {
    const int nb = gi * cnt;
    for (int n = nb; n < nb + cnt - skip; ++n) {
      if (PD != 8) wait_blocks<PPB>(min(NS - 2, total - 1 - n));
      __syncthreads();
      if (PD != 8 && n + NS - 1 < total) issue();  // into the slot block n - 1 used
      const int qb = nqb - 1 - (n - nb);
      const char* qimg = smem + use_slot * SLOT;
      use_slot = use_slot == NS - 1 ? 0 : use_slot + 1;
      const char* dimg = qimg + IMG;
      const float* stat = (const float*)(qimg + 2 * IMG);
      const char* rimg = role ? dimg : qimg;
      const int q0 = qb * QB;
      // lane-derived values re-materialised per block (empty asm): hipcc would otherwise hoist
      // the 16 per-fragment LDS offsets of the two phases out of the block loop, which took it
      // past 256 registers; computed at their use they cost ~3 VALU per fragment
      int lo;  // the lane id by v_mbcnt inside the loop (a hoisted copy is spilled, and its
               // reload's vmcnt(0) would drain the ring DMA: guide, attention pitfalls)
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lo));
      const int li = lo & 15, gg = lo >> 4;
      // slab images (Img<256>::off<QB>: 8 slabs of 32 rows x 64 B): one per-lane base for the row
      // fragments and two for the transposed ones (d-tile parity), the rest compile-time offsets
      constexpr int SS = QB * 64;  // slab bytes
      const int rbase = li * 64 + ((gg ^ I::fs(li)) << 4);
      // row fragment (Img::row_frag): rows 16qt + li, d chunk 4ks + gg
      auto rowf = [&](const char* img, int qt, int ks) -> v8s {
        return *(const v8s*)(img + ks * SS + qt * 1024 + rbase);
      };
      const int r1 = 4 * gg + (li >> 2), f1 = I::fs(r1) >> 1, pp = li & 3;
      const int tb0 = r1 * 64 + (((2 * f1) | (pp >> 1)) << 4) + (pp & 1) * 8;
      const int tb1 = r1 * 64 + (((2 * (f1 ^ 1)) | (pp >> 1)) << 4) + (pp & 1) * 8;
      // transposed fragment (Img::tr_frag, s = 0) of d-tile d0 + dt: rows r1 and r1 + 16, chunk
      // 2(d0 + dt) + (pp >> 1) = slab (d0 + dt) / 2, in-slab chunk 2((d0 + dt) & 1) + (pp >> 1)
      auto trf = [&](const char* img, int dt) -> v8s {
        const char* a = img + (d0 >> 1) * SS + (dt >> 1) * SS + ((dt & 1) ? tb1 : tb0);
        const v4s x = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a));
        const v4s y = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a + 16 * 64));
        return v8s{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
      };
      v4f acc[KT][2];
  #pragma unroll
      for (int kt = 0; kt < KT; ++kt) acc[kt][0] = acc[kt][1] = v4f{0.f, 0.f, 0.f, 0.f};
      // S^T (role 0) / dP^T (role 1): row fragments through a PA-deep register ring
      constexpr int NSA = 2 * (D / 32);
      v8s fr[PA];
  #pragma unroll
      for (int u = 0; u < PA - 1; ++u)
      fr[u] = PD == 4 ? kvf[1][u % (D / 32)] : rowf(rimg, u / (D / 32), u % (D / 32));
  #pragma unroll
      for (int u = 0; u < NSA; ++u) {
        const int qt = u / (D / 32), ks = u % (D / 32);
        if (u + PA - 1 < NSA) {
          const int v = u + PA - 1;
          fr[v % PA] = PD == 4 ? kvf[1][v % (D / 32)] : rowf(rimg, v / (D / 32), v % (D / 32));
        }
        __builtin_amdgcn_sched_barrier(0);
  #pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
        if (PD == 2) acc[kt][qt][0] += (float)(fr[u % PA][0] ^ kvf[kt][ks][1]);
        else acc[kt][qt] = mfma(fr[u % PA], kvf[kt][ks], acc[kt][qt]);
      }
        __builtin_amdgcn_sched_barrier(0);
      }
      // the first transposed fragments of this wave's D half go out before the exchange
      v8s dtr[PB], qtr[PB];
  #pragma unroll
      for (int dt = 0; dt < PB - 1; ++dt) {
        dtr[dt] = PD == 5 ? kvf[0][dt] : trf(dimg, dt);
        qtr[dt] = PD == 5 ? kvf[1][dt] : trf(qimg, dt);
      }
      const bool masked = (q0 + QB > p.S) || (kw0 + KW > p.S) || (CAUSAL && q0 < kw0 + KW - 1);
      if (role == 0) {  // P = exp(S·scale − lse); the mask as one uniform branch after
  #pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const float4 ls = *(const float4*)(stat + qt * 16 + 4 * gg);
          const float nls[4] = {-ls.x * LOG2E, -ls.y * LOG2E, -ls.z * LOG2E, -ls.w * LOG2E};
  #pragma unroll
          for (int kt = 0; kt < KT; ++kt)
  #pragma unroll
            for (int i = 0; i < 4; ++i)
              acc[kt][qt][i] = __builtin_amdgcn_exp2f(fmaf(acc[kt][qt][i], sl2, nls[i]));
        }
        if (masked) {
  #pragma unroll
          for (int qt = 0; qt < 2; ++qt)
  #pragma unroll
            for (int kt = 0; kt < KT; ++kt)
  #pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int q = q0 + qt * 16 + 4 * gg + i;
                const bool z = q >= p.S || mykey[kt] >= p.S || (CAUSAL && mykey[kt] > q);
                acc[kt][qt][i] = z ? 0.f : acc[kt][qt][i];
              }
        }
      }
  #pragma unroll
      for (int kt = 0; kt < KT; ++kt)
  #pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          if (PD != 6) *(v4f*)(xme + (kt * 2 + qt) * 1024 + lane * 16) = acc[kt][qt];
      if (PD != 1) __syncthreads();  // the pair's P and dP are in LDS
      v8s pa[KT], da[KT];
  #pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        v4f pp[2], ss[2];
  #pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const v4f pv = PD == 6 ? acc[kt][qt] : *(const v4f*)(xp + (kt * 2 + qt) * 1024 + lane * 16);
          const v4f dpv = PD == 6 ? acc[kt][qt] : *(const v4f*)(xd + (kt * 2 + qt) * 1024 + lane * 16);
          const float4 dl = *(const float4*)(stat + 32 + qt * 16 + 4 * gg);
          const float dlv[4] = {dl.x, dl.y, dl.z, dl.w};
  #pragma unroll
          for (int i = 0; i < 4; ++i) {
            pp[qt][i] = pv[i];
            ss[qt][i] = pv[i] * (dpv[i] - dlv[i]);  // dS (unscaled)
          }
        }
        pa[kt] = pack_pair(pp[0], pp[1]);
        da[kt] = pack_pair(ss[0], ss[1]);
      }
      // dS rows 16·role.. of the pair's tile, transposed into the dQ fragment order
  #pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
  #pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int L = (li >> 2) * 16 + 4 * gg + i;
          if (PD != 7)
            *(short*)(tl + (dst_pos(L) << 4) + ((li & 3) + 4 * kt) * 2) =
                role ? da[kt][4 + i] : da[kt][i];
        }
      }
      v8s dsv = v8s{0, 0, 0, 0, 0, 0, 0, 0};
  #pragma unroll
      for (int dt = 0; dt < DH; ++dt) {
        if (dt == DH - 3 && PD != 7) dsv = *(const v8s*)(tl + (dst_pos(lo) << 4));
        if (dt + PB - 1 < DH) {
          dtr[(dt + PB - 1) % PB] = PD == 5 ? kvf[0][dt % 8] : trf(dimg, dt + PB - 1);
          qtr[(dt + PB - 1) % PB] = PD == 5 ? kvf[1][dt % 8] : trf(qimg, dt + PB - 1);
        }
        __builtin_amdgcn_sched_barrier(0);
  #pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          if (PD == 3) {
            dv[kt][dt][0] += (float)(dtr[dt % PB][0] ^ pa[kt][1]);
            dk[kt][dt][0] += (float)(qtr[dt % PB][0] ^ da[kt][1]);
            continue;
          }
          dv[kt][dt] = mfma(dtr[dt % PB], pa[kt], dv[kt][dt]);
          dk[kt][dt] = mfma(qtr[dt % PB], da[kt], dk[kt][dt]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (PD != 7 && kw0 < p.S) {  // (non-causal: a pair whose keys all lie past S has no tile column)
        bf16_t* dst = p.ds + ds_tile(b * p.H + j * p.G + gi, nq, qb, kw0 / 32);
        *(v8s*)(dst + role * 512 + lane * 8) = dsv;
      }
    }
    for (int n = nb + cnt - skip; n < nb + cnt; ++n) {  // no contribution: keep the ring moving
      wait_blocks<PPB>(min(NS - 2, total - 1 - n));
      __syncthreads();
      if (n + NS - 1 < total) issue();
      use_slot = use_slot == NS - 1 ? 0 : use_slot + 1;
      __syncthreads();  // (the exchange barrier of the computing pairs)
    }
    }  // query heads of the group
  vm_wait_all();  // the ring is drained
  // the next item: K / V fragments and first ring blocks in flight under this epilogue
  const int wid_n = attn_item(nitems, it + 1);
  const int b_c = b, kw0_c = kw0;
  const long kcol_c = kcol, vcol_c = vcol;
  if (wid_n >= 0) decode(wid_n);
  __syncthreads();  // every wave is past the ring, exchange and transpose areas
  // dK then dV through slot 2 + exchange + transpose areas (16 KiB per pair: rows 0..31 of
  // 512 B, chunk c of row r at c ^ (r & 15)); each wave writes its D half, then stores 16 rows
  static_assert(2 * SLOT + NP * KW * I::RB <= TOFF + NP * 2048, "dK/dV staging exceeds LDS");
  char* st = smem + 2 * SLOT + pr * (KW * I::RB);
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int dt = 0; dt < DH; ++dt) dk[kt][dt] *= p.scale;
  if (p.rot == FUSED_ROT && role == 0) {  // (wave-uniform) dims 0..63 live in role 0's half
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
      rope_bwd_tiles(dk[kt], p, min(kw0_c + kt * 16 + (lane & 15), p.S - 1), lane >> 4);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    {
      const int g = lane >> 4;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const int r = kt * 16 + (lane & 15);
#pragma unroll
        for (int dt = 0; dt < DH; ++dt) {
          const int c = 2 * (d0 + dt) + (g >> 1);
          const v4f x = h ? dv[kt][dt] : dk[kt][dt];
          uint2 u;
          u.x = (uint32_t)f2bf(x[0]) | ((uint32_t)f2bf(x[1]) << 16);
          u.y = (uint32_t)f2bf(x[2]) | ((uint32_t)f2bf(x[3]) << 16);
          stage_w8(st + r * I::RB, c ^ (r & 15), g & 1, r, u);
        }
      }
    }
    __syncthreads();
    // the next item's K / V fragments once dV is staged (the accumulators are dead: loading
    // them earlier, under live dK/dV, made hipcc spill and drain every load with vmcnt(0))
    if (h == 1 && wid_n >= 0) {  // its first ring blocks (slots 0, 1) too
      setup();
      for (int n = 0; n < min(NS - 1, total); ++n) issue();
      load_kv();
    }
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    const int rr = ln / CPR, cc = ln % CPR;
#pragma unroll
    for (int i = 0; i < NST / 2; ++i) {
      const int r = 16 * role + i * RPI + rr;
      const uint4 v = *(const uint4*)(st + r * I::RB + ((cc ^ (r & 15)) << 4));
      if (kw0_c + r < p.S)
        *(uint4*)(p.dqkv + (long)(b_c * p.S + kw0_c + r) * p.ld + (h ? vcol_c : kcol_c) + cc * 8) = v;
    }
    if (h == 0) __syncthreads();  // dK read out before dV overwrites the area
  }
  if (wid_n < 0) break;
  // a partial key block's stores are exec-masked or skipped: count-free wait next time
  drain_all = kw0_c + KW > p.S;
  wid = wid_n;
  ++it;
  }  // items
}

// ================================ dQ =======================================
// Workgroup = NW waves = NW·16·QT queries (query on the MFMA lane); K / V blocks of 64 keys
// double-buffered in LDS by LDS-DMA.  Persistent like the forward (attn_item order): the
// next item's first K/V block is staged under the current item's last key block, dQ leaves
// through the LDS buffer that block frees, as 16-B row segments.
template <int D, bool CAUSAL, int QT, int NW, int DR = D>
__global__ __launch_bounds__(NW * 64, 1) void attn_bwd_dq_kernel(AttnParams p) {
  using I = Img<D>;
  constexpr int KS = dr_ksteps<D, DR>(), DT = DR / 16;
  __shared__ __attribute__((aligned(16))) char smem[4 * I::BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  constexpr int BQ = NW * 16 * QT;
  const int nx = (p.S + BQ - 1) / BQ;
  const int nitems = nx * p.B * p.H;
  int it = 0;
  int wid = attn_item(nitems, 0);
  if (wid < 0) return;  // (workgroup-uniform)
  const float sl2 = p.scale * LOG2E;
  const int nkb_all = (p.S + ABLK - 1) / ABLK;

  int b, h, bh, q0, nkb;
  long kcol, vcol;
  int myq[QT];
  v8s qf[QT][KS], df[QT][KS];
  float my_lse[QT], my_del[QT];
  auto decode = [&](int w, int& b_, int& h_, int& bh_, int& q0_, long& kc, long& vc) {
    const int bx = nx - 1 - w % nx;
    bh_ = w / nx;
    b_ = bh_ / p.H;
    h_ = bh_ % p.H;
    kc = p.koff + (long)(h_ / p.G) * p.khs;
    vc = p.voff + (long)(h_ / p.G) * p.khs;
    q0_ = bx * BQ;
  };
  auto load_q = [&]() {
    nkb = CAUSAL ? min(nkb_all, (q0 + BQ - 1) / ABLK + 1) : nkb_all;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      myq[qt] = q0 + wave * 16 * QT + qt * 16 + (lane & 15);
      const long tq = (long)(b * p.S + min(myq[qt], p.S - 1));
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        qf[qt][ks] = gfrag_m<D>(p.qkv + tq * p.ld + h * p.hs, ks, lane, p.dr);
        df[qt][ks] = gfrag_m<D>(p.dout + tq * p.ld_out + h * p.dr, ks, lane, p.dr);
      }
      my_lse[qt] = myq[qt] < p.S ? p.lse[(long)bh * p.S + myq[qt]] * LOG2E : 0.f;
      my_del[qt] = myq[qt] < p.S ? p.delta[(long)bh * p.S + myq[qt]] : 0.f;
    }
  };
  auto stage_kv = [&](int buf, int bb, long kc, long vc, int kb) {
    char* img = smem + buf * 2 * I::BYTES;
    if constexpr (D == 256) {
      // K and V pieces share their per-lane row / chunk offsets (32-bit, from a uniform base
      // at the batch's row 0): ~4 VALU per piece pair instead of ~8 of 64-bit math per piece
      constexpr int PPW = (D / 8) / NW;
      const char* bk = (const char*)(p.qkv + (long)bb * p.S * p.ld + kc);
      const char* bv = bk + (vc - kc) * 2;
      const int ldb = (int)p.ld * 2;
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        const int q = wave * PPW + i;
        int r, lc;
        I::template piece<ABLK>(q, lane, r, lc);
        const int off = min(kb * ABLK + r, p.S - 1) * ldb + (lc << 4);
        glds16(bk + off, img + q * 1024);
        glds16(bv + off, img + I::BYTES + q * 1024);
      }
    } else {
      I::template dma<NW>(img, p.qkv, p.ld, kc, p.S, bb, kb * ABLK, wave, lane, p.dr);
      I::template dma<NW>(img + I::BYTES, p.qkv, p.ld, vc, p.S, bb, kb * ABLK, wave, lane, p.dr);
    }
  };
  decode(wid, b, h, bh, q0, kcol, vcol);
  load_q();
  stage_kv(0, b, kcol, vcol, 0);
  int par = 0;  // LDS buffer of key block kb: (kb + par) & 1
  v4f dq[QT][DT];
  for (;;) {
  const int wid_n = attn_item(nitems, it + 1);
  int nb = 0, nh = 0, nbh = 0, nq0 = 0;
  long nkc = 0, nvc = 0;
  if (wid_n >= 0) decode(wid_n, nb, nh, nbh, nq0, nkc, nvc);
  vm_wait_all();
  __syncthreads();
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int i = 0; i < DT; ++i) dq[qt][i] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * ABLK;
    char* kimg = smem + ((kb + par) & 1) * 2 * I::BYTES;
    char* vimg = kimg + I::BYTES;
    if (kb + 1 < nkb) stage_kv((kb + 1 + par) & 1, b, kcol, vcol, kb + 1);
    else if (wid_n >= 0) stage_kv((kb + 1 + par) & 1, nb, nkc, nvc, 0);
    v4f s[QT][4], dp[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) s[qt][kt] = dp[qt][kt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const v8s kfr = I::row_frag(kimg, kt * 16, ks, lane);
        const v8s vfr = I::row_frag(vimg, kt * 16, ks, lane);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
          s[qt][kt] = mfma(kfr, qf[qt][ks], s[qt][kt]);
          dp[qt][kt] = mfma(vfr, df[qt][ks], dp[qt][kt]);
        }
      }
    v8s dsf[QT][2];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = k0 + kt * 16 + 4 * g + i;
          float pr = exp2f(s[qt][kt][i] * sl2 - my_lse[qt]);
          if (key >= p.S || myq[qt] >= p.S || (CAUSAL && key > myq[qt])) pr = 0.f;
          dp[qt][kt][i] = pr * (dp[qt][kt][i] - my_del[qt]);
        }
      dsf[qt][0] = pack_pair(dp[qt][0], dp[qt][1]);
      dsf[qt][1] = pack_pair(dp[qt][2], dp[qt][3]);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const v8s k0f = I::tr_frag(kimg, dt * 16, 0, lane);
      const v8s k1f = I::tr_frag(kimg, dt * 16, 1, lane);
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        dq[qt][dt] = mfma(k0f, dsf[qt][0], dq[qt][dt]);
        dq[qt][dt] = mfma(k1f, dsf[qt][1], dq[qt][dt]);
      }
    }
    vm_wait_all();
    __syncthreads();
  }
  // past the item's last barrier: dQ through the buffer the last key block used
  const int cb = b, cq0 = q0 + wave * 16 * QT;
  const long cqcol = (long)h * p.hs;
  char* ostage = smem + ((nkb - 1 + par) & 1) * 2 * I::BYTES + wave * (16 * QT * I::RB);
  wid = wid_n;
  ++it;
  if (wid >= 0) {
    par = (nkb + par) & 1;
    b = nb;
    h = nh;
    bh = nbh;
    q0 = nq0;
    kcol = nkc;
    vcol = nvc;
    if (MMPT_ATTN_EARLYQ) load_q();  // next item's Q / dO / lse / δ under the dQ stores
  }
#if MMPT_ATTN_DQ_STAGE
  constexpr int CPR = D / 8, RPI = 64 / CPR, SWM = (CPR < 16 ? CPR : 16) - 1;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int r = qt * 16 + (lane & 15);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      uint2 u;
      u.x = (uint32_t)f2bf(dq[qt][dt][0] * p.scale) | ((uint32_t)f2bf(dq[qt][dt][1] * p.scale) << 16);
      u.y = (uint32_t)f2bf(dq[qt][dt][2] * p.scale) | ((uint32_t)f2bf(dq[qt][dt][3] * p.scale) << 16);
      const int c = 2 * dt + (g >> 1);
      stage_w8(ostage + r * I::RB, c ^ (r & SWM), g & 1, r, u);
    }
  }
  {
    const int rr = lane / CPR, c = lane % CPR;
#pragma unroll
    for (int i = 0; i < 16 * QT / RPI; ++i) {
      const int r = i * RPI + rr;
      const uint4 v = *(const uint4*)(ostage + r * I::RB + ((c ^ (r & SWM)) << 4));
      if (cq0 + r < p.S && chunk_real<D>(c, p.dr))
        *(uint4*)(p.dqkv + (long)(cb * p.S + cq0 + r) * p.ld + cqcol + c * 8) = v;
    }
  }
#else
  (void)ostage;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    if (cq0 + qt * 16 + (lane & 15) >= p.S) continue;
    bf16_t* base = p.dqkv + (long)(cb * p.S + cq0 + qt * 16 + (lane & 15)) * p.ld + cqcol;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      if (!chunk_real<D>(dt * 2, p.dr)) break;
      uint2 u;
      u.x = (uint32_t)f2bf(dq[qt][dt][0] * p.scale) | ((uint32_t)f2bf(dq[qt][dt][1] * p.scale) << 16);
      u.y = (uint32_t)f2bf(dq[qt][dt][2] * p.scale) | ((uint32_t)f2bf(dq[qt][dt][3] * p.scale) << 16);
      *(uint2*)(base + dt * 16 + 4 * g) = u;
    }
  }
#endif
  if (wid < 0) break;
  if (!MMPT_ATTN_EARLYQ) load_q();
  }  // items
}

// ============================ dQ from dS tiles ==============================
// dQ = scale · dS·K over the dS tiles the dK/dV kernel wrote (ds_tile): one workgroup = 4
// waves x 32 query rows of one (batch, head); wave w owns 32-query block qb and reads its
// tiles (qb, kb) as B fragments straight from global memory (16 B per lane, one block
// ahead in registers); K blocks of 64 keys double-buffered in LDS by LDS-DMA, read as K^T
// fragments (ds_read_b64_tr_b16, the pi key order of the tiles).  Two workgroups per CU
// (64 KiB LDS each).  Causal: tiles past the diagonal (kb > qb) are neither written nor
// read.  dQ leaves through the K buffers as 16-B row segments.
// 16-B global load issued from inline asm: hipcc does not count it, so it inserts no
// s_waitcnt of its own before the fragment's use; `ds_wait` below orders the use
__device__ __forceinline__ v8s gload16(const bf16_t* ptr) {
  v8s r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(ptr) : "memory");
  return r;
}
// s_waitcnt vmcnt(N) tied to the four fragments it guards (their uses cannot move above it)
template <int N>
__device__ __forceinline__ void ds_wait(v8s& a, v8s& b, v8s& c, v8s& d) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N) : "memory");
}

// dQ-from-dS diagnostics (never shipped, wrong results; scripts/build_variants.sh): 1 = no
// MFMAs, 2 = no dS loads, 3 = no K DMA / K^T reads, 4 = no barrier
#ifndef MMPT_ATTN_DQDIAG
#define MMPT_ATTN_DQDIAG 0
#endif
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_ds_kernel(AttnParams p) {
  constexpr int QD = MMPT_ATTN_DQDIAG;
  using I = Img<D>;
  constexpr int NW = 4, BQ = NW * 32;
  constexpr int PPW = (D / 8) / NW;  // K DMA pieces per wave per block
  static_assert(2 * I::BYTES >= NW * 32 * I::RB, "dQ staging exceeds the K buffers");
  __shared__ __attribute__((aligned(16))) char smem[2 * I::BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  int bx, bh;
  attn_block(bx, bh);
  const int b = bh / p.H, h = bh % p.H;
  const long kcol = p.koff + (long)(h / p.G) * p.khs;
  const int q0 = bx * BQ;
  const int nq = (p.S + 31) / 32;
  const int qb = q0 / 32 + wave;  // this wave's 32-query block
  // 32-key tiles this wave reads: [0, kt_hi)
  const int kt_hi = qb >= nq ? 0 : (CAUSAL ? qb + 1 : nq);
  const int nkb_all = (p.S + ABLK - 1) / ABLK;
  const int nkb = CAUSAL ? min(nkb_all, (min(q0 + BQ, p.S) - 1) / ABLK + 1) : nkb_all;
  const bf16_t* dsw = p.ds + ds_tile(bh, nq, min(qb, nq - 1), 0) + lane * 8;
  auto stage_k = [&](int buf, int kb) {
    if (QD == 3) return;
    I::template dma<NW>(smem + buf * I::BYTES, p.qkv, p.ld, kcol, p.S, b, kb * ABLK, wave, lane,
                        p.dr);
  };
  // dS fragments of 64-key block kb: tiles 2kb, 2kb + 1 (clamped into the head's tile row, so
  // every wave always issues exactly 4 loads: the vmcnt counts stay uniform) x fragments qt
  auto load_ds = [&](int kb, v8s (&f)[4]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
        f[2 * t + qt] = QD == 2 ? v8s{0, 0, 0, 0, 0, 0, 0, (short)kb}
                                : gload16(dsw + (long)min(2 * kb + t, nq - 1) * 1024 + qt * 512);
  };
  v4f dq[2][D / 16];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int i = 0; i < D / 16; ++i) dq[qt][i] = v4f{0.f, 0.f, 0.f, 0.f};
  // ring: dS fragments two blocks ahead in registers (three named sets, the loop unrolled by
  // three so no set is ever copied), K one block ahead in the LDS double buffer.  Issue order
  // per iteration kb: K(kb+1), dS(kb+2); the prologue dS(0), K(0), dS(1) — so at the top of
  // iteration kb only dS(kb+1) (4 loads) is younger than K(kb) and dS(kb).
  v8s fa[4], fb[4], fc[4];
  load_ds(0, fa);
  stage_k(0, 0);
  load_ds(1, fb);  // (issued even past nkb: clamped, never used)
  auto body = [&](int kb, v8s (&cur)[4], v8s (&far)[4]) {
    if (QD != 2) ds_wait<4>(cur[0], cur[1], cur[2], cur[3]);  // K(kb), dS(kb) landed
    else vm_wait_all();
    if (QD != 4) __syncthreads();  // ... for every wave; block kb - 1's K buffer is free
    if (kb + 1 < nkb) stage_k((kb + 1) & 1, kb + 1);
    load_ds(kb + 2, far);
    const char* kimg = smem + (kb & 1) * I::BYTES;
    if (2 * kb < kt_hi) {  // wave-uniform
      const bool two = 2 * kb + 1 < kt_hi;
      // K^T fragments through a depth-KD register ring: the reads of d-tile dt + KD - 1 are
      // in flight under the MFMAs of dt (hipcc's order waited out the LDS latency before
      // every d-tile)
      constexpr int KD = MMPT_ATTN_KD;
      v8s kr[KD][2];
#pragma unroll
      for (int dt = 0; dt < KD - 1; ++dt) {
        kr[dt][0] = QD == 3 ? cur[dt & 3] : I::tr_frag(kimg, dt * 16, 0, lane);
        kr[dt][1] = QD == 3 ? cur[(dt + 1) & 3] : I::tr_frag(kimg, dt * 16, 1, lane);
      }
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        if (dt + KD - 1 < D / 16) {
          kr[(dt + KD - 1) % KD][0] = QD == 3 ? cur[dt & 3] : I::tr_frag(kimg, (dt + KD - 1) * 16, 0, lane);
          kr[(dt + KD - 1) % KD][1] = QD == 3 ? cur[(dt + 1) & 3] : I::tr_frag(kimg, (dt + KD - 1) * 16, 1, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          if (QD == 1) {
            dq[qt][dt][0] += (float)(kr[dt % KD][0][1] ^ cur[qt][2]);
            if (two) dq[qt][dt][1] += (float)(kr[dt % KD][1][1] ^ cur[2 + qt][2]);
            continue;
          }
          dq[qt][dt] = mfma(kr[dt % KD][0], cur[qt], dq[qt][dt]);
          if (two) dq[qt][dt] = mfma(kr[dt % KD][1], cur[2 + qt], dq[qt][dt]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  for (int kb = 0; kb < nkb; kb += 3) {
    body(kb, fa, fc);
    if (kb + 1 < nkb) body(kb + 1, fb, fa);
    if (kb + 2 < nkb) body(kb + 2, fc, fb);
  }
  (void)PPW;
  vm_wait_all();
  // the last blocks' loads run past nkb (their fragments are never used): keep every set
  // live until this wait, or hipcc would hand a dead set's registers to other values while
  // the load is still in flight and the late write would clobber them
#pragma unroll
  for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(fa[i]), "v"(fb[i]), "v"(fc[i]));
  __syncthreads();  // every wave is done with both K buffers: they stage dQ
  constexpr int CPR = D / 8, RPI = 64 / CPR, SWM = (CPR < 16 ? CPR : 16) - 1;
  char* ost = smem + wave * (32 * I::RB);
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) dq[qt][dt] *= p.scale;
  if (p.rot == FUSED_ROT) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
      rope_bwd_tiles(dq[qt], p, min(q0 + wave * 32 + qt * 16 + (lane & 15), p.S - 1), g);
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int r = qt * 16 + (lane & 15);
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      uint2 u;
      u.x = (uint32_t)f2bf(dq[qt][dt][0]) | ((uint32_t)f2bf(dq[qt][dt][1]) << 16);
      u.y = (uint32_t)f2bf(dq[qt][dt][2]) | ((uint32_t)f2bf(dq[qt][dt][3]) << 16);
      const int c = 2 * dt + (g >> 1);
      stage_w8(ost + r * I::RB, c ^ (r & SWM), g & 1, r, u);
    }
  }
  const int rr = lane / CPR, c = lane % CPR;
  const int wq0 = q0 + wave * 32;
#pragma unroll
  for (int i = 0; i < 32 / RPI; ++i) {
    const int r = i * RPI + rr;
    const uint4 v = *(const uint4*)(ost + r * I::RB + ((c ^ (r & SWM)) << 4));
    if (wq0 + r < p.S && chunk_real<D>(c, p.dr))
      *(uint4*)(p.dqkv + (long)(b * p.S + wq0 + r) * p.ld + (long)h * p.hs + c * 8) = v;
  }
}

// D = 256 backward through dS tiles (MMPT_ATTN_DS, default on): 0 = the recomputing dQ kernel
int g_attn_ds = -1;
int attn_ds_mode() {
  if (g_attn_ds < 0) {
    const char* e = getenv("MMPT_ATTN_DS");
    g_attn_ds = (e != nullptr && e[0] == '0') ? 0 : 1;
  }
  return g_attn_ds;
}
// D = 256 dK/dV through D-split wave pairs (MMPT_ATTN_PAIR, default on): 0 = the one-wave-
// per-SIMD ring kernel
int g_attn_pair = -1;  // read once; mmpt_set_switch overrides it (the bitwise A/B test)
int attn_pair_mode() {
  if (g_attn_pair < 0) {
    const char* e = getenv("MMPT_ATTN_PAIR");
    g_attn_pair = (e != nullptr && e[0] == '0') ? 0 : 1;
  }
  return g_attn_pair;
}
// head_dim 80 (Pythia-2.8B) on the D = 128 kernels computing 80 dims (MMPT_ATTN_NATIVE80, default
// on): 0 = all 128 dims with 80.. zero-filled (the round-3 path; bitwise the same results)
int g_attn_native80 = -1;
int attn_native80() {
  if (g_attn_native80 < 0) {
    const char* e = getenv("MMPT_ATTN_NATIVE80");
    g_attn_native80 = (e != nullptr && e[0] == '0') ? 0 : 1;
  }
  return g_attn_native80;
}
size_t ds_offset(int64_t batch, int64_t seq, int64_t heads) {  // after δ, 256-B aligned
  return ((size_t)(batch * seq * heads) * sizeof(float) + 255) & ~(size_t)255;
}

// Wave layout per head dim: D = 256 -> 8 waves x 16 query rows (2 waves per SIMD: one
// wave's softmax VALU runs under the other's MFMAs; O = 64 accumulator registers);
// D = 128 -> 4 waves x 32 rows; D = 64 -> 4 waves x 16 rows (short ViT sequences).
#ifndef MMPT_ATTN_FWD256
#define MMPT_ATTN_FWD256 81  // D = 256 forward: waves * 10 + query tiles per wave
#endif
#ifndef MMPT_ATTN_DKDV256
#define MMPT_ATTN_DKDV256 42  // D = 256 dK/dV kernel: waves * 10 + key tiles per wave
#endif
#ifndef MMPT_ATTN_DQ256
#define MMPT_ATTN_DQ256 81   // D = 256 dQ kernel: waves * 10 + query tiles per wave
#endif
template <int D>
#ifndef MMPT_ATTN_FWD128
#define MMPT_ATTN_FWD128 1  // D = 128 forward: query tiles per wave (round 5: 1, was 2 — C5's
                           // attention forward 1433 -> 1208 us, profiles/r05/attn128/)
#endif
constexpr int qtiles() { return D == 128 ? MMPT_ATTN_FWD128 : D == 256 ? MMPT_ATTN_FWD256 % 10 : 1; }
template <int D>
constexpr int qwaves() { return D == 256 ? MMPT_ATTN_FWD256 / 10 : 4; }
template <int D>
#ifndef MMPT_ATTN_DQ128
#define MMPT_ATTN_DQ128 1  // D = 128 (and the 80-dim native path) dQ kernel: query tiles per wave
                          // (round 5: 1, was 2 — C5's attention backward 4795 -> 3676 us,
                          // profiles/r05/attn128/)
#endif
constexpr int dq_qtiles() { return D == 128 ? MMPT_ATTN_DQ128 : D == 256 ? MMPT_ATTN_DQ256 % 10 : 1; }
template <int D>
constexpr int dq_qwaves() { return D == 256 ? MMPT_ATTN_DQ256 / 10 : 4; }

// workgroups of a persistent forward launch: the CU count rounded down to whole XCDs (one
// 128-KiB-LDS workgroup per CU); MMPT_ATTN_PERSIST=0 -> one workgroup per query block
int attn_slots() {
  static int slots = -1;
  if (slots < 0) {
    const char* e = getenv("MMPT_ATTN_PERSIST");
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    slots = (e != nullptr && e[0] == '0') ? 0 : (cus / 8) * 8;
  }
  return slots;
}

template <int D, int DR = D>
int run_fwd(const AttnParams& p, bool causal, hipStream_t s) {
  constexpr int QT = qtiles<D>(), NW = qwaves<D>();
  const long items = (long)((p.S + NW * 16 * QT - 1) / (NW * 16 * QT)) * p.B * p.H;
  // persistent grid: CUs x resident workgroups per CU (1 at D = 256: 128 KiB of LDS)
  static int occ[2] = {-1, -1};
  auto grid_for = [&](const void* kern, int& o) {
    if (o < 0 && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kern, NW * 64, 0) != hipSuccess ||
                  o < 1))
      o = 1;
    const long slots = D >= 128 ? (long)attn_slots() * o : 0;  // D = 64 (ViT): one per block
    return dim3((unsigned)(slots > 0 && items > slots ? slots : items));
  };
  if (causal)
    attn_fwd_kernel<D, true, QT, NW, DR><<<grid_for((const void*)attn_fwd_kernel<D, true, QT, NW, DR>,
                                                    occ[0]), NW * 64, 0, s>>>(p);
  else
    attn_fwd_kernel<D, false, QT, NW, DR><<<grid_for((const void*)attn_fwd_kernel<D, false, QT, NW, DR>,
                                                     occ[1]), NW * 64, 0, s>>>(p);
  return check_launch("attention_fwd");
}

template <int D, int DR = D>
int run_bwd(AttnParams p, bool causal, float* delta, hipStream_t s) {
  const long rows = (long)p.B * p.S * p.H;
  constexpr int RPB = 4 * (64 / (D / 8));  // (t, h) rows per 256-thread block
  attn_delta_kernel<D><<<(unsigned)((rows + RPB - 1) / RPB), 256, 0, s>>>(p, delta);
  int rc = check_launch("attention_bwd_delta");
  if (rc) return rc;
  p.delta = delta;
  constexpr int QT = dq_qtiles<D>(), NW = dq_qwaves<D>();
  // dK/dV: key tiles per wave and waves (D = 256: MMPT_ATTN_DKDV256 = waves·10 + tiles)
  constexpr int KT = D == 256 ? MMPT_ATTN_DKDV256 % 10 : 1;
  constexpr int KNW = D == 256 ? MMPT_ATTN_DKDV256 / 10 : 4;
  dim3 grid((p.S + KNW * 16 * KT - 1) / (KNW * 16 * KT), p.B * p.Hkv);
  const long items = (long)((p.S + NW * 16 * QT - 1) / (NW * 16 * QT)) * p.B * p.H;
  static int occ[2] = {-1, -1};
  auto gq = [&](const void* kern, int& o) {
    if (o < 0 && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kern, NW * 64, 0) != hipSuccess ||
                  o < 1))
      o = 1;
    const long slots = D >= 128 ? (long)attn_slots() * o : 0;
    return dim3((unsigned)(slots > 0 && items > slots ? slots : items));
  };
  if constexpr (D == 256 && KT == 2) {
   if (attn_ds_mode() && p.ds != nullptr) {
    // dS tiles: the dK/dV kernel writes them, dQ = scale · dS·K reads them
    dim3 gq((p.S + 127) / 128, p.B * p.H);
    if (attn_pair_mode()) {  // D-split wave pairs: 128 keys per workgroup as the ring kernel
      const long pitems = (long)((p.S + 127) / 128) * p.B * p.Hkv;  // persistent: one per CU
      const long pslots = attn_slots();
      dim3 gp((unsigned)(pslots > 0 && pitems > pslots ? pslots : pitems));
      if (causal) attn_bwd_dkdv_pair_kernel<D, true><<<gp, 512, 0, s>>>(p);
      else attn_bwd_dkdv_pair_kernel<D, false><<<gp, 512, 0, s>>>(p);
      rc = check_launch("attention_bwd_dkdv");
      if (rc) return rc;
      if (causal) attn_bwd_dq_ds_kernel<D, true><<<gq, 256, 0, s>>>(p);
      else attn_bwd_dq_ds_kernel<D, false><<<gq, 256, 0, s>>>(p);
      return check_launch("attention_bwd");
    }
    if (causal) {
      attn_bwd_dkdv_ring_kernel<D, true, KT, KNW, true><<<grid, KNW * 64, 0, s>>>(p);
      attn_bwd_dq_ds_kernel<D, true><<<gq, 256, 0, s>>>(p);
    } else {
      attn_bwd_dkdv_ring_kernel<D, false, KT, KNW, true><<<grid, KNW * 64, 0, s>>>(p);
      attn_bwd_dq_ds_kernel<D, false><<<gq, 256, 0, s>>>(p);
    }
    return check_launch("attention_bwd");
   }
  }
  if (causal) {
    attn_bwd_dkdv_ring_kernel<D, true, KT, KNW, false, DR><<<grid, KNW * 64, 0, s>>>(p);
    attn_bwd_dq_kernel<D, true, QT, NW, DR><<<gq((const void*)attn_bwd_dq_kernel<D, true, QT, NW, DR>,
                                                 occ[0]), NW * 64, 0, s>>>(p);
  } else {
    attn_bwd_dkdv_ring_kernel<D, false, KT, KNW, false, DR><<<grid, KNW * 64, 0, s>>>(p);
    attn_bwd_dq_kernel<D, false, QT, NW, DR><<<gq((const void*)attn_bwd_dq_kernel<D, false, QT, NW, DR>,
                                                  occ[1]), NW * 64, 0, s>>>(p);
  }
  return check_launch("attention_bwd");
}

int validate(int64_t batch, int64_t seq, int64_t heads, int64_t head_dim, const void* qkv,
             int64_t ld, int64_t hs, int64_t ps) {
  MMPT_REQUIRE(batch > 0 && seq > 0 && heads > 0, "attention: empty problem");
  MMPT_REQUIRE(head_dim == 64 || head_dim == 256 || (head_dim % 16 == 0 && head_dim >= 80 &&
                                                      head_dim <= 128),
               "attention: head_dim %lld unsupported (64, 80-128 in steps of 16, 256)",
               (long long)head_dim);
  MMPT_REQUIRE(qkv != nullptr, "attention: null qkv");
  MMPT_REQUIRE(((uintptr_t)qkv & 15) == 0 && ld % 8 == 0 && hs % 8 == 0 && ps % 8 == 0,
               "attention: qkv must be 16-B aligned with strides multiple of 8");
  MMPT_REQUIRE(batch * seq < (1LL << 31), "attention: too many tokens");
  MMPT_REQUIRE(seq * ld * 2 < (1LL << 31), "attention: one sequence must span < 2 GiB (32-bit offsets)");
  return MMPT_OK;
}

// GQA geometry (G = heads / kv_heads query heads per kv head, k/v at their own offsets)
int set_kv(AttnParams& p, int64_t heads, int64_t kv_heads, int64_t k_off, int64_t v_off,
           int64_t kv_stride) {
  MMPT_REQUIRE(kv_heads > 0 && heads % kv_heads == 0, "attention: heads %% kv_heads != 0");
  MMPT_REQUIRE(k_off % 8 == 0 && v_off % 8 == 0 && kv_stride % 8 == 0 && k_off >= 0 && v_off >= 0,
               "attention: k/v offsets and stride must be non-negative multiples of 8");
  p.koff = k_off;
  p.voff = v_off;
  p.khs = kv_stride;
  p.Hkv = (int)kv_heads;
  p.G = (int)(heads / kv_heads);
  return MMPT_OK;
}

}  // namespace
}  // namespace mmpt

using namespace mmpt;

extern "C" int mmpt_attention_gqa_fwd(int64_t batch, int64_t seq, int64_t heads, int64_t kv_heads,
                                      int64_t head_dim, const void* qkv, int64_t ld,
                                      int64_t head_stride, int64_t k_offset, int64_t v_offset,
                                      int causal, float scale, void* out, int64_t ld_out,
                                      float* lse, void* stream) {
  int rc = validate(batch, seq, heads, head_dim, qkv, ld, head_stride, 0);
  if (rc) return rc;
  MMPT_REQUIRE(out && lse && ld_out % 8 == 0, "attention_fwd: bad out/lse");
  AttnParams p{};
  rc = set_kv(p, heads, kv_heads, k_offset, v_offset, head_stride);
  if (rc) return rc;
  p.qkv = (const bf16_t*)qkv;
  p.ld = ld;
  p.hs = head_stride;
  p.ps = 0;
  p.B = (int)batch;
  p.S = (int)seq;
  p.H = (int)heads;
  p.scale = scale;
  p.out = (bf16_t*)out;
  p.ld_out = ld_out;
  p.lse = lse;
  p.dr = (int)head_dim;
  hipStream_t s = (hipStream_t)stream;
  switch (head_dim) {
    case 64: return run_fwd<64>(p, causal, s);
    case 256: return run_fwd<256>(p, causal, s);
    case 80: if (attn_native80()) return run_fwd<128, 80>(p, causal, s);
      return run_fwd<128>(p, causal, s);
    default: return run_fwd<128>(p, causal, s);  // 96, 112: padded to 128
  }
}

extern "C" int64_t mmpt_attention_bwd_workspace_bytes(int64_t batch, int64_t seq, int64_t heads,
                                                      int64_t head_dim) {
  // δ (fp32 per query row), then at D = 256 the dS tiles: ceil(S/32)^2 tiles of 2 KiB per
  // (batch, head)
  if (head_dim != 256 || !attn_ds_mode()) return batch * seq * heads * (int64_t)sizeof(float);
  const int64_t nq = (seq + 31) / 32;
  return (int64_t)ds_offset(batch, seq, heads) + batch * heads * nq * nq * 2048;
}

extern "C" int mmpt_attention_gqa_bwd(int64_t batch, int64_t seq, int64_t heads, int64_t kv_heads,
                                      int64_t head_dim, const void* qkv, int64_t ld,
                                      int64_t head_stride, int64_t k_offset, int64_t v_offset,
                                      int causal, float scale, const void* out, const void* dout,
                                      int64_t ld_out, const float* lse, void* dqkv,
                                      void* workspace, void* stream) {
  int rc = validate(batch, seq, heads, head_dim, qkv, ld, head_stride, 0);
  if (rc) return rc;
  MMPT_REQUIRE(out && dout && lse && dqkv && workspace && ld_out % 8 == 0,
               "attention_bwd: null pointer");
  AttnParams p{};
  rc = set_kv(p, heads, kv_heads, k_offset, v_offset, head_stride);
  if (rc) return rc;
  p.qkv = (const bf16_t*)qkv;
  p.ld = ld;
  p.hs = head_stride;
  p.ps = 0;
  p.B = (int)batch;
  p.S = (int)seq;
  p.H = (int)heads;
  p.scale = scale;
  p.ld_out = ld_out;
  p.lse = (float*)lse;
  p.o = (const bf16_t*)out;
  p.dout = (const bf16_t*)dout;
  p.dqkv = (bf16_t*)dqkv;
  p.dr = (int)head_dim;
  p.ds = head_dim == 256 && attn_ds_mode()
             ? (bf16_t*)((char*)workspace + ds_offset(batch, seq, heads)) : nullptr;
  hipStream_t s = (hipStream_t)stream;
  switch (head_dim) {
    case 64: return run_bwd<64>(p, causal, (float*)workspace, s);
    case 256: return run_bwd<256>(p, causal, (float*)workspace, s);
    case 80: if (attn_native80()) return run_bwd<128, 80>(p, causal, (float*)workspace, s);
      return run_bwd<128>(p, causal, (float*)workspace, s);
    default: return run_bwd<128>(p, causal, (float*)workspace, s);  // 96, 112: padded
  }
}

// mmpt_attention_bwd followed by the rope backward of the q and k parts (mmpt_rope_inplace,
// inverse, parts = 2) — GPTNeoX's `apply_rotary_pos_emb` backward.  On the D = 256 wave-pair +
// dS-tile path with 64 rotary dims the dK / dQ epilogues rotate before they store (no second
// pass over dQKV); otherwise the rope kernel runs after the attention backward.
extern "C" int mmpt_rope_inplace(int64_t tokens, int64_t seq, int64_t heads, int64_t head_dim,
                                 int64_t rot_dims, void* qkv, int64_t ld, int64_t head_stride,
                                 int64_t part_stride, int64_t parts, const float* cos,
                                 const float* sin, int inverse, void* stream);
extern "C" int mmpt_attention_bwd_rope(int64_t batch, int64_t seq, int64_t heads, int64_t head_dim,
                                       const void* qkv, int64_t ld, int64_t head_stride,
                                       int64_t part_stride, int causal, float scale, const void* out,
                                       const void* dout, int64_t ld_out, const float* lse,
                                       void* dqkv, void* workspace, int64_t rot_dims,
                                       const float* cos, const float* sin, void* stream) {
  MMPT_REQUIRE(rot_dims > 0 && rot_dims % 2 == 0 && rot_dims <= head_dim && cos && sin,
               "attention_bwd_rope: bad rotary tables");
  const bool fused = head_dim == 256 && rot_dims == FUSED_ROT && attn_ds_mode() &&
                     attn_pair_mode() && ((uintptr_t)cos & 15) == 0 && ((uintptr_t)sin & 15) == 0;
  if (!fused) {
    int rc = mmpt_attention_gqa_bwd(batch, seq, heads, heads, head_dim, qkv, ld, head_stride,
                                    part_stride, 2 * part_stride, causal, scale, out, dout, ld_out,
                                    lse, dqkv, workspace, stream);
    if (rc) return rc;
    return mmpt_rope_inplace(batch * seq, seq, heads, head_dim, rot_dims, dqkv, ld, head_stride,
                             part_stride, 2, cos, sin, 1, stream);
  }
  int rc = validate(batch, seq, heads, head_dim, qkv, ld, head_stride, part_stride);
  if (rc) return rc;
  MMPT_REQUIRE(out && dout && lse && dqkv && workspace && ld_out % 8 == 0,
               "attention_bwd_rope: null pointer");
  AttnParams p{};
  rc = set_kv(p, heads, heads, part_stride, 2 * part_stride, head_stride);
  if (rc) return rc;
  p.qkv = (const bf16_t*)qkv;
  p.ld = ld;
  p.hs = head_stride;
  p.ps = part_stride;
  p.B = (int)batch;
  p.S = (int)seq;
  p.H = (int)heads;
  p.scale = scale;
  p.ld_out = ld_out;
  p.lse = (float*)lse;
  p.o = (const bf16_t*)out;
  p.dout = (const bf16_t*)dout;
  p.dqkv = (bf16_t*)dqkv;
  p.dr = (int)head_dim;
  p.ds = (bf16_t*)((char*)workspace + ds_offset(batch, seq, heads));
  p.rcos = cos;
  p.rsin = sin;
  p.rot = (int)rot_dims;
  return run_bwd<256>(p, causal, (float*)workspace, (hipStream_t)stream);
}

// The fused-qkv layouts of GPTNeoX (per-head interleaved q|k|v) and ViT/CLIP (planar) as
// the G = 1 case: k of head h at h*head_stride + part_stride, v at + 2*part_stride.
extern "C" int mmpt_attention_fwd(int64_t batch, int64_t seq, int64_t heads, int64_t head_dim,
                                  const void* qkv, int64_t ld, int64_t head_stride,
                                  int64_t part_stride, int causal, float scale, void* out,
                                  int64_t ld_out, float* lse, void* stream) {
  return mmpt_attention_gqa_fwd(batch, seq, heads, heads, head_dim, qkv, ld, head_stride,
                                part_stride, 2 * part_stride, causal, scale, out, ld_out, lse,
                                stream);
}

extern "C" int mmpt_attention_bwd(int64_t batch, int64_t seq, int64_t heads, int64_t head_dim,
                                  const void* qkv, int64_t ld, int64_t head_stride,
                                  int64_t part_stride, int causal, float scale, const void* out,
                                  const void* dout, int64_t ld_out, const float* lse, void* dqkv,
                                  void* workspace, void* stream) {
  return mmpt_attention_gqa_bwd(batch, seq, heads, heads, head_dim, qkv, ld, head_stride,
                                part_stride, 2 * part_stride, causal, scale, out, dout, ld_out,
                                lse, dqkv, workspace, stream);
}

// Test / measurement hook (include/mmpt.h): override a switch that is otherwise read once
// from the environment.  Returns the previous value, or MMPT_ERR_ARG for an unknown name.
extern "C" int mmpt_set_switch(const char* name, int value) {
  MMPT_REQUIRE(name != nullptr && value >= 0 && value <= 2, "set_switch: bad arguments");
  MMPT_REQUIRE(value < 2 || strcmp(name, "MMPT_GEMM_KREV") == 0 ||
                   strcmp(name, "MMPT_GEMM_WTAIL") == 0,
               "set_switch: %s takes 0 or 1", name);
  int* slot = nullptr;
  int prev = 0;
  if (strcmp(name, "MMPT_ATTN_PAIR") == 0) {
    prev = attn_pair_mode();
    slot = &g_attn_pair;
  } else if (strcmp(name, "MMPT_ATTN_DS") == 0) {
    prev = attn_ds_mode();
    slot = &g_attn_ds;
  } else if (strcmp(name, "MMPT_ATTN_NATIVE80") == 0) {
    prev = attn_native80();
    slot = &g_attn_native80;
  } else {
    slot = gemm_switch(name, &prev);
    if (slot == nullptr) slot = misc_switch(name, &prev);
  }
  MMPT_REQUIRE(slot != nullptr, "set_switch: unknown switch %s", name);
  *slot = value;
  return prev;
}
