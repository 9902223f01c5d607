// Per-micro-batch index bookkeeping on the device: the deterministic
// embedding backward needs the text rows grouped by token id, in position order inside
// each id.  Round 2 built that order with a host numpy argsort after a device->host copy
// of the ids (28 ms per 256 x 707 micro-batch plus a sync); round 3 with a library radix
// sort.  Round 4: a hand-written stable counting sort over the vocabulary — the key space
// is small (50,304 / 128,264 ids) and dense, so one histogram, one scan and one scatter
// replace the 3-4 radix passes over 2·rows keys:
//
//   key[r]   = ids[r] in [0, vocab)  (rows with id == skip_id, the LLaVA image slots,
//              and any id outside the vocabulary get the sentinel key `vocab` and take
//              no part)
//   perm     = text rows ordered by key, stable (position order inside a key)
//   seg_off[s], seg_id[s]: first sorted index and id of segment s;  seg_off[nseg] = the
//              number of text rows;  nseg lands in DEVICE memory, the embedding backward
//              reads it there — no host round trip on the step.
//   bad[0]   = 1 if any id lies outside [0, vocab) and is not skip_id, else 0 (device
//              flag: the forward gather trusts its ids, so a caller validates them before
//              the step — engine.Batch does, for host and device inputs alike).
//
// Kernels (HBM-bound, a few µs each at 256 x 707 rows):
//   1. seg_count:   key[r]; cnt[key] += 1 (integer atomics: the counts do not depend on
//                   the order of the adds).
//   2. seg_tot / seg_scan: 4096 ids per workgroup — the blocks' row and non-empty-id totals,
//                   then each block's scan on top of the totals before it: cur[k] = start of
//                   id k, seg_id / seg_off of every non-empty id, nseg, seg_off[nseg].
//   3. seg_scatter: tmp[atomicAdd(cur[key], 1)] = r — every row lands in its id's slot
//                   range, in an order that varies from run to run.
//   4. seg_rank:    the order inside a slot range is fixed by the row numbers: slot p of id
//                   k holds row r; its stable position is start_k + #{rows of id k < r}, a
//                   count over the id's own range only (uniform ids: ≈3.6 rows per id at
//                   C3).  perm[start_k + rank] = r — deterministic, bitwise the stable sort.
#include "common.h"

namespace mmpt {
namespace {

constexpr int SCAN_KEYS = 16;                 // ids per thread in the scan kernels
constexpr int SCAN_BLOCK = 256 * SCAN_KEYS;   // ids per scan workgroup

__global__ __launch_bounds__(256) void seg_count_kernel(int rows, const int64_t* __restrict__ ids,
                                                        int vocab, long skip_id,
                                                        int32_t* __restrict__ key,
                                                        int32_t* __restrict__ cnt,
                                                        int32_t* __restrict__ bad) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const long v = ids[r];
  const bool text = v != skip_id;
  const bool ok = v >= 0 && v < vocab;
  const int k = (text && ok) ? (int)v : vocab;
  key[r] = k;
  if (k < vocab) atomicAdd(&cnt[k], 1);
  if (text && !ok) bad[0] = 1;  // benign race: every writer stores 1
}

// Inclusive scan of one int per thread over a 256-thread block (4 waves): wave prefix by
// shuffles, the 4 wave totals through LDS.  *total = the block's sum.
__device__ __forceinline__ int block_scan256(int x, int* lds, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) lds[wave] = x;
  __syncthreads();
  int before = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) before += w < wave ? lds[w] : 0;
  *total = lds[0] + lds[1] + lds[2] + lds[3];
  __syncthreads();  // lds reused by the next call
  return x + before;
}

// Pass 1: per scan block, the number of text rows and of non-empty ids.
__global__ __launch_bounds__(256) void seg_tot_kernel(int vocab, const int32_t* __restrict__ cnt,
                                                      int32_t* __restrict__ tot) {
  __shared__ int lds[4];
  const int k0 = blockIdx.x * SCAN_BLOCK + threadIdx.x * SCAN_KEYS;
  int off = 0, seg = 0;
#pragma unroll
  for (int i = 0; i < SCAN_KEYS; ++i) {
    const int c = k0 + i < vocab ? cnt[k0 + i] : 0;
    off += c;
    seg += c > 0;
  }
  int t_off, t_seg;
  block_scan256(off, lds, &t_off);
  block_scan256(seg, lds, &t_seg);
  if (threadIdx.x == 0) {
    tot[2 * blockIdx.x] = t_off;
    tot[2 * blockIdx.x + 1] = t_seg;
  }
}

// Pass 2: each block adds the totals of the blocks before it, scans its ids: cur[k] = start of
// id k, seg_id / seg_off of every non-empty id; the last block writes nseg and seg_off[nseg].
__global__ __launch_bounds__(256) void seg_scan_kernel(int vocab, const int32_t* __restrict__ cnt,
                                                       const int32_t* __restrict__ tot,
                                                       int32_t* __restrict__ cur,
                                                       int32_t* __restrict__ seg_id,
                                                       int32_t* __restrict__ seg_off,
                                                       int32_t* __restrict__ nseg) {
  __shared__ int lds[4];
  int p_off = 0, p_seg = 0;
  for (int b = threadIdx.x; b < (int)blockIdx.x; b += 256) {
    p_off += tot[2 * b];
    p_seg += tot[2 * b + 1];
  }
  int base_off, base_seg;
  block_scan256(p_off, lds, &base_off);
  block_scan256(p_seg, lds, &base_seg);
  const int k0 = blockIdx.x * SCAN_BLOCK + threadIdx.x * SCAN_KEYS;
  int c[SCAN_KEYS];
  int my_off = 0, my_seg = 0;
#pragma unroll
  for (int i = 0; i < SCAN_KEYS; ++i) {
    c[i] = k0 + i < vocab ? cnt[k0 + i] : 0;
    my_off += c[i];
    my_seg += c[i] > 0;
  }
  int t_off, t_seg;
  int o = base_off + block_scan256(my_off, lds, &t_off) - my_off;
  int sg = base_seg + block_scan256(my_seg, lds, &t_seg) - my_seg;
#pragma unroll
  for (int i = 0; i < SCAN_KEYS; ++i) {
    if (k0 + i < vocab) {
      cur[k0 + i] = o;
      if (c[i] > 0) {
        seg_id[sg] = k0 + i;
        seg_off[sg] = o;
        ++sg;
      }
    }
    o += c[i];
  }
  if (blockIdx.x + 1 == gridDim.x && threadIdx.x == 0) {
    seg_off[base_seg + t_seg] = base_off + t_off;  // the number of text rows
    nseg[0] = base_seg + t_seg;
  }
}

__global__ __launch_bounds__(256) void seg_scatter_kernel(int rows, int vocab,
                                                          const int32_t* __restrict__ key,
                                                          int32_t* __restrict__ cur,
                                                          int32_t* __restrict__ tmp) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const int k = key[r];
  if (k < vocab) tmp[atomicAdd(&cur[k], 1)] = r;
}

// After the scatter cur[k] = end of id k's range and start = end - cnt[k].  One thread per
// text row; the count loop runs over the row's own id range (broadcast loads when a wave's
// rows share an id).
__global__ __launch_bounds__(256) void seg_rank_kernel(int rows, int vocab,
                                                       const int32_t* __restrict__ key,
                                                       const int32_t* __restrict__ cnt,
                                                       const int32_t* __restrict__ cur,
                                                       const int32_t* __restrict__ tmp,
                                                       int32_t* __restrict__ perm) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const int k = key[r];
  if (k >= vocab) return;
  const int end = cur[k], start = end - cnt[k];
  int rank = 0;
  for (int j = start; j < end; ++j) rank += tmp[j] < r;
  perm[start + rank] = r;
}

// Workspace: key, tmp [rows]; cnt, cur [vocab]; tot [2 x scan blocks]; every part 256-B aligned.
struct SegWs {
  size_t key, tmp, cnt, cur, tot, total;
};
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
void seg_layout(long rows, long vocab, SegWs* w) {
  const size_t n4 = align256((size_t)rows * 4), v4 = align256((size_t)vocab * 4);
  w->key = 0;
  w->tmp = w->key + n4;
  w->cnt = w->tmp + n4;
  w->cur = w->cnt + v4;
  w->tot = w->cur + v4;
  w->total = w->tot + align256((size_t)((vocab + SCAN_BLOCK - 1) / SCAN_BLOCK) * 8);
}

}  // namespace
}  // namespace mmpt

using namespace mmpt;

extern "C" int64_t mmpt_embed_segments_workspace_bytes(int64_t rows, int64_t vocab) {
  if (rows <= 0 || vocab <= 0 || vocab >= (1L << 30) || rows >= (1L << 30)) return -1;
  SegWs w;
  seg_layout(rows, vocab, &w);
  return (int64_t)w.total;
}

extern "C" int mmpt_embed_segments(int64_t rows, const int64_t* ids, int64_t vocab,
                                   int64_t skip_id, int32_t* seg_id, int32_t* seg_off,
                                   int32_t* perm, int32_t* nseg, int32_t* bad, void* workspace,
                                   int64_t ws_bytes, void* stream) {
  MMPT_REQUIRE(rows > 0 && rows < (1L << 30) && vocab > 0 && vocab < (1L << 30),
               "embed_segments: bad sizes");
  MMPT_REQUIRE(ids && seg_id && seg_off && perm && nseg && bad && workspace,
               "embed_segments: null pointer");
  SegWs w;
  seg_layout(rows, vocab, &w);
  MMPT_REQUIRE(ws_bytes >= (int64_t)w.total, "embed_segments: workspace %lld < %lld bytes",
               (long long)ws_bytes, (long long)w.total);
  hipStream_t s = (hipStream_t)stream;
  char* base = (char*)workspace;
  int32_t* key = (int32_t*)(base + w.key);
  int32_t* tmp = (int32_t*)(base + w.tmp);
  int32_t* cnt = (int32_t*)(base + w.cnt);
  int32_t* cur = (int32_t*)(base + w.cur);
  int32_t* tot = (int32_t*)(base + w.tot);
  const unsigned nb = (unsigned)((vocab + SCAN_BLOCK - 1) / SCAN_BLOCK);
  const unsigned grid = (unsigned)((rows + 255) / 256);
  hipError_t e = hipMemsetAsync(bad, 0, sizeof(int32_t), s);
  if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, (size_t)vocab * 4, s);
  if (e != hipSuccess) {
    set_error("embed_segments: memset: %s", hipGetErrorString(e));
    return (int)e;
  }
  int rc;
  seg_count_kernel<<<grid, 256, 0, s>>>((int)rows, ids, (int)vocab, (long)skip_id, key, cnt, bad);
  if ((rc = check_launch("embed_segments count"))) return rc;
  seg_tot_kernel<<<nb, 256, 0, s>>>((int)vocab, cnt, tot);
  if ((rc = check_launch("embed_segments totals"))) return rc;
  seg_scan_kernel<<<nb, 256, 0, s>>>((int)vocab, cnt, tot, cur, seg_id, seg_off, nseg);
  if ((rc = check_launch("embed_segments scan"))) return rc;
  seg_scatter_kernel<<<grid, 256, 0, s>>>((int)rows, (int)vocab, key, cur, tmp);
  if ((rc = check_launch("embed_segments scatter"))) return rc;
  seg_rank_kernel<<<grid, 256, 0, s>>>((int)rows, (int)vocab, key, cnt, cur, tmp, perm);
  return check_launch("embed_segments rank");
}
