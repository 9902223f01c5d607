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
//   2. seg_scan:    ONE workgroup scans cnt[0..vocab) in tiles of 4096 (offsets and the
//                   number of non-empty ids, carried across tiles): cur[k] = start of id k,
//                   seg_id / seg_off of every non-empty id, nseg, seg_off[nseg].
//   3. seg_scatter: tmp[atomicAdd(cur[key], 1)] = r — every row lands in its id's slot
//                   range, in an order that varies from run to run.
//   4. seg_rank:    the order inside a slot range is fixed by the row numbers: slot p of id
//                   k holds row r; its stable position is start_k + #{rows of id k < r}, a
//                   count over the id's own range only (uniform ids: ≈3.6 rows per id at
//                   C3).  perm[start_k + rank] = r — deterministic, bitwise the stable sort.
#include "common.h"

namespace mmpt {
namespace {

constexpr int SCAN_THREADS = 1024;
constexpr int SCAN_TILE = SCAN_THREADS * 4;

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

// Inclusive block scan of one int per thread (1024 threads = 16 waves): wave prefix by
// DPP-free shuffles, wave totals through LDS.  Returns the inclusive prefix; *total = the
// block's sum.
__device__ __forceinline__ int block_scan_incl(int x, int* lds, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) lds[wave] = x;
  __syncthreads();
  if (wave == 0) {
    int w = lane < SCAN_THREADS / 64 ? lds[lane] : 0;
#pragma unroll
    for (int d = 1; d < SCAN_THREADS / 64; d <<= 1) {
      const int y = __shfl_up(w, d, 64);
      if (lane >= d) w += y;
    }
    if (lane < SCAN_THREADS / 64) lds[16 + lane] = w;  // inclusive wave-total prefix
  }
  __syncthreads();
  const int before = wave > 0 ? lds[16 + wave - 1] : 0;
  *total = lds[16 + SCAN_THREADS / 64 - 1];
  __syncthreads();  // lds reused by the next call
  return x + before;
}

__global__ __launch_bounds__(SCAN_THREADS) void seg_scan_kernel(int vocab,
                                                                const int32_t* __restrict__ cnt,
                                                                int32_t* __restrict__ cur,
                                                                int32_t* __restrict__ seg_id,
                                                                int32_t* __restrict__ seg_off,
                                                                int32_t* __restrict__ nseg) {
  __shared__ int lds[64];
  int off_carry = 0, seg_carry = 0;
  for (int base = 0; base < vocab; base += SCAN_TILE) {
    const int k0 = base + threadIdx.x * 4;
    int c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = k0 + i < vocab ? cnt[k0 + i] : 0;
    const int my_off = c[0] + c[1] + c[2] + c[3];
    const int my_seg = (c[0] > 0) + (c[1] > 0) + (c[2] > 0) + (c[3] > 0);
    int t_off, t_seg;
    const int inc_off = block_scan_incl(my_off, lds, &t_off);
    const int inc_seg = block_scan_incl(my_seg, lds, &t_seg);
    int o = off_carry + inc_off - my_off, sg = seg_carry + inc_seg - my_seg;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
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
    off_carry += t_off;
    seg_carry += t_seg;
  }
  if (threadIdx.x == 0) {
    seg_off[seg_carry] = off_carry;  // the number of text rows
    nseg[0] = seg_carry;
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

// Workspace: key, tmp [rows]; cnt, cur [vocab]; every part 256-B aligned.
struct SegWs {
  size_t key, tmp, cnt, cur, total;
};
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
void seg_layout(long rows, long vocab, SegWs* w) {
  const size_t n4 = align256((size_t)rows * 4), v4 = align256((size_t)vocab * 4);
  w->key = 0;
  w->tmp = w->key + n4;
  w->cnt = w->tmp + n4;
  w->cur = w->cnt + v4;
  w->total = w->cur + v4;
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
  seg_scan_kernel<<<1, SCAN_THREADS, 0, s>>>((int)vocab, cnt, cur, seg_id, seg_off, nseg);
  if ((rc = check_launch("embed_segments scan"))) return rc;
  seg_scatter_kernel<<<grid, 256, 0, s>>>((int)rows, (int)vocab, key, cur, tmp);
  if ((rc = check_launch("embed_segments scatter"))) return rc;
  seg_rank_kernel<<<grid, 256, 0, s>>>((int)rows, (int)vocab, key, cnt, cur, tmp, perm);
  return check_launch("embed_segments rank");
}
