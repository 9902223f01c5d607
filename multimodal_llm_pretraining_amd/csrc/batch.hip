// Per-micro-batch index bookkeeping on the device: the deterministic
// embedding backward needs the text rows grouped by token id, in position order inside
// each id.  Round 2 built that order with a host numpy argsort after a device->host copy
// of the ids (28 ms per 256 x 707 micro-batch plus a sync); here it is one stable LSD
// radix sort of (id, row) pairs (rocPRIM through hipCUB, the only library code on the
// path) and two hand-written kernels that turn the sorted ids into segments:
//
//   key[r]   = ids[r] in [0, vocab)  (rows with id == skip_id, the LLaVA image slots,
//              and any id outside the vocabulary get the sentinel key `vocab`, sorted last
//              and never part of a segment)
//   perm     = rows ordered by key, stable (position order inside a key)
//   seg_off[s], seg_id[s]: first sorted index and id of segment s;  seg_off[nseg] = the
//              number of text rows;  nseg lands in DEVICE memory, the embedding backward
//              reads it there — no host round trip on the step.
//   bad[0]   = 1 if any id lies outside [0, vocab) and is not skip_id, else 0 (device
//              flag: the host reads it lazily; the forward gather trusts its ids, so a
//              caller staging host data validates them on the host before the copy).
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace mmpt {
namespace {

__global__ __launch_bounds__(256) void seg_keys_kernel(int rows, const int64_t* __restrict__ ids,
                                                       int vocab, long skip_id,
                                                       int32_t* __restrict__ key,
                                                       int32_t* __restrict__ row,
                                                       int32_t* __restrict__ bad) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const long v = ids[r];
  const bool text = v != skip_id;
  const bool ok = v >= 0 && v < vocab;
  key[r] = (text && ok) ? (int32_t)v : vocab;
  row[r] = r;
  if (text && !ok) bad[0] = 1;  // benign race: every writer stores 1
}

// flag[i] = 1 where sorted index i starts a segment (a text key different from its left
// neighbour's); the inclusive scan of the flags numbers the segments from 1.
__global__ __launch_bounds__(256) void seg_flags_kernel(int rows, int vocab,
                                                        const int32_t* __restrict__ ks,
                                                        int32_t* __restrict__ flag) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= rows) return;
  const int k = ks[i];
  flag[i] = (k < vocab && (i == 0 || ks[i - 1] != k)) ? 1 : 0;
}

__global__ __launch_bounds__(256) void seg_write_kernel(int rows, int vocab,
                                                        const int32_t* __restrict__ ks,
                                                        const int32_t* __restrict__ flag,
                                                        const int32_t* __restrict__ pos,
                                                        int32_t* __restrict__ seg_id,
                                                        int32_t* __restrict__ seg_off,
                                                        int32_t* __restrict__ nseg) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= rows) return;
  const int k = ks[i];
  if (k >= vocab) {
    if (i == 0) nseg[0] = 0;  // no text rows at all: the only writer of nseg
    return;
  }
  if (flag[i]) {
    seg_off[pos[i] - 1] = i;
    seg_id[pos[i] - 1] = k;
  }
  if (i + 1 == rows || ks[i + 1] >= vocab) {  // the last text row: exactly one thread
    seg_off[pos[i]] = i + 1;
    nseg[0] = pos[i];
  }
}

// Workspace: keys in / out, rows in, flags, scan, then hipCUB's temporary
// storage (the larger of the sort's and the scan's), every part 256-B aligned.
struct SegWs {
  size_t key_in, key_out, row_in, flag, pos, tmp, tmp_bytes, total;
};
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
int seg_bits(long vocab) {
  int b = 1;
  while ((1L << b) <= vocab) ++b;  // keys in [0, vocab]: the sentinel included
  return b;
}
int seg_layout(long rows, long vocab, SegWs* w) {
  const size_t n4 = align256((size_t)rows * 4);
  w->key_in = 0;
  w->key_out = w->key_in + n4;
  w->row_in = w->key_out + n4;
  w->flag = w->row_in + n4;
  w->pos = w->flag + n4;
  w->tmp = w->pos + n4;
  size_t sort_b = 0, scan_b = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (const int32_t*)nullptr,
                                                    (int32_t*)nullptr, (const int32_t*)nullptr,
                                                    (int32_t*)nullptr, (int)rows, 0,
                                                    seg_bits(vocab));
  if (e != hipSuccess) return (int)e;
  e = hipcub::DeviceScan::InclusiveSum(nullptr, scan_b, (const int32_t*)nullptr,
                                       (int32_t*)nullptr, (int)rows);
  if (e != hipSuccess) return (int)e;
  w->tmp_bytes = align256(sort_b > scan_b ? sort_b : scan_b);
  w->total = w->tmp + w->tmp_bytes;
  return MMPT_OK;
}

}  // namespace
}  // namespace mmpt

using namespace mmpt;

extern "C" int64_t mmpt_embed_segments_workspace_bytes(int64_t rows, int64_t vocab) {
  if (rows <= 0 || vocab <= 0 || vocab >= (1L << 30) || rows >= (1L << 30)) return -1;
  SegWs w;
  if (seg_layout(rows, vocab, &w) != MMPT_OK) return -1;
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
  int rc = seg_layout(rows, vocab, &w);
  if (rc) {
    set_error("embed_segments: hipCUB size query failed");
    return rc;
  }
  MMPT_REQUIRE(ws_bytes >= (int64_t)w.total, "embed_segments: workspace %lld < %lld bytes",
               (long long)ws_bytes, (long long)w.total);
  hipStream_t s = (hipStream_t)stream;
  char* base = (char*)workspace;
  int32_t* key_in = (int32_t*)(base + w.key_in);
  int32_t* key_out = (int32_t*)(base + w.key_out);
  int32_t* row_in = (int32_t*)(base + w.row_in);
  int32_t* flag = (int32_t*)(base + w.flag);
  int32_t* pos = (int32_t*)(base + w.pos);
  const unsigned grid = (unsigned)((rows + 255) / 256);
  hipError_t e = hipMemsetAsync(bad, 0, sizeof(int32_t), s);
  if (e != hipSuccess) {
    set_error("embed_segments: memset: %s", hipGetErrorString(e));
    return (int)e;
  }
  seg_keys_kernel<<<grid, 256, 0, s>>>((int)rows, ids, (int)vocab, (long)skip_id, key_in, row_in,
                                       bad);
  if ((rc = check_launch("embed_segments keys"))) return rc;
  size_t tb = w.tmp_bytes;
  e = hipcub::DeviceRadixSort::SortPairs(base + w.tmp, tb, key_in, key_out, row_in,
                                                    perm, (int)rows, 0, seg_bits(vocab), s);
  if (e != hipSuccess) {
    set_error("embed_segments: radix sort: %s", hipGetErrorString(e));
    return (int)e;
  }
  seg_flags_kernel<<<grid, 256, 0, s>>>((int)rows, (int)vocab, key_out, flag);
  if ((rc = check_launch("embed_segments flags"))) return rc;
  tb = w.tmp_bytes;
  e = hipcub::DeviceScan::InclusiveSum(base + w.tmp, tb, flag, pos, (int)rows, s);
  if (e != hipSuccess) {
    set_error("embed_segments: scan: %s", hipGetErrorString(e));
    return (int)e;
  }
  seg_write_kernel<<<grid, 256, 0, s>>>((int)rows, (int)vocab, key_out, flag, pos, seg_id,
                                        seg_off, nseg);
  return check_launch("embed_segments write");
}
