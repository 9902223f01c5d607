// ZeRO++ quantized communication for `sharding = "zero_3++"` (src/train.py:196-201:
// DeepSpeed `zero_quantized_weights` + `zero_quantized_gradients`; SURVEY.md §2.3 row
// ZeRO-3++, §8(f)4): blockwise symmetric quantization around the RCCL collectives of the
// ZeRO-3 exchange (zero3.py).
//
//   qwZ  weights: each rank's bf16 shard -> int8 + one fp32 scale per 256-element block
//        (scale = absmax / 127, q = rint(x · 127 / absmax)) -> all-gather of the int8 bytes and
//        scales -> dequantized into the bf16 gather window (x' = bf16(q · scale)).
//   qgZ  gradients: the unit's fp32 gradient window, cut into the world destination shards,
//        -> int4 + fp32 scale per 256-element block (scale = absmax / 7, q in [-7, 7], two
//        per byte, low nibble first) -> all-to-all -> each rank sums the world dequantized
//        copies of its shard in rank order (fp32) into its gradient shard.
//
// Every kernel: one 64-lane wave per block, 4 elements per lane, blocks never straddle a
// part (a rank's shard), the last block of a part may be partial (parts are multiples of
// 4 elements).  HBM-bound byte work: 2 B in + 1 B out per weight, 4 B in + 0.5 B out per
// gradient element.
#include "common.h"

namespace mmpt {
namespace {

constexpr int QB = 256;  // elements per quantization block

__device__ __forceinline__ float wave_absmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

struct BlockPos {
  long base;  // first element of the block
  int len;    // valid elements (<= QB)
  long sidx;  // scale index
};
__device__ __forceinline__ BlockPos block_pos(long blk, long n_part, long nb) {
  const long part = blk / nb, j = blk % nb;
  const long lo = j * QB;
  return {part * n_part + lo, (int)min((long)QB, n_part - lo), blk};
}

__global__ __launch_bounds__(256) void quant_int8_kernel(long n_part, long nblk, long nb,
                                                         const bf16_t* __restrict__ src,
                                                         int8_t* __restrict__ dst,
                                                         float* __restrict__ scales) {
  const long blk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= nblk) return;  // (wave-uniform)
  const int lane = threadIdx.x & 63;
  const BlockPos bp = block_pos(blk, n_part, nb);
  const int e0 = lane * 4;
  float x[4] = {0.f, 0.f, 0.f, 0.f};
  if (e0 < bp.len) {
    const uint2 u = *(const uint2*)(src + bp.base + e0);
    x[0] = bf2f(u.x & 0xffff);
    x[1] = bf2f(u.x >> 16);
    x[2] = bf2f(u.y & 0xffff);
    x[3] = bf2f(u.y >> 16);
  }
  float m = fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3])));
  m = wave_absmax(m);
  const float inv = m > 0.f ? 127.0f / m : 0.f;
  if (e0 < bp.len) {
    uint32_t w = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = (int)fminf(fmaxf(rintf(x[e] * inv), -127.f), 127.f);
      w |= (uint32_t)(q & 0xff) << (8 * e);
    }
    *(uint32_t*)(dst + bp.base + e0) = w;
  }
  if (lane == 0) scales[bp.sidx] = m / 127.0f;
}

__global__ __launch_bounds__(256) void dequant_int8_kernel(long n_part, long nblk, long nb,
                                                           const int8_t* __restrict__ src,
                                                           const float* __restrict__ scales,
                                                           bf16_t* __restrict__ dst) {
  const long blk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= nblk) return;
  const int lane = threadIdx.x & 63;
  const BlockPos bp = block_pos(blk, n_part, nb);
  const int e0 = lane * 4;
  if (e0 >= bp.len) return;
  const float s = scales[bp.sidx];
  const uint32_t w = *(const uint32_t*)(src + bp.base + e0);
  float y[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) y[e] = (float)(int8_t)((w >> (8 * e)) & 0xff) * s;
  uint2 u;
  u.x = (uint32_t)f2bf(y[0]) | ((uint32_t)f2bf(y[1]) << 16);
  u.y = (uint32_t)f2bf(y[2]) | ((uint32_t)f2bf(y[3]) << 16);
  *(uint2*)(dst + bp.base + e0) = u;
}

__global__ __launch_bounds__(256) void quant_int4_kernel(long n_part, long nblk, long nb,
                                                         const float* __restrict__ src,
                                                         uint8_t* __restrict__ dst,
                                                         float* __restrict__ scales) {
  const long blk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= nblk) return;
  const int lane = threadIdx.x & 63;
  const BlockPos bp = block_pos(blk, n_part, nb);
  const int e0 = lane * 4;
  float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e0 < bp.len) x = *(const float4*)(src + bp.base + e0);
  float m = fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
  m = wave_absmax(m);
  const float inv = m > 0.f ? 7.0f / m : 0.f;
  if (e0 < bp.len) {
    const float v[4] = {x.x, x.y, x.z, x.w};
    uint32_t w = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = (int)fminf(fmaxf(rintf(v[e] * inv), -7.f), 7.f);
      w |= (uint32_t)(q & 0xf) << (4 * e);
    }
    *(uint16_t*)(dst + (bp.base + e0) / 2) = (uint16_t)w;
  }
  if (lane == 0) scales[bp.sidx] = m / 7.0f;
}

// dst[i] += Σ_{r < parts} q_r[i] · scale_r[block(i)]  (rank order, fp32)
__global__ __launch_bounds__(256) void dequant_int4_sum_kernel(long n_part, long nb, int parts,
                                                               const uint8_t* __restrict__ src,
                                                               const float* __restrict__ scales,
                                                               float* __restrict__ dst) {
  const long blk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= nb) return;
  const int lane = threadIdx.x & 63;
  const BlockPos bp = block_pos(blk, n_part, nb);  // part 0 geometry
  const int e0 = lane * 4;
  if (e0 >= bp.len) return;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < parts; ++r) {
    const float s = scales[(long)r * nb + blk];
    const uint32_t w = *(const uint16_t*)(src + ((long)r * n_part + bp.base + e0) / 2);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = (int)((w >> (4 * e)) & 0xf);
      acc[e] += (float)(q >= 8 ? q - 16 : q) * s;
    }
  }
  float4* o = (float4*)(dst + bp.base + e0);
  float4 v = *o;
  v.x += acc[0];
  v.y += acc[1];
  v.z += acc[2];
  v.w += acc[3];
  *o = v;
}

int launch_check(const char* what) { return check_launch(what); }

unsigned grid_for(long nblk) { return (unsigned)((nblk + 3) / 4); }

}  // namespace
}  // namespace mmpt

using namespace mmpt;

extern "C" int64_t mmpt_quant_blocks(int64_t n_part) { return (n_part + QB - 1) / QB; }

extern "C" int mmpt_quant_int8(int64_t n_part, int64_t parts, const void* src_bf16, void* dst_i8,
                               float* scales, void* stream) {
  MMPT_REQUIRE(n_part > 0 && parts > 0 && n_part % 4 == 0, "quant_int8: n_part must be a positive multiple of 4");
  MMPT_REQUIRE(src_bf16 && dst_i8 && scales, "quant_int8: null pointer");
  MMPT_REQUIRE(((uintptr_t)src_bf16 & 7) == 0 && ((uintptr_t)dst_i8 & 3) == 0, "quant_int8: misaligned");
  const long nb = mmpt_quant_blocks(n_part), nblk = nb * parts;
  quant_int8_kernel<<<grid_for(nblk), 256, 0, (hipStream_t)stream>>>(
      n_part, nblk, nb, (const bf16_t*)src_bf16, (int8_t*)dst_i8, scales);
  return launch_check("quant_int8");
}

extern "C" int mmpt_dequant_int8(int64_t n_part, int64_t parts, const void* src_i8, const float* scales,
                                 void* dst_bf16, void* stream) {
  MMPT_REQUIRE(n_part > 0 && parts > 0 && n_part % 4 == 0, "dequant_int8: n_part must be a positive multiple of 4");
  MMPT_REQUIRE(src_i8 && scales && dst_bf16, "dequant_int8: null pointer");
  MMPT_REQUIRE(((uintptr_t)dst_bf16 & 7) == 0 && ((uintptr_t)src_i8 & 3) == 0, "dequant_int8: misaligned");
  const long nb = mmpt_quant_blocks(n_part), nblk = nb * parts;
  dequant_int8_kernel<<<grid_for(nblk), 256, 0, (hipStream_t)stream>>>(
      n_part, nblk, nb, (const int8_t*)src_i8, scales, (bf16_t*)dst_bf16);
  return launch_check("dequant_int8");
}

extern "C" int mmpt_quant_int4(int64_t n_part, int64_t parts, const float* src, void* dst_u8,
                               float* scales, void* stream) {
  MMPT_REQUIRE(n_part > 0 && parts > 0 && n_part % 4 == 0, "quant_int4: n_part must be a positive multiple of 4");
  MMPT_REQUIRE(src && dst_u8 && scales, "quant_int4: null pointer");
  MMPT_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst_u8 & 1) == 0, "quant_int4: misaligned");
  const long nb = mmpt_quant_blocks(n_part), nblk = nb * parts;
  quant_int4_kernel<<<grid_for(nblk), 256, 0, (hipStream_t)stream>>>(
      n_part, nblk, nb, src, (uint8_t*)dst_u8, scales);
  return launch_check("quant_int4");
}

extern "C" int mmpt_dequant_int4_sum(int64_t n_part, int64_t parts, const void* src_u8,
                                     const float* scales, float* dst, void* stream) {
  MMPT_REQUIRE(n_part > 0 && parts > 0 && n_part % 4 == 0, "dequant_int4_sum: n_part must be a positive multiple of 4");
  MMPT_REQUIRE(src_u8 && scales && dst, "dequant_int4_sum: null pointer");
  MMPT_REQUIRE(((uintptr_t)dst & 15) == 0 && ((uintptr_t)src_u8 & 1) == 0, "dequant_int4_sum: misaligned");
  const long nb = mmpt_quant_blocks(n_part);
  dequant_int4_sum_kernel<<<grid_for(nb), 256, 0, (hipStream_t)stream>>>(
      n_part, nb, (int)parts, (const uint8_t*)src_u8, scales, dst);
  return launch_check("dequant_int4_sum");
}
