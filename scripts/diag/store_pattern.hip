// Store-throughput probe for the GEMM epilogue (diagnostic, not product code).
// Each workgroup (512 threads, 8 waves) writes NT 256x256 bf16 tiles to its own region, 16-B
// vector stores, no other work.  Patterns (per store instruction of one wave):
//   0: 16 rows x 64 B   (gemm256's epilogue: lane = row (lane&15), 4 column groups)
//   1:  8 rows x 128 B
//   2:  4 rows x 256 B
//   3:  1 row  x 1 KiB  (whole contiguous KiB)
// Reports GB/s chip-wide and B/clk per active CU (at the given clock) for a grid of G WGs.
// Build: hipcc -O3 --offload-arch=gfx950 store_pattern.hip -o store_pattern
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int PAT, bool LOAD = false>
__global__ __launch_bounds__(512, 1) void store_tiles(uint4* out, int nt, long ld_u4) {
  __shared__ char sm[96 * 1024];  // one workgroup per CU
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (nt < 0) {  // never: keeps the LDS allocation
    sm[tid] = (char)tid;
    __syncthreads();
    out[tid].x = sm[tid ^ 1];
  }
  const int wm = wave >> 2, wn = wave & 3;
  const uint4 v = {(unsigned)tid, 1u, 2u, 3u};
  uint4 accx = {0u, 0u, 0u, 0u};
  // a 32768 x 8192 bf16 matrix (row stride ld_u4 = 1024 uint4) cut into 256x256 tiles,
  // 32 per tile row; this WG writes tiles blockIdx.x*nt .. +nt-1 (as the GEMM's C)
  for (int t = 0; t < nt; ++t) {
    const int id = blockIdx.x * nt + t;
    uint4* tile = out + (long)(id >> 5) * 256 * ld_u4 + (id & 31) * 32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int row, col;  // col in uint4 units (8 bf16)
      if (PAT == 0) {
        const int nh = r >> 3, mh = (r >> 2) & 1, i = r & 3, g = lane >> 4;
        row = mh * 128 + wm * 64 + i * 16 + (lane & 15);
        col = nh * 16 + wn * 4 + (g & 1) * 2 + (g >> 1);
      } else if (PAT == 1) {  // 8 rows x 8 uint4
        const int blk = wave * 16 + r;  // 128 blocks of 8 rows x 64 cols... cover 256x256
        row = (blk >> 2) * 8 + (lane >> 3);
        col = (blk & 3) * 8 + (lane & 7);
      } else if (PAT == 2) {  // 4 rows x 16 uint4
        const int blk = wave * 16 + r;  // 128 blocks of 4 rows x 128 cols
        row = (blk >> 1) * 4 + (lane >> 4);
        col = (blk & 1) * 16 + (lane & 15);
      } else {  // 1 row x 64 uint4 (two rows' worth when a row is 32 uint4)
        const int blk = wave * 16 + r;  // 128 blocks of 2 rows x 256 cols
        row = blk * 2 + (lane >> 5);
        col = lane & 31;
      }
      if constexpr (LOAD) {
        const uint4 x = tile[(long)row * ld_u4 + col];
        accx.x ^= x.x; accx.y ^= x.y; accx.z ^= x.z; accx.w ^= x.w;
      } else {
        tile[(long)row * ld_u4 + col] = v;
      }
    }
  }
  if constexpr (LOAD) {
    if ((accx.x ^ accx.y ^ accx.z ^ accx.w) == 0x9e3779b9u) out[tid] = accx;  // keeps the loads
  }
}

template <int PAT, bool LOAD = false>
float run(uint4* buf, int grid, int nt, long ld_u4, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  store_tiles<PAT, LOAD><<<grid, 512>>>(buf, nt, ld_u4);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) store_tiles<PAT, LOAD><<<grid, 512>>>(buf, nt, ld_u4);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char** argv) {
  const double ghz = argc > 1 ? atof(argv[1]) : 2.1;
  const int nt = 16, iters = 20;
  const long ld_u4 = 1024;  // rows of 8192 bf16
  const int grids[] = {256, 128, 64, 32, 8};
  const size_t bytes = (size_t)256 * nt * 256 * 256 * 2;  // 256 WGs x nt tiles x 128 KiB
  uint4* buf;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 0, bytes));
  for (int gi = 0; gi < 5; ++gi) {
    const int G = grids[gi];
    const double wg_bytes = (double)nt * 256 * 256 * 2, tot = wg_bytes * G;
    float ms[4] = {run<0>(buf, G, nt, ld_u4, iters), run<1>(buf, G, nt, ld_u4, iters),
                   run<2>(buf, G, nt, ld_u4, iters), run<3>(buf, G, nt, ld_u4, iters)};
    float ml[4] = {run<0, true>(buf, G, nt, ld_u4, iters), run<1, true>(buf, G, nt, ld_u4, iters),
                   run<2, true>(buf, G, nt, ld_u4, iters), run<3, true>(buf, G, nt, ld_u4, iters)};
    for (int p = 0; p < 8; ++p) {
      const float t = p < 4 ? ms[p] : ml[p - 4];
      const double s = t * 1e-3;
      printf("{\"grid\": %d, \"op\": \"%s\", \"pattern\": %d, \"us\": %.1f, \"GBps\": %.0f, \"B_per_clk_per_CU\": %.2f}\n",
             G, p < 4 ? "store" : "load", p & 3, t * 1e3, tot / s * 1e-9, wg_bytes / (s * ghz * 1e9));
    }
  }
  CK(hipFree(buf));
  return 0;
}
