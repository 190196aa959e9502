// Probe: global -> LDS staging throughput on gfx950 for the access shapes the
// sweep kernel can use.  Each workgroup repeatedly stages `per_wg` bytes of a
// window (region `span` bytes, L2-resident when small) into a 32 KiB LDS
// buffer and touches one word so nothing is dead.
//   mode 0: global_load_lds_dword, 256 contiguous bytes per wave-instruction
//   mode 1: global_load_lds_dword, 4 stripes x 64 B per wave-instruction
//   mode 2: global_load_lds_dwordx4, 1 KiB contiguous per wave-instruction
//   mode 3: global_load_dwordx4 to VGPRs + ds_write_b128 (register staging)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef __attribute__((address_space(3))) float lds_float_t;

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(const lds_float_t*)p; }

template <int MODE>
__global__ __launch_bounds__(512) void k(const float* __restrict__ src, int64_t region_floats,
                                         int iters, float* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  const int64_t wg_off = ((int64_t)blockIdx.x * 9973 * 256) % (region_floats - 65536);
  const float* base = src + wg_off;
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    // 32 KiB per iteration per workgroup
    const float* b = base + (it % 4) * 8192;
    if constexpr (MODE == 0 || MODE == 1) {
      for (int q = w; q < 128; q += nw) {   // 128 x 256 B
        const float* s;
        if (MODE == 0) s = b + q * 64 + lane;
        else s = b + q * 16 + (lane >> 2) + (lane & 3) * 2048;
        uint32_t la = lds_addr(sm + q * 64), keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(s), "s"(__builtin_amdgcn_readfirstlane(la)) : "memory");
      }
    } else if constexpr (MODE == 2) {
      for (int q = w; q < 32; q += nw) {    // 32 x 1 KiB
        const float* s = b + q * 256 + lane * 4 + 1;  // dword- but not 16B-aligned, like the sweep
        uint32_t la = lds_addr(sm + q * 256), keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(s), "s"(__builtin_amdgcn_readfirstlane(la)) : "memory");
      }
    } else {
      for (int q = w; q < 32; q += nw) {
        const float4 v = *(const float4*)(b + q * 256 + lane * 4);
        *(float4*)(sm + q * 256 + lane * 4) = v;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    acc += sm[(threadIdx.x * 7 + it) & 8191];
    __syncthreads();
  }
  if (acc == 12345.f) sink[threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int64_t big = 1ll << 30;  // 4 GiB of floats
  float* src;
  float* sink;
  hipMalloc(&src, big * 4);
  hipMalloc(&sink, 4096);
  hipMemset(src, 0, big * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 64;
  for (int64_t region : {(int64_t)(1 << 20), (int64_t)(64 << 20), big}) {   // floats: 4 MB, 256 MB, 4 GB
    for (int wgs_per_cu : {1, 2, 4}) {
      for (int mode = 0; mode < 4; ++mode) {
        const int grid = 256 * wgs_per_cu * 4;
        auto launch = [&]() {
          if (mode == 0) k<0><<<grid, 512, 32768>>>(src, region, iters, sink);
          if (mode == 1) k<1><<<grid, 512, 32768>>>(src, region, iters, sink);
          if (mode == 2) k<2><<<grid, 512, 32768>>>(src, region, iters, sink);
          if (mode == 3) k<3><<<grid, 512, 32768>>>(src, region, iters, sink);
        };
        launch();
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double bytes = (double)grid * iters * 32768;
        printf("region %6.0f MB  wg/cu %d  mode %d : %7.3f ms  %8.2f TB/s\n", region * 4 / 1e6,
               wgs_per_cu, mode, ms, bytes / ms / 1e9);
      }
    }
  }
  return 0;
}
