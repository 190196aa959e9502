// Probe: LDS-DMA staging of sweep-like channel windows.  Each workgroup (4
// waves) walks `nch` channel rows; per row it DMAs a window of `we` 16-B
// elements starting at its time offset into a double-buffered LDS ring (8 rows
// per chunk, one barrier per chunk), like k_sweep_il's loaders without compute.
// Row stride `rs` elements: the production image (rs = nR ~ 146k elements,
// 2.3 MB) or compact (rs small, rows adjacent) -- isolates address-translation
// and DRAM-page effects from the byte count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef __attribute__((address_space(3))) float lds_float_t;
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(const lds_float_t*)p; }

__global__ __launch_bounds__(256) void k(const float4* __restrict__ R, int64_t rs, int nch, int we,
                                         int ntile, int tq, float* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t t0 = (int64_t)(blockIdx.x % ntile) * tq;
  const int nq = (we + 63) / 64;
  const int per_chunk = 8;
  const int buf_e = per_chunk * nq * 64;
  for (int c0 = 0; c0 < nch; c0 += per_chunk) {
    const int b = (c0 / per_chunk) & 1;
    for (int i = 0; i < per_chunk; ++i) {
      const float4* row = R + (int64_t)(c0 + i) * rs + t0;
      for (int q = w; q < nq; q += 4) {
        const float4* s = row + q * 64 + lane;
        uint32_t la = lds_addr(sm) + (uint32_t)((b * buf_e + (i * nq + q) * 64) * 16), keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(s), "s"(__builtin_amdgcn_readfirstlane(la)) : "memory");
      }
    }
    // keep one chunk in flight: wait for the previous chunk's DMAs
    if (c0 > 0) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __syncthreads();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (sm[threadIdx.x] == 12345.f) sink[threadIdx.x] = 1.f;
}

int main(int argc, char** argv) {
  const int nch = 4096, we = 200, tq = 128;
  const int64_t nR = 146000;
  const size_t bytes = (size_t)nch * nR * 16;
  float4* R;
  float* sink;
  if (hipMalloc(&R, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMalloc(&sink, 4096);
  hipMemset(R, 0, bytes);
  const int nq = (we + 63) / 64;
  const int lds = 2 * 8 * nq * 64 * 16;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  struct Cfg { const char* name; int64_t rs; int ntile; int grid; };
  // production-like: 1016 time tiles x 4 trial blocks (same windows reread by 4)
  Cfg cfgs[] = {{"rows 2.3MB stride, 1016 tiles", nR, 1016, 4096},
                {"rows 2.3MB stride, 32 tiles (L2-friendly)", nR, 32, 4096},
                {"compact rows (stride 8192 el), 32 tiles", 8192, 32, 4096},
                {"compact rows (stride 256 el), 1 tile", 256, 1, 4096},
                {"rows 2.3MB stride, 1 tile", nR, 1, 4096}};
  for (auto& c : cfgs) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(c.grid), dim3(256), lds, 0, R, c.rs, nch, we, c.ntile, tq, sink);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double staged = (double)c.grid * nch * nq * 64 * 16;
      if (rep == 2) printf("%-45s %8.3f ms  staged %.1f GB  %.2f TB/s  %.1f B/clk/CU\n", c.name, ms, staged / 1e9,
                           staged / ms / 1e9, staged / (ms * 1e-3) / 256 / 2.4e9);
    }
  }
  return 0;
}
