// HBM write-rate probe: streaming 16-B-per-lane stores (plain and
// non-temporal) over a 16 GiB buffer, the access shape of the factorised
// stage 1 (k_fx_patterns_x writes every pattern element once).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <bool NT>
__global__ __launch_bounds__(256) void k_write(uint4* __restrict__ p, int64_t n, uint32_t v) {
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const u32x4v s = {v, v + 1, v + 2, v + 3};
    if (NT) __builtin_nontemporal_store(s, reinterpret_cast<u32x4v*>(p + i));
    else *reinterpret_cast<u32x4v*>(p + i) = s;
  }
}
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) b[i] = a[i];
}

int main() {
  const int64_t bytes = (int64_t)16 << 30, n = bytes / 16;
  uint4 *p, *q;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&q, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int grid : {2048, 8192, 32768}) {
    for (int mode = 0; mode < 3; ++mode) {
      float best = 1e30f;
      for (int r = 0; r < 4; ++r) {
        hipEventRecord(e0);
        if (mode == 0) hipLaunchKernelGGL(k_write<false>, dim3(grid), dim3(256), 0, 0, p, n, (uint32_t)r);
        else if (mode == 1) hipLaunchKernelGGL(k_write<true>, dim3(grid), dim3(256), 0, 0, p, n, (uint32_t)r);
        else hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, p, q, n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double b = mode == 2 ? 2.0 * bytes : (double)bytes;
      printf("grid %6d %-12s %7.2f ms  %.2f TB/s\n", grid, mode == 0 ? "store" : (mode == 1 ? "nt-store" : "copy r+w"),
             best, b / (best * 1e-3) / 1e12);
    }
  }
  hipFree(p);
  hipFree(q);
  return 0;
}
