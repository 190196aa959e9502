// Probe: does the instruction offset of global_load_lds_dwordx4 move the LDS
// destination too (LDS_ADDR = M0 + inst_offset + lane*16)?  One M0 write, four
// 1 KiB DMAs at offsets 0/1024/2048/3072 of a contiguous 4 KiB source; the
// LDS image is copied out and compared with the source.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef __attribute__((address_space(3))) float lds_float_t;
__global__ __launch_bounds__(64) void k(const float4* __restrict__ src, float4* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float4 sm[];
  for (int i = threadIdx.x; i < 512; i += 64) sm[i] = make_float4(-1.f, -1.f, -1.f, -1.f);
  __syncthreads();
  const uint32_t base = (uint32_t)(uintptr_t)(const lds_float_t*)(sm + 64);  // 1 KiB in
  const float4* s = src + threadIdx.x;
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "global_load_lds_dwordx4 %1, off offset:1024\n\t"
      "global_load_lds_dwordx4 %1, off offset:2048\n\t"
      "global_load_lds_dwordx4 %1, off offset:3072\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep) : "v"(s), "s"(__builtin_amdgcn_readfirstlane(base)) : "memory");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = sm[i];
}
int main() {
  std::vector<float4> h(256);
  for (int i = 0; i < 256; ++i) h[i] = make_float4(4 * i, 4 * i + 1, 4 * i + 2, 4 * i + 3);
  float4 *d, *o;
  hipMalloc(&d, 256 * 16);
  hipMalloc(&o, 512 * 16);
  hipMemcpy(d, h.data(), 256 * 16, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 512 * 16, 0, d, o);
  std::vector<float4> r(512);
  hipMemcpy(r.data(), o, 512 * 16, hipMemcpyDeviceToHost);
  int bad = 0, untouched_after = 0;
  for (int i = 0; i < 64; ++i) bad += r[i].x != -1.f;  // before the base: untouched
  for (int i = 0; i < 256; ++i) bad += r[64 + i].x != h[i].x || r[64 + i].w != h[i].w;
  for (int i = 320; i < 512; ++i) untouched_after += r[i].x == -1.f;
  printf("offset moves the LDS destination: %s (mismatches %d, untouched after %d/192)\n",
         bad == 0 ? "YES" : "NO", bad, untouched_after);
  return bad != 0;
}
