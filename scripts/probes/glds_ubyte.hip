// Probe: what does global_load_lds_ubyte / _ushort write into LDS on gfx950?
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void g_void;
__global__ void k(const unsigned char* src, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned sm[512];
  for (int i = threadIdx.x; i < 512; i += 64) sm[i] = 0xdeadbeefu;
  __syncthreads();
  __builtin_amdgcn_global_load_lds((g_void*)(src + threadIdx.x * 3), (lds_void*)(sm), 1, 0, 0);
  __builtin_amdgcn_global_load_lds((g_void*)(src + threadIdx.x * 2), (lds_void*)(sm + 256), 2, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = sm[i];
}
int main() {
  unsigned char h[256];
  for (int i = 0; i < 256; ++i) h[i] = (unsigned char)i;
  unsigned char* d; unsigned* o; unsigned ho[512];
  hipMalloc(&d, 256); hipMalloc(&o, 2048);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, o);
  hipMemcpy(ho, o, 2048, hipMemcpyDeviceToHost);
  printf("ubyte: "); for (int i = 0; i < 20; ++i) printf("%08x ", ho[i]); printf("\n");
  printf("ushort: "); for (int i = 256; i < 276; ++i) printf("%08x ", ho[i]); printf("\n");
  return 0;
}
