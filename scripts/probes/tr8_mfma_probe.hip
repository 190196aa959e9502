// Probe (gfx950): (1) ds_read_b64_tr_b8 lane mapping, (2) i8 16x16x64 MFMA
// operand maps. Single workgroup of 64 threads; writes results to host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

// mode 0: LDS byte a = (a >> 3) & 0xff (chunk id); mode 1: byte a = a & 7
__global__ void k_tr8(uint32_t* out, int mode, const int* lane_chunk) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4096];
  for (int a = threadIdx.x; a < 4096; a += 64)
    lds[a] = mode == 0 ? (uint8_t)((a >> 3) & 0xff) : (uint8_t)(a & 7);
  __syncthreads();
  const int l = threadIdx.x;
  typedef __attribute__((address_space(3))) i32x2 lds_v2;
  typedef __attribute__((address_space(3))) uint8_t lds_u8;
  const uint32_t addr = (uint32_t)lane_chunk[l] * 8u;
  lds_u8* base = (lds_u8*)lds;
  i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2*)(base + addr));
  out[128 + l] = lds[(l * 67) & 4095];
  out[2 * l] = (uint32_t)v.x;
  out[2 * l + 1] = (uint32_t)v.y;
}

// MFMA i8 16x16x64: for each (g0, j0), A[l][j] = (j==j0 && l>>4==g0) ? (l&15)+1 : 0,
// B[l][j] = (j==j0 && l>>4==g0) ? 1 : 0; expect C[m][n] = m+1 (C map:
// lane l holds rows 4(l>>4)+i, col l&15). Count mismatches.
__global__ void k_mfma(int* bad, int* sample) {
  const int l = threadIdx.x;
  int nbad = 0;
  for (int g0 = 0; g0 < 4; ++g0)
    for (int j0 = 0; j0 < 16; ++j0) {
      i32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
      if ((l >> 4) == g0) {
        a[j0 >> 2] = ((l & 15) + 1) << (8 * (j0 & 3));
        b[j0 >> 2] = 1 << (8 * (j0 & 3));
      }
      i32x4 c = {0, 0, 0, 0};
      c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
      for (int i = 0; i < 4; ++i) {
        const int m = 4 * (l >> 4) + i;
        if (c[i] != m + 1) ++nbad;
        if (g0 == 1 && j0 == 5) sample[4 * l + i] = c[i];
      }
    }
  bad[l] = nbad;
}

// signed check: A = -128..127 values, B = ones -> C = sum over k of A row
__global__ void k_mfma_signed(int* out) {
  const int l = threadIdx.x;
  i32x4 a, b;
  for (int w = 0; w < 4; ++w) {
    uint32_t v = 0;
    for (int bb = 0; bb < 4; ++bb) v |= (uint32_t)(uint8_t)(int8_t)(-128 + ((l * 7 + w * 4 + bb) & 255)) << (8 * bb);
    a[w] = (int)v;
    b[w] = 0x01010101;
  }
  i32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) out[4 * l + i] = c[i];
}

int main() {
  uint32_t* d_out; int* d_lc; int *d_bad, *d_s;
  hipMalloc(&d_out, 64 * 8 + 256); hipMalloc(&d_lc, 64 * 4); hipMalloc(&d_bad, 64 * 4); hipMalloc(&d_s, 256 * 4);
  std::vector<int> lc(64);
  for (int l = 0; l < 64; ++l) lc[l] = (l * 37 + 11) % 64 + 64 * (l & 1);  // distinct chunk ids < 256
  hipMemcpy(d_lc, lc.data(), 256, hipMemcpyHostToDevice);
  std::vector<uint32_t> o0(128), o1(128);
  hipLaunchKernelGGL(k_tr8, dim3(1), dim3(64), 0, 0, d_out, 0, d_lc);
  hipMemcpy(o0.data(), d_out, 512, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(k_tr8, dim3(1), dim3(64), 0, 0, d_out, 1, d_lc);
  hipMemcpy(o1.data(), d_out, 512, hipMemcpyDeviceToHost);
  // invert chunk id -> source lane
  std::vector<int> src(256, -1);
  for (int l = 0; l < 64; ++l) src[lc[l] & 0xff] = l;
  printf("RAW mode0 lanes 0..17:\n");
  for (int l = 0; l < 18; ++l) printf("%2d: %08x %08x | %08x %08x  chunk=%d\n", l, o0[2*l], o0[2*l+1], o1[2*l], o1[2*l+1], lc[l]);
  printf("TR8: lane: (srclane.byteoff) x8\n");
  for (int l = 0; l < 64; ++l) {
    printf("%2d:", l);
    for (int b = 0; b < 8; ++b) {
      const uint32_t w0 = o0[2 * l + b / 4], w1 = o1[2 * l + b / 4];
      const int cid = (w0 >> (8 * (b & 3))) & 0xff, off = (w1 >> (8 * (b & 3))) & 0xff;
      printf(" %2d.%d", src[cid], off);
    }
    printf("\n");
  }
  hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, d_bad, d_s);
  std::vector<int> bad(64), s(256);
  hipMemcpy(bad.data(), d_bad, 256, hipMemcpyDeviceToHost);
  hipMemcpy(s.data(), d_s, 1024, hipMemcpyDeviceToHost);
  int tb = 0; for (int v : bad) tb += v;
  printf("MFMA map mismatches: %d of %d\n", tb, 64 * 64 * 4);
  printf("sample (g0=1,j0=5) lanes 0,16,33: %d %d %d %d | %d %d %d %d | %d %d %d %d\n", s[0], s[1], s[2], s[3], s[64], s[65], s[66], s[67], s[132], s[133], s[134], s[135]);
  hipLaunchKernelGGL(k_mfma_signed, dim3(1), dim3(64), 0, 0, d_s);
  hipMemcpy(s.data(), d_s, 1024, hipMemcpyDeviceToHost);
  // expected: C[m][n] = sum_k A[m][k], A[m] = rows held by lanes with l&15==m
  int sbad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int m = 4 * (l >> 4) + i;
      long ex = 0;
      for (int ll = 0; ll < 64; ++ll) if ((ll & 15) == m)
        for (int w = 0; w < 4; ++w) for (int bb = 0; bb < 4; ++bb) ex += -128 + ((ll * 7 + w * 4 + bb) & 255);
      if (s[4 * l + i] != ex) ++sbad;
    }
  printf("signed ones-B mismatches: %d\n", sbad);
  return 0;
}
