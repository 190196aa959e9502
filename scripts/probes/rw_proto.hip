// Probe: compute-side rate of the register-window sweep (no staging).
//
// A static LDS image of NCH channel windows (u16 pairs, random), 8 compute
// waves x DPW = 8 trials each, K = 4 elements (8 samples) per lane per trial.
// The per-(trial block, wave, channel) records come from the BASELINE
// configs[3] grid (4096 ch, 1250-1550 MHz, 64 us, 4096 DMs 0..1000).
// Checks every output against a host sum; prints adds/s and adds/clk/CU.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o rw_proto rw_proto.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include <stdint.h>

#ifdef RW_NOP
#include "rw_asm_nop.inc"
#else
#include "rw_asm.inc"
#endif

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

typedef unsigned u32x32 __attribute__((ext_vector_type(32)));
constexpr int NW = 8, DB = NW * RW_DPW, NCH = 32, LW = 512;  // LW: words per channel window

__global__ __launch_bounds__(512) void k_rw(const uint4* __restrict__ gimg, const uint4* __restrict__ meta,
                                            int C, int n_dblk, int recs, uint32_t* __restrict__ out,
                                            int check_blocks) {
  extern __shared__ uint4 lds[];
  for (int i = threadIdx.x; i < NCH * LW / 4; i += 512) lds[i] = gimg[i];
  __syncthreads();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int dblk = blockIdx.x % n_dblk;
  const uint4* mp = meta + (size_t)(dblk * NW + w) * recs;
  const uint32_t vl = lane * 16;
  u32x32 acc = (u32x32)0u, f0 = (u32x32)0u, f1 = (u32x32)0u;
  for (int c0 = 0; c0 < C; c0 += 256) {
    const int n = __builtin_amdgcn_readfirstlane(min(256, C - c0));
    const uint4* p = mp + c0;
    asm volatile(RW_BLOCK_ASM
                 : "+{v[192:223]}"(acc), "+{v[64:95]}"(f0), "+{v[96:127]}"(f1)
                 : [mp] "s"(p), [n] "s"(n), [vl] "v"(vl)
                 : RW_BLOCK_CLOBBERS);
  }
  if ((int)blockIdx.x < check_blocks) {
    uint32_t* o = out + ((size_t)(blockIdx.x * NW + w) * 64 + lane) * 64;
#pragma unroll
    for (int q = 0; q < 32; ++q) o[q] = f0[q];
#pragma unroll
    for (int q = 0; q < 32; ++q) o[32 + q] = f1[q];
  } else if (f0[0] == 0xdeadbeef) {
    out[0] = f1[3];
  }
}

int main(int argc, char** argv) {
  const int C = 4096, D = 4096;
  const int n_dblk = 16;
  const int reps = argc > 1 ? atoi(argv[1]) : 256 * 16;
  const double dt = 64e-6;
  std::vector<double> f(C);
  const double foff = -300.0 / C;
  for (int c = 0; c < C; ++c) f[c] = 1550.0 + foff / 2 + foff * c;
  auto bin = [&](int d, int c) {
    const double dm = 1000.0 * d / (D - 1);
    const double del = dm / (0.000241 * f[c] * f[c]) - dm / (0.000241 * f[0] * f[0]);
    return (int)std::nearbyint(del / dt);
  };
  // trial blocks spread over the grid
  const int recs = C + 16;
  std::vector<uint32_t> meta((size_t)n_dblk * NW * recs * 4, 0);
  std::vector<int> rec_ws((size_t)n_dblk * NW * C), rec_idx((size_t)n_dblk * NW * C * RW_DPW);
  int worst = 0;
  double ng_sum = 0;
  for (int b = 0; b < n_dblk; ++b) {
    const int tb = b * (D / DB / n_dblk);
    for (int c = 0; c < C; ++c) {
      int bmin = 1 << 30;
      for (int d = 0; d < DB; ++d) bmin = std::min(bmin, bin(tb * DB + d, c));
      for (int w = 0; w < NW; ++w) {
        int lo = 1 << 30, hi = -1;
        int s[RW_DPW];
        for (int j = 0; j < RW_DPW; ++j) {
          s[j] = bin(tb * DB + w * RW_DPW + j, c) - bmin;
          lo = std::min(lo, s[j]);
          hi = std::max(hi, s[j]);
        }
        int ws = lo & ~3;
        int mx = 0;
        uint32_t z = 0, ww = 0;
        for (int j = 0; j < RW_DPW; ++j) {
          int idx = s[j] - ws;
          if (idx > RW_W - RW_K) { idx = RW_W - RW_K; }
          mx = std::max(mx, idx);
          worst = std::max(worst, s[j] - ws + RW_K);
          if (j < 4) z |= (uint32_t)idx << (8 * j); else ww |= (uint32_t)idx << (8 * (j - 4));
          rec_idx[((size_t)(b * NW + w) * C + c) * RW_DPW + j] = idx;
        }
        if (ws + 4 * 64 + RW_W > LW) ws = (LW - 4 * 64 - RW_W) & ~3;
        rec_ws[(size_t)(b * NW + w) * C + c] = ws;
        const int ng = (mx + RW_K + 3) / 4;
        ng_sum += ng;
        uint32_t* r = &meta[(((size_t)(b * NW + w)) * recs + c) * 4];
        r[0] = (uint32_t)(((c % NCH) * LW + ws) * 4);
        r[1] = ng;
        r[2] = z;
        r[3] = ww;
      }
    }
  }
  printf("worst window words %d (W=%d), mean granules %.2f\n", worst, RW_W,
         ng_sum / ((double)n_dblk * NW * C));
  std::vector<uint32_t> img(NCH * LW);
  srand(1);
  for (auto& v : img) v = (uint32_t)(rand() & 255) | ((uint32_t)(rand() & 255) << 16);
  uint4 *d_img, *d_meta;
  uint32_t* d_out;
  const int check_blocks = n_dblk;
  CK(hipMalloc(&d_img, img.size() * 4));
  CK(hipMalloc(&d_meta, meta.size() * 4));
  CK(hipMalloc(&d_out, (size_t)check_blocks * NW * 64 * 64 * 4));
  CK(hipMemcpy(d_img, img.data(), img.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_meta, meta.data(), meta.size() * 4, hipMemcpyHostToDevice));
  const int lds = NCH * LW * 4;
  CK(hipFuncSetAttribute((const void*)k_rw, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipLaunchKernelGGL(k_rw, dim3(reps), dim3(512), lds, 0, d_img, d_meta, C, n_dblk, recs, d_out,
                     check_blocks);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> out((size_t)check_blocks * NW * 64 * 64);
  CK(hipMemcpy(out.data(), d_out, out.size() * 4, hipMemcpyDeviceToHost));
  long bad = 0;
  for (int b = 0; b < check_blocks; ++b)
    for (int w = 0; w < NW; ++w)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < RW_DPW; ++j)
          for (int m = 0; m < RW_K; ++m) {
            uint32_t lo = 0, hi = 0;
            for (int c = 0; c < C; ++c) {
              const size_t r = (size_t)(b * NW + w) * C + c;
              const uint32_t v = img[(c % NCH) * LW + rec_ws[r] + 4 * lane + rec_idx[r * RW_DPW + j] + m];
              lo += v & 0xffff;
              hi += v >> 16;
            }
            const uint32_t* o = &out[((size_t)(b * NW + w) * 64 + lane) * 64];
            const int q = j * RW_K + m;
            if (o[2 * q] != lo || o[2 * q + 1] != hi) {
              if (bad < 5) printf("mismatch b%d w%d l%d j%d m%d: %u/%u vs %u/%u\n", b, w, lane, j, m,
                                  o[2 * q], o[2 * q + 1], lo, hi);
              ++bad;
            }
          }
  printf("check: %ld mismatches\n", bad);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int it = 0; it < 3; ++it) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_rw, dim3(reps), dim3(512), lds, 0, d_img, d_meta, C, n_dblk, recs, d_out,
                       0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double adds = (double)reps * DB * 64 * RW_K * 2 * C;
    printf("reps %d: %.3f ms, %.2f T adds/s, %.1f adds/clk/CU at 2.4 GHz\n", reps, ms,
           adds / ms / 1e9, adds / (ms * 1e-3) / 256 / 2.4e9);
  }
  return bad ? 1 : 0;
}
