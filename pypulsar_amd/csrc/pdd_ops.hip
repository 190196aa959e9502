// libpdd: single-pass (HBM-bound) kernels of the Spectra hot path, gfx950.
//
// Every kernel here reads its input once and writes its output once; they are
// bounded by HBM (≈8 TB/s spec).  Algorithmic bytes per launch are documented
// in DESIGN.md §Kernels.  Coalescing: consecutive lanes always touch
// consecutive samples of one channel row (wave-strided, 64 lanes x 4 B).
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "pdd_internal.h"

namespace pdd {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

namespace {
struct ScratchBuf {
  int dev;  // the null stream is per device: key by device too
  hipStream_t st;
  std::thread::id tid;  // per calling thread: two host threads queueing on one
                        // stream (torch's default stream is shared) must not
                        // interleave their launches on one buffer
  int slot;
  void* ptr;
  size_t bytes;
};
std::mutex g_scratch_mu;
std::vector<ScratchBuf> g_scratch;
}  // namespace

void* scratch(hipStream_t st, int slot, size_t bytes) {
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  bytes = std::max<size_t>(bytes, 256);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    set_error("device scratch: hipGetDevice failed");
    return nullptr;
  }
  const std::thread::id tid = std::this_thread::get_id();
  for (auto& b : g_scratch) {
    if (b.dev != dev || b.st != st || b.tid != tid || b.slot != slot) continue;
    if (b.bytes >= bytes) return b.ptr;
    // grow: the stream's queued work may still read the old buffer
    hipError_t e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = hipFree(b.ptr);
    b.ptr = nullptr;
    b.bytes = 0;
    if (e == hipSuccess) e = hipMalloc(&b.ptr, bytes);
    if (e != hipSuccess) {
      b.ptr = nullptr;
      set_error("device scratch (%zu bytes): %s", bytes, hipGetErrorString(e));
      return nullptr;
    }
    b.bytes = bytes;
    return b.ptr;
  }
  void* p = nullptr;
  const hipError_t e = hipMalloc(&p, bytes);
  if (e != hipSuccess) {
    set_error("device scratch (%zu bytes): %s", bytes, hipGetErrorString(e));
    return nullptr;
  }
  g_scratch.push_back({dev, st, tid, slot, p, bytes});
  return p;
}

size_t scratch_held(hipStream_t st, int slot) {
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const std::thread::id tid = std::this_thread::get_id();
  for (const auto& b : g_scratch)
    if (b.dev == dev && b.st == st && b.tid == tid && b.slot == slot) return b.bytes;
  return 0;
}

// ---------------------------------------------------------------- loaders
template <typename T>
__device__ __forceinline__ float to_f32(T v) { return static_cast<float>(v); }

// ---------------------------------------------------------------- corner turn
// [nspec][nchan] -> [nchan][nspec] through a 64x65 LDS tile (padding breaks
// the power-of-two column stride on the transposed read).
template <typename InT, typename OutT>
__global__ __launch_bounds__(256) void k_corner_turn(const InT* __restrict__ in, int64_t nspec,
                                                     int64_t nchan, int64_t ld_in,
                                                     OutT* __restrict__ out, int64_t ld_out,
                                                     int64_t tiles_c) {
  __shared__ OutT tile[64][65];
  const int64_t tt = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int64_t t0 = tt * 64, c0 = tc * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int64_t t = t0 + i, c = c0 + tx;
    if (t < nspec && c < nchan) tile[i][tx] = static_cast<OutT>(in[t * ld_in + c]);
  }
  __syncthreads();
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, t = t0 + tx;
    if (t < nspec && c < nchan) out[c * ld_out + t] = tile[tx][i];
  }
}

// The same to float32 with 16-byte row loads (8 lanes cover one 128-byte
// line of a spectrum): tile = 64 spectra x 8*VEC channels, VEC = elements per
// 16 bytes.  Rows must be 16-B aligned and nchan*sizeof(InT) a multiple of 16
// (the launcher checks).
template <typename InT>
__global__ __launch_bounds__(256) void k_corner_turn_vec(const InT* __restrict__ in, int64_t nspec,
                                                         int64_t nchan, int64_t ld_in,
                                                         float* __restrict__ out, int64_t ld_out,
                                                         int64_t tiles_c) {
  constexpr int VEC = 16 / sizeof(InT);
  constexpr int TC = 8 * VEC;
  __shared__ float tile[TC][65];
  const int64_t tt = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int64_t t0 = tt * 64, c0 = tc * TC;
  const int seg = threadIdx.x & 7, r0 = threadIdx.x >> 3;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int i = r0 + 32 * pass;
    const int64_t t = t0 + i, c = c0 + seg * VEC;
    union { uint4 q; InT e[VEC]; } u;
    if (t < nspec && c < nchan) u.q = *reinterpret_cast<const uint4*>(in + t * ld_in + c);
    else u.q = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int e = 0; e < VEC; ++e) tile[seg * VEC + e][i] = static_cast<float>(u.e[e]);
  }
  __syncthreads();
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t t = t0 + tx;
#pragma unroll 4
  for (int i = ty; i < TC; i += 4) {
    const int64_t c = c0 + i;
    if (t < nspec && c < nchan) out[c * ld_out + t] = tile[i][tx];
  }
}

// 8-bit raw corner turn [nspec][nchan] -> [nchan][nspec] through a
// 128-spectra x 128-channel LDS tile (rows of 33 dwords): every input row and
// every output row is read / written as whole 128-byte lines (16 bytes per
// lane), each output vector gathering 16 spectra of one channel byte by
// byte.  Rows and nchan must be 16-B aligned (the launcher checks); the
// nspec tail is stored bytewise.
__global__ __launch_bounds__(256) void k_corner_turn_b8w(const uint8_t* __restrict__ in,
                                                         int64_t nspec, int64_t nchan, int64_t ld_in,
                                                         uint8_t* __restrict__ out, int64_t ld_out,
                                                         int64_t tiles_c) {
  __shared__ uint32_t tile[128][33];
  const int64_t tt = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int64_t t0 = tt * 128, c0 = tc * 128;
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int r = (threadIdx.x >> 3) + 32 * pass, seg = threadIdx.x & 7;
    const int64_t t = t0 + r, c = c0 + seg * 16;
    uint4 q = make_uint4(0u, 0u, 0u, 0u);
    if (t < nspec && c < nchan) q = *reinterpret_cast<const uint4*>(in + t * ld_in + c);
    tile[r][seg * 4 + 0] = q.x;
    tile[r][seg * 4 + 1] = q.y;
    tile[r][seg * 4 + 2] = q.z;
    tile[r][seg * 4 + 3] = q.w;
  }
  __syncthreads();
  const auto* tb = reinterpret_cast<const uint8_t*>(&tile[0][0]);
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int cl = (threadIdx.x >> 3) + 32 * pass, ts = threadIdx.x & 7;
    const int64_t c = c0 + cl, t = t0 + ts * 16;
    if (c >= nchan || t >= nspec) continue;
    uint32_t w[4];
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      uint32_t v = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) v |= (uint32_t)tb[(ts * 16 + k4 * 4 + k) * 132 + cl] << (8 * k);
      w[k4] = v;
    }
    uint8_t* o = out + c * ld_out + t;
    if (t + 16 <= nspec) {
      *reinterpret_cast<uint4*>(o) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      for (int k = 0; k < (int)(nspec - t); ++k) o[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
  }
}

template <typename InT>
__global__ __launch_bounds__(256) void k_convert(const InT* __restrict__ in, int64_t rows,
                                                 int64_t cols, int64_t ld_in,
                                                 float* __restrict__ out, int64_t ld_out) {
  const int64_t total = rows * cols;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cols, c = i % cols;
    out[r * ld_out + c] = to_f32(in[r * ld_in + c]);
  }
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

// Per-channel mean in float64 (one workgroup per channel); 16-byte loads,
// four in flight per lane, when the rows are 16-B aligned.
__global__ __launch_bounds__(256) void k_channel_mean(const float* __restrict__ x, int64_t N,
                                                      int64_t ld, float* __restrict__ out) {
  __shared__ double part[4];
  const float* row = x + (int64_t)blockIdx.x * ld;
  double s = 0.0;
  int64_t i0 = 0;
  if (((uintptr_t)row & 15) == 0) {
    const float4* r4 = reinterpret_cast<const float4*>(row);
    const int64_t n4 = N / 4;
    int64_t i = threadIdx.x;
    for (; i + 768 < n4; i += 1024) {
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = r4[i + 256 * k];
#pragma unroll
      for (int k = 0; k < 4; ++k) s += ((double)v[k].x + (double)v[k].y) + ((double)v[k].z + (double)v[k].w);
    }
    for (; i < n4; i += 256) {
      const float4 v = r4[i];
      s += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
    }
    i0 = n4 * 4;
  }
  for (int64_t i = i0 + threadIdx.x; i < N; i += 256) s += (double)row[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (float)(((part[0] + part[1]) + (part[2] + part[3])) / (double)N);
}

// Orderable key of a float (total order for non-NaN values).
__device__ __forceinline__ uint32_t fkey(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// k-th smallest of a row by 4 passes of 8-bit radix selection (LDS histogram).
__device__ float radix_select_row(const float* __restrict__ row, int64_t N, int64_t k,
                                  uint32_t* hist, uint32_t* shared_state) {
  uint32_t prefix = 0, mask = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) {
      const uint32_t key = fkey(row[i]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t kk = k;
      uint32_t d = 0;
      for (; d < 256; ++d) {
        if (kk < (int64_t)hist[d]) break;
        kk -= hist[d];
      }
      shared_state[0] = d;
      shared_state[1] = (uint32_t)kk;
    }
    __syncthreads();
    const uint32_t d = shared_state[0];
    k = shared_state[1];
    prefix |= d << shift;
    mask |= 255u << shift;
    __syncthreads();
  }
  return fkey_inv(prefix);
}

// Per-channel median with numpy semantics (mean of the two middle values when
// N is even).  One workgroup per channel.
__global__ __launch_bounds__(256) void k_channel_median(const float* __restrict__ x, int64_t N,
                                                        int64_t ld, float* __restrict__ out) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t st[2];
  const float* row = x + (int64_t)blockIdx.x * ld;
  const float hi = radix_select_row(row, N, N / 2, hist, st);
  float med = hi;
  if ((N & 1) == 0) {
    const float lo = radix_select_row(row, N, N / 2 - 1, hist, st);
    med = (float)(((double)lo + (double)hi) * 0.5);
  }
  if (threadIdx.x == 0) out[blockIdx.x] = med;
}

// ---------------------------------------------------------------- shift / pad
// out[c][t] = X(c, t + bins[c]).  Block = 1024 consecutive outputs of one
// channel; lane-consecutive samples per wave instruction.
__global__ __launch_bounds__(256) void k_shift_pad(const float* __restrict__ x, int64_t N,
                                                   int64_t ld, const int32_t* __restrict__ bins,
                                                   int pad_mode, const float* __restrict__ padvals,
                                                   float* __restrict__ out, int64_t ld_out,
                                                   int64_t n_out, int64_t tiles) {
  const int64_t c = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const float* row = x + c * ld;
  float* orow = out + c * ld_out;
  int64_t b = bins[c];
  if (pad_mode == PDD_PAD_ROTATE) b = ((b % N) + N) % N;
  const float pad = (pad_mode == PDD_PAD_VALUE) ? padvals[c] : 0.f;
  const int64_t t0 = tile * 1024 + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t t = t0 + 64 * k;
    v[k] = (t < n_out) ? fetch_padded(row, t + b, N, pad_mode, pad) : 0.f;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t t = t0 + 64 * k;
    if (t < n_out) orow[t] = v[k];
  }
}

// ---------------------------------------------------------------- shift + group sum
// out[g][t] = sum_{c in group g} X(c, t + bins[c]).  Block = 256 outputs of
// one group (4 per lane) and one of `csplit` channel slices of it; wave w of
// 8 sums channels w, w+8, ... of the slice in float64, four channels' loads
// in flight at once (16 per lane: enough bytes in flight to reach HBM rate);
// the 8 partials are added in a fixed order (deterministic).  csplit > 1
// (few outputs per group) writes float64 partials that k_group_sum_reduce
// adds in slice order.
constexpr int kGsWaves = 8;
__global__ __launch_bounds__(kGsWaves * 64) void k_shift_group_sum(
    const float* __restrict__ x, int64_t N, int64_t ld, const int32_t* __restrict__ bins,
    int pad_mode, const float* __restrict__ padvals, int64_t cps, int64_t csplit,
    float* __restrict__ out, double* __restrict__ part_out, int64_t ld_out, int64_t n_out,
    int64_t tiles, int64_t ngrp) {
  __shared__ double part[kGsWaves][256];
  const int64_t gp = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const int64_t g = gp % ngrp, sl = gp / ngrp;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t cpp = (cps + csplit - 1) / csplit;
  const int64_t cbeg = sl * cpp, cend = min(cps, cbeg + cpp);
  const int64_t t0 = tile * 256 + lane;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t ci = cbeg + w; ci < cend; ci += 4 * kGsWaves) {
    float v[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t cj = ci + j * kGsWaves;
      if (cj < cend) {
        const int64_t c = g * cps + cj;
        const float* row = x + c * ld;
        int64_t b = bins ? (int64_t)bins[c] : 0;
        if (pad_mode == PDD_PAD_ROTATE) b = ((b % N) + N) % N;
        const float pad = (pad_mode == PDD_PAD_VALUE && padvals) ? padvals[c] : 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t t = t0 + 64 * k;
          v[j][k] = (t < n_out) ? fetch_padded(row, t + b, N, pad_mode, pad) : 0.f;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[j][k] = 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += (double)v[j][k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) part[w][lane + 64 * k] = acc[k];
  __syncthreads();
  if (threadIdx.x < 256) {
    const int i = threadIdx.x;
    const int64_t t = tile * 256 + i;
    if (t < n_out) {
      const double sum = ((part[0][i] + part[1][i]) + (part[2][i] + part[3][i])) +
                         ((part[4][i] + part[5][i]) + (part[6][i] + part[7][i]));
      if (csplit == 1) out[g * ld_out + t] = (float)sum;
      else part_out[(sl * ngrp + g) * n_out + t] = sum;
    }
  }
}

__global__ __launch_bounds__(256) void k_group_sum_reduce(const double* __restrict__ part,
                                                          int64_t csplit, int64_t ngrp,
                                                          int64_t n_out, float* __restrict__ out,
                                                          int64_t ld_out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= ngrp * n_out) return;
  const int64_t g = i / n_out, t = i % n_out;
  double s = 0.0;
  for (int64_t p = 0; p < csplit; ++p) s += part[(p * ngrp + g) * n_out + t];
  out[g * ld_out + t] = (float)s;
}

// ---------------------------------------------------------------- downsample
__global__ __launch_bounds__(256) void k_downsample(const float* __restrict__ x, int64_t ld,
                                                    int64_t factor, int64_t nout,
                                                    float* __restrict__ out, int64_t ld_out,
                                                    int64_t tiles) {
  const int64_t c = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const int64_t j = tile * 256 + threadIdx.x;
  if (j >= nout) return;
  const float* p = x + c * ld + j * factor;
  double s = 0.0;
  for (int64_t k = 0; k < factor; ++k) s += (double)p[k];
  out[c * ld_out + j] = (float)s;
}

// factor % 4 == 0 and 16-B aligned rows: float4 loads (factor/4 per output)
__global__ __launch_bounds__(256) void k_downsample_v4(const float* __restrict__ x, int64_t ld,
                                                       int64_t factor, int64_t nout,
                                                       float* __restrict__ out, int64_t ld_out,
                                                       int64_t tiles) {
  const int64_t c = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const int64_t j = tile * 256 + threadIdx.x;
  if (j >= nout) return;
  const float4* p = reinterpret_cast<const float4*>(x + c * ld + j * factor);
  double s = 0.0;
  for (int64_t k = 0; k < factor / 4; ++k) {
    const float4 v = p[k];
    s += (double)v.x;
    s += (double)v.y;
    s += (double)v.z;
    s += (double)v.w;
  }
  out[c * ld_out + j] = (float)s;
}

// 8-bit input (a Spectra's raw bytes): integer sums (exact), one 16-byte load
// per lane when the factor divides 16 and the rows are 16-B aligned -- a
// quarter of the float32 image's bytes (DDplan executor, spectra.py:329-351)
template <int F, typename OutT>
__global__ __launch_bounds__(256) void k_downsample_u8v(const uint8_t* __restrict__ x, int64_t ld,
                                                        int64_t nvec, OutT* __restrict__ out,
                                                        int64_t ld_out, int64_t nout,
                                                        int64_t tiles, bool vstore) {
  constexpr int PER = 16 / F;  // outputs per 16-byte vector
  const int64_t c = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const int64_t v = tile * 256 + threadIdx.x;  // 16-byte vector index in the row
  if (v >= nvec) return;
  const uint4 q = *reinterpret_cast<const uint4*>(x + c * ld + v * 16);
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
  uint32_t r[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    uint32_t s = 0;
#pragma unroll
    for (int b = 0; b < F; ++b) {
      const int e = k * F + b;
      s += (w[e >> 2] >> (8 * (e & 3))) & 0xffu;
    }
    r[k] = s;
  }
  OutT* o = out + c * ld_out + v * PER;
  if constexpr (sizeof(OutT) == 4) {
    if constexpr (PER >= 4) {
      if (vstore && v * PER + PER <= nout) {
#pragma unroll
        for (int k = 0; k < PER; k += 4)
          *reinterpret_cast<float4*>(o + k) =
              make_float4((float)r[k], (float)r[k + 1], (float)r[k + 2], (float)r[k + 3]);
        return;
      }
    } else if constexpr (PER == 2) {
      if (vstore && v * PER + PER <= nout) {
        *reinterpret_cast<float2*>(o) = make_float2((float)r[0], (float)r[1]);
        return;
      }
    }
  } else {
    // uint16 sums (F <= 4: <= 1020), packed two per dword
    if constexpr (PER >= 4) {
      if (vstore && v * PER + PER <= nout) {
#pragma unroll
        for (int k = 0; k < PER; k += 4)
          *reinterpret_cast<uint2*>(o + k) = make_uint2(r[k] | (r[k + 1] << 16),
                                                        r[k + 2] | (r[k + 3] << 16));
        return;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (v * PER + k < nout) o[k] = (OutT)r[k];
}

template <typename OutT>
__global__ __launch_bounds__(256) void k_downsample_u8(const uint8_t* __restrict__ x, int64_t ld,
                                                       int64_t factor, int64_t nout,
                                                       OutT* __restrict__ out, int64_t ld_out,
                                                       int64_t tiles) {
  const int64_t c = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const int64_t j = tile * 256 + threadIdx.x;
  if (j >= nout) return;
  const uint8_t* p = x + c * ld + j * factor;
  uint64_t s = 0;
  for (int64_t k = 0; k < factor; ++k) s += p[k];
  out[c * ld_out + j] = (OutT)s;
}

// ---------------------------------------------------------------- zero-DM
// Integer data: avg = rint(float64(sum)/nchan) cast to the dtype, out = x - avg
// modulo 2^nbits (bin/zero_dm_filter.py:35-39).  float32: float32 mean.
template <typename T>
__device__ __forceinline__ T zd_apply(T v, double mean) {
  if constexpr (sizeof(T) == 4) {
    return v - (float)mean;
  } else {
    const uint32_t a = (uint32_t)rint(mean);
    return (T)((uint32_t)v - a);
  }
}

// one wave per spectrum, time-major [nspec][nchan]
template <typename T>
__global__ __launch_bounds__(256) void k_zero_dm_tm(const T* __restrict__ in, int64_t nspec,
                                                    int64_t nchan, int64_t ld,
                                                    T* __restrict__ out, int64_t ld_out) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= nspec) return;
  const T* row = in + s * ld;
  double mean;
  if constexpr (sizeof(T) == 4) {
    double acc = 0.0;
    for (int64_t c = lane; c < nchan; c += 64) acc += (double)row[c];
    acc = wave_sum(acc);
    acc = __shfl(acc, 0, 64);
    mean = (double)((float)acc / (float)nchan);
  } else {
    unsigned long long acc = 0;
    for (int64_t c = lane; c < nchan; c += 64) acc += (unsigned long long)row[c];
    acc = wave_sum_u64(acc);
    acc = __shfl(acc, 0, 64);
    mean = (double)acc / (double)nchan;
  }
  T* orow = out + s * ld_out;
  for (int64_t c = lane; c < nchan; c += 64) orow[c] = zd_apply<T>(row[c], mean);
}

// 8/16-bit time-major rows, 16 bytes per lane per load (rows 16-B aligned,
// nchan*sizeof(T) a multiple of 16; the launcher checks): one wave per
// spectrum, the byte/halfword sum by masked SWAR adds, and the modular
// subtraction of the rounded mean applied to whole words without borrows
// between lanes: ((x | H) - (a & ~H)) ^ ((x ^ ~a) & H), H = the lane sign bits.
template <typename T>
__global__ __launch_bounds__(256) void k_zero_dm_tm_vec(const T* __restrict__ in, int64_t nspec,
                                                        int64_t nchan, int64_t ld,
                                                        T* __restrict__ out, int64_t ld_out) {
  static_assert(sizeof(T) == 1 || sizeof(T) == 2, "8/16-bit only");
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= nspec) return;
  const uint4* row = reinterpret_cast<const uint4*>(in + s * ld);
  const int64_t nv = nchan * (int64_t)sizeof(T) / 16;
  constexpr uint32_t M = sizeof(T) == 1 ? 0x00ff00ffu : 0x0000ffffu;
  constexpr int SH = sizeof(T) == 1 ? 8 : 16;
  unsigned long long acc = 0;
  for (int64_t v = lane; v < nv; v += 64) {
    const uint4 q = row[v];
    const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
    uint32_t p = 0;  // two 16-bit (u8) / one 32-bit-safe (u16: split below) partial lanes
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (sizeof(T) == 1) p += (w4[i] & M) + ((w4[i] >> SH) & M);
      else acc += (unsigned long long)((w4[i] & M) + (w4[i] >> SH));
    }
    if constexpr (sizeof(T) == 1) acc += (unsigned long long)((p & 0xffffu) + (p >> 16));
  }
  acc = wave_sum_u64(acc);
  acc = __shfl(acc, 0, 64);
  const uint32_t a = (uint32_t)rint((double)acc / (double)nchan);
  constexpr uint32_t H = sizeof(T) == 1 ? 0x80808080u : 0x80008000u;
  const uint32_t ar = sizeof(T) == 1 ? (a & 0xffu) * 0x01010101u : (a & 0xffffu) * 0x00010001u;
  uint4* orow = reinterpret_cast<uint4*>(out + s * ld_out);
  for (int64_t v = lane; v < nv; v += 64) {
    const uint4 q = row[v];
    uint4 r;
    r.x = ((q.x | H) - (ar & ~H)) ^ ((q.x ^ ~ar) & H);
    r.y = ((q.y | H) - (ar & ~H)) ^ ((q.y ^ ~ar) & H);
    r.z = ((q.z | H) - (ar & ~H)) ^ ((q.z ^ ~ar) & H);
    r.w = ((q.w | H) - (ar & ~H)) ^ ((q.w ^ ~ar) & H);
    orow[v] = r;
  }
}

// one thread per spectrum, channel-major [nchan][nspec] (Spectra layout)
template <typename T>
__global__ __launch_bounds__(256) void k_zero_dm_cm(const T* __restrict__ in, int64_t nspec,
                                                    int64_t nchan, int64_t ld,
                                                    T* __restrict__ out, int64_t ld_out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= nspec) return;
  double mean;
  if constexpr (sizeof(T) == 4) {
    double acc = 0.0;
    for (int64_t c = 0; c < nchan; ++c) acc += (double)in[c * ld + t];
    mean = (double)((float)acc / (float)nchan);
  } else {
    unsigned long long acc = 0;
    for (int64_t c = 0; c < nchan; ++c) acc += (unsigned long long)in[c * ld + t];
    mean = (double)acc / (double)nchan;
  }
  for (int64_t c = 0; c < nchan; ++c) out[c * ld_out + t] = zd_apply<T>(in[c * ld + t], mean);
}

// ---------------------------------------------------------------- waterfaller post-chain
// (Spectra.scaled / scaled2 / masked / smooth, formats/spectra.py:140-303)

// Per-channel population std (two passes in float64) or min / max.
__global__ __launch_bounds__(256) void k_channel_std(const float* __restrict__ x, int64_t N,
                                                     int64_t ld, float* __restrict__ out) {
  __shared__ double part[4];
  __shared__ double mean_s;
  const float* row = x + (int64_t)blockIdx.x * ld;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < N; i += 256) s += (double)row[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) mean_s = ((part[0] + part[1]) + (part[2] + part[3])) / (double)N;
  __syncthreads();
  const double m = mean_s;
  double q = 0.0;
  for (int64_t i = threadIdx.x; i < N; i += 256) {
    const double d = (double)row[i] - m;
    q += d * d;
  }
  q = wave_sum(q);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (float)sqrt(((part[0] + part[1]) + (part[2] + part[3])) / (double)N);
}

__device__ __forceinline__ float wave_minmax(float v, bool want_max) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_down(v, o, 64);
    v = want_max ? fmaxf(v, u) : fminf(v, u);
  }
  return v;
}

__global__ __launch_bounds__(256) void k_channel_minmax(const float* __restrict__ x, int64_t N,
                                                        int64_t ld, int want_max,
                                                        float* __restrict__ out) {
  __shared__ float part[4];
  const float* row = x + (int64_t)blockIdx.x * ld;
  float v = want_max ? -INFINITY : INFINITY;
  for (int64_t i = threadIdx.x; i < N; i += 256) v = want_max ? fmaxf(v, row[i]) : fminf(v, row[i]);
  v = wave_minmax(v, want_max);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = part[0];
    for (int i = 1; i < 4; ++i) r = want_max ? fmaxf(r, part[i]) : fminf(r, part[i]);
    out[blockIdx.x] = r;
  }
}

// Global statistics of a [C][N] array: fixed grid (kGlobBlocks x 256), every
// partial in float64, combined in a fixed order (deterministic).
constexpr int kGlobBlocks = 1024;

__global__ __launch_bounds__(256) void k_global_partial(const float* __restrict__ x, int64_t C,
                                                        int64_t N, int64_t ld, int pass,
                                                        const double* __restrict__ fin,
                                                        double* __restrict__ part) {
  __shared__ double ps[4][3];
  const int64_t total = C * N;
  const double m = pass ? fin[0] : 0.0;
  double a = 0.0, mn = INFINITY, mx = -INFINITY;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)kGlobBlocks * 256) {
    const double v = (double)x[(i / N) * ld + (i % N)];
    if (pass) {
      a += (v - m) * (v - m);
    } else {
      a += v;
      mn = fmin(mn, v);
      mx = fmax(mx, v);
    }
  }
  a = wave_sum(a);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fmin(mn, __shfl_down(mn, o, 64));
    mx = fmax(mx, __shfl_down(mx, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    ps[threadIdx.x >> 6][0] = a;
    ps[threadIdx.x >> 6][1] = mn;
    ps[threadIdx.x >> 6][2] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x * 3 + 0] = (ps[0][0] + ps[1][0]) + (ps[2][0] + ps[3][0]);
    part[blockIdx.x * 3 + 1] = fmin(fmin(ps[0][1], ps[1][1]), fmin(ps[2][1], ps[3][1]));
    part[blockIdx.x * 3 + 2] = fmax(fmax(ps[0][2], ps[1][2]), fmax(ps[2][2], ps[3][2]));
  }
}

// pass 0: fin[0] = mean, out[0] = mean, out[2] = min, out[3] = max;
// pass 1: out[1] = population std
__global__ __launch_bounds__(256) void k_global_reduce(const double* __restrict__ part, int pass,
                                                       int64_t total, double* __restrict__ fin,
                                                       float* __restrict__ out) {
  __shared__ double ps[4][3];
  double a = 0.0, mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < kGlobBlocks; i += 256) {
    a += part[i * 3 + 0];
    mn = fmin(mn, part[i * 3 + 1]);
    mx = fmax(mx, part[i * 3 + 2]);
  }
  a = wave_sum(a);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fmin(mn, __shfl_down(mn, o, 64));
    mx = fmax(mx, __shfl_down(mx, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    ps[threadIdx.x >> 6][0] = a;
    ps[threadIdx.x >> 6][1] = mn;
    ps[threadIdx.x >> 6][2] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double s = (ps[0][0] + ps[1][0]) + (ps[2][0] + ps[3][0]);
    if (pass == 0) {
      fin[0] = s / (double)total;
      out[0] = (float)(s / (double)total);
      out[2] = (float)fmin(fmin(ps[0][1], ps[1][1]), fmin(ps[2][1], ps[3][1]));
      out[3] = (float)fmax(fmax(ps[0][2], ps[1][2]), fmax(ps[2][2], ps[3][2]));
    } else {
      out[1] = (float)sqrt(s / (double)total);
    }
  }
}

// out[c][t] = (x[c][t] - sub[c * sub_inc]) / div[c * div_inc]  (float64 arithmetic)
__global__ __launch_bounds__(256) void k_scale_rows(const float* __restrict__ x, int64_t N,
                                                    int64_t ld, const float* __restrict__ sub,
                                                    int64_t sub_inc, const float* __restrict__ dv,
                                                    int64_t div_inc, float* __restrict__ out,
                                                    int64_t ld_out, int64_t tiles) {
  const int64_t c = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const double s = (double)sub[c * sub_inc], d = (double)dv[c * div_inc];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t t = tile * 1024 + k * 256 + threadIdx.x;
    if (t < N) out[c * ld_out + t] = (float)(((double)x[c * ld + t] - s) / d);
  }
}

// out = mask ? vals[c] : x
__global__ __launch_bounds__(256) void k_masked_fill(const float* __restrict__ x, int64_t N,
                                                     int64_t ld, const uint8_t* __restrict__ mask,
                                                     int64_t ld_mask, const float* __restrict__ vals,
                                                     float* __restrict__ out, int64_t ld_out,
                                                     int64_t tiles) {
  const int64_t c = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const float v = vals[c];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t t = tile * 1024 + k * 256 + threadIdx.x;
    if (t < N) out[c * ld_out + t] = mask[c * ld_mask + t] ? v : x[c * ld + t];
  }
}

// Boxcar smooth: out[c][t] = (1/sqrt(w)) * sum_{j = t - w/2}^{t + (w-1)/2} P(c, j)
// with P the padded channel (value pad, or wrap for PDD_PAD_ROTATE).  The
// window of one 4096-output tile is staged in LDS (w <= kSmoothLds - 1023);
// sums in float64.
constexpr int kSmoothLds = 8192;

__device__ __forceinline__ float smooth_src(const float* row, int64_t j, int64_t N, int pad_mode,
                                            float pad) {
  if (j >= 0 && j < N) return row[j];
  if (pad_mode == PDD_PAD_ROTATE) {
    int64_t r = j % N;
    return row[r < 0 ? r + N : r];
  }
  return pad;
}

constexpr int kSmoothOpt = 16;                 // outputs per thread
constexpr int kSmoothTile = 256 * kSmoothOpt;  // outputs per workgroup
// LDS slot of window sample j: one pad float after every 16, so the lanes'
// sliding reads (16 samples apart) fall in distinct banks (was 8-way)
__device__ __forceinline__ int64_t smooth_slot(int64_t j) { return j + (j >> 4); }
__global__ __launch_bounds__(256) void k_smooth(const float* __restrict__ x, int64_t N, int64_t ld,
                                                int64_t w, int pad_mode,
                                                const float* __restrict__ padvals,
                                                float* __restrict__ out, int64_t ld_out,
                                                int64_t tiles) {
  extern __shared__ float win[];  // kSmoothTile + w floats (sized by the launcher)
  const int64_t c = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const float* row = x + c * ld;
  const float pad = (pad_mode == PDD_PAD_VALUE) ? padvals[c] : 0.f;
  const int64_t t0 = tile * kSmoothTile;
  const int64_t j0 = t0 - w / 2;
  const int64_t nw = kSmoothTile + w - 1;
  {
    // all of a thread's window loads in flight before its LDS stores
    float v[kSmoothOpt];
#pragma unroll
    for (int q = 0; q < kSmoothOpt; ++q)
      v[q] = smooth_src(row, j0 + q * 256 + threadIdx.x, N, pad_mode, pad);
#pragma unroll
    for (int q = 0; q < kSmoothOpt; ++q) win[smooth_slot(q * 256 + threadIdx.x)] = v[q];
    for (int64_t i = kSmoothTile + threadIdx.x; i < nw; i += 256)
      win[smooth_slot(i)] = smooth_src(row, j0 + i, N, pad_mode, pad);
    if (threadIdx.x == 0) win[smooth_slot(nw)] = 0.f;  // the spare slot the sliding window reads last
  }
  __syncthreads();
  const double k = 1.0 / sqrt((double)w);
  // thread = kSmoothOpt consecutive outputs; each window summed from its first
  // sample in order (the arithmetic of one output is unchanged), the windows
  // share a sliding register window: w + kSmoothOpt - 1 LDS reads
  const int o = kSmoothOpt * threadIdx.x;
  float r[kSmoothOpt];
  double sm[kSmoothOpt];
#pragma unroll
  for (int q = 0; q < kSmoothOpt; ++q) {
    r[q] = win[smooth_slot(o + q)];
    sm[q] = 0.0;
  }
  for (int64_t i = 0; i < w; ++i) {
#pragma unroll
    for (int q = 0; q < kSmoothOpt; ++q) sm[q] += (double)r[q];
#pragma unroll
    for (int q = 0; q < kSmoothOpt - 1; ++q) r[q] = r[q + 1];
    r[kSmoothOpt - 1] = win[smooth_slot(o + kSmoothOpt + i)];
  }
  // results through the LDS window (free after the barrier) so every store
  // instruction writes 1 KiB of consecutive outputs (a thread's own 16
  // contiguous outputs would spread each instruction over 4 KiB)
  float* orow = out + c * ld_out;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kSmoothOpt; ++q) win[smooth_slot(o + q)] = (float)(sm[q] * k);
  __syncthreads();
  const bool vec = (((uintptr_t)(orow + t0)) & 15) == 0;
#pragma unroll
  for (int q = 0; q < kSmoothOpt / 4; ++q) {
    const int i0 = q * 1024 + 4 * threadIdx.x;
    const int64_t t = t0 + i0;
    const float a = win[smooth_slot(i0)], b = win[smooth_slot(i0 + 1)],
                d = win[smooth_slot(i0 + 2)], e = win[smooth_slot(i0 + 3)];
    if (vec && t + 4 <= N) {
      *reinterpret_cast<float4*>(orow + t) = make_float4(a, b, d, e);
    } else {
      if (t < N) orow[t] = a;
      if (t + 1 < N) orow[t + 1] = b;
      if (t + 2 < N) orow[t + 2] = d;
      if (t + 3 < N) orow[t + 3] = e;
    }
  }
}


// ---------------------------------------------------------------- streaming prologue
// Per-spectrum channel mean (float64) of a time-major block.
template <typename T>
__global__ __launch_bounds__(256) void k_spectrum_mean(const T* __restrict__ in, int64_t nspec,
                                                       int64_t nchan, int64_t ld,
                                                       double* __restrict__ mean) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= nspec) return;
  const T* row = in + s * ld;
  double acc = 0.0;
  for (int64_t c = lane; c < nchan; c += 64) acc += (double)row[c];
  acc = wave_sum(acc);
  if (lane == 0) mean[s] = acc / (double)nchan;
}

// Fused corner turn + zero-DM (float mode) + downsample:
//   out[c][j] = sum_{k < f} (x[j*f + k][c] - mean[j*f + k]),   mean = 0 if !mean
// through a 64-spectrum x 64-channel LDS tile (f divides 64).
template <typename T>
__global__ __launch_bounds__(256) void k_zdm_ds(const T* __restrict__ in, int64_t nspec,
                                                int64_t nchan, int64_t ld,
                                                const double* __restrict__ mean, int f,
                                                float* __restrict__ out, int64_t ld_out,
                                                int64_t tiles_c) {
  __shared__ float tile[64][65];
  const int64_t tt = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int64_t t0 = tt * 64, c0 = tc * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int64_t t = t0 + i, c = c0 + tx;
    float v = 0.f;
    if (t < nspec && c < nchan) v = (float)((double)in[t * ld + c] - (mean ? mean[t] : 0.0));
    tile[i][tx] = v;
  }
  __syncthreads();
  const int per = 64 / f;  // outputs per channel in this tile
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i;
    if (c >= nchan || tx >= per) continue;
    const int64_t j = t0 / f + tx;
    if ((j + 1) * f > nspec) continue;  // trailing partial group dropped (downsample trim)
    float acc = 0.f;
    for (int k = 0; k < f; ++k) acc += tile[tx * f + k][i];
    out[c * ld_out + j] = acc;
  }
}

// Vectorised streaming prologue for 16-B aligned rows (nchan*sizeof(T) a
// multiple of 16).  Spectrum means: one wave per spectrum, 16-byte loads,
// exact integer (8/16-bit) or float64 (float32) sums.
template <typename T>
__global__ __launch_bounds__(256) void k_spectrum_mean_vec(const T* __restrict__ in, int64_t nspec,
                                                           int64_t nchan, int64_t ld,
                                                           double* __restrict__ mean) {
  constexpr int VEC = 16 / sizeof(T);
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= nspec) return;
  const uint4* row = reinterpret_cast<const uint4*>(in + s * ld);
  const int64_t nv = nchan / VEC;
  double acc = 0.0;
  for (int64_t v = lane; v < nv; v += 64) {
    union { uint4 q; T e[VEC]; } u;
    u.q = row[v];
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc += (double)u.e[e];
    } else {
      uint32_t p = 0;  // <= 8 x 65535: exact in 32 bits
#pragma unroll
      for (int e = 0; e < VEC; ++e) p += (uint32_t)u.e[e];
      acc += (double)p;
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) mean[s] = acc / (double)nchan;
}

// Fused corner turn + zero-DM (float mode) + downsample, one block = 64
// outputs (64*f spectra) x 8*VEC channels: each thread sums f 16-byte rows of
// VEC channels (in the order of k_zdm_ds) into the LDS tile, then every wave
// writes whole 64-output channel rows.
template <typename T>
__global__ __launch_bounds__(256) void k_zdm_ds_vec(const T* __restrict__ in, int64_t nspec,
                                                    int64_t nchan, int64_t ld,
                                                    const double* __restrict__ mean, int f,
                                                    float* __restrict__ out, int64_t ld_out,
                                                    int64_t nout, int64_t tiles_c) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int TC = 8 * VEC;
  __shared__ float tile[TC][65];
  const int64_t tj = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int64_t j0 = tj * 64, c0 = tc * TC;
  const int seg = threadIdx.x & 7, r0 = threadIdx.x >> 3;
  const int64_t c = c0 + seg * VEC;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int jl = r0 + 32 * pass;
    const int64_t j = j0 + jl;
    float acc[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = 0.f;
    if (j < nout && c < nchan) {
      for (int k = 0; k < f; ++k) {
        const int64_t t = j * f + k;
        union { uint4 q; T e[VEC]; } u;
        u.q = *reinterpret_cast<const uint4*>(in + t * ld + c);
        const double m = mean ? mean[t] : 0.0;
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] += (float)((double)u.e[e] - m);
      }
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) tile[seg * VEC + e][jl] = acc[e];
  }
  __syncthreads();
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t j = j0 + tx;
#pragma unroll 4
  for (int i = ty; i < TC; i += 4) {
    const int64_t cc = c0 + i;
    if (j < nout && cc < nchan) out[cc * ld_out + j] = tile[i][tx];
  }
}

// 8-bit prologue of the exact 16-bit sweep: zero-DM (bin/zero_dm_filter.py:
// 30-39, the spectrum's channel mean rounded half-to-even as np.round) +
// downsample (formats/spectra.py:329-351, co-added) + corner turn, 16-B
// aligned rows:
//   out[c][j] = offset + sum_{k < f} z(x[j f + k][c], m[j f + k])
// as uint16, z = x (MODE 0: no filter), x - m as a signed value (MODE 1:
// integer zero-DM without the uint8 wrap) or (x - m) mod 256 (MODE 2: the
// reference's uint8 arithmetic).  Integer math throughout (exact); the tile
// order is that of k_zdm_ds_vec.
template <int MODE>
__global__ __launch_bounds__(256) void k_zdm_int_ds_vec(const uint8_t* __restrict__ in,
                                                        int64_t nchan, int64_t ld,
                                                        const double* __restrict__ mean, int f,
                                                        uint16_t* __restrict__ out, int64_t ld_out,
                                                        int64_t nout, int64_t tiles_c, int offset) {
  constexpr int VEC = 16;
  constexpr int TC = 8 * VEC;
  __shared__ int tile[TC][65];
  const int64_t tj = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int64_t j0 = tj * 64, c0 = tc * TC;
  const int seg = threadIdx.x & 7, r0 = threadIdx.x >> 3;
  const int64_t c = c0 + seg * VEC;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int jl = r0 + 32 * pass;
    const int64_t j = j0 + jl;
    int acc[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = offset;
    if (j < nout && c < nchan) {
      for (int k = 0; k < f; ++k) {
        const int64_t t = j * f + k;
        union { uint4 q; uint8_t e[VEC]; } u;
        u.q = *reinterpret_cast<const uint4*>(in + t * ld + c);
        const int m = MODE ? (int)rint(mean[t]) : 0;
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const int z = (int)u.e[e] - m;
          acc[e] += MODE == 2 ? (z & 255) : z;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) tile[seg * VEC + e][jl] = acc[e];
  }
  __syncthreads();
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t j = j0 + tx;
#pragma unroll 4
  for (int i = ty; i < TC; i += 4) {
    const int64_t cc = c0 + i;
    if (j < nout && cc < nchan) out[cc * ld_out + j] = (uint16_t)tile[i][tx];
  }
}

static int grid_1d(int64_t n, int per_block = 256) {
  int64_t g = cdiv(n, per_block);
  if (g > 2048 * 8) g = 2048 * 8;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace pdd

using namespace pdd;

extern "C" {

int pdd_version(void) { return 1; }

// PDD_SRC_DIGEST: set by the build (__graft_entry__.build, pypulsar_amd/_digest.py)
// to the digest of the sources and flags; the marker lets build() read it
// from the file without loading the library
#ifndef PDD_SRC_DIGEST
#define PDD_SRC_DIGEST "unstamped"
#endif
static const char kPddDigest[] = "pdd-src-digest:" PDD_SRC_DIGEST;
const char* pdd_source_digest(void) { return kPddDigest + 15; }

const char* pdd_last_error(void) { return pdd::g_err; }

int pdd_scratch_release(void) {
  // Every entry is freed and dropped even when a HIP call fails part way (a
  // kept entry would hand out a freed pointer); the first error is returned.
  std::lock_guard<std::mutex> lock(pdd::g_scratch_mu);
  hipError_t first = hipSuccess;
  auto note = [&](hipError_t e) { if (first == hipSuccess && e != hipSuccess) first = e; };
  int cur = 0;
  note(hipGetDevice(&cur));
  for (auto& b : pdd::g_scratch) {
    if (!b.ptr) continue;
    note(hipSetDevice(b.dev));
    note(hipDeviceSynchronize());
    note(hipFree(b.ptr));
    b.ptr = nullptr;
  }
  pdd::g_scratch.clear();
  note(hipSetDevice(cur));
  if (first != hipSuccess) {
    pdd::set_error("pdd_scratch_release: %s", hipGetErrorString(first));
    return -3;
  }
  return 0;
}

int pdd_sync(void* stream) {
  PDD_HIP(hipStreamSynchronize(as_stream(stream)));
  return 0;
}

int pdd_corner_turn(const void* in, int in_dtype, int64_t nspec, int64_t nchan, int64_t ld_in,
                    void* out, int out_dtype, int64_t ld_out, void* stream) {
  PDD_REQUIRE(in && out, "pdd_corner_turn: null pointer");
  PDD_REQUIRE(nspec >= 0 && nchan >= 0 && ld_in >= nchan && ld_out >= nspec,
              "pdd_corner_turn: bad shape nspec=%lld nchan=%lld ld_in=%lld ld_out=%lld",
              (long long)nspec, (long long)nchan, (long long)ld_in, (long long)ld_out);
  if (nspec == 0 || nchan == 0) return 0;
  const int64_t tiles_c = cdiv(nchan, 64);
  const int64_t blocks = cdiv(nspec, 64) * tiles_c;
  PDD_REQUIRE(blocks < (1ll << 31), "pdd_corner_turn: too large");
  hipStream_t s = as_stream(stream);
#define CT(IT, OT)                                                                           \
  k_corner_turn<IT, OT><<<(unsigned)blocks, 256, 0, s>>>((const IT*)in, nspec, nchan, ld_in, \
                                                         (OT*)out, ld_out, tiles_c)
  const int64_t es = in_dtype == PDD_U8 ? 1 : (in_dtype == PDD_U16 ? 2 : 4);
  if (out_dtype == PDD_F32 && (uintptr_t)in % 16 == 0 && (ld_in * es) % 16 == 0 &&
      (nchan * es) % 16 == 0 && (in_dtype == PDD_U8 || in_dtype == PDD_U16 || in_dtype == PDD_F32)) {
    const int64_t tcv = cdiv(nchan, 8 * (16 / es));
    const int64_t bv = cdiv(nspec, 64) * tcv;
#define CV(IT)                                                                                \
  k_corner_turn_vec<IT><<<(unsigned)bv, 256, 0, s>>>((const IT*)in, nspec, nchan, ld_in,       \
                                                    (float*)out, ld_out, tcv)
    if (in_dtype == PDD_U8) CV(uint8_t);
    else if (in_dtype == PDD_U16) CV(uint16_t);
    else CV(float);
#undef CV
  } else if (out_dtype == PDD_F32) {
    if (in_dtype == PDD_U8) CT(uint8_t, float);
    else if (in_dtype == PDD_U16) CT(uint16_t, float);
    else if (in_dtype == PDD_F32) CT(float, float);
    else PDD_REQUIRE(false, "pdd_corner_turn: bad in_dtype %d", in_dtype);
  } else {
    PDD_REQUIRE(out_dtype == in_dtype, "pdd_corner_turn: out dtype must be F32 or the input dtype");
    if (in_dtype == PDD_U8 && (uintptr_t)in % 16 == 0 && (uintptr_t)out % 16 == 0 &&
        ld_in % 16 == 0 && nchan % 16 == 0 && ld_out % 16 == 0) {
      // (128 x 128 tiles: 1.94 -> 1.63 ms per 2^20 x 4096 batch against the
      // round-4 128 x 64 tiles, which read half lines of their input rows)
      const int64_t tcb = cdiv(nchan, 128);
      const int64_t bb = cdiv(nspec, 128) * tcb;
      PDD_REQUIRE(bb < (1ll << 31), "pdd_corner_turn: too large");
      k_corner_turn_b8w<<<(unsigned)bb, 256, 0, s>>>((const uint8_t*)in, nspec, nchan, ld_in,
                                                     (uint8_t*)out, ld_out, tcb);
    } else if (in_dtype == PDD_U8) CT(uint8_t, uint8_t);
    else if (in_dtype == PDD_U16) CT(uint16_t, uint16_t);
    else PDD_REQUIRE(false, "pdd_corner_turn: bad in_dtype %d", in_dtype);
  }
#undef CT
  PDD_LAUNCHED();
  return 0;
}

int pdd_convert_f32(const void* in, int in_dtype, int64_t rows, int64_t cols, int64_t ld_in,
                    float* out, int64_t ld_out, void* stream) {
  PDD_REQUIRE(in && out, "pdd_convert_f32: null pointer");
  PDD_REQUIRE(rows >= 0 && cols >= 0 && ld_in >= cols && ld_out >= cols,
              "pdd_convert_f32: bad shape");
  if (rows == 0 || cols == 0) return 0;
  const int g = grid_1d(rows * cols);
  hipStream_t s = as_stream(stream);
  if (in_dtype == PDD_U8)
    k_convert<uint8_t><<<g, 256, 0, s>>>((const uint8_t*)in, rows, cols, ld_in, out, ld_out);
  else if (in_dtype == PDD_U16)
    k_convert<uint16_t><<<g, 256, 0, s>>>((const uint16_t*)in, rows, cols, ld_in, out, ld_out);
  else if (in_dtype == PDD_F32)
    k_convert<float><<<g, 256, 0, s>>>((const float*)in, rows, cols, ld_in, out, ld_out);
  else
    PDD_REQUIRE(false, "pdd_convert_f32: bad dtype %d", in_dtype);
  PDD_LAUNCHED();
  return 0;
}

int pdd_channel_stats(const float* x, int64_t C, int64_t N, int64_t ld, int stat, float* out,
                      void* stream) {
  PDD_REQUIRE(x && out, "pdd_channel_stats: null pointer");
  PDD_REQUIRE(C >= 0 && N > 0 && ld >= N, "pdd_channel_stats: bad shape");
  PDD_REQUIRE(C < (1ll << 31), "pdd_channel_stats: too many channels");
  if (C == 0) return 0;
  hipStream_t s = as_stream(stream);
  if (stat == PDD_STAT_MEAN)
    k_channel_mean<<<(unsigned)C, 256, 0, s>>>(x, N, ld, out);
  else if (stat == PDD_STAT_MEDIAN)
    k_channel_median<<<(unsigned)C, 256, 0, s>>>(x, N, ld, out);
  else if (stat == PDD_STAT_STD)
    k_channel_std<<<(unsigned)C, 256, 0, s>>>(x, N, ld, out);
  else if (stat == PDD_STAT_MIN || stat == PDD_STAT_MAX)
    k_channel_minmax<<<(unsigned)C, 256, 0, s>>>(x, N, ld, stat == PDD_STAT_MAX, out);
  else
    PDD_REQUIRE(false, "pdd_channel_stats: bad stat %d", stat);
  PDD_LAUNCHED();
  return 0;
}

int pdd_shift_pad(const float* x, int64_t C, int64_t N, int64_t ld, const int32_t* bins,
                  int pad_mode, const float* padvals, float* out, int64_t ld_out, int64_t n_out,
                  void* stream) {
  PDD_REQUIRE(x && out && bins, "pdd_shift_pad: null pointer");
  PDD_REQUIRE(x != out, "pdd_shift_pad: out must not alias x");
  PDD_REQUIRE(C >= 0 && N > 0 && ld >= N && n_out >= 0 && ld_out >= n_out,
              "pdd_shift_pad: bad shape");
  PDD_REQUIRE(pad_mode == PDD_PAD_ROTATE || (pad_mode == PDD_PAD_VALUE && padvals),
              "pdd_shift_pad: bad pad mode %d", pad_mode);
  if (C == 0 || n_out == 0) return 0;
  const int64_t tiles = cdiv(n_out, 1024);
  PDD_REQUIRE(C * tiles < (1ll << 31), "pdd_shift_pad: too large");
  k_shift_pad<<<(unsigned)(C * tiles), 256, 0, as_stream(stream)>>>(x, N, ld, bins, pad_mode,
                                                                    padvals, out, ld_out, n_out,
                                                                    tiles);
  PDD_LAUNCHED();
  return 0;
}

int pdd_shift_group_sum(const float* x, int64_t C, int64_t N, int64_t ld, const int32_t* bins,
                        int pad_mode, const float* padvals, int64_t nsub, float* out,
                        int64_t ld_out, int64_t n_out, void* stream) {
  PDD_REQUIRE(x && out, "pdd_shift_group_sum: null pointer");
  PDD_REQUIRE(nsub > 0 && C % nsub == 0, "pdd_shift_group_sum: nsub must divide C");
  PDD_REQUIRE(C >= 0 && N > 0 && ld >= N && n_out >= 0 && ld_out >= n_out,
              "pdd_shift_group_sum: bad shape");
  PDD_REQUIRE(pad_mode == PDD_PAD_ROTATE || pad_mode == PDD_PAD_VALUE,
              "pdd_shift_group_sum: bad pad mode %d", pad_mode);
  if (C == 0 || n_out == 0) return 0;
  const int64_t tiles = cdiv(n_out, 256);
  const int64_t cps = C / nsub;
  // channel slices: enough workgroups to fill 256 CUs with 8-wave blocks
  int64_t csplit = std::max<int64_t>(1, std::min<int64_t>(cdiv(2048, nsub * tiles),
                                                          cps / (4 * kGsWaves)));
  PDD_REQUIRE(csplit * nsub * tiles < (1ll << 31), "pdd_shift_group_sum: too large");
  hipStream_t st = as_stream(stream);
  double* part = nullptr;
  if (csplit > 1) {
    part = static_cast<double*>(
        scratch(st, kScratchPartial, (size_t)(csplit * nsub * n_out) * sizeof(double)));
    if (!part) return -2;
  }
  k_shift_group_sum<<<(unsigned)(csplit * nsub * tiles), kGsWaves * 64, 0, st>>>(
      x, N, ld, bins, pad_mode, padvals, cps, csplit, out, part, ld_out, n_out, tiles, nsub);
  if (csplit > 1) {
    k_group_sum_reduce<<<(unsigned)cdiv(nsub * n_out, 256), 256, 0, st>>>(part, csplit, nsub,
                                                                          n_out, out, ld_out);
  }
  PDD_LAUNCHED();
  return 0;
}

int pdd_downsample(const float* x, int64_t C, int64_t N, int64_t ld, int64_t factor, float* out,
                   int64_t ld_out, void* stream) {
  PDD_REQUIRE(x && out, "pdd_downsample: null pointer");
  PDD_REQUIRE(factor >= 1 && C >= 0 && N >= 0 && ld >= N, "pdd_downsample: bad shape");
  const int64_t nout = N / factor;
  PDD_REQUIRE(ld_out >= nout, "pdd_downsample: ld_out too small");
  if (C == 0 || nout == 0) return 0;
  const int64_t tiles = cdiv(nout, 256);
  PDD_REQUIRE(C * tiles < (1ll << 31), "pdd_downsample: too large");
  if (factor % 4 == 0 && (uintptr_t)x % 16 == 0 && ld % 4 == 0)
    k_downsample_v4<<<(unsigned)(C * tiles), 256, 0, as_stream(stream)>>>(x, ld, factor, nout,
                                                                          out, ld_out, tiles);
  else
    k_downsample<<<(unsigned)(C * tiles), 256, 0, as_stream(stream)>>>(x, ld, factor, nout, out,
                                                                       ld_out, tiles);
  PDD_LAUNCHED();
  return 0;
}

}  // extern "C"

template <typename OutT>
static int downsample_u8(const uint8_t* x, int64_t C, int64_t N, int64_t ld, int64_t factor,
                         OutT* out, int64_t ld_out, void* stream) {
  PDD_REQUIRE(x && out, "pdd_downsample_u8: null pointer");
  PDD_REQUIRE(factor >= 1 && C >= 0 && N >= 0 && ld >= N, "pdd_downsample_u8: bad shape");
  const int64_t nout = N / factor;
  PDD_REQUIRE(ld_out >= nout, "pdd_downsample_u8: ld_out too small");
  if (C == 0 || nout == 0) return 0;
  hipStream_t s = as_stream(stream);
  const bool vec = (16 % factor == 0) && ((uintptr_t)x % 16 == 0) && (ld % 16 == 0);
  if (vec) {
    const int64_t nvec = cdiv(nout * factor, 16);  // the last vector may read past nout*factor
    PDD_REQUIRE(nvec * 16 <= ld, "pdd_downsample_u8: row padding");
    const int64_t tiles = cdiv(nvec, 256);
    PDD_REQUIRE(C * tiles < (1ll << 31), "pdd_downsample_u8: too large");
    const int per = (int)(16 / factor);
    const int64_t vb = sizeof(OutT) == 4 ? (per >= 4 ? 16 : 8) : 8;  // vector store bytes
    const bool vstore = (uintptr_t)out % vb == 0 && (ld_out * (int64_t)sizeof(OutT)) % vb == 0 &&
                        per >= (sizeof(OutT) == 4 ? 2 : 4);
#define DV(F_)                                                                                 \
  k_downsample_u8v<F_, OutT><<<(unsigned)(C * tiles), 256, 0, s>>>(x, ld, nvec, out, ld_out, nout, \
                                                                   tiles, vstore)
    if (factor == 1) DV(1);
    else if (factor == 2) DV(2);
    else if (factor == 4) DV(4);
    else if (factor == 8) DV(8);
    else DV(16);
#undef DV
  } else {
    const int64_t tiles = cdiv(nout, 256);
    PDD_REQUIRE(C * tiles < (1ll << 31), "pdd_downsample_u8: too large");
    k_downsample_u8<OutT><<<(unsigned)(C * tiles), 256, 0, s>>>(x, ld, factor, nout, out, ld_out,
                                                               tiles);
  }
  PDD_LAUNCHED();
  return 0;
}

extern "C" {

int pdd_downsample_u8(const uint8_t* x, int64_t C, int64_t N, int64_t ld, int64_t factor,
                      float* out, int64_t ld_out, void* stream) {
  return downsample_u8<float>(x, C, N, ld, factor, out, ld_out, stream);
}

int pdd_downsample_u8_u16(const uint8_t* x, int64_t C, int64_t N, int64_t ld, int64_t factor,
                          uint16_t* out, int64_t ld_out, void* stream) {
  PDD_REQUIRE(factor >= 1 && factor <= 4, "pdd_downsample_u8_u16: factor must be 1..4 (sums <= 1020)");
  return downsample_u8<uint16_t>(x, C, N, ld, factor, out, ld_out, stream);
}

int pdd_zero_dm(const void* in, int dtype, int64_t nspec, int64_t nchan, int64_t ld, int layout,
                void* out, int64_t ld_out, void* stream) {
  PDD_REQUIRE(in && out, "pdd_zero_dm: null pointer");
  PDD_REQUIRE(nspec >= 0 && nchan > 0, "pdd_zero_dm: bad shape");
  if (nspec == 0) return 0;
  hipStream_t s = as_stream(stream);
  if (layout == PDD_LAYOUT_TIME_MAJOR) {
    PDD_REQUIRE(ld >= nchan && ld_out >= nchan, "pdd_zero_dm: bad ld");
    const int64_t g = cdiv(nspec, 4);
    PDD_REQUIRE(g < (1ll << 31), "pdd_zero_dm: too large");
#define ZT(T) k_zero_dm_tm<T><<<(unsigned)g, 256, 0, s>>>((const T*)in, nspec, nchan, ld, (T*)out, ld_out)
#define ZV(T) k_zero_dm_tm_vec<T><<<(unsigned)g, 256, 0, s>>>((const T*)in, nspec, nchan, ld, (T*)out, ld_out)
    const int64_t es = dtype == PDD_U8 ? 1 : (dtype == PDD_U16 ? 2 : 4);
    const bool vec = es < 4 && ((uintptr_t)in | (uintptr_t)out) % 16 == 0 &&
                     (nchan * es) % 16 == 0 && (ld * es) % 16 == 0 && (ld_out * es) % 16 == 0;
    if (dtype == PDD_U8 && vec) ZV(uint8_t);
    else if (dtype == PDD_U16 && vec) ZV(uint16_t);
    else if (dtype == PDD_U8) ZT(uint8_t);
    else if (dtype == PDD_U16) ZT(uint16_t);
    else if (dtype == PDD_F32) ZT(float);
    else PDD_REQUIRE(false, "pdd_zero_dm: bad dtype %d", dtype);
#undef ZT
#undef ZV
  } else if (layout == PDD_LAYOUT_CHAN_MAJOR) {
    PDD_REQUIRE(ld >= nspec && ld_out >= nspec, "pdd_zero_dm: bad ld");
    const int64_t g = cdiv(nspec, 256);
#define ZC(T) k_zero_dm_cm<T><<<(unsigned)g, 256, 0, s>>>((const T*)in, nspec, nchan, ld, (T*)out, ld_out)
    if (dtype == PDD_U8) ZC(uint8_t);
    else if (dtype == PDD_U16) ZC(uint16_t);
    else if (dtype == PDD_F32) ZC(float);
    else PDD_REQUIRE(false, "pdd_zero_dm: bad dtype %d", dtype);
#undef ZC
  } else {
    PDD_REQUIRE(false, "pdd_zero_dm: bad layout %d", layout);
  }
  PDD_LAUNCHED();
  return 0;
}

int pdd_global_stats(const float* x, int64_t C, int64_t N, int64_t ld, float* out4, void* stream) {
  PDD_REQUIRE(x && out4, "pdd_global_stats: null pointer");
  PDD_REQUIRE(C > 0 && N > 0 && ld >= N, "pdd_global_stats: bad shape");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(scratch(s, kScratchSmall, (kGlobBlocks * 3 + 1) * sizeof(double)));
  if (!part) return -2;
  double* fin = part + kGlobBlocks * 3;
  k_global_partial<<<kGlobBlocks, 256, 0, s>>>(x, C, N, ld, 0, fin, part);
  k_global_reduce<<<1, 256, 0, s>>>(part, 0, C * N, fin, out4);
  k_global_partial<<<kGlobBlocks, 256, 0, s>>>(x, C, N, ld, 1, fin, part);
  k_global_reduce<<<1, 256, 0, s>>>(part, 1, C * N, fin, out4);
  const hipError_t e = hipGetLastError();
  PDD_REQUIRE(e == hipSuccess, "pdd_global_stats: launch failed: %s", hipGetErrorString(e));
  return 0;
}

int pdd_scale_rows(const float* x, int64_t C, int64_t N, int64_t ld, const float* sub,
                   int64_t sub_inc, const float* div, int64_t div_inc, float* out, int64_t ld_out,
                   void* stream) {
  PDD_REQUIRE(x && out && sub && div, "pdd_scale_rows: null pointer");
  PDD_REQUIRE(C >= 0 && N >= 0 && ld >= N && ld_out >= N && sub_inc >= 0 && div_inc >= 0,
              "pdd_scale_rows: bad shape");
  if (C == 0 || N == 0) return 0;
  const int64_t tiles = cdiv(N, 1024);
  PDD_REQUIRE(C * tiles < (1ll << 31), "pdd_scale_rows: too large");
  k_scale_rows<<<(unsigned)(C * tiles), 256, 0, as_stream(stream)>>>(x, N, ld, sub, sub_inc, div,
                                                                     div_inc, out, ld_out, tiles);
  PDD_LAUNCHED();
  return 0;
}

int pdd_masked_fill(const float* x, int64_t C, int64_t N, int64_t ld, const uint8_t* mask,
                    int64_t ld_mask, const float* vals, float* out, int64_t ld_out, void* stream) {
  PDD_REQUIRE(x && out && mask && vals, "pdd_masked_fill: null pointer");
  PDD_REQUIRE(C >= 0 && N >= 0 && ld >= N && ld_mask >= N && ld_out >= N,
              "pdd_masked_fill: bad shape");
  if (C == 0 || N == 0) return 0;
  const int64_t tiles = cdiv(N, 1024);
  PDD_REQUIRE(C * tiles < (1ll << 31), "pdd_masked_fill: too large");
  k_masked_fill<<<(unsigned)(C * tiles), 256, 0, as_stream(stream)>>>(x, N, ld, mask, ld_mask, vals,
                                                                      out, ld_out, tiles);
  PDD_LAUNCHED();
  return 0;
}

int pdd_smooth(const float* x, int64_t C, int64_t N, int64_t ld, int64_t width, int pad_mode,
               const float* padvals, float* out, int64_t ld_out, void* stream) {
  PDD_REQUIRE(x && out, "pdd_smooth: null pointer");
  PDD_REQUIRE(x != out, "pdd_smooth: out must not alias x");
  PDD_REQUIRE(C >= 0 && N > 0 && ld >= N && ld_out >= N, "pdd_smooth: bad shape");
  PDD_REQUIRE(width >= 1 && width <= kSmoothLds - 1023, "pdd_smooth: width %lld out of range",
              (long long)width);
  PDD_REQUIRE(pad_mode == PDD_PAD_ROTATE || (pad_mode == PDD_PAD_VALUE && padvals),
              "pdd_smooth: bad pad mode %d", pad_mode);
  PDD_REQUIRE(pad_mode != PDD_PAD_ROTATE || width <= N, "pdd_smooth: wrap needs width <= N");
  if (C == 0) return 0;
  const int64_t tiles = cdiv(N, kSmoothTile);
  PDD_REQUIRE(C * tiles < (1ll << 31), "pdd_smooth: too large");
  const int64_t nslot = kSmoothTile + width;  // window + the spare sample
  const size_t lds = (size_t)(nslot + nslot / 16 + 1) * sizeof(float);  // <= 48 KiB
  k_smooth<<<(unsigned)(C * tiles), 256, lds, as_stream(stream)>>>(x, N, ld, width, pad_mode,
                                                                   padvals, out, ld_out, tiles);
  PDD_LAUNCHED();
  return 0;
}

int pdd_zdm_downsample(const void* in, int dtype, int64_t nspec, int64_t nchan, int64_t ld,
                       int64_t factor, int zero_dm, float* out, int64_t ld_out, void* stream) {
  PDD_REQUIRE(in && out, "pdd_zdm_downsample: null pointer");
  PDD_REQUIRE(nspec >= 0 && nchan > 0 && ld >= nchan, "pdd_zdm_downsample: bad shape");
  PDD_REQUIRE(factor >= 1 && factor <= 64 && 64 % factor == 0,
              "pdd_zdm_downsample: factor must divide 64");
  PDD_REQUIRE(ld_out >= nspec / factor, "pdd_zdm_downsample: ld_out too small");
  if (nspec < factor) return 0;
  hipStream_t s = as_stream(stream);
  double* mean = nullptr;
  if (zero_dm) {
    mean = static_cast<double*>(scratch(s, kScratchSmall, (size_t)nspec * sizeof(double)));
    if (!mean) return -2;
  }
  const int64_t tiles_c = cdiv(nchan, 64);
  const int64_t blocks = cdiv(nspec, 64) * tiles_c;
  PDD_REQUIRE(blocks < (1ll << 31), "pdd_zdm_downsample: too large");
#define ZD(T)                                                                                   \
  do {                                                                                          \
    if (zero_dm)                                                                                \
      k_spectrum_mean<T><<<(unsigned)cdiv(nspec, 4), 256, 0, s>>>((const T*)in, nspec, nchan, ld, \
                                                                   mean);                       \
    k_zdm_ds<T><<<(unsigned)blocks, 256, 0, s>>>((const T*)in, nspec, nchan, ld, mean,          \
                                                 (int)factor, out, ld_out, tiles_c);            \
  } while (0)
#define ZV(T)                                                                                   \
  do {                                                                                          \
    if (zero_dm)                                                                                \
      k_spectrum_mean_vec<T><<<(unsigned)cdiv(nspec, 4), 256, 0, s>>>((const T*)in, nspec,     \
                                                                       nchan, ld, mean);        \
    const int64_t tcv = cdiv(nchan, 8 * (16 / (int64_t)sizeof(T)));                            \
    k_zdm_ds_vec<T><<<(unsigned)(cdiv(nout, 64) * tcv), 256, 0, s>>>(                           \
        (const T*)in, nspec, nchan, ld, mean, (int)factor, out, ld_out, nout, tcv);             \
  } while (0)
  const int64_t es = dtype == PDD_U8 ? 1 : (dtype == PDD_U16 ? 2 : 4);
  const int64_t nout = nspec / factor;
  const bool vec = (uintptr_t)in % 16 == 0 && (ld * es) % 16 == 0 && (nchan * es) % 16 == 0;
  if (vec && dtype == PDD_U8) ZV(uint8_t);
  else if (vec && dtype == PDD_U16) ZV(uint16_t);
  else if (vec && dtype == PDD_F32) ZV(float);
  else if (dtype == PDD_U8) ZD(uint8_t);
  else if (dtype == PDD_U16) ZD(uint16_t);
  else if (dtype == PDD_F32) ZD(float);
  else PDD_REQUIRE(false, "pdd_zdm_downsample: bad dtype %d", dtype);
#undef ZD
#undef ZV
  const hipError_t e = hipGetLastError();
  PDD_REQUIRE(e == hipSuccess, "pdd_zdm_downsample: launch failed: %s", hipGetErrorString(e));
  return 0;
}

int pdd_zdm_int_downsample(const void* in, int dtype, int64_t nspec, int64_t nchan, int64_t ld,
                           int64_t factor, int mode, int offset, uint16_t* out, int64_t ld_out,
                           void* stream) {
  PDD_REQUIRE(in && out, "pdd_zdm_int_downsample: null pointer");
  PDD_REQUIRE(dtype == PDD_U8, "pdd_zdm_int_downsample: 8-bit input only");
  PDD_REQUIRE(mode >= PDD_ZDM_NONE && mode <= PDD_ZDM_WRAP, "pdd_zdm_int_downsample: bad mode %d",
              mode);
  PDD_REQUIRE(nspec >= 0 && nchan > 0 && ld >= nchan, "pdd_zdm_int_downsample: bad shape");
  PDD_REQUIRE(factor >= 1 && factor <= 64 && 64 % factor == 0,
              "pdd_zdm_int_downsample: factor must divide 64");
  const int lo = mode == PDD_ZDM_INT ? -255 * (int)factor : 0, hi = 255 * (int)factor;
  PDD_REQUIRE(offset + lo >= 0 && offset + hi <= 65535,
              "pdd_zdm_int_downsample: offset %d cannot hold [%d, %d] in uint16", offset, lo, hi);
  PDD_REQUIRE(ld_out >= nspec / factor, "pdd_zdm_int_downsample: ld_out too small");
  PDD_REQUIRE((uintptr_t)in % 16 == 0 && ld % 16 == 0 && nchan % 16 == 0,
              "pdd_zdm_int_downsample: rows must be 16-byte aligned (nchan %% 16 == 0)");
  if (nspec < factor) return 0;
  hipStream_t s = as_stream(stream);
  double* mean = nullptr;
  if (mode != PDD_ZDM_NONE) {
    mean = static_cast<double*>(scratch(s, kScratchSmall, (size_t)nspec * sizeof(double)));
    if (!mean) return -2;
    k_spectrum_mean_vec<uint8_t><<<(unsigned)cdiv(nspec, 4), 256, 0, s>>>(
        (const uint8_t*)in, nspec, nchan, ld, mean);
  }
  const int64_t nout = nspec / factor;
  const int64_t tcv = cdiv(nchan, 8 * 16);
  const dim3 grid((unsigned)(cdiv(nout, 64) * tcv));
  const uint8_t* x = (const uint8_t*)in;
  if (mode == PDD_ZDM_NONE)
    k_zdm_int_ds_vec<0><<<grid, 256, 0, s>>>(x, nchan, ld, mean, (int)factor, out, ld_out, nout,
                                             tcv, offset);
  else if (mode == PDD_ZDM_INT)
    k_zdm_int_ds_vec<1><<<grid, 256, 0, s>>>(x, nchan, ld, mean, (int)factor, out, ld_out, nout,
                                             tcv, offset);
  else
    k_zdm_int_ds_vec<2><<<grid, 256, 0, s>>>(x, nchan, ld, mean, (int)factor, out, ld_out, nout,
                                             tcv, offset);
  const hipError_t e = hipGetLastError();
  PDD_REQUIRE(e == hipSuccess, "pdd_zdm_int_downsample: launch failed: %s", hipGetErrorString(e));
  return 0;
}

}  // extern "C"
