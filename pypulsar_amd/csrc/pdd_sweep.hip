// libpdd: batched brute-force DM sweep, gfx950.
//
//   plane[d][t] = sum_c X(c, t + table[d][c]),  t < n_out
//
// which is, per DM trial, Spectra.dedisperse(dm, padval, trim) followed by the
// channel sum of bin/waterfaller.py:140 (formats/spectra.py:229-260).
//
// Design:
//  * a workgroup owns a tile of DB = NW*DPW DM trials x TB = S*64*G samples;
//    each wave owns DPW trials, each lane G*S output samples per trial;
//  * channels are processed in chunks of `cc`; for every channel of a chunk
//    the workgroup stages X(c, t0 + bmin_c + e), e < 64*G + span_c, into LDS
//    ONCE (bmin_c / span_c = min / extent of the tile's shifts at channel c)
//    and all DB trials read it from there: one coalesced HBM/L2 read feeds
//    DB trials;
//  * the LDS image is STRIPED: element e packs the S samples
//    e, e+Q, e+2Q, ... (Q = 64*G) of the tile, so one aligned 8- or 16-byte
//    ds_read per lane returns S samples that share the SAME shift -- the
//    shift is wave-uniform per (trial, channel), read from the channel-major
//    table through the scalar cache;
//  * float32 input accumulates in float32 registers (exact for integer data);
//  * 8-bit input is staged as packed u16 pairs and accumulated with plain
//    32-bit integer adds (two u16 lanes per add, no carry while <= 257
//    channels are summed), flushed to float32 every 256 channels -- exact;
//  * blockIdx is remapped so the n_dblk DM blocks of one time tile run
//    back to back on ONE XCD and re-read the tile's input from that XCD's L2.
#include <algorithm>
#include <cstring>
#include <type_traits>
#include <vector>

#include "pdd_internal.h"

namespace pdd {

template <bool U8, int S>
struct ElemOf {
  static constexpr int bytes = U8 ? 2 * S : 4 * S;
  static_assert(bytes == 8 || bytes == 16, "LDS element must be 8 or 16 bytes");
  using type = typename std::conditional<bytes == 8, uint2, uint4>::type;
};

__device__ __forceinline__ uint32_t get_w(const uint2& v, int i) { return i == 0 ? v.x : v.y; }
__device__ __forceinline__ uint32_t get_w(const uint4& v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}
__device__ __forceinline__ void set_w(uint2& v, int i, uint32_t x) {
  if (i == 0) v.x = x; else v.y = x;
}
__device__ __forceinline__ void set_w(uint4& v, int i, uint32_t x) {
  if (i == 0) v.x = x; else if (i == 1) v.y = x; else if (i == 2) v.z = x; else v.w = x;
}

__device__ __forceinline__ int64_t wrap_mod(int64_t s, int64_t N) {
  int64_t r = s % N;
  return r < 0 ? r + N : r;
}

template <bool U8, int S, int G, int DPW, int NW>
__global__ __launch_bounds__(NW * 64) void k_sweep(
    const void* __restrict__ xv, int64_t ld, int C, int64_t N, const int* __restrict__ tab,
    int Dpad, int D, const int* __restrict__ bmin, const int* __restrict__ bspan, int pad_mode,
    const float* __restrict__ padvals, float* __restrict__ out, int64_t ld_out, int64_t n_out,
    int cc, int stride, int n_tblk, int n_dblk) {
  constexpr int Q = 64 * G;
  constexpr int TB = S * Q;
  constexpr int DB = NW * DPW;
  constexpr int NT = NW * 64;
  constexpr int WORDS = U8 ? S / 2 : S;  // 32-bit words per LDS element
  using E = typename ElemOf<U8, S>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  E* lds = reinterpret_cast<E*>(smem);

  // XCD-aware tile order: blocks b and b+8 share an XCD; give each XCD a
  // contiguous run of L so the DM blocks of one time tile share its L2.
  const int total = n_tblk * n_dblk;
  const int full = (total / 8) * 8;
  const int bid = blockIdx.x;
  const int L = (bid < full) ? (bid % 8) * (total / 8) + bid / 8 : bid;
  const int dblk = L % n_dblk, tblk = L / n_dblk;
  const int64_t t0 = (int64_t)tblk * TB;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int d0 = dblk * DB + w * DPW;
  const int* bmin_b = bmin + (int64_t)dblk * C;
  const int* bspan_b = bspan + (int64_t)dblk * C;

  float accf[DPW][G][S];
#pragma unroll
  for (int j = 0; j < DPW; ++j)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int k = 0; k < S; ++k) accf[j][g][k] = 0.f;
  uint32_t acc16[U8 ? DPW : 1][U8 ? G : 1][U8 ? WORDS : 1];
  if constexpr (U8) {
#pragma unroll
    for (int j = 0; j < DPW; ++j)
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int h = 0; h < WORDS; ++h) acc16[j][g][h] = 0u;
  }
  int since_flush = 0;

  for (int c0 = 0; c0 < C; c0 += cc) {
    const int ncc = min(cc, C - c0);
    __syncthreads();
    // ---- stage the chunk's channels into the striped LDS image
    for (int i = 0; i < ncc; ++i) {
      const int c = c0 + i;
      const int bm = bmin_b[c];
      const int ne = Q + bspan_b[c];
      const int64_t sb = t0 + bm;
      E* dst = lds + (int64_t)i * stride;
      if constexpr (U8) {
        const uint8_t* row = reinterpret_cast<const uint8_t*>(xv) + (int64_t)c * ld;
        const uint32_t pv = (pad_mode == PDD_PAD_VALUE) ? (uint32_t)padvals[c] : 0u;
        for (int e = threadIdx.x; e < ne; e += NT) {
          E v;
#pragma unroll
          for (int h = 0; h < WORDS; ++h) {
            uint32_t lo, hi;
            const int64_t s0 = sb + e + (2 * h) * Q, s1 = s0 + Q;
            if (pad_mode == PDD_PAD_ROTATE) {
              lo = row[wrap_mod(s0, N)];
              hi = row[wrap_mod(s1, N)];
            } else {
              lo = (s0 >= 0 && s0 < N) ? (uint32_t)row[s0] : pv;
              hi = (s1 >= 0 && s1 < N) ? (uint32_t)row[s1] : pv;
            }
            set_w(v, h, lo | (hi << 16));
          }
          dst[e] = v;
        }
      } else {
        const float* row = reinterpret_cast<const float*>(xv) + (int64_t)c * ld;
        const float pv = (pad_mode == PDD_PAD_VALUE) ? padvals[c] : 0.f;
        for (int e = threadIdx.x; e < ne; e += NT) {
          E v;
#pragma unroll
          for (int k = 0; k < S; ++k) {
            const int64_t s = sb + e + k * Q;
            float f;
            if (pad_mode == PDD_PAD_ROTATE) f = row[wrap_mod(s, N)];
            else f = (s >= 0 && s < N) ? row[s] : pv;
            set_w(v, k, __float_as_uint(f));
          }
          dst[e] = v;
        }
      }
    }
    __syncthreads();
    // ---- accumulate: every wave reads the image at its trials' shifts
    for (int i = 0; i < ncc; ++i) {
      const int c = c0 + i;
      const int bm = bmin_b[c];
      const int* tb = tab + (int64_t)c * Dpad + d0;
      const E* base = lds + (int64_t)i * stride + lane;
#pragma unroll
      for (int j = 0; j < DPW; ++j) {
        const E* p = base + (tb[j] - bm);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const E v = p[g * 64];
          if constexpr (U8) {
#pragma unroll
            for (int h = 0; h < WORDS; ++h) acc16[j][g][h] += get_w(v, h);
          } else {
#pragma unroll
            for (int k = 0; k < S; ++k) accf[j][g][k] += __uint_as_float(get_w(v, k));
          }
        }
      }
      if constexpr (U8) {
        if (++since_flush == 256) {
          since_flush = 0;
#pragma unroll
          for (int j = 0; j < DPW; ++j)
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
              for (int h = 0; h < WORDS; ++h) {
                accf[j][g][2 * h] += (float)(acc16[j][g][h] & 0xffffu);
                accf[j][g][2 * h + 1] += (float)(acc16[j][g][h] >> 16);
                acc16[j][g][h] = 0u;
              }
        }
      }
    }
  }
  if constexpr (U8) {
#pragma unroll
    for (int j = 0; j < DPW; ++j)
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int h = 0; h < WORDS; ++h) {
          accf[j][g][2 * h] += (float)(acc16[j][g][h] & 0xffffu);
          accf[j][g][2 * h + 1] += (float)(acc16[j][g][h] >> 16);
        }
  }
  // ---- write the tile (lane-consecutive samples: coalesced rows)
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
    const int d = d0 + j;
    if (d >= D) continue;
    float* orow = out + (int64_t)d * ld_out;
#pragma unroll
    for (int k = 0; k < S; ++k)
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int64_t t = t0 + k * Q + g * 64 + lane;
        if (t < n_out) orow[t] = accf[j][g][k];
      }
  }
}

// ------------------------------------------------------------------ variants
struct Variant {
  bool u8;
  int S, G, DPW, NW;
  int elem_bytes() const { return u8 ? 2 * S : 4 * S; }
  int Q() const { return 64 * G; }
  int TB() const { return S * 64 * G; }
  int DB() const { return NW * DPW; }
};

// Candidate tilings, best first; the plan takes the first whose LDS image of
// one channel fits the budget.
static const Variant kF32Variants[] = {{false, 2, 4, 8, 4}, {false, 2, 4, 2, 4}, {false, 2, 4, 1, 1}};
static const Variant kU8Variants[] = {{true, 4, 2, 8, 4}, {true, 4, 2, 2, 4}, {true, 4, 2, 1, 1}};

static constexpr int kLdsBudget = 48 * 1024;   // per workgroup, 3 workgroups per CU
static constexpr int kLdsMax = 160 * 1024;

typedef void (*sweep_fn)(const void*, int64_t, int, int64_t, const int*, int, int, const int*,
                         const int*, int, const float*, float*, int64_t, int64_t, int, int, int,
                         int);

static sweep_fn kernel_for(const Variant& v) {
#define V(U, S_, G_, DPW_, NW_)                                                                 \
  if (v.u8 == U && v.S == S_ && v.G == G_ && v.DPW == DPW_ && v.NW == NW_)                     \
    return k_sweep<U, S_, G_, DPW_, NW_>;
  V(false, 2, 4, 8, 4)
  V(false, 2, 4, 2, 4)
  V(false, 2, 4, 1, 1)
  V(true, 4, 2, 8, 4)
  V(true, 4, 2, 2, 4)
  V(true, 4, 2, 1, 1)
#undef V
  return nullptr;
}

}  // namespace pdd

struct pdd_sweep_plan {
  pdd::Variant v;
  int64_t D, C, Dpad, n_dblk;
  int max_span, stride, cc, lds_bytes;
  int* d_tab = nullptr;    // [C][Dpad]
  int* d_bmin = nullptr;   // [n_dblk][C]
  int* d_bspan = nullptr;  // [n_dblk][C]
  int max_bin = 0, min_bin = 0;
};

using namespace pdd;

extern "C" {

int pdd_sweep_plan_create(const int32_t* host_table, int64_t D, int64_t C, int dtype,
                          pdd_sweep_plan** plan_out) {
  PDD_REQUIRE(host_table && plan_out, "pdd_sweep_plan_create: null pointer");
  PDD_REQUIRE(D > 0 && C > 0 && D < (1 << 24) && C < (1 << 20),
              "pdd_sweep_plan_create: bad extents D=%lld C=%lld", (long long)D, (long long)C);
  PDD_REQUIRE(dtype == PDD_F32 || dtype == PDD_U8, "pdd_sweep_plan_create: dtype must be F32 or U8");
  const Variant* cands = dtype == PDD_U8 ? kU8Variants : kF32Variants;
  const int ncand = 3;

  for (int vi = 0; vi < ncand; ++vi) {
    const Variant v = cands[vi];
    const int64_t DB = v.DB();
    const int64_t n_dblk = cdiv(D, DB);
    const int64_t Dpad = n_dblk * DB;
    std::vector<int> tab((size_t)(C * Dpad));
    std::vector<int> bmin((size_t)(n_dblk * C)), bspan((size_t)(n_dblk * C));
    int max_span = 0, mx = INT32_MIN, mn = INT32_MAX;
    for (int64_t d = 0; d < Dpad; ++d) {
      const int32_t* row = host_table + std::min(d, D - 1) * C;
      for (int64_t c = 0; c < C; ++c) tab[(size_t)(c * Dpad + d)] = row[c];
    }
    for (int64_t b = 0; b < n_dblk; ++b) {
      for (int64_t c = 0; c < C; ++c) {
        int lo = INT32_MAX, hi = INT32_MIN;
        for (int64_t d = b * DB; d < (b + 1) * DB; ++d) {
          const int x = tab[(size_t)(c * Dpad + d)];
          lo = std::min(lo, x);
          hi = std::max(hi, x);
        }
        bmin[(size_t)(b * C + c)] = lo;
        bspan[(size_t)(b * C + c)] = hi - lo;
        max_span = std::max(max_span, hi - lo);
        mx = std::max(mx, hi);
        mn = std::min(mn, lo);
      }
    }
    const int64_t stride = v.Q() + max_span;
    const int64_t per_chan = stride * v.elem_bytes();
    const bool last = (vi == ncand - 1);
    if (per_chan > kLdsBudget && !(last && per_chan <= kLdsMax)) {
      if (last) {
        set_error("pdd_sweep_plan_create: DM grid too sparse for one LDS tile (span %d bins)", max_span);
        return -1;
      }
      continue;
    }
    int cc = (int)std::max<int64_t>(1, kLdsBudget / per_chan);
    cc = (int)std::min<int64_t>(cc, C);
    pdd_sweep_plan* p = new pdd_sweep_plan();
    p->v = v;
    p->D = D;
    p->C = C;
    p->Dpad = Dpad;
    p->n_dblk = n_dblk;
    p->max_span = max_span;
    p->stride = (int)stride;
    p->cc = cc;
    p->lds_bytes = (int)(cc * per_chan);
    p->max_bin = mx;
    p->min_bin = mn;
    hipError_t e = hipMalloc(&p->d_tab, tab.size() * sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&p->d_bmin, bmin.size() * sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&p->d_bspan, bspan.size() * sizeof(int));
    if (e == hipSuccess) e = hipMemcpy(p->d_tab, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_bmin, bmin.data(), bmin.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_bspan, bspan.data(), bspan.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      set_error("pdd_sweep_plan_create: %s", hipGetErrorString(e));
      pdd_sweep_plan_destroy(p);
      return -2;
    }
    if (p->lds_bytes > 64 * 1024) {
      e = hipFuncSetAttribute((const void*)kernel_for(v), hipFuncAttributeMaxDynamicSharedMemorySize,
                              p->lds_bytes);
      if (e != hipSuccess) {
        set_error("pdd_sweep_plan_create: hipFuncSetAttribute: %s", hipGetErrorString(e));
        pdd_sweep_plan_destroy(p);
        return -2;
      }
    }
    *plan_out = p;
    return 0;
  }
  set_error("pdd_sweep_plan_create: no variant");
  return -1;
}

int pdd_sweep_plan_info(const pdd_sweep_plan* p, int64_t* info) {
  PDD_REQUIRE(p && info, "pdd_sweep_plan_info: null pointer");
  info[0] = p->D;
  info[1] = p->C;
  info[2] = p->v.DB();
  info[3] = p->v.TB();
  info[4] = p->lds_bytes;
  info[5] = p->max_bin;
  info[6] = p->min_bin;
  info[7] = p->cc;
  return 0;
}

int pdd_sweep_execute(const pdd_sweep_plan* p, const void* x, int64_t N, int64_t ld, int pad_mode,
                      const float* padvals, float* out, int64_t ld_out, int64_t n_out,
                      void* stream) {
  PDD_REQUIRE(p && x && out, "pdd_sweep_execute: null pointer");
  PDD_REQUIRE(N > 0 && ld >= N && n_out >= 0 && ld_out >= n_out, "pdd_sweep_execute: bad shape");
  PDD_REQUIRE(pad_mode == PDD_PAD_ROTATE || (pad_mode == PDD_PAD_VALUE && padvals),
              "pdd_sweep_execute: bad pad mode %d", pad_mode);
  if (n_out == 0) return 0;
  // every staged index must stay inside int64 / the LDS image: the shifts are
  // bounded by the plan, the samples by N + n_out.
  const int64_t n_tblk = cdiv(n_out, p->v.TB());
  const int64_t blocks = n_tblk * p->n_dblk;
  PDD_REQUIRE(blocks < (1ll << 31), "pdd_sweep_execute: grid too large");
  sweep_fn fn = kernel_for(p->v);
  PDD_REQUIRE(fn != nullptr, "pdd_sweep_execute: no kernel");
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(p->v.NW * 64), p->lds_bytes,
                     as_stream(stream), x, ld, (int)p->C, N, p->d_tab, (int)p->Dpad, (int)p->D,
                     p->d_bmin, p->d_bspan, pad_mode, padvals, out, ld_out, n_out, p->cc,
                     p->stride, (int)n_tblk, (int)p->n_dblk);
  PDD_LAUNCHED();
  return 0;
}

int pdd_sweep_plan_destroy(pdd_sweep_plan* p) {
  if (!p) return 0;
  if (p->d_tab) (void)hipFree(p->d_tab);
  if (p->d_bmin) (void)hipFree(p->d_bmin);
  if (p->d_bspan) (void)hipFree(p->d_bspan);
  delete p;
  return 0;
}

}  // extern "C"
