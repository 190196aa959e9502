// libpdd: single-pulse boxcar search over DM-time planes (SURVEY.md §8(f)
// rank 4 -- the consumer of the sweep's plane, so planes stay resident per
// rank instead of being gathered).  gfx950.
//
// The reference has no search; the boxcar it would feed is pulse.smooth
// (formats/pulse.py:217-241: tophat ones(w)/sqrt(w), "taken from PRESTO's
// single_pulse_search.py").  The definition implemented here, restated in
// oracle/search_oracle.py (parity against that restatement; PRESTO parity
// unpinned -- PRESTO is absent):
//   1. detrend + normalise per chunk of L samples of each DM row:
//        z[t] = (x[t] - mean_k) / std_k,   k = t / L,
//      std_k = sqrt(mean((x - mean_k)^2)) over the chunk (the last chunk may
//      be short); z = 0 in a chunk with std_k == 0;
//   2. boxcar S/N for every width w of the list and every start t <= n - w:
//        snr_w[t] = (z[t] + ... + z[t + w - 1]) / sqrt(w);
//   3. one candidate per (DM row, window of 1024 starts): the maximum of snr_w[t]
//      over the window's starts and all widths (ties: smallest width, then
//      smallest start), kept when >= threshold.
//
// Kernels (each reads the plane once; k_sp_search is VALU-bound, DESIGN.md
// §6b):
//   k_sp_stats   one wave per chunk: single-pass shifted sums, one butterfly
//   k_sp_search  one 256-thread block per (row, 4 windows of 1024 starts): z
//                of the starts + halo (max width - 1) into LDS, block prefix
//                sum (exclusive, relative to the block start), then every
//                (start, width) is one LDS difference; per-window max, then
//                an exact arg-max pass only for windows over the threshold;
//                compact candidate list through one atomic counter.
#include <algorithm>
#include <cmath>

#include "pdd_internal.h"

namespace pdd {

namespace {

constexpr int kSpThreads = 256;
constexpr int kSpWin = 1024;            // starts per candidate window
constexpr int kSpMaxHalo = 1024;        // max width - 1 <= 1024
constexpr int kSpMaxWidths = 32;
constexpr int kSpWpb = 4;                          // windows per block
constexpr int kSpStarts = kSpWin * kSpWpb;         // 4096 starts per block
constexpr int kSpSpan = kSpStarts + kSpMaxHalo;    // 5120 z values
constexpr int kSpPer = kSpSpan / kSpThreads;       // 20 per thread (scan)
constexpr int kSpR = kSpStarts / kSpThreads;       // 16 starts per thread
constexpr int kSpStat = 64;                        // chunk statistics staged per block

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Widths {
  int n;
  int maxw;
  int w[kSpMaxWidths];
  float inv_sqrt[kSpMaxWidths];
};

// Lane 0's value after an xor butterfly over the wave (the same association
// as __shfl_xor steps 1, 2, ..., 32): steps 1..16 by ds_swizzle within each
// 32-lane half (no address arithmetic), step 32 by two readlanes.
template <int XOR>
__device__ __forceinline__ float swz_xor(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v),
                                                               0x1F | (XOR << 10)));
}
template <typename Op>
__device__ __forceinline__ float wave_reduce0(float v, Op op) {
  v = op(v, swz_xor<1>(v));
  v = op(v, swz_xor<2>(v));
  v = op(v, swz_xor<4>(v));
  v = op(v, swz_xor<8>(v));
  v = op(v, swz_xor<16>(v));
  return op(__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0)),
            __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32)));
}

// one wave per (row, chunk), 4 per block: the chunk is read once, coalesced,
// as shifted sums S1 = sum(x - K), S2 = sum((x - K)^2) with K the chunk's
// first sample, so var = S2/len - (S1/len)^2 does not cancel against a large
// mean (plane rows sit at ~C x 128 for 8-bit input) and f32 is enough; both
// sums go through one butterfly reduction (wave_reduce0).
__global__ __launch_bounds__(256) void k_sp_stats(const float* __restrict__ x, int64_t D, int64_t n,
                                                  int64_t ld, int64_t L, int64_t nchunk,
                                                  float* __restrict__ mean_out,
                                                  float* __restrict__ istd_out) {
  const int lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= D * nchunk) return;
  const int64_t d = item / nchunk, k = item % nchunk;
  const int64_t t0 = k * L;
  const int len = (int)((t0 + L <= n) ? L : n - t0);
  const float* row = x + d * ld + t0;
  const float K = row[0];
  // lane l sums samples 4 (l + 64 i) + e in (i, e) order, by 16-byte loads
  // where the chunk start is 16-byte aligned and its length a multiple of 4,
  // by single loads otherwise: the same float sums either way (a streamed
  // plane's chunks land at other alignments than the one-shot plane's).
  // Loads past the chunk re-read its last group / sample (in bounds) and add
  // K (i.e. 0), so each pass issues its loads before any use.
  float s1 = 0.f, s2 = 0.f;
  auto add = [&](const float (&a)[4][4], int i0) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float c = (4 * (lane + 64 * (i0 + u)) + e < len) ? a[u][e] - K : 0.f;
        s1 += c;
        s2 += c * c;
      }
  };
  if (((uintptr_t)row & 15) == 0 && (len & 3) == 0) {
    for (int i0 = 0; 256 * i0 < len; i0 += 4) {
      float a[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int b = 4 * (lane + 64 * (i0 + u));
        const f32x4 q =
            __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row + min(b, len - 4)));
#pragma unroll
        for (int e = 0; e < 4; ++e) a[u][e] = q[e];
      }
      add(a, i0);
    }
  } else {
    for (int i0 = 0; 256 * i0 < len; i0 += 4) {
      float a[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) a[u][e] = row[min(4 * (lane + 64 * (i0 + u)) + e, len - 1)];
      add(a, i0);
    }
  }
  const auto plus = [](float a, float b) { return a + b; };
  s1 = wave_reduce0(s1, plus);
  s2 = wave_reduce0(s2, plus);
  if (lane == 0) {
    const float m1 = s1 / (float)len;
    const float var = fmaxf(s2 / (float)len - m1 * m1, 0.f);
    mean_out[item] = K + m1;
    istd_out[item] = var > 0.f ? 1.f / sqrtf(var) : 0.f;
  }
}

// P[zoff + i] (LDS) is the exclusive prefix sum of z over the block's starts
// + halo, relative to the block start, so snr(i, w) = (P[zoff + i + w] -
// P[zoff + i]) / sqrt(w); zoff = the row's misalignment on the 16-byte-load
// path (z at P[zoff + i], zoff leading zeros), else 0.
//   pass 1: per window, the maximum S/N over (width, start)  (sub, mul, max)
//   pass 2: only for windows whose maximum reaches the threshold (rare): the
//           first (width, start) in (width, start) order whose S/N -- the
//           same float ops, hence bit-identical -- equals that maximum.
__global__ __launch_bounds__(kSpThreads) void k_sp_search(
    const float* __restrict__ x, int64_t na, int64_t ld, const float* __restrict__ xn,
    int64_t ldn, int64_t n, int64_t n_starts, int64_t L, int64_t nchunk, int64_t nchunk_n,
    const float* __restrict__ mean, const float* __restrict__ istd,
    const float* __restrict__ mean_n, const float* __restrict__ istd_n, Widths W, float thr,
    int64_t nblk, int32_t* __restrict__ cands, int64_t max_cands,
    unsigned long long* __restrict__ count) {
  __shared__ __attribute__((aligned(16))) float P[kSpSpan + 4];
  __shared__ float wtot[kSpThreads / 64];
  __shared__ float wmax[kSpThreads / 64][kSpWpb];
  __shared__ int wkey[kSpThreads / 64][kSpWpb];
  __shared__ float bmax[kSpWpb];
  __shared__ float smean[kSpStat], sistd[kSpStat];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // (32-bit: D * nblk < 2^31, checked by the host)
  const int64_t d = blockIdx.x / (uint32_t)nblk, blk = blockIdx.x % (uint32_t)nblk;
  const int64_t t0 = blk * kSpStarts;
  // the row is x[d][0:na] followed by xn[d][0:n-na] (a stream's next plane);
  // chunks k < nchunk use mean/istd, later ones mean_n/istd_n (na % L == 0)
  const float* row = x + d * ld;
  const float* nrow = xn ? xn + d * ldn - na : row;
  const float* mrow = mean + d * nchunk;
  const float* irow = istd + d * nchunk;
  const float* mnrow = mean_n ? mean_n + d * nchunk_n - nchunk : mrow;
  const float* inrow = istd_n ? istd_n + d * nchunk_n - nchunk : irow;
  const int64_t span = min((int64_t)kSpStarts + W.maxw - 1, n - t0);  // z values needed
  const int64_t nst = n - t0;  // start i is valid for width w when i + w <= nst
  const int64_t nss = n_starts - t0;  // ... and i < nss

  // z of the starts + halo, coalesced, into P[zoff..]: (x - mean_k) * istd_k
  // (32-bit quotients: t0 + span <= nt < 2^31, checked by the host; L
  // clamped, which changes no quotient)
  const uint32_t L32 = (uint32_t)min(L, (int64_t)0x7fffffff);
  const int64_t k_lo = (uint32_t)t0 / L32, nks = (uint32_t)(t0 + span - 1) / L32 - k_lo + 1;
  // (16-byte loads need the block inside the first plane and, with the row's
  // misalignment mis, the span plus mis inside the block's LDS span)
  const int mis = (int)(((uintptr_t)(row + t0) >> 2) & 3);
  const bool staged = L >= 4 && nks <= kSpStat && t0 + span <= na && span + mis <= kSpSpan;
  const int zoff = staged ? mis : 0;  // where z[0] sits in P
  if (staged) {
    // the block's chunk statistics staged in LDS; thread tid loads the
    // 16-byte-aligned groups 4 (tid + 256 j) of the row from mis elements
    // before the block start (element i = 4 (tid + 256 j) + e - mis; a group
    // past the last valid element re-reads that element's group, so every
    // load stays in the 16-byte granules holding the row's own elements);
    // every load is issued before the statistics are staged and used (at
    // most one chunk boundary in 4 samples: L >= 4)
    constexpr int NJ = kSpSpan / (4 * kSpThreads);
    const float* rowA = row + t0 - mis;
    const int amax = (mis + (int)span - 1) & ~3;
    // (the statistics first: their LDS stores wait for them alone)
    float sm = 0.f, si = 0.f;
    if (tid < nks) {
      const int64_t k = k_lo + tid;
      sm = (k < nchunk ? mrow : mnrow)[k];
      si = (k < nchunk ? irow : inrow)[k];
    }
    f32x4 q[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      q[j] = __builtin_nontemporal_load(
          reinterpret_cast<const f32x4*>(rowA + min(4 * (tid + kSpThreads * j), amax)));
    if (tid < nks) {
      smean[tid] = sm;
      sistd[tid] = si;
    }
    // (z lands at P[i + mis], 16-byte aligned, after mis zeros)
    // chunk index of the thread's first element
    const int64_t k = (uint32_t)(t0 + max(4 * tid - mis, 0)) / L32;
    // block-relative: chunk kr (of the staged ones) ends before element rb
    int kr = (int)(k - k_lo);
    int rb = (int)min((k + 1) * L - t0, (int64_t)0x7fffffff);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = 4 * (tid + kSpThreads * j) - mis;
      while (i >= rb) {
        ++kr;
        rb = (int)min((int64_t)rb + L32, (int64_t)0x7fffffff);
      }
      // the group's chunk and, past rb, the next one
      const int ka = min(kr, (int)nks - 1), kb = min(kr + 1, (int)nks - 1);
      const float ma = smean[ka], ia = sistd[ka], mb = smean[kb], ib = sistd[kb];
      f32x4 z;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool nx = i + e >= rb;
        z[e] = (i + e >= 0 && i + e < span) ? (q[j][e] - (nx ? mb : ma)) * (nx ? ib : ia) : 0.f;
      }
      *reinterpret_cast<f32x4*>(P + i + mis) = z;
    }
  } else {
    // (short chunks or a block over many: per sample, the chunk index
    // advancing incrementally -- one 64-bit division per thread)
    int64_t k = (t0 + tid) / L, nb = (k + 1) * L;
    for (int i = tid; i < kSpSpan; i += kSpThreads) {
      float z = 0.f;
      if (i < span) {
        const int64_t t = t0 + i;
        while (t >= nb) {
          ++k;
          nb += L;
        }
        const bool a = t < na;
        const float v = __builtin_nontemporal_load((a ? row : nrow) + t);
        z = (v - (k < nchunk ? mrow : mnrow)[k]) * (k < nchunk ? irow : inrow)[k];
      }
      P[i] = z;
    }
  }
  __syncthreads();
  // thread-contiguous kSpPer values -> block exclusive prefix
  float v[kSpPer];
  float loc = 0.f;
#pragma unroll
  for (int j = 0; j < kSpPer; ++j) {
    v[j] = P[tid * kSpPer + j];
    loc += v[j];
  }
  float inc = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wtot[wv] = inc;
  __syncthreads();
  float run = inc - loc;
  for (int i = 0; i < wv; ++i) run += wtot[i];
#pragma unroll
  for (int j = 0; j < kSpPer; ++j) {
    P[tid * kSpPer + j] = run;
    run += v[j];
  }
  if (tid == kSpThreads - 1) P[kSpSpan] = run;
  __syncthreads();

  // pass 1: per-window maxima; start i = tid + 256 r lies in window r / 4
  float p0[kSpR];
  const float* Pz = P + zoff;
#pragma unroll
  for (int r = 0; r < kSpR; ++r) p0[r] = Pz[tid + kSpThreads * r];
  float m[kSpWpb];
#pragma unroll
  for (int q = 0; q < kSpWpb; ++q) m[q] = -INFINITY;
  if (nst >= kSpStarts - 1 + W.maxw && nss >= kSpStarts) {
    // interior block: every (start, width) valid; starts in pairs through
    // packed f32 (v_pk_add_f32), maxima through v_max3_f32.  Per width the
    // window's largest sum first, scaled once: rounding x -> x * (1/sqrt w)
    // is monotonic, so max((a - b) * s) == max(a - b) * s bit for bit (and
    // pass 2 finds the same float)
    for (int wi = 0; wi < W.n; ++wi) {
      const int w = W.w[wi];
      float mw[kSpWpb];
#pragma unroll
      for (int q = 0; q < kSpWpb; ++q) mw[q] = -INFINITY;
#pragma unroll
      for (int r = 0; r < kSpR; r += 2) {
        const int i = tid + kSpThreads * r;
        const f32x2 a = {Pz[i + w], Pz[i + kSpThreads + w]};
        const f32x2 b = {p0[r], p0[r + 1]};
        const f32x2 sum = a - b;
        const int q = r / (kSpR / kSpWpb);
        mw[q] = fmaxf(fmaxf(mw[q], sum.x), sum.y);
      }
#pragma unroll
      for (int q = 0; q < kSpWpb; ++q) m[q] = fmaxf(m[q], mw[q] * W.inv_sqrt[wi]);
    }
  } else {
    for (int wi = 0; wi < W.n; ++wi) {
      const int w = W.w[wi];
      const float iw = W.inv_sqrt[wi];
#pragma unroll
      for (int r = 0; r < kSpR; ++r) {
        const int i = tid + kSpThreads * r;
        const float snr = (i + w <= nst && i < nss) ? (Pz[i + w] - p0[r]) * iw : -INFINITY;
        m[r / (kSpR / kSpWpb)] = fmaxf(m[r / (kSpR / kSpWpb)], snr);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kSpWpb; ++q) {
    m[q] = wave_reduce0(m[q], [](float a, float b) { return fmaxf(a, b); });
    if (lane == 0) wmax[wv][q] = m[q];
  }
  __syncthreads();
  if (tid < kSpWpb) {
    float b = wmax[0][tid];
    for (int i = 1; i < kSpThreads / 64; ++i) b = fmaxf(b, wmax[i][tid]);
    bmax[tid] = b;
  }
  __syncthreads();
  bool any = false;
#pragma unroll
  for (int q = 0; q < kSpWpb; ++q) any |= (bmax[q] >= thr);
  if (!any) return;  // uniform over the block

  // pass 2: first (width, start) reaching each hit window's maximum; the key
  // wi * kSpStarts + i orders (width, start) and is minimised.
  int key[kSpWpb];
#pragma unroll
  for (int q = 0; q < kSpWpb; ++q) key[q] = 0x7fffffff;
  for (int wi = 0; wi < W.n; ++wi) {
    const int w = W.w[wi];
    const float iw = W.inv_sqrt[wi];
#pragma unroll
    for (int r = 0; r < kSpR; ++r) {
      const int i = tid + kSpThreads * r, q = r / (kSpR / kSpWpb);
      const float snr = (i + w <= nst && i < nss) ? (Pz[i + w] - p0[r]) * iw : -INFINITY;
      if (bmax[q] >= thr && snr == bmax[q]) key[q] = min(key[q], wi * kSpStarts + i);
    }
  }
#pragma unroll
  for (int q = 0; q < kSpWpb; ++q) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) key[q] = min(key[q], __shfl_xor(key[q], o, 64));
    if (lane == 0) wkey[wv][q] = key[q];
  }
  __syncthreads();
  if (tid < kSpWpb && bmax[tid] >= thr) {
    int kk = wkey[0][tid];
    for (int i = 1; i < kSpThreads / 64; ++i) kk = min(kk, wkey[i][tid]);
    const int wi = kk / kSpStarts, i = kk % kSpStarts;
    const unsigned long long slot = atomicAdd(count, 1ull);
    if ((int64_t)slot < max_cands) {
      int32_t* c = cands + slot * 4;
      c[0] = (int32_t)d;
      c[1] = (int32_t)(t0 + i);
      c[2] = W.w[wi];
      c[3] = __float_as_int(bmax[tid]);
    }
  }
}

}  // namespace

}  // namespace pdd

using namespace pdd;

extern "C" {

int pdd_sp_chunk_stats(const float* x, int64_t D, int64_t n, int64_t ld, int64_t L, float* mean,
                       float* istd, void* stream) {
  PDD_REQUIRE(x && mean && istd, "pdd_sp_chunk_stats: null pointer");
  PDD_REQUIRE(D >= 0 && n > 0 && ld >= n && L > 0, "pdd_sp_chunk_stats: bad shape");
  const int64_t nchunk = cdiv(n, L);
  const int64_t blocks = cdiv(D * nchunk, 4);
  PDD_REQUIRE(blocks < (1ll << 31) && L < (1ll << 30), "pdd_sp_chunk_stats: too large");
  if (D == 0) return 0;
  k_sp_stats<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(x, D, n, ld, L, nchunk, mean, istd);
  PDD_LAUNCHED();
  return 0;
}

int pdd_sp_search(const float* x, int64_t D, int64_t n, int64_t ld, int64_t L, const float* mean,
                  const float* istd, const float* x_next, int64_t n_next, int64_t ld_next,
                  const float* mean_next, const float* istd_next, int64_t n_starts,
                  const int32_t* widths, int n_widths, float threshold, int32_t* cands,
                  int64_t max_cands, unsigned long long* count, void* stream) {
  PDD_REQUIRE(x && mean && istd && widths && count && (cands || max_cands == 0),
              "pdd_sp_search: null pointer");
  PDD_REQUIRE(D >= 0 && n > 0 && ld >= n && L > 0 && max_cands >= 0, "pdd_sp_search: bad shape");
  PDD_REQUIRE(n_next >= 0 && (n_next == 0 || (x_next && mean_next && istd_next &&
                                               ld_next >= n_next && n % L == 0)),
              "pdd_sp_search: next plane needs x/mean/istd, ld >= n_next and n %% L == 0");
  PDD_REQUIRE(n_starts >= 0 && n_starts <= n + n_next, "pdd_sp_search: n_starts out of range");
  PDD_REQUIRE(n_widths >= 1 && n_widths <= kSpMaxWidths, "pdd_sp_search: 1..%d widths",
              kSpMaxWidths);
  Widths W;
  W.n = n_widths;
  W.maxw = 0;
  for (int i = 0; i < n_widths; ++i) {
    PDD_REQUIRE(widths[i] >= 1 && widths[i] <= kSpMaxHalo + 1,
                "pdd_sp_search: width %d out of range 1..%d", widths[i], kSpMaxHalo + 1);
    PDD_REQUIRE(i == 0 || widths[i] > widths[i - 1], "pdd_sp_search: widths must ascend");
    W.w[i] = widths[i];
    W.inv_sqrt[i] = (float)(1.0 / std::sqrt((double)widths[i]));
    W.maxw = widths[i];
  }
  const int64_t nchunk = cdiv(n, L), nchunk_n = cdiv(n_next, L);
  const int64_t nt = n + n_next;
  const int64_t nblk = cdiv(std::min(n_starts, nt), kSpStarts);
  PDD_REQUIRE(D * nblk < (1ll << 31) && nt < (1ll << 31) - kSpSpan, "pdd_sp_search: too large");
  if (D == 0 || nblk == 0) return 0;
  k_sp_search<<<(unsigned)(D * nblk), kSpThreads, 0, as_stream(stream)>>>(
      x, n, ld, n_next ? x_next : nullptr, ld_next, nt, n_starts, L, nchunk, nchunk_n, mean, istd,
      n_next ? mean_next : nullptr, n_next ? istd_next : nullptr, W, threshold, nblk, cands,
      max_cands, count);
  PDD_LAUNCHED();
  return 0;
}

}  // extern "C"
