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
// Kernels (both meant to be HBM-bound: each reads the plane once):
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

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct Widths {
  int n;
  int maxw;
  int w[kSpMaxWidths];
  float inv_sqrt[kSpMaxWidths];
};

// one wave per (row, chunk), 4 per block: the chunk is read once, coalesced,
// as shifted sums S1 = sum(x - K), S2 = sum((x - K)^2) with K the chunk's
// first sample, so var = S2/len - (S1/len)^2 does not cancel against a large
// mean (plane rows sit at ~C x 128 for 8-bit input) and f32 is enough; both
// sums go through one butterfly reduction (two independent chains).
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
  float s1 = 0.f, s2 = 0.f;
  int i = lane;
#pragma unroll 4
  for (; i + 192 < len; i += 256) {
    const float a = __builtin_nontemporal_load(row + i) - K;
    const float b = __builtin_nontemporal_load(row + i + 64) - K;
    const float c = __builtin_nontemporal_load(row + i + 128) - K;
    const float e = __builtin_nontemporal_load(row + i + 192) - K;
    s1 += (a + b) + (c + e);
    s2 += (a * a + b * b) + (c * c + e * e);
  }
  for (; i < len; i += 64) {
    const float a = row[i] - K;
    s1 += a;
    s2 += a * a;
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if (lane == 0) {
    const float m1 = s1 / (float)len;
    const float var = fmaxf(s2 / (float)len - m1 * m1, 0.f);
    mean_out[item] = K + m1;
    istd_out[item] = var > 0.f ? 1.f / sqrtf(var) : 0.f;
  }
}

// P[i] (LDS) is the exclusive prefix sum of z over the block's starts + halo,
// relative to the block start, so snr(i, w) = (P[i + w] - P[i]) / sqrt(w).
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
  __shared__ float P[kSpSpan + 1];
  __shared__ float wtot[kSpThreads / 64];
  __shared__ float wmax[kSpThreads / 64][kSpWpb];
  __shared__ int wkey[kSpThreads / 64][kSpWpb];
  __shared__ float bmax[kSpWpb];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t d = blockIdx.x / nblk, blk = blockIdx.x % nblk;
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

  // z of the starts + halo, coalesced, into P[1..]; the chunk index advances
  // incrementally (one 64-bit division per thread, not per sample)
  {
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
      P[i + 1] = z;
    }
  }
  __syncthreads();
  // thread-contiguous kSpPer values -> block exclusive prefix
  float v[kSpPer];
  float loc = 0.f;
#pragma unroll
  for (int j = 0; j < kSpPer; ++j) {
    v[j] = P[1 + tid * kSpPer + j];
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
#pragma unroll
  for (int r = 0; r < kSpR; ++r) p0[r] = P[tid + kSpThreads * r];
  float m[kSpWpb];
#pragma unroll
  for (int q = 0; q < kSpWpb; ++q) m[q] = -INFINITY;
  if (nst >= kSpStarts - 1 + W.maxw && nss >= kSpStarts) {
    // interior block: every (start, width) valid; starts in pairs through
    // packed f32 (v_pk_add_f32 / v_pk_mul_f32), maxima through v_max3_f32
    for (int wi = 0; wi < W.n; ++wi) {
      const int w = W.w[wi];
      const f32x2 iw = {W.inv_sqrt[wi], W.inv_sqrt[wi]};
#pragma unroll
      for (int r = 0; r < kSpR; r += 2) {
        const int i = tid + kSpThreads * r;
        const f32x2 a = {P[i + w], P[i + kSpThreads + w]};
        const f32x2 b = {p0[r], p0[r + 1]};
        const f32x2 snr = (a - b) * iw;
        const int q = r / (kSpR / kSpWpb);
        m[q] = fmaxf(fmaxf(m[q], snr.x), snr.y);
      }
    }
  } else {
    for (int wi = 0; wi < W.n; ++wi) {
      const int w = W.w[wi];
      const float iw = W.inv_sqrt[wi];
#pragma unroll
      for (int r = 0; r < kSpR; ++r) {
        const int i = tid + kSpThreads * r;
        const float snr = (i + w <= nst && i < nss) ? (P[i + w] - p0[r]) * iw : -INFINITY;
        m[r / (kSpR / kSpWpb)] = fmaxf(m[r / (kSpR / kSpWpb)], snr);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kSpWpb; ++q) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m[q] = fmaxf(m[q], __shfl_xor(m[q], o, 64));
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
      const float snr = (i + w <= nst && i < nss) ? (P[i + w] - p0[r]) * iw : -INFINITY;
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
