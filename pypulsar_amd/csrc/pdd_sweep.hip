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
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <unordered_map>
#include <map>
#include <utility>
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

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

// Stage one channel of the striped image with the reference pad semantics
// (register path: used for 8-bit data and for float32 channels whose window
// leaves [0, N), i.e. edge tiles, pads and rotation).
template <bool U8, int S, int Q, int NT>
__device__ __forceinline__ void stage_channel_regs(typename ElemOf<U8, S>::type* dst,
                                                   const void* xv, int64_t ld, int c, int64_t N,
                                                   int64_t sb, int ne, bool inside, int pad_mode,
                                                   const float* __restrict__ padvals) {
  using E = typename ElemOf<U8, S>::type;
  constexpr int WORDS = U8 ? S / 2 : S;
  if constexpr (U8) {
    const uint8_t* row = reinterpret_cast<const uint8_t*>(xv) + (int64_t)c * ld;
    if (inside) {
      const uint8_t* rb = row + sb;
      for (int e = threadIdx.x; e < ne; e += NT) {
        E v;
#pragma unroll
        for (int h = 0; h < WORDS; ++h)
          set_w(v, h, (uint32_t)rb[e + (2 * h) * Q] | ((uint32_t)rb[e + (2 * h + 1) * Q] << 16));
        dst[e] = v;
      }
    } else {
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
        if (inside) f = row[s];
        else if (pad_mode == PDD_PAD_ROTATE) f = row[wrap_mod(s, N)];
        else f = (s >= 0 && s < N) ? row[s] : pv;
        set_w(v, k, __float_as_uint(f));
      }
      dst[e] = v;
    }
  }
}

// float32 channel fully inside [0, N): asynchronous LDS-DMA
// (global_load_lds_dword) straight into the striped image.  One
// wave-instruction writes 256 contiguous LDS bytes = 16 elements x 4 stripes;
// lane l loads sample (e0 + l/4) of stripe l%4.  Elements past ne are filled
// from a clamped (valid) address and never read.
template <int Q, int NW>
__device__ __forceinline__ int stage_channel_dma(uint4* dst, const float* rb, int ne, int w,
                                                 int lane) {
  // Issued through inline asm: hipcc would otherwise treat the DMA as a
  // pending LDS write and put vmcnt(0) in front of every ds_read of the OTHER
  // buffer.  The kernel waits for it explicitly (vmcnt(0) before the barrier
  // that publishes the chunk).
  const int nq = (ne + 15) >> 4;
  const int k = lane & 3;
  for (int q = w; q < nq; q += NW) {
    const int e = min(q * 16 + (lane >> 2), ne - 1);
    const float* src = rb + e + k * Q;
    const uint32_t lds_addr = (uint32_t)(uintptr_t)(lds_void_t*)(dst + q * 16);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
        : "memory");
  }
  return w < nq ? (nq - 1 - w) / NW + 1 : 0;  // DMAs this wave issued
}

// s_waitcnt vmcnt(n) for a run-time n (the counter field is an immediate):
// "all but the youngest n vector-memory operations of this wave are done".
__device__ __forceinline__ void wait_vmcnt(int n) {
  n = __builtin_amdgcn_readfirstlane(n);
  switch (n < 63 ? n : 63) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    case 23: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 25: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
    case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
    case 27: asm volatile("s_waitcnt vmcnt(27)" ::: "memory"); break;
    case 28: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 29: asm volatile("s_waitcnt vmcnt(29)" ::: "memory"); break;
    case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
    case 31: asm volatile("s_waitcnt vmcnt(31)" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 33: asm volatile("s_waitcnt vmcnt(33)" ::: "memory"); break;
    case 34: asm volatile("s_waitcnt vmcnt(34)" ::: "memory"); break;
    case 35: asm volatile("s_waitcnt vmcnt(35)" ::: "memory"); break;
    case 36: asm volatile("s_waitcnt vmcnt(36)" ::: "memory"); break;
    case 37: asm volatile("s_waitcnt vmcnt(37)" ::: "memory"); break;
    case 38: asm volatile("s_waitcnt vmcnt(38)" ::: "memory"); break;
    case 39: asm volatile("s_waitcnt vmcnt(39)" ::: "memory"); break;
    case 40: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 41: asm volatile("s_waitcnt vmcnt(41)" ::: "memory"); break;
    case 42: asm volatile("s_waitcnt vmcnt(42)" ::: "memory"); break;
    case 43: asm volatile("s_waitcnt vmcnt(43)" ::: "memory"); break;
    case 44: asm volatile("s_waitcnt vmcnt(44)" ::: "memory"); break;
    case 45: asm volatile("s_waitcnt vmcnt(45)" ::: "memory"); break;
    case 46: asm volatile("s_waitcnt vmcnt(46)" ::: "memory"); break;
    case 47: asm volatile("s_waitcnt vmcnt(47)" ::: "memory"); break;
    case 48: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
    case 49: asm volatile("s_waitcnt vmcnt(49)" ::: "memory"); break;
    case 50: asm volatile("s_waitcnt vmcnt(50)" ::: "memory"); break;
    case 51: asm volatile("s_waitcnt vmcnt(51)" ::: "memory"); break;
    case 52: asm volatile("s_waitcnt vmcnt(52)" ::: "memory"); break;
    case 53: asm volatile("s_waitcnt vmcnt(53)" ::: "memory"); break;
    case 54: asm volatile("s_waitcnt vmcnt(54)" ::: "memory"); break;
    case 55: asm volatile("s_waitcnt vmcnt(55)" ::: "memory"); break;
    case 56: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
    case 57: asm volatile("s_waitcnt vmcnt(57)" ::: "memory"); break;
    case 58: asm volatile("s_waitcnt vmcnt(58)" ::: "memory"); break;
    case 59: asm volatile("s_waitcnt vmcnt(59)" ::: "memory"); break;
    case 60: asm volatile("s_waitcnt vmcnt(60)" ::: "memory"); break;
    case 61: asm volatile("s_waitcnt vmcnt(61)" ::: "memory"); break;
    case 62: asm volatile("s_waitcnt vmcnt(62)" ::: "memory"); break;
    case 63: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
  }
}

template <bool U8, int S, int G, int DPW, int NW, int CC, int NBUF>
__global__ __launch_bounds__(NW * 64) void k_sweep(
    const void* __restrict__ xv, int64_t ld, int C, int64_t N, const int* __restrict__ rel,
    int Dpad, int D, const int* __restrict__ bmin, const int* __restrict__ bspan, int pad_mode,
    const float* __restrict__ padvals, float* __restrict__ out, int64_t ld_out, int64_t n_out,
    int dbg, int stride, int n_tblk, int n_dblk) {
  constexpr int cc = CC;
  constexpr int Q = 64 * G;
  constexpr int TB = S * Q;
  constexpr int DB = NW * DPW;
  constexpr int NT = NW * 64;
  constexpr int WORDS = U8 ? S / 2 : S;  // 32-bit words per LDS element
  constexpr bool DMA = !U8 && S == 4;
  using E = typename ElemOf<U8, S>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  E* lds = reinterpret_cast<E*>(smem);
  const int64_t buf_elems = (int64_t)cc * stride;  // one of the two chunk buffers

  // XCD-aware tile order: blocks b and b+8 share an XCD; give each XCD a
  // contiguous run of L so the DM blocks of one time tile share its L2.
  const int total = n_tblk * n_dblk;
  const int full = (total / 8) * 8;
  const int bid = blockIdx.x;
  const int L = (bid < full) ? (bid % 8) * (total / 8) + bid / 8 : bid;
  const int dblk = L % n_dblk, tblk = L / n_dblk;
  const int64_t t0 = (int64_t)tblk * TB;
  // wave index as a scalar so the per-(channel, trial) offsets are fetched by
  // scalar loads (one s_load per channel for the wave's DPW trials)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int d0 = dblk * DB + w * DPW;
  const int* bmin_b = bmin + (int64_t)dblk * C;
  const int* bspan_b = bspan + (int64_t)dblk * C;

  // stage chunk [c0, c0 + ncc) into buffer `b`; returns the number of
  // LDS-DMA instructions this wave left in flight
  auto stage = [&](int c0, int b) -> int {
    const int ncc = min(cc, C - c0);
    int ndma = 0;
    E* base = lds + b * buf_elems;
    for (int i = 0; i < ncc; ++i) {
      const int c = c0 + i;
      const int bm = bmin_b[c];
      const int ne = Q + bspan_b[c];
      const int64_t sb = t0 + bm;
      const bool inside = (sb >= 0) && (sb + (int64_t)(S - 1) * Q + ne <= N);
      E* dst = base + (int64_t)i * stride;
      if constexpr (DMA) {
        if (inside) {
          ndma += stage_channel_dma<Q, NW>(reinterpret_cast<uint4*>(dst),
                                           reinterpret_cast<const float*>(xv) + (int64_t)c * ld + sb,
                                           ne, w, lane);
          continue;
        }
      }
      stage_channel_regs<U8, S, Q, NT>(dst, xv, ld, c, N, sb, ne, inside, pad_mode, padvals);
    }
    return ndma;
  };

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

  // Ring of NBUF channel-chunk buffers: chunks k+1 .. k+NBUF-1 are staged
  // (LDS-DMA in flight for float32) while chunk k is accumulated.  One
  // barrier per chunk; before it every wave waits with a COUNTED vmcnt that
  // retires only chunk k's DMAs and keeps the younger chunks in flight.
  int pend[NBUF];  // pend[s] = DMAs this wave has in flight for chunk k+s
#pragma unroll
  for (int s2 = 0; s2 < NBUF; ++s2) pend[s2] = 0;
#pragma unroll
  for (int s2 = 0; s2 < NBUF - 1; ++s2)
    if (s2 * cc < C) pend[s2] = stage(s2 * cc, s2);
  int cur = 0;
  for (int c0 = 0; c0 < C; c0 += cc) {
    const int ncc = min(cc, C - c0);
    if constexpr (DMA) {
      int younger = 0;
#pragma unroll
      for (int s2 = 1; s2 < NBUF - 1; ++s2) younger += pend[s2];
      wait_vmcnt(younger);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // offsets of this chunk's channels for the wave's trials, into SGPRs
    // before any LDS read is issued (scalar loads share lgkmcnt with LDS):
    // rel[c][d] = table[d][c] - bmin(block, c) >= 0
    int off[CC][DPW];
#pragma unroll
    for (int i = 0; i < CC; ++i) {
      const int* rp = rel + (int64_t)(c0 + (i < ncc ? i : 0)) * Dpad + d0;
#pragma unroll
      for (int j = 0; j < DPW; ++j) off[i][j] = rp[j];
    }
    {
      // refill the buffer chunk k-1 used (every wave is past it: barrier)
      const int cn = c0 + (NBUF - 1) * cc;
      int b = cur + NBUF - 1;
      b = b >= NBUF ? b - NBUF : b;
      const int n = cn < C ? stage(cn, b) : 0;
#pragma unroll
      for (int s2 = 0; s2 < NBUF - 2; ++s2) pend[s2] = pend[s2 + 1];
      pend[NBUF - 2] = n;
    }
    // ---- accumulate: every wave reads the image at its trials' shifts
    const E* img = lds + cur * buf_elems;
#pragma unroll
    for (int i = 0; i < CC; ++i) {
      if (i >= ncc) break;
      const E* base = img + (int64_t)i * stride + lane;
#pragma unroll
      for (int j = 0; j < DPW; ++j) {
        const E* p = base + off[i][j];
        E v[G];
#pragma unroll
        for (int g = 0; g < G; ++g) v[g] = p[g * 64];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          if constexpr (U8) {
#pragma unroll
            for (int h = 0; h < WORDS; ++h) acc16[j][g][h] += get_w(v[g], h);
          } else {
#pragma unroll
            for (int k = 0; k < S; ++k) accf[j][g][k] += __uint_as_float(get_w(v[g], k));
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
    cur = cur + 1 == NBUF ? 0 : cur + 1;
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

// ------------------------------------------------------------------ LDS helpers
typedef __attribute__((address_space(3))) float lds_float_t;
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) f32x2_t lds_f32x2_t;
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f32x4_t lds_f32x4_t;

__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
  return (uint32_t)(uintptr_t)(const lds_float_t*)p;
}

// 256 consecutive ints (1 KiB) -> LDS by one dwordx4 LDS-DMA
// wave-instruction (lane l: ints 4l .. 4l + 3); lanes past n (a multiple of
// 4) stay idle, so nothing lands past the n ints; src and lds_dst 16-B
// aligned.  Used for the per-chunk metadata rows, so they travel on the same
// counted vmcnt as the sample DMAs and never touch a VGPR early.  (Measured
// and dropped, round 5: the rows one chunk further ahead, kept in flight
// through the next barrier by the compiler's LDS-DMA builtin -- the
// staging-free skeleton 48 -> 32 ms per configs[3] launch, but production
// 102.2 -> 107.1 ms.)
__device__ __forceinline__ void dma_ints4(int* lds_dst, const int* src, int n, int lane) {
  const uint32_t la = __builtin_amdgcn_readfirstlane(lds_addr_of(lds_dst));
  if (lane * 4 < n) {
    const int* p = src + lane * 4;
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(p), "s"(la)
        : "memory");
  }
}


// ------------------------------------------------------------------ interleaved
// The production sweep.  A pre-pass (k_interleave) rewrites each channel of
// the input segment as 16-byte ELEMENTS that hold 4 samples a quarter of the
// segment apart:
//     R[c][j] = ( X(c, b+j), X(c, b+j+Qs), X(c, b+j+2Qs), X(c, b+j+3Qs) ),
//     b = t_base + lo,  j < nR = Qs + hi - lo + 64
// with the reference pad semantics (value / rotate) baked in, so the sweep
// never sees an edge.  It is a pure re-layout (each sample is read once and
// written once, ~1x the input bytes; u8/f32 input both become float32).
// A sweep tile (DB trials x Tq elements) then stages each channel's window
// R[c][t0 + bmin_c - lo + e], e < Tq + span_c, with 1 KiB LDS-DMA
// instructions (global_load_lds_dwordx4, one element per lane) issued by
// dedicated loader waves, and every compute-wave ds_read_b128 at a trial's
// (wave-uniform) shift returns 4 samples -- one per quarter -- that share it.
// Output (trial d, element e, quarter k) is plane[d][t_base + e + k*Qs].
// Each thread writes kIlPer elements 256 apart, issuing all their loads
// before any store (memory-level parallelism for the strided quarter reads).
constexpr int kIlPer = 4;
// Input layouts of the pre-pass: channel-major rows (x[c * ld + s]) or the
// "pieces" layout an all-gather of channel-major time slices produces,
// x[(s / P) * C * P + c * P + s % P] (P = piece, a power of two; C = all
// channels of the plan).
struct InLayout {
  int64_t ld;      // channel-major row stride (piece == 0)
  int64_t piece;   // P, 0 = channel-major
  int psh;         // log2(P)
  int64_t pstride; // C * P
  __device__ __forceinline__ int64_t at(int c, int64_t s) const {
    return piece ? (s >> psh) * pstride + (int64_t)c * piece + (s & (piece - 1))
                 : (int64_t)c * ld + s;
  }
};

template <typename InT>
__global__ __launch_bounds__(256) void k_interleave(const InT* __restrict__ x, InLayout lay, int64_t N,
                                                    int64_t base, int64_t Qs, int64_t nR,
                                                    int pad_mode, const float* __restrict__ padvals,
                                                    float4* __restrict__ R) {
  const int c = blockIdx.y;
  const int64_t j0 = (int64_t)blockIdx.x * (256 * kIlPer) + threadIdx.x;
  const float pv = (pad_mode == PDD_PAD_VALUE) ? padvals[c] : 0.f;
  float v[kIlPer][4];
#pragma unroll
  for (int i = 0; i < kIlPer; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t s = base + j0 + i * 256 + k * Qs;
      if (s >= 0 && s < N) v[i][k] = (float)x[lay.at(c, s)];
      else if (pad_mode == PDD_PAD_ROTATE) v[i][k] = (float)x[lay.at(c, wrap_mod(s, N))];
      else v[i][k] = pv;
    }
#pragma unroll
  for (int i = 0; i < kIlPer; ++i) {
    const int64_t j = j0 + i * 256;
    if (j < nR) R[(int64_t)c * nR + j] = make_float4(v[i][0], v[i][1], v[i][2], v[i][3]);
  }
}

// u16 eighths for 8-bit data (and for 16-bit data <= 1023): R[c][j] = 8
// samples X(c, b + j + k*Qs), k < 8, as packed u16 pairs (word h = sample 2h |
// sample 2h+1 << 16); pads (integer values, checked by the caller) and
// rotation baked in as for float32.
template <typename InT>
__global__ __launch_bounds__(256) void k_interleave_u16(const InT* __restrict__ x, InLayout lay,
                                                        int64_t N, int64_t base, int64_t Qs,
                                                        int64_t nR, int pad_mode,
                                                        const float* __restrict__ padvals,
                                                        uint4* __restrict__ R) {
  const int c = blockIdx.y;
  const int64_t j0 = (int64_t)blockIdx.x * (256 * kIlPer) + threadIdx.x;
  const uint32_t pv = (pad_mode == PDD_PAD_VALUE) ? (uint32_t)padvals[c] : 0u;
  uint32_t v[kIlPer][8];
#pragma unroll
  for (int i = 0; i < kIlPer; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t s = base + j0 + i * 256 + k * Qs;
      if (s >= 0 && s < N) v[i][k] = x[lay.at(c, s)];
      else if (pad_mode == PDD_PAD_ROTATE) v[i][k] = x[lay.at(c, wrap_mod(s, N))];
      else v[i][k] = pv;
    }
#pragma unroll
  for (int i = 0; i < kIlPer; ++i) {
    const int64_t j = j0 + i * 256;
    if (j < nR)
      R[(int64_t)c * nR + j] = make_uint4(v[i][0] | (v[i][1] << 16), v[i][2] | (v[i][3] << 16),
                                          v[i][4] | (v[i][5] << 16), v[i][6] | (v[i][7] << 16));
  }
}

// The same u16 eighths of an 8-bit block DOWNSAMPLED by F <= 4 on the fly
// (formats/spectra.py:329-351: sample s = the co-add of raw samples
// s*F .. s*F + F - 1, <= 1020, exact), so a downsampled DDplan step never
// writes and re-reads its downsampled copy; pads and rotation act on the
// downsampled series (N = raw length / F) as for k_interleave_u16.  VEC: the
// F raw bytes of a sample are one aligned 2- or 4-byte load (summed by
// v_sad_u8 against zero).
template <int F, bool VEC>
__global__ __launch_bounds__(256) void k_interleave_u16_ds(const uint8_t* __restrict__ x, int64_t ld,
                                                           int64_t N, int64_t base, int64_t Qs,
                                                           int64_t nR, int pad_mode,
                                                           const float* __restrict__ padvals,
                                                           uint4* __restrict__ R) {
  const int c = blockIdx.y;
  const int64_t j0 = (int64_t)blockIdx.x * (256 * kIlPer) + threadIdx.x;
  const uint32_t pv = (pad_mode == PDD_PAD_VALUE) ? (uint32_t)padvals[c] : 0u;
  const uint8_t* row = x + (int64_t)c * ld;
  auto coadd = [&](int64_t s) -> uint32_t {
    const uint8_t* q = row + s * F;
    if constexpr (VEC && F == 4) {
      return __builtin_amdgcn_sad_u8(*reinterpret_cast<const uint32_t*>(q), 0u, 0u);
    } else if constexpr (VEC && F == 2) {
      return __builtin_amdgcn_sad_u8((uint32_t)*reinterpret_cast<const uint16_t*>(q), 0u, 0u);
    } else {
      uint32_t a = 0;
#pragma unroll
      for (int k = 0; k < F; ++k) a += q[k];
      return a;
    }
  };
  uint32_t v[kIlPer][8];
#pragma unroll
  for (int i = 0; i < kIlPer; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t s = base + j0 + i * 256 + k * Qs;
      if (s >= 0 && s < N) v[i][k] = coadd(s);
      else if (pad_mode == PDD_PAD_ROTATE) v[i][k] = coadd(wrap_mod(s, N));
      else v[i][k] = pv;
    }
#pragma unroll
  for (int i = 0; i < kIlPer; ++i) {
    const int64_t j = j0 + i * 256;
    if (j < nR)
      R[(int64_t)c * nR + j] = make_uint4(v[i][0] | (v[i][1] << 16), v[i][2] | (v[i][3] << 16),
                                          v[i][4] | (v[i][5] << 16), v[i][6] | (v[i][7] << 16));
  }
}

// Vector form for 16-B aligned rows (F = 2 or 4): a thread builds J = 16 / F
// CONSECUTIVE elements from one 16-byte load per eighth (J co-adds), and
// stores them as J contiguous 16-byte elements (a wave writes 4-8 KiB in one
// piece); the element run's base must be a multiple of J (base % J == 0,
// Qs % J == 0).  Runs that touch a pad or the wrap take the per-sample path.
template <int F>
__global__ __launch_bounds__(256) void k_interleave_u16_ds_v(const uint8_t* __restrict__ x,
                                                             int64_t ld, int64_t N, int64_t base,
                                                             int64_t Qs, int64_t nR, int pad_mode,
                                                             const float* __restrict__ padvals,
                                                             uint4* __restrict__ R) {
  static_assert(F == 2 || F == 4, "16-byte loads of 4 or 8 co-adds");
  constexpr int J = 16 / F;
  const int c = blockIdx.y;
  const int64_t j0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * J;
  if (j0 >= nR) return;
  const uint32_t pv = (pad_mode == PDD_PAD_VALUE) ? (uint32_t)padvals[c] : 0u;
  const uint8_t* row = x + (int64_t)c * ld;
  uint32_t v[8][J];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t s0 = base + j0 + k * Qs;
    if (s0 >= 0 && s0 + J <= N) {
      const uint4 q = *reinterpret_cast<const uint4*>(row + s0 * F);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        if constexpr (F == 4) {
          v[k][h] = __builtin_amdgcn_sad_u8(w[h], 0u, 0u);
        } else {
          v[k][2 * h] = __builtin_amdgcn_sad_u8(w[h] & 0xffffu, 0u, 0u);
          v[k][2 * h + 1] = __builtin_amdgcn_sad_u8(w[h] >> 16, 0u, 0u);
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < J; ++e) {
        const int64_t s = s0 + e;
        const int64_t sw = (s >= 0 && s < N) ? s : (pad_mode == PDD_PAD_ROTATE ? wrap_mod(s, N) : -1);
        uint32_t a = pv;
        if (sw >= 0) {
          a = 0;
#pragma unroll
          for (int f = 0; f < F; ++f) a += row[sw * F + f];
        }
        v[k][e] = a;
      }
    }
  }
  uint4* dst = R + (int64_t)c * nR + j0;
#pragma unroll
  for (int e = 0; e < J; ++e)
    if (j0 + e < nR)
      dst[e] = make_uint4(v[0][e] | (v[1][e] << 16), v[2][e] | (v[3][e] << 16),
                          v[4][e] | (v[5][e] << 16), v[6][e] | (v[7][e] << 16));
}

// ------------------------------------------------------------------ factorised sweep
// Exact factorisation of the 8-bit sweep over groups of fx = 4 (or 2)
// adjacent channels.  Within a group (channels c0..c0+3) trial d's shifts are its base
// shift b = table[d][c0] plus a RELATIVE pattern r = (0, r1, r2, r3); the
// group's contribution to plane[d][t] is
//     sum_k X(c0 + k, t + b + r_k) = S_r(t + b),  S_r(u) = sum_k X(c0 + k, u + r_k),
// the same samples summed in integers, so the plane is bit-identical to the
// channel-by-channel sum.  Across a DM grid a group takes few distinct
// patterns (configs[3]: 27 769 over 1024 groups, 6.8 per group): stage 1
// (k_fx_patterns) writes every pattern series S_r once as a u16-eighths image
// row (sums of four samples <= 1020 stay exact in the packed u16 lanes), and
// stage 2 is k_sweep_il over the GROUPS, each trial reading its pattern's
// window at its base shift: a quarter of the LDS reads and adds of the
// channel sweep, the same window staging (a tile stages every pattern its
// trials use: 3.8 of a group's patterns per 48-trial block, 0.88 x the
// channel windows' elements).
__global__ __launch_bounds__(256) void k_fx_patterns(const uint4* __restrict__ R, int64_t nR,
                                                     const int4* __restrict__ pat, int fx,
                                                     uint4* __restrict__ P) {
  const int64_t p = blockIdx.x;
  const int4 q = pat[p];  // {c0, r1, r2, r3}
  const uint4* r0 = R + (int64_t)q.x * nR;
  const int64_t j0 = (int64_t)blockIdx.y * (256 * kIlPer) + threadIdx.x;
  auto at = [&](int k, int r, int64_t j) -> uint4 {
    const int64_t e = j + r;  // elements no trial reads may fall outside the row
    return (e >= 0 && e < nR) ? r0[(int64_t)k * nR + e] : make_uint4(0u, 0u, 0u, 0u);
  };
  uint4 v[kIlPer];
#pragma unroll
  for (int i = 0; i < kIlPer; ++i) {
    const int64_t j = j0 + i * 256;
    if (j >= nR) continue;
    const uint4 a = at(0, 0, j), b = at(1, q.y, j);
    const uint4 c = fx > 2 ? at(2, q.z, j) : make_uint4(0u, 0u, 0u, 0u);
    const uint4 d = fx > 3 ? at(3, q.w, j) : make_uint4(0u, 0u, 0u, 0u);
    v[i] = make_uint4(a.x + b.x + c.x + d.x, a.y + b.y + c.y + d.y, a.z + b.z + c.z + d.z,
                      a.w + b.w + c.w + d.w);
  }
#pragma unroll
  for (int i = 0; i < kIlPer; ++i) {
    const int64_t j = j0 + i * 256;
    if (j < nR) P[p * nR + j] = v[i];
  }
}

// Stage 1 through LDS: one workgroup per (group, kFxE-element block) loads
// the group's four rows over the block (+ the group's relative-shift range)
// ONCE and writes every pattern of the group from them (the plain kernel
// above reads four rows per pattern element from L2: 4 x 16 B per 16 B
// written).  gtab: [NG + 1] first pattern of each group, then [NG] x {lo,
// hi} = the group's min(0, r) / max(0, r) over its patterns (hi - lo <=
// kFxRspan, checked by the plan), then [n_pat] x {first, last - nR}: the
// pattern row's elements stage 2 reads (fx_build): kFxE-element blocks
// outside that range are not written.
constexpr int kFxE = 512, kFxRspan = 512;

// float32 stage 1 (k_fx_patterns_xf) builds 1024-element blocks: configs[1]
// f32 7.31 -> 7.10 ms per launch against 512 (8-bit stage 1: 512 best, 12.5
// against 14.2 ms at 1024)
constexpr int kFxEf = 1024;
// The group's pattern descriptors 64 at a time, one wave-wide load: lane i
// holds pattern pb + i's relative shifts and row range (fx_build), which the
// pattern loops take by v_readlane -- no dependent scalar loads per pattern.
struct FxBatch {
  int y, z, w, lo, hi;
};
__device__ __forceinline__ FxBatch fx_batch(const int4* __restrict__ pat, const int* __restrict__ rng,
                                            int pb, int p1) {
  const int pl = min(pb + (int)(threadIdx.x & 63), p1 - 1);
  const int4 q = pat[pl];
  return {q.y, q.z, q.w, rng[2 * pl], rng[2 * pl + 1]};
}
__global__ __launch_bounds__(256) void k_fx_patterns_lds(const uint4* __restrict__ R, int64_t nR,
                                                         const int4* __restrict__ pat,
                                                         const int* __restrict__ gtab, int NG,
                                                         int fx, uint4* __restrict__ P) {
  extern __shared__ __attribute__((aligned(16))) uint4 L[];
  const int g = blockIdx.x;
  const int64_t j0 = (int64_t)blockIdx.y * kFxE;
  const int p0 = gtab[g], p1 = gtab[g + 1];
  const int lo = gtab[NG + 1 + 2 * g], hi = gtab[NG + 2 + 2 * g];
  const int W = kFxE + hi - lo;
  const uint4* r0 = R + (int64_t)(g * fx) * nR;
  for (int k = 0; k < fx; ++k)
    for (int e = threadIdx.x; e < W; e += 256) {
      const int64_t i = j0 + lo + e;
      L[k * W + e] = (i >= 0 && i < nR) ? r0[(int64_t)k * nR + i] : make_uint4(0u, 0u, 0u, 0u);
    }
  __syncthreads();
  const int* rng = gtab + 3 * NG + 1;
  for (int pb = p0; pb < p1; pb += 64) {
    const FxBatch B = fx_batch(pat, rng, pb, p1);
    for (int i = 0; i < min(64, p1 - pb); ++i) {
      const int p = pb + i;
      const int4 q = make_int4(0, __builtin_amdgcn_readlane(B.y, i), __builtin_amdgcn_readlane(B.z, i),
                               __builtin_amdgcn_readlane(B.w, i));
      const int64_t jlo = __builtin_amdgcn_readlane(B.lo, i), jhi = nR + __builtin_amdgcn_readlane(B.hi, i);
      if (j0 >= jhi || j0 + kFxE <= jlo) continue;  // no trial of p reads this block
#pragma unroll
      for (int e = threadIdx.x; e < kFxE; e += 256) {
        const int64_t j = j0 + e;
        if (j >= nR) break;  // (a block's elements outside [jlo, jhi): written, unread)
        const uint4 a = L[e - lo], b = L[W + e - lo + q.y];
        const uint4 c = fx > 2 ? L[2 * W + e - lo + q.z] : make_uint4(0u, 0u, 0u, 0u);
        const uint4 d = fx > 3 ? L[3 * W + e - lo + q.w] : make_uint4(0u, 0u, 0u, 0u);
        P[(int64_t)p * nR + j] = make_uint4(a.x + b.x + c.x + d.x, a.y + b.y + c.y + d.y,
                                            a.z + b.z + c.z + d.z, a.w + b.w + c.w + d.w);
      }
    }
  }
}

// Stage 1 straight from the input (no u16-eighths image R in HBM): the
// load phase builds each of the group's row elements the way
// k_interleave_u16 would -- 8 samples X(c, base + i + m*Qs), m < 8, as packed
// u16 pairs, with the reference pads (value / rotate) -- then writes every
// pattern of the group as k_fx_patterns_lds does.  Saves the image's write
// and read, and the interleave launch, per segment (the per-rank work of a
// DM-sharded step that does not shrink with the world size).
template <typename InT, int FXG>
__global__ __launch_bounds__(256) void k_fx_patterns_x(const InT* __restrict__ x, InLayout lay,
                                                       int64_t N, int64_t base, int64_t Qs,
                                                       int64_t nR, int pad_mode,
                                                       const float* __restrict__ padvals,
                                                       const int4* __restrict__ pat,
                                                       const int* __restrict__ gtab, int NG, int fx,
                                                       uint4* __restrict__ P) {
  extern __shared__ __attribute__((aligned(16))) uint4 L[];
  const int g = blockIdx.x;
  const int64_t j0 = (int64_t)blockIdx.y * kFxE;
  const int p0 = gtab[g], p1 = gtab[g + 1];
  const int lo = gtab[NG + 1 + 2 * g], hi = gtab[NG + 2 + 2 * g];
  const int W = kFxE + hi - lo;
  // a block whose rows lie inside [0, nR) and whose samples inside [0, N)
  // (every block but the segment's edges) loads without per-sample tests
  const int64_t s_lo = base + j0 + lo, s_hi = s_lo + W - 1 + 7 * Qs;
  const bool inner = j0 + lo >= 0 && j0 + lo + W <= nR && s_lo >= 0 && s_hi < N;
  for (int k = 0; k < FXG; ++k) {
    const int c = g * FXG + k;
    const uint32_t pv = (pad_mode == PDD_PAD_VALUE) ? (uint32_t)padvals[c] : 0u;
    if (inner) {
      for (int e = threadIdx.x; e < W; e += 256) {
        const int64_t sm = s_lo + e;
        uint32_t v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = x[lay.at(c, sm + m * Qs)];
        L[k * W + e] = make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16),
                                  v[6] | (v[7] << 16));
      }
      continue;
    }
    for (int e = threadIdx.x; e < W; e += 256) {
      const int64_t i = j0 + lo + e;
      uint32_t v[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int64_t sm = base + i + m * Qs;
        if (i < 0 || i >= nR) v[m] = 0u;
        else if (sm >= 0 && sm < N) v[m] = x[lay.at(c, sm)];
        else if (pad_mode == PDD_PAD_ROTATE) v[m] = x[lay.at(c, wrap_mod(sm, N))];
        else v[m] = pv;
      }
      L[k * W + e] = make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16),
                                v[6] | (v[7] << 16));
    }
  }
  __syncthreads();
  const int* rng = gtab + 3 * NG + 1;
  for (int pb = p0; pb < p1; pb += 64) {
    const FxBatch B = fx_batch(pat, rng, pb, p1);
    for (int i = 0; i < min(64, p1 - pb); ++i) {
      const int p = pb + i;
      const int4 q = make_int4(0, __builtin_amdgcn_readlane(B.y, i), __builtin_amdgcn_readlane(B.z, i),
                               __builtin_amdgcn_readlane(B.w, i));
      const int64_t jlo = __builtin_amdgcn_readlane(B.lo, i), jhi = nR + __builtin_amdgcn_readlane(B.hi, i);
      if (j0 >= jhi || j0 + kFxE <= jlo) continue;  // no trial of p reads this block
#pragma unroll
      for (int e = threadIdx.x; e < kFxE; e += 256) {
        const int64_t j = j0 + e;
        if (j >= nR) break;  // (a block's elements outside [jlo, jhi): written, unread)
        const uint4 a = L[e - lo], b = L[W + e - lo + q.y];
        const uint4 c = FXG > 2 ? L[2 * W + e - lo + q.z] : make_uint4(0u, 0u, 0u, 0u);
        const uint4 d = FXG > 3 ? L[3 * W + e - lo + q.w] : make_uint4(0u, 0u, 0u, 0u);
        // non-temporal: the pattern image is read back only after the whole
        // stage (12.6 against 13.0 ms per configs[3] launch, same box; the
        // float32 stage 1 measured 8.6 ms with it against 7.5 without, on
        // another box, so it keeps plain stores)
        typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
        const u32x4v sv = {a.x + b.x + c.x + d.x, a.y + b.y + c.y + d.y, a.z + b.z + c.z + d.z,
                           a.w + b.w + c.w + d.w};
        __builtin_nontemporal_store(sv, reinterpret_cast<u32x4v*>(P + (int64_t)p * nR + j));
      }
    }
  }
}

// Stage 1 of factorised float32 sweeps: the same from float32 rows into the
// float32 QUARTERS image of k_interleave (element = 4 samples X(c, base + i +
// m*Qs), m < 4), each pattern element the float sum of its group's fx
// elements in channel order (x_c0 + x_c0+1 [+ x_c0+2 + x_c0+3]); the sweep
// then adds pattern series instead of channels -- the reference's float64
// channel sum regrouped, within the float32 parity bar (and exact for
// integer-valued data).  Pads as k_interleave: value (per channel) / rotate.
template <int FXG>
__global__ __launch_bounds__(256) void k_fx_patterns_xf(const float* __restrict__ x, InLayout lay,
                                                        int64_t N, int64_t base, int64_t Qs,
                                                        int64_t nR, int pad_mode,
                                                        const float* __restrict__ padvals,
                                                        const int4* __restrict__ pat,
                                                        const int* __restrict__ gtab, int NG, int fx,
                                                        float4* __restrict__ P) {
  extern __shared__ __attribute__((aligned(16))) float4 Lf[];
  const int g = blockIdx.x;
  const int64_t j0 = (int64_t)blockIdx.y * kFxEf;
  const int p0 = gtab[g], p1 = gtab[g + 1];
  const int lo = gtab[NG + 1 + 2 * g], hi = gtab[NG + 2 + 2 * g];
  const int W = kFxEf + hi - lo;
  // interior blocks load without per-sample tests (as k_fx_patterns_x)
  const int64_t s_lo = base + j0 + lo, s_hi = s_lo + W - 1 + 3 * Qs;
  const bool inner = j0 + lo >= 0 && j0 + lo + W <= nR && s_lo >= 0 && s_hi < N;
  for (int k = 0; k < FXG; ++k) {
    const int c = g * FXG + k;
    const float pv = (pad_mode == PDD_PAD_VALUE) ? padvals[c] : 0.f;
    if (inner) {
      for (int e = threadIdx.x; e < W; e += 256) {
        const int64_t sm = s_lo + e;
        Lf[k * W + e] = make_float4(x[lay.at(c, sm)], x[lay.at(c, sm + Qs)], x[lay.at(c, sm + 2 * Qs)],
                                    x[lay.at(c, sm + 3 * Qs)]);
      }
      continue;
    }
    for (int e = threadIdx.x; e < W; e += 256) {
      const int64_t i = j0 + lo + e;
      float v[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int64_t sm = base + i + m * Qs;
        if (i < 0 || i >= nR) v[m] = 0.f;
        else if (sm >= 0 && sm < N) v[m] = x[lay.at(c, sm)];
        else if (pad_mode == PDD_PAD_ROTATE) v[m] = x[lay.at(c, wrap_mod(sm, N))];
        else v[m] = pv;
      }
      Lf[k * W + e] = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  __syncthreads();
  const int* rng = gtab + 3 * NG + 1;
  for (int pb = p0; pb < p1; pb += 64) {
    const FxBatch B = fx_batch(pat, rng, pb, p1);
    for (int i = 0; i < min(64, p1 - pb); ++i) {
      const int p = pb + i;
      const int4 q = make_int4(0, __builtin_amdgcn_readlane(B.y, i), __builtin_amdgcn_readlane(B.z, i),
                               __builtin_amdgcn_readlane(B.w, i));
      const int64_t jlo = __builtin_amdgcn_readlane(B.lo, i), jhi = nR + __builtin_amdgcn_readlane(B.hi, i);
      if (j0 >= jhi || j0 + kFxEf <= jlo) continue;  // (as k_fx_patterns_lds)
#pragma unroll
      for (int e = threadIdx.x; e < kFxEf; e += 256) {
        const int64_t j = j0 + e;
        if (j >= nR) break;  // (a block's elements outside [jlo, jhi): written, unread)
        float4 s = Lf[e - lo];
        const float4 b = Lf[W + e - lo + q.y];
        s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
        if constexpr (FXG > 2) {
          const float4 c = Lf[2 * W + e - lo + q.z], d = Lf[3 * W + e - lo + q.w];
          s.x += c.x; s.y += c.y; s.z += c.z; s.w += c.w;
          s.x += d.x; s.y += d.y; s.z += d.z; s.w += d.w;
        }
        P[(int64_t)p * nR + j] = s;
      }
    }
  }
}

// A whole window from ONE wave: runs of up to four consecutive 1 KiB DMAs
// share one M0 value, the instruction offset (0 / 1024 / 2048 / 3072 bytes)
// moving both the global source and the LDS destination
// (scripts/probes/dma_offset.hip checks the LDS side on the device).
__device__ __forceinline__ int stage_il_dma_win(uint32_t lds_dst, const float4* src, int ne,
                                                int lane) {
  const int nq = (ne + 63) >> 6;
  uint32_t keep;
#define PDD_DMA_RUN(TEXT)                                                                      \
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t" TEXT "s_mov_b32 m0, %0" \
               : "=&s"(keep) : "v"(s), "s"(m) : "memory")
  for (int q = 0; q < nq; q += 4) {
    const float4* s = src + q * 64 + lane;
    const uint32_t m = __builtin_amdgcn_readfirstlane(lds_dst + q * 1024);
    switch (min(4, nq - q)) {
      case 1: PDD_DMA_RUN("global_load_lds_dwordx4 %1, off\n\t"); break;
      case 2: PDD_DMA_RUN("global_load_lds_dwordx4 %1, off\n\t"
                          "global_load_lds_dwordx4 %1, off offset:1024\n\t"); break;
      case 3: PDD_DMA_RUN("global_load_lds_dwordx4 %1, off\n\t"
                          "global_load_lds_dwordx4 %1, off offset:1024\n\t"
                          "global_load_lds_dwordx4 %1, off offset:2048\n\t"); break;
      default: PDD_DMA_RUN("global_load_lds_dwordx4 %1, off\n\t"
                           "global_load_lds_dwordx4 %1, off offset:1024\n\t"
                           "global_load_lds_dwordx4 %1, off offset:2048\n\t"
                           "global_load_lds_dwordx4 %1, off offset:3072\n\t"); break;
#undef PDD_DMA_RUN
    }
  }
  return nq;
}

// A factorised window of nq pieces from a wave-uniform source address in an
// SGPR pair (the saddr form; the lanes' VGPR offset is lane * 16 for every
// DMA: no VALU address arithmetic), as ONE asm block per run of up to four:
// M0 set once, then the pieces with instruction offsets, each after the
// first behind an s_cmp / s_cbranch on the remaining count (a compiler switch
// over min(4, nq - q) became a tree of ~20 scalar instructions and four
// branches per run).  Returns the DMAs issued.
__device__ __forceinline__ int stage_il_dma_s2(uint32_t lds_dst, const float4* src, int nq,
                                               uint32_t voff) {
  for (int q = 0; q < nq; q += 4) {
    const float4* s = src + q * 64;
    const uint32_t m = __builtin_amdgcn_readfirstlane(lds_dst + q * 1024);
    const int left = __builtin_amdgcn_readfirstlane(nq - q);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_cmp_lt_i32 %4, 2\n\t"
        "s_cbranch_scc1 1f\n\t"
        "global_load_lds_dwordx4 %1, %2 offset:1024\n\t"
        "s_cmp_lt_i32 %4, 3\n\t"
        "s_cbranch_scc1 1f\n\t"
        "global_load_lds_dwordx4 %1, %2 offset:2048\n\t"
        "s_cmp_lt_i32 %4, 4\n\t"
        "s_cbranch_scc1 1f\n\t"
        "global_load_lds_dwordx4 %1, %2 offset:3072\n"
        "1:\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(s), "s"(m), "s"(left)
        : "memory", "scc");
  }
  return nq;
}

// The last rem (< 64) elements of a window: one DMA piece from a
// wave-uniform source with lanes >= rem masked off, so nothing lands past
// the window's end in LDS.  Returns the DMAs issued (1).
__device__ __forceinline__ int stage_il_dma_tail(uint32_t lds_dst, const float4* src, int rem,
                                                 uint32_t voff, int lane) {
  if (lane < rem) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(src), "s"(lds_dst)
        : "memory");
  }
  return 1;
}


// Synchronisation of k_sweep_il: one s_barrier per chunk.  Before barrier k
// the loader waves retire chunk k's DMAs with a counted vmcnt (chunks k+1 ..
// k+NBUF-2 stay in flight); after it they refill the buffer chunk k-1 used.
// (Measured and dropped, DESIGN.md §3: an LDS-counter hand-off without
// barriers; the compute waves reading their shifts by scalar loads.)
// Metadata: mt[dblk][c][ROW], ROW = DB + 4: the tile's DB shifts at channel c
// relative to their minimum bmin, as byte offsets into the channel's LDS
// image (16 x elements), then {bmin, span, 0, 0} (in elements).  Loader 0 DMAs
// the rows of chunk j into ONE shared ring (slot j % MR) MA = 2(NBUF-1)
// chunks ahead, before the samples of chunk j - MA + NBUF - 1; its counted
// vmcnt before barrier k therefore also retires the rows of chunk
// k + NBUF - 1, which every loader reads after barrier k to issue that
// chunk's samples, and the compute waves read the shifts of chunk k after
// the same barrier.
__host__ __device__ constexpr int il_ma(int nbuf) { return 2 * nbuf - 2; }
// (ring slots: chunk j's rows are written after barrier j - MA and read by
// the end of chunk j's compute -- factorised tiles read them a chunk early
// -- and every wave has finished its reads of chunk j before barrier j + 1,
// after which chunk j + MA + 1 may overwrite the slot: MA + 1 slots suffice.
// Two buffers: 3 slots; the fourth slot's 3.2 KiB went to the chunk buffers,
// configs[3] stage 2 90.76 -> 90.08 ms, north star 59.42 -> 58.57 ms per
// launch.)
__host__ __device__ constexpr int il_mr(int nbuf) { return nbuf <= 2 ? 3 : (nbuf <= 4 ? 8 : (nbuf <= 8 ? 16 : 32)); }
__host__ __device__ constexpr int il_slot(int cc, int db) { return (cc * (db + 4) + 63) / 64 * 64; }
__host__ __device__ constexpr int il_meta_bytes(int nbuf, int cc, int db) {
  return il_mr(nbuf) * il_slot(cc, db) * 4;
}

// Tile order of k_sweep_il.  Blocks b and b+8 share an XCD (and its L2).
// XCD x walks its time tiles in bands of GT time tiles, each band in 2-D
// groups of GT time tiles x GJ trial blocks: at one channel the concurrent
// windows of such a group overlap along both axes (a trial block's window
// extends its neighbour's by the span, a time tile's by Tq), so the group
// re-reads each staged element ~GT*GJ*(Tq+S)/(GT*Tq + GJ*S) times from L2.
// Channel sweeps: XCD x owns the time tiles [x*TX, (x+1)*TX), TX = n_tblk / 8
// (8 x 4 groups).  Factorised sweeps (XI): band b of XCD x is global band
// 8b + x, so the eight XCDs sweep eight ADJACENT bands with the same
// trial-block groups at the same time and the windows two neighbouring bands
// share are fetched from HBM once, into the Infinity Cache (8 x 2 groups
// since the chunk packing orders each trial block's groups by its own
// windows, so that neighbouring trial blocks no longer stage the same
// group at the same time: configs[3] 94.23 -> 93.03 ms per launch, north
// star 61.34 -> 59.20 ms, L2-side fetch 478 -> 412 GB).  Leftover time tiles (n_tblk % 8) follow in natural order.
#ifndef PDD_IL_GT
#define PDD_IL_GT 8
#endif
#ifndef PDD_IL_GJ
#define PDD_IL_GJ 4
#endif
#ifndef PDD_FX_GT
#define PDD_FX_GT 8
#endif
#ifndef PDD_FX_GJ
#define PDD_FX_GJ 2
#endif
// float32 factorised tiles: 8 x 1 groups (their plans do not pair trial
// blocks: configs[1] f32 stage 2 23.45-23.53 -> 22.95-23.01 ms against 8 x 2)
#ifndef PDD_FX_GJF
#define PDD_FX_GJF 1
#endif
template <int GT = PDD_IL_GT, int GJ = PDD_IL_GJ, bool XI = false>
__device__ __forceinline__ void il_tile_of(int bid, int n_tblk, int n_dblk, int& dblk, int& tblk) {
  const int TX = n_tblk / 8;
  const int owned = 8 * TX * n_dblk;
  if (bid >= owned) {
    const int L = bid - owned;
    dblk = L % n_dblk;
    tblk = 8 * TX + L / n_dblk;
    return;
  }
  const int x = bid % 8, k = bid / 8;  // k-th tile of XCD x
  const int band = k / (GT * n_dblk);
  const int gtb = min(GT, TX - band * GT);  // time tiles in this band
  int r = k - band * GT * n_dblk;
  const int nj = (n_dblk + GJ - 1) / GJ;
  const int jg = min(r / (gtb * GJ), nj - 1);
  const int gj = min(GJ, n_dblk - jg * GJ);  // trial blocks in this group
  r -= jg * gtb * GJ;
  dblk = jg * GJ + r % gj;
  if constexpr (XI) {
    const int nb = (TX + GT - 1) / GT;
    tblk = (band < nb - 1 ? (band * 8 + x) * GT : 8 * (nb - 1) * GT + x * gtb) + r / gj;
  } else {
    tblk = x * TX + band * GT + r / gj;
  }
}

// Eight consecutive metadata rows' window fields {bmin, span, offset,
// source row} (row stride ROW ints) by eight scalar loads and one wait
// (the sweep's loader waves; they read no LDS).  The plan pads the table so
// eight rows from any chunk start are inside the allocation.
typedef int i32x4s_t __attribute__((ext_vector_type(4)));
struct il_rows8 {
  i32x4s_t r0, r1, r2, r3, r4, r5, r6, r7;
};
template <int ROW>
__device__ __forceinline__ il_rows8 il_load_rows8(const int* p) {
  il_rows8 o;
  asm volatile(
      "s_load_dwordx4 %0, %8, %9\n\ts_load_dwordx4 %1, %8, %10\n\t"
      "s_load_dwordx4 %2, %8, %11\n\ts_load_dwordx4 %3, %8, %12\n\t"
      "s_load_dwordx4 %4, %8, %13\n\ts_load_dwordx4 %5, %8, %14\n\t"
      "s_load_dwordx4 %6, %8, %15\n\ts_load_dwordx4 %7, %8, %16\n\t"
      "s_waitcnt lgkmcnt(0)"
      // early-clobber outputs: a row's registers must not overlap the base
      // address the later loads of the block still read (a load returning
      // before the next one issues would change its address)
      : "=&s"(o.r0), "=&s"(o.r1), "=&s"(o.r2), "=&s"(o.r3), "=&s"(o.r4), "=&s"(o.r5),
        "=&s"(o.r6), "=&s"(o.r7)
      : "s"(p), "i"(0), "i"(ROW * 4), "i"(2 * ROW * 4), "i"(3 * ROW * 4), "i"(4 * ROW * 4),
        "i"(5 * ROW * 4), "i"(6 * ROW * 4), "i"(7 * ROW * 4));
  return o;
}

// a + b + c: one v_add3_u32 (two packed-u16 sample adds per lane)
__device__ __forceinline__ uint32_t add3_u32(uint32_t a, uint32_t b, uint32_t c) {
  return a + b + c;
}

// Factorised sweeps (FX): the kernel's "channels" are the channel groups;
// a chunk's windows (one per pattern its trials use) come from the plan's
// window records wt[dblk][chunk][kFxWin] = {bmin, length, buffer offset,
// pattern row | window count << 20}, one vector load per loader lane, two
// chunks ahead.
constexpr int kFxWin = 64;
template <int G, int DPW, int NCW, int NLW, int CC, int NBUF, bool U16 = false, bool FX = false>
__global__ __launch_bounds__((NCW + NLW) * 64) void k_sweep_il(
    const float4* __restrict__ R0, int64_t nR, int C, int lo, const int* __restrict__ mt,
    const int* __restrict__ cht, int maxch, float* __restrict__ out, int64_t ld_out, int D,
    int64_t Qs, int64_t t_base, int64_t n_out, int buf_e, int n_tblk, int n_dblk, int dbg,
    int64_t row_g, int64_t row_d, int flush_n, float out_bias, const float* __restrict__ r2_pad,
    int64_t r2_nR, int64_t r2_ov, const int4* __restrict__ wt, const int* __restrict__ sig) {
  // Grouped sweeps: C is the channel count of ONE group; blockIdx.x / (tiles
  // per group) is the group, whose channels are R rows [grp*C, grp*C + C),
  // whose tables are mt[grp][...], and whose trial d lands in plane row
  // grp*row_g + d*row_d (ungrouped: 0, 0, 1).
  constexpr int Tq = 64 * G;
  constexpr int DB = NCW * DPW;
  constexpr int ROW = DB + 4;
  constexpr int SLOT = il_slot(CC, DB);
  constexpr int MA = il_ma(NBUF), MR = il_mr(NBUF);
  static_assert(ROW % 4 == 0, "metadata rows land as 16-byte quads");
  constexpr int S = U16 ? 8 : 4;  // samples per 16-byte element (quarters / eighths)
  static_assert((U16 ? (DPW >= 4 && DPW <= 8) : DPW == 4) && G == (U16 ? 2 : 4) &&
                    DPW * CC <= 64 && CC % 2 == 0,
                "4 (f32) or 4..8 (u16) trials per wave, 4 (f32) or 2 (u16) groups; one lane "
                "per (channel, trial)");
  static_assert(NBUF >= 2 && MA >= 2 * NBUF - 2 && MR > MA, "ring geometry");
  extern __shared__ __attribute__((aligned(16))) float smf[];
  uint4* img = reinterpret_cast<uint4*>(smf);
  int* metar = reinterpret_cast<int*>(img + NBUF * buf_e);  // [MR][SLOT]

  const int per_grp = n_tblk * n_dblk;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  // developer builds only (PDD_SWEEP_DEBUG bit 2): per-wave cycle stamps
  // written into `out` instead of the plane
  const bool stamps = (dbg & 4) != 0;

  // One tile per workgroup.  (A persistent grid -- 256 workgroups walking
  // their XCD's tiles -- measured no faster for the channel sweep: the L2 hit
  // rate of the staging fell from 77% to 48% at unchanged kernel time.)
  int dblk, tblk;
  const int grp = blockIdx.x / per_grp;
  il_tile_of<FX ? PDD_FX_GT : PDD_IL_GT, FX ? (U16 ? PDD_FX_GJ : PDD_FX_GJF) : PDD_IL_GJ, FX>(
      blockIdx.x - grp * per_grp, n_tblk, n_dblk, dblk, tblk);
  const float4* R = R0 + (int64_t)grp * C * nR;
  const int64_t t0 = (int64_t)tblk * Tq;
  const int* mt_b = mt + ((int64_t)grp * n_dblk + dblk) * (C + 1) * ROW;
  const int* cht_t = cht + ((int64_t)grp * n_dblk + dblk) * (maxch + 1);
  const int nchunk = cht_t[0];
  const uint32_t img_lds = lds_addr_of(img);
  const uint32_t voff16 = (uint32_t)lane * 16u;
  // FX tiles: the chunk's window records (lane i = window i, one vector load)
  const int4* wt_b = FX ? wt + ((int64_t)grp * n_dblk + dblk) * maxch * kFxWin : nullptr;
  auto fx_rec = [&](int k) -> int4 {
    if constexpr (FX) return wt_b[(int64_t)min(k, nchunk - 1) * kFxWin + lane];
    else return make_int4(0, 0, 0, 0);
  };
  // one loader's share of chunk k's window DMAs (windows first, first +
  // step, ...): lane i computes window i's source, LDS address and piece
  // count once, then the loader issues its own windows from SGPRs.
  // (Measured and dropped: every wave of the workgroup issuing a share of
  // the DMAs -- configs[3] 101.6 -> 116.4 ms per launch.)
  auto fx_issue = [&](int k, const int4& rec, int first, int step) -> int {
    // the compiler's wait for the record (vmcnt(0): it cannot see the DMAs)
    // lands here, before any DMA of this chunk
    asm volatile("" ::"v"(rec.x), "v"(rec.y), "v"(rec.z), "v"(rec.w));
    const int b = k % NBUF;
    const int nw = __builtin_amdgcn_readlane(rec.w, 0) >> 20;
    const uint64_t sv = (uint64_t)(R + (int64_t)(rec.w & 0xfffff) * nR + (t0 + rec.x - lo));
    const uint32_t dv = img_lds + (uint32_t)((b * buf_e + rec.z) * 16);
    // whole 64-element pieces, then the window's last rv < 64 elements as
    // one piece under an EXEC mask: windows sit back to back in the buffer.
    // (Every window in whole pieces, round 4's layout: configs[3] stage 2
    // 99.25 against 95.36 ms per launch, north star 69.17 against 64.94.)
    const int qv = rec.y >> 6;
    const int rv = rec.y & 63;
    int n = 0;
    for (int i = first; i < nw; i += step) {
      const uint32_t lo32 = __builtin_amdgcn_readlane((uint32_t)sv, i);
      const uint32_t hi32 = __builtin_amdgcn_readlane((uint32_t)(sv >> 32), i);
      const float4* src = (const float4*)(((uint64_t)hi32 << 32) | lo32);
      const uint32_t dst = __builtin_amdgcn_readlane(dv, i);
      const int nq = __builtin_amdgcn_readlane(qv, i);
      n += stage_il_dma_s2(dst, src, nq, voff16);
      const int rem = __builtin_amdgcn_readlane(rv, i);
      if (rem) n += stage_il_dma_tail(dst + (uint32_t)nq * 1024u, src + nq * 64, rem, voff16, lane);
    }
    return n;
  };
  if (w >= NCW) {
    // ---------------- loader waves: metadata rows + sample windows
    // Top issue priority: a loader shares its SIMD with compute waves that
    // have an LDS read or add ready every cycle.
    __builtin_amdgcn_s_setprio(3);
    const int lw = w - NCW;
    int* ring = metar;  // the shared ring (loader 0 fills it)
    // (Measured and dropped, round 5: windows to the loaders in reverse
    // order, so that loader 0, which also issues the metadata rows, takes the
    // fewest -- configs[3] 97.2 / north star 81.7 ms per launch either way.)
    // chunk k = channels c0 .. c0 + ncc - 1 (cht: c0 | ncc << 20), packed
    // into its buffer at the per-channel offsets of the metadata rows
    // (loader 0 reads chunk k + MA's table entry one iteration ahead: a
    // scalar load's latency is not on the loaders' per-chunk path)
    int e_next = (lw == 0 && MA < nchunk) ? cht_t[1 + MA] : 0;
    auto issue_meta = [&](int k) -> int {
      if (k >= nchunk || lw != 0) return 0;
      const int e = k < MA ? cht_t[1 + k] : e_next;
      if (k >= MA && k + 1 < nchunk) e_next = cht_t[2 + k];
      const int n_int = (e >> 20) * ROW;
      int n = 0;
      // 1 KiB per DMA: a chunk's rows in ceil(n_int / 256) instructions (the
      // metadata DMAs of a 96-trial chunk: 4 instead of 13 dword DMAs;
      // configs[3] stage 2 103.1 -> 102.2 ms per launch)
#pragma unroll
      for (int m = 0; m < (SLOT + 255) / 256; ++m) {
        if (m * 256 >= n_int) break;
        dma_ints4(ring + (k % MR) * SLOT + m * 256, mt_b + (int64_t)(e & 0xfffff) * ROW + m * 256,
                  n_int - m * 256, lane);
        ++n;
      }
      return n;
    };
    // FX: the records are loaded two chunks ahead; the load issued after a
    // chunk's DMAs (and the metadata DMAs) is the wave's youngest vector-memory
    // operation, so the counted wait before the next barrier leaves it in
    // flight and its latency is off the per-chunk path
    int4 rec_next = fx_rec(0);
    int4 rec_next2 = fx_rec(1);
    int rec_tail = 0;  // a record load issued after the last chunk's DMAs
    auto issue_samples = [&](int k) -> int {
      if constexpr (FX) {
        const int4 rec = rec_next;
        rec_next = rec_next2;  // (chunk k + 2's record: rec_ahead)
        return fx_issue(k, rec, lw, NLW);
      }
      const int b = k % NBUF;
      // the chunk's window rows {bmin, span, offset, source row} by scalar
      // loads from the global table, all eight issued before one wait: the
      // loaders read no LDS.  (They used to read these fields from the
      // metadata ring, 4 LDS reads per channel queued behind the compute
      // waves' read stream: configs[3] u8 260.1 -> 239.0 ms per launch.)
      static_assert(CC <= 8, "at most eight rows per chunk");
      const int e = cht_t[1 + k];
      const int ncc = e >> 20;
      const il_rows8 r8 = il_load_rows8<ROW>(mt_b + (int64_t)(e & 0xfffff) * ROW + DB);
      const i32x4s_t rr[8] = {r8.r0, r8.r1, r8.r2, r8.r3, r8.r4, r8.r5, r8.r6, r8.r7};
      int n = 0;
#pragma unroll
      for (int i = 0; i < CC; ++i) {
        if (i >= ncc) break;
        // window i from loader i mod NLW, its DMAs in runs sharing M0
        if (i % NLW == lw)
          n += stage_il_dma_win(img_lds + (uint32_t)((b * buf_e + rr[i].z) * 16),
                                R + (int64_t)(rr[i].w & 0xfffff) * nR + (t0 + rr[i].x - lo),
                                Tq + rr[i].y, lane);
      }
      return n;
    };
    auto rec_ahead = [&](int c) -> int {
      rec_tail = 0;
      if constexpr (FX) {
        if (c + 2 < nchunk) {
          rec_next2 = fx_rec(c + 2);
          rec_tail = 1;
          return 1;
        }
      }
      return 0;
    };
    for (int k = 0; k < MA; ++k) issue_meta(k);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // prologue: every ring's first MA slots landed
    asm volatile("" ::: "memory");
    int hist[NBUF];  // hist[i]: DMAs this wave issued i+1 iterations ago
#pragma unroll
    for (int i = 0; i < NBUF; ++i) hist[i] = 0;
#pragma unroll
    for (int s2 = 0; s2 < NBUF - 1; ++s2) {
#pragma unroll
      for (int i = NBUF - 1; i > 0; --i) hist[i] = hist[i - 1];
      hist[0] = s2 < nchunk ? issue_samples(s2) + rec_ahead(s2) : 0;
    }
    uint64_t ts_poll = 0, ts_issue = 0, ts_wait = 0, tA = 0, tB = 0;
    for (int k = 0; k < nchunk; ++k) {
      // retire chunk k (and everything older); the NBUF-2 younger chunks stay in flight
      if (stamps) tA = __builtin_amdgcn_s_memtime();
      int younger = FX ? rec_tail : 0;
#pragma unroll
      for (int i = 0; i < NBUF - 2; ++i) younger += hist[i];
      wait_vmcnt(younger);
      if (stamps) { tB = __builtin_amdgcn_s_memtime(); ts_wait += tB - tA; tA = tB; }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (stamps) { tB = __builtin_amdgcn_s_memtime(); ts_poll += tB - tA; tA = tB; }
      // metadata rows first (loader 0), then the chunk's windows: the rows'
      // latency overlaps the window DMAs instead of trailing them (configs[3]
      // stage 2 101.4 -> 96.3 ms per launch, north star 83.9 -> 82.2).  The
      // compiler's wait for the window records (vmcnt(0): it cannot see the
      // DMAs) is forced here, before any DMA of this iteration, on records
      // loaded one and two chunks ago
      if constexpr (FX)
        asm volatile("" ::"v"(rec_next.x), "v"(rec_next.y), "v"(rec_next.z), "v"(rec_next.w),
                     "v"(rec_next2.x), "v"(rec_next2.y), "v"(rec_next2.z), "v"(rec_next2.w));
      int n = issue_meta(k + MA);
      n += k + NBUF - 1 < nchunk ? issue_samples(k + NBUF - 1) : 0;
      if (k + NBUF - 1 < nchunk) n += rec_ahead(k + NBUF - 1);
      else rec_tail = 0;
#pragma unroll
      for (int i = NBUF - 1; i > 0; --i) hist[i] = hist[i - 1];
      hist[0] = n;
      if (stamps) ts_issue += __builtin_amdgcn_s_memtime() - tA;
    }
    if (stamps && lane == 0) {
      float* o = out + ((int64_t)blockIdx.x * (NCW + NLW) + w) * 4;
      o[0] = (float)ts_wait; o[1] = (float)ts_poll; o[2] = (float)ts_issue; o[3] = 0.f;
    }
    return;
  }

  // ---------------- compute waves: ds_read_b128 at the trial's shift + adds
  // float32 elements: 4 quarter samples per read, float accumulators as float
  // pairs (the adds issue as v_pk_add_f32: two samples per VALU instruction).
  // u16 elements (8/16-bit data): 8 eighth samples per read as packed u16
  // pairs, accumulated with plain 32-bit adds into `lo` (two u16 lanes per
  // add, one v_add3_u32 per channel pair) and normalised every flush_n
  // channels: each lane's bit 15 moves into `hi` (a count of 2^15 per lane,
  // also packed) and `lo` keeps the low 15 bits, so a lane never carries
  // into its neighbour while flush_n * (input bound) <= 32767 (the plan's
  // flush_n).  The total hi * 2^15 + lo is exact (float32-exact below 2^24,
  // the same bound as float accumulators).  16 registers per trial instead
  // of 24 (u16 partial sums + float totals): the tile holds DPW = 6 trials
  // per wave (DB 72) in the registers DPW = 4 took.
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  constexpr int AJ = U16 ? 1 : DPW, AG = U16 ? 1 : G, AH = U16 ? 1 : S / 2;
  f32x2_t acc[AJ][AG][AH];
#pragma unroll
  for (int j = 0; j < AJ; ++j)
#pragma unroll
    for (int g = 0; g < AG; ++g)
#pragma unroll
      for (int h = 0; h < AH; ++h) acc[j][g][h] = (f32x2_t){0.f, 0.f};
  // carries: HI8 (DPW > 6) -- one byte per sample, four samples per
  // register (totals < 255 * 2^15 + 2^16, checked by the plan: 12 registers
  // per trial, DPW = 8 fits); else one u16 per sample, two per register
  // (totals < 2^24: 16 registers per trial)
  constexpr bool HI8 = U16 && DPW > 6;
  constexpr int NHI = U16 ? (HI8 ? 2 : 4) : 1;
  uint32_t lo16[U16 ? DPW : 1][U16 ? G : 1][4], hic[U16 ? DPW : 1][U16 ? G : 1][NHI];
  if constexpr (U16) {
#pragma unroll
    for (int j = 0; j < DPW; ++j)
#pragma unroll
      for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int h = 0; h < 4; ++h) lo16[j][g][h] = 0u;
#pragma unroll
        for (int h = 0; h < NHI; ++h) hic[j][g][h] = 0u;
      }
  }
  auto normalise16 = [&]() {
    if constexpr (U16) {
#pragma unroll
      for (int j = 0; j < DPW; ++j)
#pragma unroll
        for (int g = 0; g < G; ++g) {
          if constexpr (HI8) {
            // lo words 2q and 2q + 1 -> carry bytes 0 / 2 and 1 / 3 of hic[q]
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const uint32_t ca = (lo16[j][g][2 * q] >> 15) & 0x00010001u;
              const uint32_t cb = (lo16[j][g][2 * q + 1] >> 15) & 0x00010001u;
              hic[j][g][q] += ca + (cb << 8);
            }
          } else {
#pragma unroll
            for (int h = 0; h < 4; ++h) hic[j][g][h] += (lo16[j][g][h] >> 15) & 0x00010001u;
          }
#pragma unroll
          for (int h = 0; h < 4; ++h) lo16[j][g][h] &= 0x7fff7fffu;
        }
    }
  };
  // plane value of trial j, group g, eighth / quarter k2 (before out_bias)
  auto value = [&](int j, int g, int k2) -> float {
    if constexpr (U16) {
      const int h = k2 >> 1, half = k2 & 1;
      const uint32_t l = half ? (lo16[j][g][h] >> 16) : (lo16[j][g][h] & 0xffffu);
      uint32_t c;
      if constexpr (HI8)
        c = (hic[j][g][h >> 1] >> (8 * ((h & 1) + 2 * half))) & 0xffu;
      else
        c = half ? (hic[j][g][h] >> 16) : (hic[j][g][h] & 0xffffu);
      return (float)(c * 32768u + l);
    } else {
      return acc[j][g][k2 >> 1][k2 & 1];
    }
  };
  int since_flush = 0;
  const uint32_t lane_byte = lds_addr_of(img) + lane * 16;
  const uint32_t meta_base = lds_addr_of(metar) + w * DPW * 4;  // loader 0's ring
  typedef int i32x4_t __attribute__((ext_vector_type(4)));
  typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
  static_assert(!U16 || DPW * CC <= 64, "one lane per (channel, trial) shift");
  typedef __attribute__((address_space(3))) u32x4_t lds_u32x4_t;
  uint64_t ts_poll = 0, ts_comp = 0, tA = 0, tB = 0;
  int vmeta_n = 0, ncc_n = 0;  // FX: the next chunk's shifts and count
  // (Measured and dropped, round 6: compute-wave issue priorities by age,
  // raised for the youngest third, or rotating by chunk -- the older waves
  // finish a chunk ~20% earlier and wait at its barrier, but the LDS stays
  // saturated to the end of the chunk: configs[3] 89.5 ms per launch either
  // way, DESIGN.md appendix.)
  __builtin_amdgcn_s_barrier();  // prologue barrier (metadata landed)
  asm volatile("" ::: "memory");
  if (stamps) tB = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < nchunk; ++k) {
    const int b = k % NBUF;
    if (stamps) {
      tA = __builtin_amdgcn_s_memtime();
      ts_comp += tA - tB;
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (stamps) { tB = __builtin_amdgcn_s_memtime(); ts_poll += tB - tA; }
    const int slot = k % MR;
    // ONE ds_read_b32 brings the wave's DPW shifts of all CC channels of the
    // chunk (lane DPW*i + j = trial j at channel i, as LDS byte offsets: the
    // plan stores them pre-scaled by 16), each broadcast by v_readlane when
    // its reads issue.  (A ds_read_b128 of 4 shifts per channel costs 4 LDS
    // cycles per channel; this costs 2 per chunk plus one VALU per shift:
    // configs[3] u8 288 -> 280 ms, configs[1] u8 32.7 -> 27.3 ms.)
    // (the shifts include the channel's offset in the packed buffer; row 0's
    // last field is the chunk's channel count)
    typedef __attribute__((address_space(3))) int lds_int_t;
    const int ml = min(lane / DPW, CC - 1) * ROW + lane % DPW;
    auto read_shifts = [&](int sl) -> int {
      return *(const lds_int_t*)(uintptr_t)(meta_base + (uint32_t)((sl * SLOT + ml) * 4));
    };
    auto read_count = [&](int sl) -> int {
      return *(const lds_int_t*)(uintptr_t)(lds_addr_of(metar) + (uint32_t)((sl * SLOT + DB + 3) * 4));
    };
    int vmeta, ncc;
    if constexpr (FX) {
      // chunk k + 1's shifts and count are read during chunk k (its ring
      // slot landed before barrier k), so no dependent LDS round trip stands
      // between a barrier and the first sample read
      vmeta = k == 0 ? read_shifts(slot) : vmeta_n;
      ncc = __builtin_amdgcn_readfirstlane(k == 0 ? read_count(slot) : ncc_n) >> 20;
      if (k + 1 < nchunk) {
        vmeta_n = read_shifts((k + 1) % MR);
        ncc_n = read_count((k + 1) % MR);
      }
    } else {
      vmeta = read_shifts(slot);
      // (the channel count rides in a separate read: folding it into the shift
      // read -- lanes >= DPW * CC -- measured 1.6% slower for u16, neutral for f32)
      ncc = __builtin_amdgcn_readfirstlane(read_count(slot)) >> 20;
    }
    const uint32_t cb = lane_byte + (uint32_t)(b * buf_e * 16);
    if constexpr (U16) {
      // normalise before a chunk could carry a u16 lane past 65535
      if (since_flush + ncc > flush_n) {
        since_flush = 0;
        normalise16();
      }
      since_flush += ncc;
      // channel pairs (acc + x_c + x_c+1: one v_add3_u32 per two samples);
      // u16 chunks always hold an even count (an odd channel count ends in
      // a pad channel whose window is a row of zeros)
      u32x4_t v0[G], v1[G];
      auto pair = [&](int i) {
#pragma unroll
        for (int j = 0; j < DPW; ++j) {
          const uint32_t s0 = (uint32_t)__builtin_amdgcn_readlane(vmeta, DPW * i + j);
          const uint32_t s1 = (uint32_t)__builtin_amdgcn_readlane(vmeta, DPW * (i + 1) + j);
#pragma unroll
          for (int g2 = 0; g2 < G; ++g2) {
            v0[g2] = *(const lds_u32x4_t*)(uintptr_t)(cb + s0 + g2 * 1024);
            v1[g2] = *(const lds_u32x4_t*)(uintptr_t)(cb + s1 + g2 * 1024);
          }
#pragma unroll
          for (int g2 = 0; g2 < G; ++g2) {
            lo16[j][g2][0] = add3_u32(lo16[j][g2][0], v0[g2].x, v1[g2].x);
            lo16[j][g2][1] = add3_u32(lo16[j][g2][1], v0[g2].y, v1[g2].y);
            lo16[j][g2][2] = add3_u32(lo16[j][g2][2], v0[g2].z, v1[g2].z);
            lo16[j][g2][3] = add3_u32(lo16[j][g2][3], v0[g2].w, v1[g2].w);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
#pragma unroll
      for (int i = 0; i < CC; i += 2)
        if (i < ncc) pair(i);
    } else {
#pragma unroll
      for (int i = 0; i < CC; ++i) {
        if (i >= ncc) break;
        // the channel's DPW read addresses first (readlane + add each), then
        // two trials of reads in flight: trial j's adds overlap trial j+1's
        // reads (the accumulators take 64 of the 128 VGPRs, the reads 2 x 4G)
        uint32_t a[DPW];
#pragma unroll
        for (int j = 0; j < DPW; ++j)
          a[j] = cb + (uint32_t)__builtin_amdgcn_readlane(vmeta, DPW * i + j);
        f32x4_t v[DPW][G];
#pragma unroll
        for (int j = 0; j < DPW; ++j)
#pragma unroll
          for (int g2 = 0; g2 < G; ++g2)
            v[j][g2] = *(const lds_f32x4_t*)(uintptr_t)(a[j] + g2 * 1024);
#pragma unroll
        for (int j = 0; j < DPW; ++j)
#pragma unroll
          for (int g2 = 0; g2 < G; ++g2) {
            acc[j][g2][0] += v[j][g2].xy;
            acc[j][g2][1] += v[j][g2].zw;
          }
        __builtin_amdgcn_sched_group_barrier(0x002, 2 * DPW, 0);  // addresses
        __builtin_amdgcn_sched_group_barrier(0x100, G, 0);        // reads, trial 0
        __builtin_amdgcn_sched_group_barrier(0x100, G, 0);        // reads, trial 1
#pragma unroll
        for (int j = 0; j < DPW; ++j) {
          __builtin_amdgcn_sched_group_barrier(0x002, 2 * G, 0);  // adds, trial j
          if (j + 2 < DPW) __builtin_amdgcn_sched_group_barrier(0x100, G, 0);  // reads, j+2
        }
      }
    }
  }
  if (stamps) ts_comp += __builtin_amdgcn_s_memtime() - tB;
  if (stamps) {
    if (lane == 0) {
      float* o = out + ((int64_t)blockIdx.x * (NCW + NLW) + w) * 4;
      o[0] = 0.f; o[1] = (float)ts_poll; o[2] = (float)ts_comp; o[3] = 1.f;
    }
    return;
  }
  const int d0 = dblk * DB + w * DPW;
  if constexpr (S == 8) {
    if (r2_pad) {
      // Output as the NEXT sweep's float32 quarters image (subband chain,
      // pdd_subband_chain): row r = grp*row_g + d*row_d of R2 ([rows][r2_nR]
      // float4, quarter length Q2 = 2 Qs, single segment, t_base 0) holds
      //   R2[r][j] = (X(j), X(j + Q2), X(j + 2 Q2), X(j + 3 Q2)),  j < r2_nR,
      // X(t) = this sweep's sample t (t < n_out) or the next sweep's pad
      // r2_pad[r].  A lane's eighths (e + k Qs, k < 8) are elements e (even k)
      // and e + Qs (odd k), and its even eighths 2, 4, 6 + the pad are element
      // Q2 + e of the overlap tail (e < r2_ov = r2_nR - Q2 <= Qs).
      float4* R2 = reinterpret_cast<float4*>(out);
#pragma unroll
      for (int j = 0; j < DPW; ++j) {
        const int d = d0 + j;
        if (d >= D) continue;
        const int64_t r = (int64_t)grp * row_g + (int64_t)d * row_d;
        const float pv = r2_pad[r];
        float4* rrow = R2 + r * r2_nR;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int64_t e = t0 + g * 64 + lane;
          if (e >= Qs) continue;
          float x8[8];
#pragma unroll
          for (int k2 = 0; k2 < 8; ++k2)
            x8[k2] = (e + k2 * Qs < n_out) ? value(j, g, k2) + out_bias : pv;
          rrow[e] = make_float4(x8[0], x8[2], x8[4], x8[6]);
          rrow[e + Qs] = make_float4(x8[1], x8[3], x8[5], x8[7]);
          if (e < r2_ov) rrow[2 * Qs + e] = make_float4(x8[2], x8[4], x8[6], pv);
        }
      }
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
    const int d = d0 + j;
    if (d >= D) continue;
    float* orow = out + ((int64_t)grp * row_g + (int64_t)d * row_d) * ld_out + t_base;
    // delay-aligned factorised tiles (fx_skew): trial d's tile covers the
    // elements [t0 - sig[d], t0 - sig[d] + Tq); each element of [0, Qs) is
    // stored by exactly one tile of the trial
    const int64_t ts = t0 - ((FX && sig) ? (int64_t)sig[d] : 0);
#pragma unroll
    for (int k2 = 0; k2 < S; ++k2)
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int64_t t = ts + g * 64 + lane;
        if (t >= 0 && t < Qs && t_base + t + k2 * Qs < n_out)
          orow[t + k2 * Qs] = value(j, g, k2) + out_bias;
      }
  }
}

// ------------------------------------------------------------------ variants
// kind 0: interleaved image + k_sweep_il (dedicated loader waves, NLW);
// kind 1: generic striped k_sweep (register staging; sparse-grid fallback).
struct Variant {
  int kind;
  bool u8;     // kind 1: 8-bit input staged as u16 pairs
  int S, G, DPW, NW, CC, NBUF;
  int NLW;     // kind 0: loader waves (NW = compute waves)
  int threads() const { return (NW + (kind == 0 ? NLW : 0)) * 64; }
  int elem_bytes() const { return kind == 0 ? 16 : (u8 ? 2 * S : 4 * S); }
  int Q() const { return 64 * G; }
  int TB() const { return S * 64 * G; }
  int DB() const { return NW * DPW; }
  // LDS "stride" (elements per channel per buffer) for a max span
  int64_t stride_for(int max_span) const {
    if (kind == 0) return (64 * G + max_span + 63) / 64 * 64;  // whole 64-element DMA granules
    return (Q() + max_span + 15) / 16 * 16;
  }
  int64_t chan_bytes(int64_t stride) const { return stride * elem_bytes(); }
};

// Candidate tilings, best first; the plan takes the first whose LDS fits (a
// sparser grid -- wider shift span per trial block -- moves down the list;
// grouped sweeps skip the kinds that cannot sweep groups).
// Every entry is reached by a named test (tests/test_gpu_parity.py
// test_sweep_variant_ladder).
static const Variant kF32Variants[] = {
    {0, false, 4, 4, 4, 14, 8, 2, 2},  // DB 56, 2 packed buffers of <= 8 channels (configs[1]:
                                       //   37.9 ms against 39.4 with 3 buffers)
    {0, false, 4, 4, 4, 8, 8, 2, 2},   // DB 32
    {1, false, 4, 4, 1, 8, 1, 2, 0},   // generic, DB 8
    {1, false, 4, 1, 1, 1, 1, 2, 0}    // generic, DB 1 (any span that fits 160 KB)
};
// 8-bit input: u16 eighths (12 compute + 4 loader waves: with half the
// compute per staged byte the extra loaders pay off), then the float32-image
// tilings, then the generic u16 kernel.
// Factorised 8/16-bit plans try these first (before their channel tiling):
// u16 eighths, DB 96 -- 8 trials per compute wave with byte-wide carry
// counts (plane sums < 255 * 2^15: C * input bound checked by the plan).
// configs[3] g 4 101.8 -> 97.2 ms per launch, north star g 2 83.3 -> 81.6
// against DB 72; the channel kernel is 2% slower at DB 96 (configs[1] u8
// 21.0 -> 21.5 ms), so channel plans keep DB 72.
#ifndef PDD_FX_DPW
#define PDD_FX_DPW 8
#endif
static const Variant kU8FxVariants[] = {{0, false, 8, 2, PDD_FX_DPW, 12, 8, 2, 4}};
// 8-bit input, short grids (plan_create): u16 eighths, DB 40 in 8-wave
// tiles (5 compute waves of 8 trials + 3 loaders, <= 78 KB of LDS, 120
// VGPRs): two tiles per CU, so one tile's first window DMAs and plane stores
// run under the other's reads.  Reported as variant kShortVi.  (configs[2]
// stage-1 sweep 1.34 -> 1.12 ms against 10 + 4 waves, one tile per CU;
// float32 short grids in 7 + 1-wave DB-28 tiles, two per CU: 1.60 -> 1.57
// ms, not kept: each of the two trial blocks stages every window again.)
static const Variant kU8Short = {0, false, 8, 2, 8, 5, 8, 2, 3};
// float32 input, grouped short grids: quarters, DB 52 (13 compute + 3 loader
// waves; configs[2] stage 2: 50 trials per pass in 52 slots instead of 56)
static const Variant kF32Short = {0, false, 4, 4, 4, 13, 8, 2, 3};
static constexpr int kShortVi = 100;
static const Variant kU8Variants[] = {
    {0, false, 8, 2, 6, 12, 8, 2, 4},   // u16 eighths, DB 72: 6 trials per compute wave in the
                                        //   registers 4 took with float totals (k_sweep_il's
                                        //   15-bit normalised sums), 2 packed buffers
    {0, false, 8, 2, 4, 12, 8, 2, 4},   // u16 eighths, DB 48 (configs[3]: 236.7 ms against 239.0
                                        //   with 3 buffers, once the loaders read no LDS)
    {0, false, 4, 4, 4, 8, 8, 2, 2},    // f32 image of u8 data, DB 32
    {1, true, 8, 2, 1, 8, 1, 2, 0},     // generic u16, DB 8
    {1, true, 8, 1, 1, 1, 1, 2, 0}      // generic u16, DB 1
};

// LDS per workgroup: 16-wave (il) tiles run one per CU, <= 8-wave tiles two
static int64_t lds_budget(const Variant& v) {
  if (v.kind == 0) return (v.NW + v.NLW) * 2 <= 16 ? 78 * 1024 : 158 * 1024;
  return v.NW >= 16 ? 150 * 1024 : 76 * 1024;
}
static constexpr int kLdsMax = 160 * 1024;

typedef void (*sweep_il_fn)(const float4*, int64_t, int, int, const int*, const int*, int, float*,
                            int64_t, int, int64_t, int64_t, int64_t, int, int, int, int, int64_t,
                            int64_t, int, float, const float*, int64_t, int64_t, const int4*,
                            const int*);
static sweep_il_fn il_kernel_for(const Variant& v, bool fx = false) {
  if (fx) {
    // factorised stage 2: u16 eighths (8/16-bit input) or float32 quarters
    if (v.S == 8 && v.NW == 12 && v.NLW == 4 && v.G == 2 && v.CC == 8 && v.NBUF == 2) {
      if (v.DPW == 8) return k_sweep_il<2, 8, 12, 4, 8, 2, true, true>;
      if (v.DPW == 6) return k_sweep_il<2, 6, 12, 4, 8, 2, true, true>;
      if (v.DPW == 4) return k_sweep_il<2, 4, 12, 4, 8, 2, true, true>;
    }
    if (v.S == 4 && v.NW == 14 && v.NLW == 2 && v.G == 4 && v.DPW == 4 && v.CC == 8 && v.NBUF == 2)
      return k_sweep_il<4, 4, 14, 2, 8, 2, false, true>;
    return nullptr;
  }
  if (v.S == 8 && v.NW == 5 && v.NLW == 3 && v.G == 2 && v.CC == 8 && v.NBUF == 2 && v.DPW == 8)
    return k_sweep_il<2, 8, 5, 3, 8, 2, true>;
  if (v.S == 8 && v.NW == 12 && v.NLW == 4 && v.G == 2 && v.CC == 8 && v.NBUF == 2) {
    if (v.DPW == 6) return k_sweep_il<2, 6, 12, 4, 8, 2, true>;
    if (v.DPW == 4) return k_sweep_il<2, 4, 12, 4, 8, 2, true>;
  }
  if (v.S == 4 && v.G == 4 && v.DPW == 4 && v.CC == 8 && v.NBUF == 2) {
    if (v.NW == 13 && v.NLW == 3) return k_sweep_il<4, 4, 13, 3, 8, 2>;
    if (v.NW == 14 && v.NLW == 2) return k_sweep_il<4, 4, 14, 2, 8, 2>;
    if (v.NW == 8 && v.NLW == 2) return k_sweep_il<4, 4, 8, 2, 8, 2>;
  }
  return nullptr;
}

typedef void (*sweep_fn)(const void*, int64_t, int, int64_t, const int*, int, int, const int*,
                         const int*, int, const float*, float*, int64_t, int64_t, int, int, int,
                         int);

static sweep_fn kernel_for(const Variant& v) {
#define V(U, S_, G_, DPW_, NW_, CC_, NB_)                                                     \
  if (v.u8 == U && v.S == S_ && v.G == G_ && v.DPW == DPW_ && v.NW == NW_ && v.CC == CC_ &&  \
      v.NBUF == NB_)                                                                         \
    return k_sweep<U, S_, G_, DPW_, NW_, CC_, NB_>;
  V(false, 4, 4, 1, 8, 1, 2)
  V(false, 4, 1, 1, 1, 1, 2)
  V(true, 8, 2, 1, 8, 1, 2)
  V(true, 8, 1, 1, 1, 1, 2)
#undef V
  return nullptr;
}

// Developer knobs (kernel stamps, timing-only decompositions, forced
// tilings) live in scripts/probes/dev_knobs.patch, applied to a copy of this
// file by scripts/build_dev.sh; the production library reads no environment
// variable: no debug bits, no forced tiling.
static int debug_flags() { return 0; }
static int forced_variant() { return -1; }

}  // namespace pdd

struct pdd_sweep_plan {
  pdd::Variant v;
  int64_t D, C, Dpad, n_dblk;
  int max_span, stride, cc, lds_bytes;
  int* d_tab = nullptr;    // [C][Dpad] shifts relative to the block minimum
  int* d_bmin = nullptr;   // [n_dblk][C]; interleaved kernel: chunk tables
  int maxch = 0;           // interleaved kernel: most chunks of a trial block
  int* d_bspan = nullptr;  // [n_dblk][C]
  int max_bin = 0, min_bin = 0;
  int vi = 0;              // index of the chosen tiling in its candidate list
  int fx = 0;              // factorised sweep: channels per group (0 = channel by channel)
  int64_t n_pat = 0;       // factorised: pattern series (stage-1 rows, + 1 zero row)
  int64_t fx_rows = 0;     // factorised: metadata rows per trial block (groups + pad groups)
  int fx_rspan = 0;        // factorised: widest relative-shift range of a group (stage-1 LDS)
  int* d_pat = nullptr;    // factorised: [n_pat][4] {c0, r1, r2, r3}
  int* d_wt = nullptr;     // factorised: [n_dblk][maxch][kFxWin][4] window records
  int* d_gtab = nullptr;   // factorised: per group first pattern + relative-shift range (LDS stage 1)
  int* d_sig = nullptr;    // factorised, delay-aligned tiles: [Dpad] per-trial skew (fx_skew)
  int fx_lo = 0, fx_hi = 0;  // factorised: pattern-row sample range (skewed shifts; fx_build)
  int fx_tpad = 0;         // factorised: extra time-tile elements per segment (max skew, whole tiles)
  int fx_sig_max = 0;      // factorised: largest per-trial skew
  int dtype = PDD_F32;     // input element type
  int input_max = 0;       // largest input value (integer input; 0 = the dtype's bound)
  int poison = 0;          // pdd_sweep_plan_set_poison: 0xFF-fill the pattern image (tests)
  int64_t seg_bytes = 0;   // pdd_sweep_plan_set_segment_bytes: segment budget cap (0 = default)
  int64_t n_grp = 1;       // independent channel groups (grouped sweep)
  // timing of the sweep kernel (pdd_sweep_set_timing): one event pair per
  // bracketed launch, recorded on the execute stream without host syncs
  static constexpr int kEvPairs = 1024;
  hipEvent_t* ev = nullptr;  // [2 * kEvPairs]
  int timing = 0;
  int timed = 0;             // launches bracketed since the last query
  int dropped = 0;           // launches past the pool (not bracketed)
};

using namespace pdd;

// Interleaved path: the output is produced in time segments whose
// interleaved copy R fits a scratch budget (the library's per-stream
// scratch, pdd::scratch, reused across calls); each segment is one k_interleave + one k_sweep_il.
// IlExtra.ds > 1: x is the 8-bit block at the raw rate (channel-major rows
// of N * ds samples, lay.ld apart), co-added by ds in the interleave
// pre-pass.  IlExtra.r2_pad: the output is the next sweep's quarters image
// (k_sweep_il's R2 epilogue; one segment).  IlExtra.R_pre: the image of this
// sweep was built by the previous one (quarter length Qs_pre, nR_pre
// elements per row): no interleave pre-pass, one segment.
// Output samples one segment of the interleaved path can hold (<= 0: the
// delay span alone exceeds the scratch budget of R).  The budget is capped
// by the device memory free now (plus what this stream's image / pattern
// slots already hold): a smaller GPU or a busier one gets more, shorter
// segments instead of a scratch allocation failure.
// Sample range [lo, hi] of an image row around the segment's columns:
// channel plans min(0, min bin) .. max(0, max bin); factorised plans the
// skewed shifts' range plus the extra time tiles of delay-aligned tiles.
static void il_lohi(const pdd_sweep_plan* p, int64_t& lo, int64_t& hi) {
  if (p->fx) {
    lo = p->fx_lo;
    hi = (int64_t)p->fx_hi + p->fx_tpad;
  } else {
    lo = std::min(0, p->min_bin);
    hi = std::max(0, p->max_bin);
  }
}

static int64_t il_seg_samples(const pdd_sweep_plan* p, hipStream_t st) {
  const int Tq = 64 * p->v.G;
  const int64_t C = p->C * p->n_grp;
  int64_t lo, hi;
  il_lohi(p, lo, hi);
  // bytes of R per segment: 16 GiB = one segment per quarter of a 4096 x
  // 2^22 block (configs[3] at 4 time batches), few launches per step
  int64_t budget = (int64_t)16 << 30;
  // factorised plans also hold the stage-1 pattern image (n_pat + 1 rows)
  const int64_t rows = C + (p->fx ? p->n_pat + 2 : 0);
  // (80 GiB: configs[3] in 4 launches of 1.04 M columns -- 572.9 against 578.3
  // ms per step with 8 launches of 40 GiB; the free-memory cap below keeps
  // smaller or busier GPUs on more, shorter segments)
  if (p->fx) budget = (int64_t)80 << 30;
  if (p->seg_bytes > 0) {
    // a caller's cap (pdd_sweep_plan_set_segment_bytes: tests of the
    // multi-segment path on small blocks)
    budget = std::max<int64_t>(p->seg_bytes, 1 << 16);
  } else {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
      const int64_t avail = (int64_t)fr + (int64_t)scratch_held(st, kScratchImage) +
                            (p->fx ? (int64_t)scratch_held(st, kScratchPattern) : 0);
      // keep 1/8 of it and 512 MiB for the caller
      budget = std::min(budget, std::max<int64_t>(avail - avail / 8 - ((int64_t)512 << 20),
                                                  (int64_t)64 << 20));
    }
  }
  const int64_t nr_max = budget / (rows * 16);
  return (nr_max - (hi - lo) - 64) / Tq * Tq * p->v.S;
}

struct IlExtra {
  int ds = 1;
  bool one_seg = false;  // the caller checked that one segment fits (pdd_subband_chain)
  const float* r2_pad = nullptr;
  int64_t r2_nR = 0, r2_ov = 0;
  const float4* R_pre = nullptr;
  int64_t Qs_pre = 0, nR_pre = 0;
  // factorised plans, staged execution (pdd_sweep_execute_stage): bit 0 =
  // stage 1 (pattern image), bit 1 = stage 2 (the sweep), into the caller's
  // pattern buffer P_ext of P_bytes (one segment)
  int stages = 3;
  uint4* P_ext = nullptr;
  int64_t P_bytes = 0;
};
static int execute_il(const pdd_sweep_plan* p, const void* x, int64_t N, InLayout lay,
                      int64_t x_off, int pad_mode, const float* padvals, float* out,
                      int64_t ld_out, int64_t n_out, int64_t row_g, int64_t row_d, float out_bias,
                      void* stream, const IlExtra& ex = IlExtra()) {
  const int ds = ex.ds;
  const int Tq = 64 * p->v.G;
  const int SP = p->v.S;  // samples per element: 4 (float32 quarters) or 8 (u16 eighths)
  const bool u16 = (SP == 8);
  PDD_REQUIRE(!u16 || p->dtype != PDD_F32, "pdd_sweep_execute: u16 path needs integer input");
  // packed u16 lanes are normalised to 15 bits every floor(32767 / max value)
  // channels (k_sweep_il): 128 channels of 8-bit values, 32 of 16-bit values
  // <= 1023, 64 of the wrap-mode zero-DM image downsampled by 2 (<= 510;
  // pdd_sweep_plan_set_input_max); factorised plans sum patterns of fx samples
  const int vmax = p->input_max > 0 ? p->input_max : (p->dtype == PDD_U8 ? 255 : 1023);
  const int flush_n = std::min(256, 32767 / (vmax * std::max(1, p->fx)));
  PDD_REQUIRE(!u16 || flush_n >= p->v.CC, "pdd_sweep_execute: input bound %d too large for the "
              "packed 16-bit sums", vmax);
  const int64_t C = p->C * p->n_grp;  // all channels (groups are contiguous channel ranges)
  int64_t lo, hi;
  il_lohi(p, lo, hi);
  // output samples per segment
  int64_t seg = (ex.one_seg || ex.P_ext) ? std::max<int64_t>(n_out, 1)
                                         : il_seg_samples(p, as_stream(stream));
  PDD_REQUIRE(seg > 0, "pdd_sweep_execute: delay span %lld too wide for the segment budget",
              (long long)(hi - lo));
  // equal segments (whole tiles): every launch does the same work
  const int64_t tile_s = (int64_t)SP * Tq;
  const int64_t nseg = cdiv(n_out, seg);
  seg = cdiv(cdiv(n_out, nseg), tile_s) * tile_s;
  const int64_t qs_max = seg / SP;
  const int64_t nr_alloc = qs_max + (hi - lo) + 64;
  PDD_REQUIRE(!(ex.r2_pad || ex.R_pre) || nseg == 1,
              "pdd_subband_chain: the stages need one segment each (%lld)", (long long)nseg);
  if (ex.R_pre)
    PDD_REQUIRE(lo == 0 && n_out <= SP * ex.Qs_pre && ex.Qs_pre % Tq == 0 &&
                    ex.nR_pre >= ex.Qs_pre + hi + 64 && !u16,
                "pdd_subband_chain: stage-2 image does not cover this plan");
  float4* R = nullptr;
  hipStream_t st = as_stream(stream);
  // factorised plans with the LDS stage 1 build their pattern image straight
  // from x (k_fx_patterns_x): no u16-eighths image R
  const bool fx_direct = p->fx && p->d_gtab && !ex.R_pre && ds == 1;
  // C rows of the image + one row of zeros (the u16 kernel's pad channel)
  if (!ex.R_pre && !fx_direct) {
    R = static_cast<float4*>(scratch(st, kScratchImage, (size_t)((C + 1) * nr_alloc) * sizeof(float4)));
    if (!R) return -2;
  }
  // factorised plans: the pattern image (stage 1), n_pat rows + a row of zeros
  uint4* P = nullptr;
  if (ex.P_ext) {
    PDD_REQUIRE(p->fx && (int64_t)(p->n_pat + 1) * nr_alloc * 16 <= ex.P_bytes,
                "pdd_sweep_execute_stage: pattern buffer of %lld bytes < %lld",
                (long long)ex.P_bytes, (long long)((p->n_pat + 1) * nr_alloc * 16));
    P = ex.P_ext;
  }
  if (p->fx) {
    // (ds > 1: the interleave pre-pass co-adds the raw rows into R and stage
    // 1 builds the patterns from R: sums of fx co-adds <= 4 * 1020 stay exact)
    PDD_REQUIRE(u16 == (p->dtype != PDD_F32) && !ex.r2_pad && !ex.R_pre && p->n_grp == 1 &&
                    (u16 || fx_direct),
                "pdd_sweep_execute: factorised plans take single-group input (float32: raw rate)");
    if (!P)
      P = static_cast<uint4*>(scratch(st, kScratchPattern, (size_t)((p->n_pat + 1) * nr_alloc) * sizeof(uint4)));
    if (!P) return -2;
  }
  const int dbg = debug_flags();
  int rc = 0;
  for (int64_t t_base = 0; t_base < n_out && rc == 0; t_base += seg) {
    const int64_t cnt = std::min(seg, n_out - t_base);
    const int64_t Qs = ex.R_pre ? ex.Qs_pre : cdiv(cdiv(cnt, SP), Tq) * Tq;
    const int64_t nR = ex.R_pre ? ex.nR_pre : Qs + (hi - lo) + 64;
    if (ex.r2_pad && ex.r2_nR != 2 * Qs + ex.r2_ov) { rc = -4; break; }
    dim3 g1((unsigned)cdiv(nR, 256 * kIlPer), (unsigned)C);
    if (ex.R_pre || fx_direct) {
      // image built by the previous sweep / none (factorised stage 1 reads x)
    } else if (hipMemsetAsync(R + C * nR, 0, (size_t)nR * sizeof(float4), st) != hipSuccess) {
      rc = -3;
      break;
    } else if (ds > 1) {
      const bool vec = ds != 3 && (uintptr_t)x % ds == 0 && lay.ld % ds == 0;
      const int64_t b0 = t_base + lo + x_off;
      const int J = 16 / (int)ds;
      const bool vec16 = ds != 3 && (uintptr_t)x % 16 == 0 && lay.ld % 16 == 0 && b0 % J == 0 &&
                         Qs % J == 0;
      const dim3 gv((unsigned)cdiv(nR, 256 * J), (unsigned)C);
#define ILDS(F_, V_)                                                                           \
  hipLaunchKernelGGL((k_interleave_u16_ds<F_, V_>), g1, dim3(256), 0, st, (const uint8_t*)x, \
                     lay.ld, N, b0, Qs, nR, pad_mode, padvals, (uint4*)R)
      if (vec16 && ds == 2)
        hipLaunchKernelGGL(k_interleave_u16_ds_v<2>, gv, dim3(256), 0, st, (const uint8_t*)x,
                           lay.ld, N, b0, Qs, nR, pad_mode, padvals, (uint4*)R);
      else if (vec16)
        hipLaunchKernelGGL(k_interleave_u16_ds_v<4>, gv, dim3(256), 0, st, (const uint8_t*)x,
                           lay.ld, N, b0, Qs, nR, pad_mode, padvals, (uint4*)R);
      else if (ds == 2 && vec) ILDS(2, true);
      else if (ds == 2) ILDS(2, false);
      else if (ds == 3) ILDS(3, false);
      else if (vec) ILDS(4, true);
      else ILDS(4, false);
#undef ILDS
    } else if (u16 && p->dtype == PDD_U8)
      hipLaunchKernelGGL(k_interleave_u16<uint8_t>, g1, dim3(256), 0, st, (const uint8_t*)x, lay, N,
                         t_base + lo + x_off, Qs, nR, pad_mode, padvals, (uint4*)R);
    else if (u16)
      hipLaunchKernelGGL(k_interleave_u16<uint16_t>, g1, dim3(256), 0, st, (const uint16_t*)x, lay,
                         N, t_base + lo + x_off, Qs, nR, pad_mode, padvals, (uint4*)R);
    else if (p->dtype == PDD_U16)
      hipLaunchKernelGGL(k_interleave<uint16_t>, g1, dim3(256), 0, st, (const uint16_t*)x, lay, N,
                         t_base + lo + x_off, Qs, nR, pad_mode, padvals, R);
    else if (p->dtype == PDD_U8)
      hipLaunchKernelGGL(k_interleave<uint8_t>, g1, dim3(256), 0, st, (const uint8_t*)x, lay, N,
                         t_base + lo + x_off, Qs, nR, pad_mode, padvals, R);
    else
      hipLaunchKernelGGL(k_interleave<float>, g1, dim3(256), 0, st, (const float*)x, lay, N,
                         t_base + lo + x_off, Qs, nR, pad_mode, padvals, R);
    if (hipGetLastError() != hipSuccess) { rc = -3; break; }
    if (p->fx && (ex.stages & 1)) {
      // pdd_sweep_plan_set_poison (a parity-test switch): the pattern rows
      // are filled with 0xFF bytes first, so a sum that read an element stage
      // 1 did not write (the per-pattern ranges of fx_build) shows as a NaN /
      // an overflowed lane instead of a stale-but-plausible value
      if (p->poison && hipMemsetAsync(P, 0xFF, (size_t)(p->n_pat * nR) * sizeof(uint4), st) != hipSuccess) {
        rc = -3;
        break;
      }
      if (hipMemsetAsync(P + p->n_pat * nR, 0, (size_t)nR * sizeof(uint4), st) != hipSuccess) {
        rc = -3;
        break;
      }
      const int NG = (int)(p->C / p->fx);
      const int fxe = p->dtype == PDD_F32 ? kFxEf : kFxE;  // stage-1 block length
      const dim3 gp((unsigned)NG, (unsigned)cdiv(nR, fxe));
      const size_t lds_p = (size_t)(p->fx * (fxe + p->fx_rspan)) * sizeof(uint4);
      const int64_t b0 = t_base + lo + x_off;
      // (stage-1 kernels are instanced per group size: fx_build makes groups of 2 or 4)
#define PDD_FX_S1(K2, K4, ...)                                                     \
  do {                                                                             \
    if (p->fx == 4) hipLaunchKernelGGL(K4, gp, dim3(256), lds_p, st, __VA_ARGS__); \
    else hipLaunchKernelGGL(K2, gp, dim3(256), lds_p, st, __VA_ARGS__);            \
  } while (0)
      if (fx_direct && p->dtype == PDD_F32) {
        PDD_FX_S1(k_fx_patterns_xf<2>, k_fx_patterns_xf<4>, (const float*)x, lay, N, b0, Qs, nR,
                  pad_mode, padvals, (const int4*)p->d_pat, p->d_gtab, NG, p->fx, (float4*)P);
      } else if (fx_direct && p->dtype == PDD_U8) {
        PDD_FX_S1((k_fx_patterns_x<uint8_t, 2>), (k_fx_patterns_x<uint8_t, 4>), (const uint8_t*)x,
                  lay, N, b0, Qs, nR, pad_mode, padvals, (const int4*)p->d_pat, p->d_gtab, NG, p->fx,
                  P);
      } else if (fx_direct) {
        PDD_FX_S1((k_fx_patterns_x<uint16_t, 2>), (k_fx_patterns_x<uint16_t, 4>), (const uint16_t*)x,
                  lay, N, b0, Qs, nR, pad_mode, padvals, (const int4*)p->d_pat, p->d_gtab, NG, p->fx,
                  P);
#undef PDD_FX_S1
      } else if (p->d_gtab) {
        hipLaunchKernelGGL(k_fx_patterns_lds, gp, dim3(256), lds_p, st, (const uint4*)R, nR,
                           (const int4*)p->d_pat, p->d_gtab, NG, p->fx, P);
      } else {
        hipLaunchKernelGGL(k_fx_patterns, dim3((unsigned)p->n_pat, (unsigned)cdiv(nR, 256 * kIlPer)),
                           dim3(256), 0, st, (const uint4*)R, nR, (const int4*)p->d_pat, p->fx, P);
      }
      if (hipGetLastError() != hipSuccess) { rc = -3; break; }
    }
    // (delay-aligned factorised tiles: fx_tpad / Tq more time tiles, whose
    // trials cover the columns their skew moved past the last tile)
    if (!(ex.stages & 2)) continue;  // (staged: stage 1 only)
    const int64_t n_tblk = Qs / Tq + (p->fx ? p->fx_tpad / Tq : 0);
    const int64_t blocks = n_tblk * p->n_dblk * p->n_grp;
    if (blocks >= (1ll << 31)) { rc = -1; break; }
    pdd_sweep_plan* pm = const_cast<pdd_sweep_plan*>(p);
    const bool bracket = p->timing && p->timed < pdd_sweep_plan::kEvPairs;
    if (p->timing && !bracket) pm->dropped++;
    if (bracket) (void)hipEventRecord(p->ev[2 * p->timed], st);
    hipLaunchKernelGGL(il_kernel_for(p->v, p->fx != 0), dim3((unsigned)blocks), dim3(p->v.threads()),
                       p->lds_bytes, st, ex.R_pre ? ex.R_pre : (p->fx ? (const float4*)P : R), nR,
                       (int)(p->fx ? p->fx_rows - 1 : p->C), (int)lo, p->d_tab,
                       p->d_bmin, p->maxch, out, ld_out, (int)p->D, Qs, t_base, t_base + cnt,
                       p->stride, (int)n_tblk, (int)p->n_dblk, dbg, row_g, row_d, flush_n, out_bias,
                       ex.r2_pad, ex.r2_nR, ex.r2_ov, (const int4*)p->d_wt, p->d_sig);
    if (hipGetLastError() != hipSuccess) rc = -3;
    if (bracket) {
      (void)hipEventRecord(p->ev[2 * p->timed + 1], st);
      pm->timed++;
    }
  }
  if (rc == -4) set_error("pdd_subband_chain: stage-2 image geometry mismatch");
  if (rc == -1) set_error("pdd_sweep_execute: grid too large");
  if (rc == -3) set_error("pdd_sweep_execute: kernel launch failed");
  return rc;
}

extern "C" {

// Tables of a factorised plan (module comment at k_fx_patterns): the
// pattern pool, the per-(trial block, group) metadata rows in the layout of
// the channel sweep (DB LDS byte offsets -- the trial's pattern window +
// base shift -- then {0, 0, 0, group | groups in the chunk << 20}), the chunk
// tables, and the window records of every chunk.  Returns false when a chunk
// cannot hold a group pair's windows or the factorisation does not pay.
struct FxTables {
  std::vector<int> pat, mt, cht, wt, gtab;  // gtab empty: a group's shift range exceeds kFxRspan
  int64_t n_pat = 0, rows_pb = 0;  // metadata rows per trial block
  int rspan = 0;                   // widest relative-shift range of a group
  int maxch = 0;
  double cost_b = 0, cost_f = 0;   // modelled cycles per time tile: channel sweep / factorised
  double el_f = 0, el_b = 0;       // staged elements per time tile (the model's inputs)
  double pair_ratio = 1.0;         // mean chunks of the re-chunked pair order / own packing
  // delay-aligned tiles: trial d's tile covers output elements [t0 - sig[d],
  // t0 - sig[d] + Tq) (sig per padded trial, >= 0); the pattern rows cover
  // samples lo_f .. hi_f (+ tpad) around the segment (fx_skew below)
  std::vector<int> sig;
  int sig_max = 0, lo_f = 0, hi_f = 0;
};

// Delay-aligned tiles (factorised plans).  A trial block's tile reads, at
// group g, the windows [t0 + b[d][g], t0 + b[d][g] + Tq) of its trials: the
// window of a pattern spans the drift of b[d][g] over the block's trials (up
// to ~680 samples at the bottom of the north star's band against Tq = 128
// elements).  Trial d's tile may as well cover the output elements [t0 -
// sig[d], t0 - sig[d] + Tq) for any per-trial skew sig[d]: it then reads
// group g at b[d][g] - sig[d].  With sig[d] = b[d][gr] - min over the block
// (gr: a reference group near the middle of the band, the one minimising the
// summed drift of b - sig over the groups) the drift of group g becomes
// |drift(g) - drift(gr)|: the north star stages 24% fewer window elements,
// configs[3] 19% (scripts/probes/fx_model.cpp).  The plane is the same
// sum at the same (trial, column): only which tile produces a column changes
// (each segment gets ceil(max sig / Tq) more time tiles; the kernel stores
// elements inside [0, Qs) only).
static void fx_skew(const int32_t* tab, int64_t D, int64_t C, int64_t DB, int fx,
                    std::vector<int>& sig) {
  const int64_t NG = C / fx, n_dblk = cdiv(D, DB);
  sig.assign((size_t)(n_dblk * DB), 0);
  std::vector<int> lo((size_t)NG), hi((size_t)NG);
  for (int64_t b = 0; b < n_dblk; ++b) {
    auto base = [&](int64_t j, int64_t g) -> int {
      return tab[std::min(b * DB + j, D - 1) * C + g * fx];
    };
    // candidate reference groups: 17 evenly spaced, then the neighbourhood
    // of the best at the finest step
    auto drift = [&](int64_t gr) -> int64_t {
      std::fill(lo.begin(), lo.end(), INT32_MAX);
      std::fill(hi.begin(), hi.end(), INT32_MIN);
      for (int64_t j = 0; j < DB; ++j) {
        const int s = base(j, gr);
        for (int64_t g = 0; g < NG; ++g) {
          const int x = base(j, g) - s;
          lo[(size_t)g] = std::min(lo[(size_t)g], x);
          hi[(size_t)g] = std::max(hi[(size_t)g], x);
        }
      }
      int64_t t = 0;
      for (int64_t g = 0; g < NG; ++g) t += (int64_t)hi[(size_t)g] - lo[(size_t)g];
      return t;
    };
    int64_t best = -1, best_t = INT64_MAX;
    const int64_t step = std::max<int64_t>(1, NG / 16);
    for (int64_t gr = 0; gr < NG; gr += step) {
      const int64_t t = drift(gr);
      if (t < best_t) { best_t = t; best = gr; }
    }
    for (int64_t gr = std::max<int64_t>(0, best - step + 1); gr < std::min(NG, best + step); gr += std::max<int64_t>(1, step / 8)) {
      const int64_t t = drift(gr);
      if (t < best_t) { best_t = t; best = gr; }
    }
    int mn = INT32_MAX;
    for (int64_t j = 0; j < DB; ++j) mn = std::min(mn, base(j, best));
    for (int64_t j = 0; j < DB; ++j) sig[(size_t)(b * DB + j)] = base(j, best) - mn;
  }
}

static bool fx_build(const int32_t* tab, int64_t D, int64_t C, const Variant& v, int64_t buf_e,
                     int fx, bool force, FxTables& T, bool pairs = true, bool skew = true) {
  if (C % fx != 0 || C < 2 * fx) return false;
  T.el_f = T.el_b = 0;
  const int64_t NG = C / fx, DB = v.DB(), ROW = DB + 4, Tq = 64 * v.G;
  const int64_t n_dblk = cdiv(D, DB);
  // per-trial skew (fx_skew; all zero: tiles aligned on the plane's columns)
  if (skew) fx_skew(tab, D, C, DB, fx, T.sig);
  else T.sig.assign((size_t)(n_dblk * DB), 0);
  const std::vector<int>& sig = T.sig;
  T.sig_max = 0;
  for (int s : sig) T.sig_max = std::max(T.sig_max, s);
  // the group base shift of (padded trial dp, group g) as the tile reads it
  auto bsk = [&](int64_t dp, int64_t g) -> int {
    return tab[std::min(dp, D - 1) * C + g * fx] - sig[(size_t)dp];
  };
  // the pattern rows' sample range relative to the segment: every channel's
  // shift less its trial's skew (a pattern sums its channels at r_k more)
  int32_t lo_all = 0, hi_all = 0;
  for (int64_t d = 0; d < D; ++d)
    for (int64_t c = 0; c < C; ++c) {
      lo_all = std::min(lo_all, tab[d * C + c] - sig[(size_t)d]);
      hi_all = std::max(hi_all, tab[d * C + c] - sig[(size_t)d]);
    }
  // (rounded down to 16 samples: the downsampling pre-pass of the stream
  // takes its 16-byte vector form only on aligned segment starts)
  lo_all = -((-lo_all + 15) / 16 * 16);
  T.lo_f = lo_all;
  T.hi_f = hi_all;
  // pattern of (trial, group): relative shifts r1..r3 (packed key) -> pool row
  std::vector<int> pid((size_t)(D * NG));
  std::unordered_map<uint64_t, int> idx;
  T.pat.clear();
  for (int64_t g = 0; g < NG; ++g) {
    idx.clear();
    for (int64_t d = 0; d < D; ++d) {
      const int32_t* r = tab + d * C + g * fx;
      uint64_t key = 0;
      for (int k = 1; k < fx; ++k) {
        const int64_t rel = (int64_t)r[k] - r[0];
        if (rel < -(1 << 20) || rel >= (1 << 20)) return false;
        key = (key << 21) | (uint64_t)(rel + (1 << 20));
      }
      auto it = idx.find(key);
      int id;
      if (it == idx.end()) {
        id = (int)(T.pat.size() / 4);
        idx.emplace(key, id);
        T.pat.push_back((int)(g * fx));
        for (int k = 1; k < 4; ++k) T.pat.push_back(k < fx ? r[k] - r[0] : 0);
      } else {
        id = it->second;
      }
      pid[(size_t)(d * NG + g)] = id;
    }
  }
  T.n_pat = (int64_t)T.pat.size() / 4;
  {
    // per group: first pattern, then the relative-shift range (stage 1 via LDS)
    T.gtab.assign((size_t)(NG + 1 + 2 * NG), 0);
    bool fits = true;
    int64_t g = -1;
    for (int64_t p = 0; p < T.n_pat; ++p) {
      const int64_t pg = T.pat[(size_t)(4 * p)] / fx;
      while (g < pg) T.gtab[(size_t)(++g)] = (int)p;
      int& lo = T.gtab[(size_t)(NG + 1 + 2 * pg)];
      int& hi = T.gtab[(size_t)(NG + 2 + 2 * pg)];
      for (int k = 1; k < fx; ++k) {
        lo = std::min(lo, T.pat[(size_t)(4 * p + k)]);
        hi = std::max(hi, T.pat[(size_t)(4 * p + k)]);
      }
      if (hi - lo > kFxRspan) fits = false;
      T.rspan = std::max(T.rspan, hi - lo);
    }
    while (g < NG) T.gtab[(size_t)(++g)] = (int)T.n_pat;
    if (!fits) T.gtab.clear();
  }
  if (!T.gtab.empty()) {
    // then [n_pat] x {first, last - nR} = the pattern row's elements stage 2
    // reads: trials of pattern p have base shifts b in [bmin_p, bmax_p], so
    // its windows cover elements [bmin_p - lo, Qs + bmax_p - lo) of a
    // segment's row (nR = Qs + hi - lo + 64; lo = min(0, min bin), hi =
    // max(0, max bin)); stage 1 skips its kFxE-element blocks outside them
    // (5-10% of the image's bytes are delay overhang no trial of the pattern
    // reads)
    // (skewed: b = the base shift less the trial's skew; rows cover [lo_f,
    // Qs + tpad + hi_f), tpad = the skew rounded up to whole time tiles)
    const size_t o = (size_t)(3 * NG + 1);
    T.gtab.resize(o + 2 * (size_t)T.n_pat);
    for (int64_t p = 0; p < T.n_pat; ++p) {
      T.gtab[o + 2 * p] = INT32_MAX;
      T.gtab[o + 2 * p + 1] = INT32_MIN;
    }
    for (int64_t d = 0; d < D; ++d)
      for (int64_t g = 0; g < NG; ++g) {
        const size_t q = o + 2 * (size_t)pid[(size_t)(d * NG + g)];
        const int32_t b = bsk(d, g);
        T.gtab[q] = std::min(T.gtab[q], b - lo_all);
        T.gtab[q + 1] = std::max(T.gtab[q + 1], b - hi_all - 64);
      }
  }
  // float32 patterns are built only by the LDS stage 1 from the input rows
  // (k_fx_patterns_xf: float adds)
  if (v.S == 4 && T.gtab.empty()) return false;
  // (a quick screen: stage 1 + stage 2 adds against the channel sweep's)
  if (!force && (double)T.n_pat * fx + (double)D * NG > 0.75 * (double)D * C) return false;
  if (T.n_pat + 1 >= (1 << 20)) return false;
  const int zero_row = (int)T.n_pat;  // pad groups read a window of this row of zeros
  // Rows (metadata) are laid out per trial block in chunk order: the groups,
  // in pairs (the u16 loop adds two per v_add3_u32), and a pad group wherever
  // a group goes alone -- the last of an odd count, or one whose pair's
  // windows do not fit a chunk buffer together.
  std::vector<std::vector<int>> rows_of((size_t)n_dblk);  // per block: mt rows [row][ROW]
  std::vector<std::vector<int>> chunks((size_t)n_dblk);
  std::vector<std::vector<std::vector<std::array<int, 4>>>> cw((size_t)n_dblk);
  auto gran = [&](int span) -> int64_t { return (Tq + span + 63) / 64 * 64; };
  // a pattern window takes exactly its Tq + span elements of the chunk
  // buffer: its last DMA piece lands under an EXEC mask (k_sweep_il fx_issue)
  auto gran_fx = [&](int span) -> int64_t { return Tq + span; };
  int64_t rows_pb = 0;
  double cost_b = 0, cost_f = 0;
  std::vector<int64_t> prev_seq;  // the even trial block's group order
  double ratio_sum = 0;            // (pair order) replayed / own chunks, summed over odd blocks
  int64_t ratio_n = 0;
  for (int64_t b = 0; b < n_dblk; ++b) {
    std::vector<int>& M = rows_of[(size_t)b];
    int64_t r0 = 0, nrow = 0, used = 0;
    std::vector<std::array<int, 4>> rec;  // the open chunk's window records
    auto close = [&]() {
      if (nrow == 0) return;
      for (int64_t r = r0; r < r0 + nrow; ++r) M[(size_t)(r * ROW + DB + 3)] = (int)(r | (nrow << 20));
      chunks[(size_t)b].push_back((int)(r0 | (nrow << 20)));
      for (auto& x : rec) x[3] |= (int)rec.size() << 20;
      cw[(size_t)b].push_back(rec);
      rec.clear();
      r0 += nrow;
      nrow = 0;
      used = 0;
    };
    // windows of group g in this block: {pattern row, bmin, span}, first-use order
    auto windows = [&](int64_t g, std::vector<std::array<int, 3>>& w) {
      w.clear();
      if (g < 0 || g >= NG) {
        w.push_back({zero_row, 0, 0});
        return;
      }
      for (int64_t j = 0; j < DB; ++j) {
        const int64_t d = std::min(b * DB + j, D - 1);
        const int id = pid[(size_t)(d * NG + g)];
        const int base = bsk(b * DB + j, g);
        size_t i = 0;
        while (i < w.size() && w[i][0] != id) ++i;
        if (i == w.size()) w.push_back({id, base, base});
        else {
          w[i][1] = std::min(w[i][1], base);
          w[i][2] = std::max(w[i][2], base);
        }
      }
      for (auto& x : w) x[2] -= x[1];  // span
    };
    auto need_of = [&](const std::vector<std::array<int, 3>>& w) {
      int64_t n = 0;
      for (auto& x : w) n += gran_fx(x[2]);
      return n;
    };
    // one row (group g, or a pad group for g < 0) with its windows
    auto place = [&](int64_t g, const std::vector<std::array<int, 3>>& w) {
      const size_t base_row = M.size();
      M.resize(base_row + (size_t)ROW, 0);
      std::vector<int64_t> off(w.size());
      for (size_t i = 0; i < w.size(); ++i) {
        off[i] = used;
        rec.push_back({w[i][1], (int)(Tq + w[i][2]), (int)used, w[i][0]});
        used += gran_fx(w[i][2]);
      }
      for (int64_t j = 0; j < DB; ++j) {
        int o = (int)(16 * off[0]);
        if (g >= 0 && g < NG) {
          const int64_t d = std::min(b * DB + j, D - 1);
          const int id = pid[(size_t)(d * NG + g)];
          const int base = bsk(b * DB + j, g);
          size_t i = 0;
          while (w[i][0] != id) ++i;
          o = (int)(16 * (off[i] + base - w[i][1]));
        }
        M[base_row + (size_t)j] = o;
      }
      ++nrow;
    };
    // Packing: a plane row sums over all groups and the sums are exact in
    // any order (float32 plans: regrouped within tolerance), so the groups
    // go into the chunks in any order, in pairs.  Two packings are built
    // per trial block and the one with the lower modelled time is placed:
    //  - best fit: the largest remaining group that fits, then the largest
    //    partner that fits beside it (fewest chunks);
    //  - balanced: the largest remaining group, then the SMALLEST partner
    //    that fits, so every chunk mixes large and small window sets and its
    //    compute (groups) tracks its staging (elements).
    // A chunk's compute overlaps the next chunk's staging, so the model sums
    // max(compute of chunk k, staging of chunk k + 1) plus a fixed cost per
    // chunk.  A group with no partner closes the chunk (or, alone in a fresh
    // chunk, takes a pad group).  (Measured, round 5, stage 2 per launch:
    // best fit / balanced / the model's choice, configs[3] 93.55 / 92.53 /
    // 92.42 ms, north star 62.02 / 66.95 / 61.77 ms.  Best fit over in-order
    // pairs, configs[3] 305 -> 256 chunks per trial block, stage 2 95.1 ms
    // either way; north star 461 -> 361, 65.2 -> 63.1 ms; configs[1] f32 23.9
    // -> 23.7 ms.  Best fit among the 16 lowest unplaced groups only, to keep
    // neighbouring trial blocks in step: configs[3] 97.0 ms.)
    std::vector<std::array<int, 3>> wz;
    windows(-1, wz);
    {
      std::vector<std::vector<std::array<int, 3>>> wg((size_t)NG);
      std::vector<int64_t> need_g((size_t)NG);
      for (int64_t g = 0; g < NG; ++g) {
        windows(g, wg[(size_t)g]);
        need_g[(size_t)g] = need_of(wg[(size_t)g]);
      }
      const int64_t need_z = need_of(wz);
      auto nw = [&](int64_t g) -> int64_t { return g < 0 ? 1 : (int64_t)wg[(size_t)g].size(); };
      auto nd = [&](int64_t g) -> int64_t { return g < 0 ? need_z : need_g[(size_t)g]; };
      // chunks as group lists (-1: a pad group); false when a group cannot fit
      auto pack = [&](bool balanced, std::vector<std::vector<int64_t>>& out) -> bool {
        out.clear();
        std::multimap<int64_t, int64_t> pool;  // need -> group
        for (int64_t g = 0; g < NG; ++g) pool.emplace(need_g[(size_t)g], g);
        auto largest = [&](int64_t room, int64_t wroom) -> int64_t {
          auto it = pool.upper_bound(room);
          while (it != pool.begin()) {
            --it;
            if (nw(it->second) <= wroom) {
              const int64_t g = it->second;
              pool.erase(it);
              return g;
            }
          }
          return -1;
        };
        auto smallest = [&](int64_t room, int64_t wroom) -> int64_t {
          for (auto it = pool.begin(); it != pool.end() && it->first <= room; ++it)
            if (nw(it->second) <= wroom) {
              const int64_t g = it->second;
              pool.erase(it);
              return g;
            }
          return -1;
        };
        std::vector<int64_t> cur;
        int64_t used_c = 0, win_c = 0;
        auto flush = [&]() {
          out.push_back(cur);
          cur.clear();
          used_c = win_c = 0;
        };
        while (!pool.empty()) {
          const bool fresh = cur.empty();
          const int64_t room = buf_e - used_c, wroom = kFxWin - win_c;
          const int64_t a = (int64_t)cur.size() + 2 <= v.CC ? largest(room, wroom) : -1;
          if (a < 0) {
            if (fresh) return false;
            flush();
            continue;
          }
          const int64_t bg = balanced ? smallest(room - nd(a), wroom - nw(a))
                                      : largest(room - nd(a), wroom - nw(a));
          if (bg >= 0 || (fresh && nd(a) + need_z <= room && nw(a) + 1 <= wroom)) {
            cur.push_back(a);
            cur.push_back(bg);
            used_c += nd(a) + nd(bg);
            win_c += nw(a) + nw(bg);
          } else if (fresh) {
            return false;
          } else {
            pool.emplace(nd(a), a);
            flush();
          }
        }
        if (!cur.empty()) flush();
        return true;
      };
      const double kc_g = v.S == 8 ? 440.0 * (double)DB / 48.0 : 1156.0 * (double)DB / 56.0;
      const double st_e = v.S == 8 ? 1.0 : 1.28;
      auto model = [&](const std::vector<std::vector<int64_t>>& ch) -> double {
        auto bytes = [&](const std::vector<int64_t>& c) {
          int64_t n = 0;
          for (int64_t g : c) n += nd(g);
          return (double)n;
        };
        double t = ch.empty() ? 0.0 : st_e * bytes(ch[0]);
        for (size_t k = 0; k < ch.size(); ++k)
          t += std::max(kc_g * (double)ch[k].size(), k + 1 < ch.size() ? st_e * bytes(ch[k + 1]) : 0.0) +
               1200.0;
        return t;
      };
      // (float32 tiles keep best fit: balanced chunks measured 23.24 -> 24.08
      // ms per configs[1] launch although the model preferred them)
      std::vector<std::vector<int64_t>> ch_f, ch_b, ch_r;
      const bool ok_f = pack(false, ch_f);
      const bool ok_b = v.S == 8 && pack(true, ch_b);
      if (!ok_f && !ok_b) return false;
      const auto* ch = !ok_b ? &ch_f : (!ok_f ? &ch_b : (model(ch_b) < model(ch_f) ? &ch_b : &ch_f));
      // The second trial block of an XCD tile group (PDD_FX_GJ = 2) stages
      // its groups in the first block's order, re-chunked to its own window
      // sizes, so the two blocks' concurrent tiles stage the same group's
      // pattern rows at about the same time (L2 hits).  The plan uses it
      // only where the re-chunked orders cost at most 5% more chunks than
      // the blocks' own packings on average (fx_build runs again without it
      // otherwise).  (Measured, round 5: configs[3], +2% chunks, stage 2
      // 90.84 -> 88.69 ms per launch, L2-side fetch 418 -> 329 GB; the north
      // star, +11% chunks, 59.01 -> 59.99 ms with it; a 2.5% per-block gate
      // instead: configs[3] 90.48 -> 91.08, north star 60.76 -> 59.44.)
      if (pairs && v.S == 8 && PDD_FX_GJ == 2 && (b & 1) && !prev_seq.empty()) {
        bool ok = true;
        std::vector<int64_t> cur;
        int64_t used_c = 0, win_c = 0;
        for (size_t i = 0; i + 1 < prev_seq.size() && ok; i += 2) {
          const int64_t ga = prev_seq[i], gb = prev_seq[i + 1];
          const int64_t need = nd(ga) + nd(gb), w = nw(ga) + nw(gb);
          if (need > buf_e || w > kFxWin) { ok = false; break; }
          if ((int64_t)cur.size() + 2 > v.CC || used_c + need > buf_e || win_c + w > kFxWin) {
            ch_r.push_back(cur);
            cur.clear();
            used_c = win_c = 0;
          }
          cur.push_back(ga);
          cur.push_back(gb);
          used_c += need;
          win_c += w;
        }
        if (ok && !cur.empty()) ch_r.push_back(cur);
        if (ok) {
          ratio_sum += (double)ch_r.size() / (double)std::max<size_t>(1, ch->size());
          ++ratio_n;
          ch = &ch_r;
        }
      }
      prev_seq.clear();
      if (!(b & 1))
        for (const auto& c : *ch) prev_seq.insert(prev_seq.end(), c.begin(), c.end());
      for (const auto& c : *ch) {
        for (int64_t g : c) place(g, g < 0 ? wz : wg[(size_t)g]);
        close();
      }
    }
    close();
    rows_pb = std::max(rows_pb, r0);
    // cost model of one tile of this trial block (CU cycles; calibrated on
    // MI355X, round 5): the compute waves take ~440 cycles per channel of a
    // 48-trial u16 tile (~110 per group of 4 once factorised: the adds and
    // LDS reads scale with C / g and with the tile's trials), the loaders
    // ~1.0 per staged element (LDS-DMA issue and landing); the tile pays
    // 1.016 x the larger plus 0.203 x the smaller (the DMAs' LDS writes take
    // LDS cycles from the compute waves' reads).  Fitted on the DB 96 tiles
    // of configs[3] g 4 (1.37 M cycles per tile, staging-bound), the north
    // star g 4 (1.89 M) and g 2 (2.22 M, both terms ~1.8 M).
    int64_t el_b = 0, el_f = 0;  // staged elements: channel sweep / factorised
    for (int64_t c = 0; c < C; ++c) {
      int lo_ = INT32_MAX, hi_ = INT32_MIN;
      for (int64_t j = 0; j < DB; ++j) {
        const int x = tab[std::min(b * DB + j, D - 1) * C + c];
        lo_ = std::min(lo_, x);
        hi_ = std::max(hi_, x);
      }
      el_b += gran(hi_ - lo_);
    }
    for (const auto& ch : cw[(size_t)b])
      for (const auto& r : ch) el_f += (r[1] + 63) / 64 * 64;
    T.el_f += (double)el_f;
    T.el_b += (double)el_b;
    if (v.S == 8) {
      const double kc = 440.0 * (double)DB / 48.0;  // compute cycles per channel of the tile
      auto tile = [](double comp, double st) {
        return 1.016 * std::max(comp, st) + 0.203 * std::min(comp, st);
      };
      cost_b += tile(kc * (double)C, (double)el_b);
      cost_f += tile(kc * (double)C / fx, (double)el_f);
    } else {
      // float32 quarters (configs[1] f32: 1.18 M cycles per 56-trial tile,
      // compute-bound at ~1156 cycles per channel; staging ~1.28 per element)
      const double kc = 1156.0 * (double)DB / 56.0;
      cost_b += std::max(kc * (double)C, 1.28 * (double)el_b);
      cost_f += std::max(kc * (double)C / fx, 1.28 * (double)el_f);
    }
  }
  // stage 1 per time tile: every pattern's Tq elements (2 KiB of eighths, 4 KiB
  // of quarters), written once for all trial blocks, ~251 CU cycles per 2 KiB
  // pattern row plus ~655 per channel group (its input rows and shift range
  // staged once): fitted on k_fx_patterns_x, configs[3] g 4 (12.6 ms per
  // 1.04 M-column launch) and the north star g 4 / g 2 (12.65 / 6.48 ms)
  cost_f += ((double)T.n_pat * 251.0 + (double)NG * 655.0) * (double)Tq / 128.0;
  // the channel sweep's interleave pre-pass: every channel's Tq elements per
  // time tile, written and read once (factorised plans build their pattern
  // rows from the input directly)
  cost_b += (double)C * (double)(Tq * 16) * 2.0 / 6.7;
  T.cost_b = cost_b;
  T.cost_f = cost_f;
  T.pair_ratio = ratio_n ? ratio_sum / (double)ratio_n : 1.0;
  // (the plan takes the factorised tables below 0.95 of the channel sweep's
  // modelled cost: configs[1] u8 g 2 models at 0.927 and measures 18.6
  // against 21.6 ms per step; the margin was 0.9.  Developer builds print the
  // model's numbers with PDD_SWEEP_DEBUG bit 3.)
  if (!force && cost_f > 0.95 * cost_b) return false;
  T.rows_pb = rows_pb;
  T.mt.assign((size_t)(n_dblk * rows_pb * ROW), 0);
  for (int64_t b = 0; b < n_dblk; ++b)
    std::copy(rows_of[(size_t)b].begin(), rows_of[(size_t)b].end(),
              T.mt.begin() + (size_t)(b * rows_pb * ROW));
  size_t maxch = 0;
  for (const auto& l : chunks) maxch = std::max(maxch, l.size());
  T.maxch = (int)maxch;
  T.cht.assign((size_t)(n_dblk * (maxch + 1)), 0);
  T.wt.assign((size_t)(n_dblk * maxch * kFxWin * 4), 0);
  for (int64_t b = 0; b < n_dblk; ++b) {
    const auto& l = chunks[(size_t)b];
    T.cht[(size_t)(b * (maxch + 1))] = (int)l.size();
    for (size_t k = 0; k < l.size(); ++k) {
      T.cht[(size_t)(b * (maxch + 1) + 1 + k)] = l[k];
      const auto& r = cw[(size_t)b][k];
      int* o = &T.wt[((size_t)b * maxch + k) * kFxWin * 4];
      for (size_t i = 0; i < r.size(); ++i)
        for (int f = 0; f < 4; ++f) o[i * 4 + f] = r[i][f];
    }
  }
  return true;
}

static int plan_create(const int32_t* host_table, int64_t n_grp, int64_t D, int64_t C, int dtype,
                       int flags, pdd_sweep_plan** plan_out);

int pdd_sweep_plan_create(const int32_t* host_table, int64_t D, int64_t C, int dtype,
                          pdd_sweep_plan** plan_out) {
  return plan_create(host_table, 1, D, C, dtype, PDD_SWEEP_FACTOR, plan_out);
}

int pdd_sweep_plan_create_ex(const int32_t* host_table, int64_t D, int64_t C, int dtype, int flags,
                             pdd_sweep_plan** plan_out) {
  return plan_create(host_table, 1, D, C, dtype, flags, plan_out);
}

int pdd_sweep_plan_create_grouped(const int32_t* host_table, int64_t n_grp, int64_t D, int64_t C,
                                  int dtype, pdd_sweep_plan** plan_out) {
  return plan_create(host_table, n_grp, D, C, dtype, 0, plan_out);
}

}  // extern "C"

// Largest mean chunk ratio (re-chunked pair order / own packing) at which a
// factorised plan keeps the pair order of its trial blocks (fx_build).
#ifndef PDD_FX_PAIR_MAX
#define PDD_FX_PAIR_MAX 1.06
#endif
static int plan_create(const int32_t* host_table, int64_t n_grp, int64_t D, int64_t C, int dtype,
                       int flags, pdd_sweep_plan** plan_out) {
  PDD_REQUIRE(host_table && plan_out, "pdd_sweep_plan_create: null pointer");
  PDD_REQUIRE(n_grp >= 1 && n_grp * C < (1 << 20), "pdd_sweep_plan_create: bad group count");
  PDD_REQUIRE(D > 0 && C > 0 && D < (1 << 24) && C < (1 << 20),
              "pdd_sweep_plan_create: bad extents D=%lld C=%lld", (long long)D, (long long)C);
  PDD_REQUIRE(dtype == PDD_F32 || dtype == PDD_U8 || dtype == PDD_U16,
              "pdd_sweep_plan_create: dtype must be F32, U8 or U16");
  // 16-bit input (<= 1023) shares the 8-bit tilings minus the generic kernel
  const bool int_in = dtype != PDD_F32;
  const Variant* cands = int_in ? kU8Variants : kF32Variants;
  const int ncand = int_in ? (int)(sizeof(kU8Variants) / sizeof(Variant))
                           : (int)(sizeof(kF32Variants) / sizeof(Variant));

  const int fv = forced_variant();
  // Short grids (the grouped sweeps of a DDplan step: 40-50 trials per
  // group) waste most of a 72-trial tile: 8/16-bit plans start at the
  // 48-trial tiling when it pads the grid to >= 3% fewer trial slots
  // (configs[2] stage 1: 40 trials in 48 slots instead of 72)
  int v0 = 0;
  auto slots = [&](const Variant& x) { return cdiv(D, (int64_t)x.DB()) * x.DB(); };
  if (int_in && slots(kU8Variants[1]) * 103 < slots(kU8Variants[0]) * 100) v0 = 1;
  // ... and grouped plans at the 40-trial tiling (kU8Short, reported as
  // variant kShortVi) when that pads to >= 3% fewer slots again (configs[2]
  // stage 1: 40 trials in 40 slots)
  // (grouped plans only: single-group plans keep the tilings their
  // factorised sweeps are instanced for; kU8Short's 8 trials per wave keep
  // byte-wide carry counts: plane sums <= 255 * 2^15)
  const bool short_first =
      fv < 0 && n_grp > 1 &&
      (int_in ? slots(kU8Short) * 103 < std::min(slots(kU8Variants[0]), slots(kU8Variants[1])) * 100 &&
                    C * (dtype == PDD_U8 ? 255 : 1023) <= 255 * 32768
              : slots(kF32Short) * 103 < slots(kF32Variants[0]) * 100);
  std::vector<std::pair<Variant, int>> cl;  // (tiling, its reported index)
  if (short_first) cl.push_back({int_in ? kU8Short : kF32Short, kShortVi});
  for (int vi = (fv >= 0 && fv < ncand) ? fv : v0; vi < ncand; ++vi) cl.push_back({cands[vi], vi});
  for (const auto& cv : cl) {
    const Variant v = cv.first;
    const int vi = cv.second;
    const bool il = v.kind == 0;
    if (n_grp > 1 && !il) continue;  // only the interleaved kernel sweeps groups
    if (dtype == PDD_U16 && !il) {     // the generic kernel reads 8-bit or float32 rows
      set_error("pdd_sweep_plan_create: DM grid too sparse for a 16-bit-input tile");
      return -1;
    }
    const int64_t DB = v.DB();
    const int64_t n_dblk = cdiv(D, DB);
    const int64_t Dpad = n_dblk * DB;
    std::vector<int> mt_all;  // interleaved path: mt of every group, concatenated
    std::vector<std::vector<int>> chunks;  // interleaved path: per (group, block) chunk list
    int max_span = 0, mx = INT32_MIN, mn = INT32_MAX;
    std::vector<int> tab, bmin, bspan;
    const bool last = (vi == ncand - 1);
    // interleaved kernel: NBUF chunk buffers of buf_e 16-B elements each
    // (what the LDS holds beside the metadata ring); a chunk packs up to CC
    // channel windows of 64-element DMA granules, Tq + span each
    int64_t buf_e = 0;
    bool fits = true;
    if (il) {
      const int64_t room = (last ? kLdsMax : lds_budget(v)) - il_meta_bytes(v.NBUF, v.CC, v.DB());
      buf_e = std::max<int64_t>(0, room / (v.NBUF * 16) / 64 * 64);
    }
    for (int64_t grp = 0; grp < n_grp; ++grp) {
    const int32_t* htab = host_table + grp * D * C;
    tab.assign((size_t)(C * Dpad), 0);
    bmin.assign((size_t)(n_dblk * C), 0);
    bspan.assign((size_t)(n_dblk * C), 0);
    for (int64_t d = 0; d < Dpad; ++d) {
      const int32_t* row = htab + std::min(d, D - 1) * C;
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
    // offsets relative to the block's minimum shift at each channel (what the
    // kernel adds to its LDS base): rel[c][d] = table[d][c] - bmin[d / DB][c]
    for (int64_t c = 0; c < C; ++c)
      for (int64_t d = 0; d < Dpad; ++d) tab[(size_t)(c * Dpad + d)] -= bmin[(size_t)((d / DB) * C + c)];
    if (il) {
      // mt[grp][dblk][c][DB + 4] = the DB shifts as LDS byte offsets in the
      // chunk buffer (16 x (shift - bmin + channel offset)), then {bmin, span,
      // channel offset (elements), c | channels in the chunk << 20}; chunks filled
      // greedily, channel order, up to CC channels or buf_e elements
      const int64_t ROWN = DB + 4;
      const int64_t Tq = 64 * v.G;
      const size_t moff = mt_all.size();
      mt_all.resize(moff + (size_t)(n_dblk * (C + 1) * ROWN), 0);
      const bool pairs = v.S == 8;  // the u16 kernel sums channel pairs
      for (int64_t b = 0; b < n_dblk && fits; ++b) {
        std::vector<int> list;
        int64_t c0 = 0, used = 0, ncc = 0;
        auto close = [&]() {
          for (int64_t c = c0; c < c0 + ncc; ++c)
            mt_all[moff + (size_t)((b * (C + 1) + c) * ROWN + DB + 3)] =
                (int)((c < C ? c : (n_grp - grp) * C) | (ncc << 20));
          list.push_back((int)(c0 | (ncc << 20)));
        };
        // window of channel c (c == C: the pad channel, Tq elements of zeros)
        auto win_of = [&](int64_t c) -> int64_t {
          return (Tq + (c < C ? bspan[(size_t)(b * C + c)] : 0) + 63) / 64 * 64;
        };
        auto place = [&](int64_t c) {
          const size_t base = moff + (size_t)((b * (C + 1) + c) * ROWN);
          for (int64_t d = 0; d < DB; ++d)
            mt_all[base + d] = (int)(16 * ((c < C ? tab[(size_t)(c * Dpad + b * DB + d)] : 0) + used));
          mt_all[base + DB] = c < C ? bmin[(size_t)(b * C + c)] : 0;
          mt_all[base + DB + 1] = c < C ? bspan[(size_t)(b * C + c)] : 0;
          mt_all[base + DB + 2] = (int)used;
          used += win_of(c);
          ++ncc;
        };
        const int64_t step = pairs ? 2 : 1;
        for (int64_t c = 0; c < C; c += step) {
          const int64_t w = win_of(c) + (pairs ? win_of(c + 1) : 0);
          if (w > buf_e) { fits = false; break; }
          if (ncc + step > v.CC || used + w > buf_e) {
            close();
            c0 = c;
            used = 0;
            ncc = 0;
          }
          place(c);
          if (pairs) place(c + 1);  // c + 1 == C: the pad channel
        }
        if (fits) close();
        chunks.push_back(std::move(list));
      }
    }
    }  // groups
    // generic kernel: stride rounded to 16 elements, NBUF chunk buffers of
    // CC channels; interleaved kernel: NBUF packed buffers + the metadata ring
    const int64_t stride = il ? buf_e : v.stride_for(max_span);
    const int64_t need = il ? v.NBUF * buf_e * 16 + il_meta_bytes(v.NBUF, v.CC, v.DB())
                            : v.NBUF * v.chan_bytes(stride) * v.CC;
    if (il && (int64_t)max_span + 64 * v.G > (int64_t)1 << 20) continue;  // windows too wide
    if (il && !fits) {
      if (last) {
        set_error("pdd_sweep_plan_create: DM grid too sparse for one LDS tile (span %d bins)", max_span);
        return -1;
      }
      continue;
    }
    if (!il && need > lds_budget(v) && !(last && need <= kLdsMax)) {
      if (last) {
        set_error("pdd_sweep_plan_create: DM grid too sparse for one LDS tile (span %d bins)", max_span);
        return -1;
      }
      continue;
    }
    const int cc = v.CC;
    pdd_sweep_plan* p = new pdd_sweep_plan();
    p->v = v;
    p->D = D;
    p->C = C;
    p->Dpad = Dpad;
    p->n_dblk = n_dblk;
    p->max_span = max_span;
    p->stride = (int)stride;
    p->cc = cc;
    p->lds_bytes = (int)need;
    p->vi = vi;
    p->dtype = dtype;
    p->n_grp = n_grp;
    if (il) {
      // (+ 8 rows of zeros: the loaders' scalar loads of a chunk's window
      // rows read 8 rows from its first channel)
      mt_all.resize(mt_all.size() + (size_t)(8 * (DB + 4)), 0);
      tab.swap(mt_all);
      // chunk tables [n_grp * n_dblk][1 + maxch]: count, then c0 | ncc << 20
      size_t maxch = 0;
      for (const auto& l : chunks) maxch = std::max(maxch, l.size());
      bmin.assign(chunks.size() * (maxch + 1), 0);
      for (size_t i = 0; i < chunks.size(); ++i) {
        bmin[i * (maxch + 1)] = (int)chunks[i].size();
        for (size_t k = 0; k < chunks[i].size(); ++k) bmin[i * (maxch + 1) + 1 + k] = chunks[i][k];
      }
      p->maxch = (int)maxch;
      // 8/16-bit single-group sweeps: the factorised tables when they pay
      // groups of 4 channels, or of 2 where 4 do not fit or pay (the
      // cheaper by the cost model; PDD_SWEEP_FACTOR_G2 / _G4: that size only)
      // Factorised u16 plans first try their own 96-trial tiling
      // (kU8FxVariants: measured faster for factorised stage 2, slower for
      // the channel kernel), then the channel plan's tiling.
      FxTables T, T2;
      const bool force = (flags & PDD_SWEEP_FACTOR_FORCE) != 0;
      const bool skew = (flags & PDD_SWEEP_NO_SKEW) == 0;
      int fxg = 0;
      if ((flags & PDD_SWEEP_FACTOR) && n_grp == 1 && v.S == (dtype == PDD_F32 ? 4 : 8) &&
          il_kernel_for(v, true)) {
        std::vector<Variant> fc;
        if (v.S == 8)
          for (const Variant& x : kU8FxVariants)
            if (C * (dtype == PDD_U8 ? 255 : 1023) <= 255 * 32768 && il_kernel_for(x, true))
              fc.push_back(x);
        fc.push_back(v);
        for (const Variant& f : fc) {
          const int64_t room_f = lds_budget(f) - il_meta_bytes(f.NBUF, f.CC, f.DB());
          const int64_t buf_f = std::max<int64_t>(0, room_f / (f.NBUF * 16) / 64 * 64);
          // (the pair order of the trial blocks is kept where it costs <= 5%
          // more chunks on average, fx_build)
          auto build = [&](int g, FxTables& X) {
            if (!fx_build(host_table, D, C, f, buf_f, g, force, X, true, skew)) return false;
            if (X.pair_ratio <= PDD_FX_PAIR_MAX || fx_build(host_table, D, C, f, buf_f, g, force, X, false, skew))
              return true;
            // (the cost screen may turn the plan down without the pair order:
            // keep it then)
            return fx_build(host_table, D, C, f, buf_f, g, force, X, true, skew);
          };
          if (!(flags & PDD_SWEEP_FACTOR_G2) && build(4, T))
            fxg = 4;
          if (!(flags & PDD_SWEEP_FACTOR_G4) && build(2, T2) &&
              (fxg == 0 || T2.cost_f < T.cost_f)) {
            fxg = 2;
            std::swap(T, T2);
          }
          if (fxg) {
            // the plan runs the factorised tiling: its trial blocks, LDS
            p->v = f;
            p->n_dblk = cdiv(D, f.DB());
            p->Dpad = p->n_dblk * f.DB();
            p->stride = (int)buf_f;
            p->lds_bytes = (int)(f.NBUF * buf_f * 16 + il_meta_bytes(f.NBUF, f.CC, f.DB()));
            break;
          }
        }
      }
      if (fxg) {
        p->fx = fxg;
        p->n_pat = T.n_pat;
        p->fx_rows = T.rows_pb;
        p->fx_rspan = T.rspan;  // stage 1 sizes its LDS to it: more workgroups per CU
        p->fx_lo = T.lo_f;
        p->fx_hi = T.hi_f;
        p->fx_tpad = (int)(cdiv(T.sig_max, 64 * p->v.G) * 64 * p->v.G);
        p->fx_sig_max = T.sig_max;
        p->maxch = T.maxch;
        tab.swap(T.mt);
        bmin.swap(T.cht);
        hipError_t e = hipMalloc(&p->d_pat, T.pat.size() * sizeof(int));
        if (e == hipSuccess) e = hipMalloc(&p->d_wt, T.wt.size() * sizeof(int));
        if (e == hipSuccess)
          e = hipMemcpy(p->d_pat, T.pat.data(), T.pat.size() * sizeof(int), hipMemcpyHostToDevice);
        if (e == hipSuccess)
          e = hipMemcpy(p->d_wt, T.wt.data(), T.wt.size() * sizeof(int), hipMemcpyHostToDevice);
        if (e == hipSuccess && T.sig_max > 0) e = hipMalloc(&p->d_sig, T.sig.size() * sizeof(int));
        if (e == hipSuccess && T.sig_max > 0)
          e = hipMemcpy(p->d_sig, T.sig.data(), T.sig.size() * sizeof(int), hipMemcpyHostToDevice);
        if (e == hipSuccess && !T.gtab.empty()) e = hipMalloc(&p->d_gtab, T.gtab.size() * sizeof(int));
        if (e == hipSuccess && !T.gtab.empty())
          e = hipMemcpy(p->d_gtab, T.gtab.data(), T.gtab.size() * sizeof(int), hipMemcpyHostToDevice);
        for (const void* kf :
             {(const void*)k_fx_patterns_lds, (const void*)k_fx_patterns_x<uint8_t, 2>,
              (const void*)k_fx_patterns_x<uint8_t, 4>, (const void*)k_fx_patterns_x<uint16_t, 2>,
              (const void*)k_fx_patterns_x<uint16_t, 4>, (const void*)k_fx_patterns_xf<2>,
              (const void*)k_fx_patterns_xf<4>})
          if (e == hipSuccess && !T.gtab.empty())
            e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)(4 * (kFxEf + kFxRspan) * sizeof(uint4)));
        if (e != hipSuccess) {
          set_error("pdd_sweep_plan_create: %s", hipGetErrorString(e));
          pdd_sweep_plan_destroy(p);
          return -2;
        }
      }
    }
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
      const void* kf = il ? (const void*)il_kernel_for(p->v, p->fx != 0) : (const void*)kernel_for(v);
      e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, p->lds_bytes);
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

extern "C" {

int pdd_sweep_plan_factor(const pdd_sweep_plan* p, int64_t* n_patterns) {
  PDD_REQUIRE(p, "pdd_sweep_plan_factor: null pointer");
  if (n_patterns) *n_patterns = p->n_pat;
  return p->fx;
}

int pdd_sweep_plan_skew(const pdd_sweep_plan* p, int64_t* extra_tiles) {
  PDD_REQUIRE(p, "pdd_sweep_plan_skew: null pointer");
  if (extra_tiles) *extra_tiles = p->fx ? p->fx_tpad / (64 * p->v.G) : 0;
  return p->fx ? p->fx_sig_max : 0;
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
  info[7] = p->vi;
  return 0;
}

int pdd_sweep_execute(const pdd_sweep_plan* p, const void* x, int64_t N, int64_t ld, int pad_mode,
                      const float* padvals, float* out, int64_t ld_out, int64_t n_out,
                      void* stream) {
  return pdd_sweep_execute_ex(p, x, N, ld, 0, 0, pad_mode, padvals, out, ld_out, n_out, 0.f,
                              stream);
}

int pdd_sweep_execute_ex(const pdd_sweep_plan* p, const void* x, int64_t N, int64_t ld,
                         int64_t piece, int64_t x_off, int pad_mode, const float* padvals,
                         float* out, int64_t ld_out, int64_t n_out, float out_bias, void* stream) {
  PDD_REQUIRE(p && x && out, "pdd_sweep_execute: null pointer");
  PDD_REQUIRE(N > 0 && n_out >= 0 && ld_out >= n_out && x_off >= 0, "pdd_sweep_execute: bad shape");
  PDD_REQUIRE(piece > 0 || ld >= N, "pdd_sweep_execute: row stride %lld < N", (long long)ld);
  PDD_REQUIRE(piece == 0 || (piece & (piece - 1)) == 0, "pdd_sweep_execute: piece must be 2^k");
  PDD_REQUIRE(pad_mode == PDD_PAD_ROTATE || (pad_mode == PDD_PAD_VALUE && padvals),
              "pdd_sweep_execute: bad pad mode %d", pad_mode);
  if (n_out == 0) return 0;
  InLayout lay{ld, piece, 0, 0};
  if (piece) {
    while ((1ll << lay.psh) < piece) ++lay.psh;
    lay.pstride = p->C * p->n_grp * piece;
  }
  if (p->v.kind == 0)
    return execute_il(p, x, N, lay, x_off, pad_mode, padvals, out, ld_out, n_out, 0, 1, out_bias,
                      stream);
  PDD_REQUIRE(piece == 0 && x_off == 0 && out_bias == 0.f,
              "pdd_sweep_execute: the generic (sparse-grid) kernel reads channel-major input "
              "at offset 0 without an output bias");
  // every staged index must stay inside int64 / the LDS image: the shifts are
  // bounded by the plan, the samples by N + n_out.
  const int64_t n_tblk = cdiv(n_out, p->v.TB());
  const int64_t blocks = n_tblk * p->n_dblk;
  PDD_REQUIRE(blocks < (1ll << 31), "pdd_sweep_execute: grid too large");
  sweep_fn fn = kernel_for(p->v);
  PDD_REQUIRE(fn != nullptr, "pdd_sweep_execute: no kernel");
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(p->v.threads()), p->lds_bytes,
                     as_stream(stream), x, ld, (int)p->C, N, p->d_tab, (int)p->Dpad, (int)p->D,
                     p->d_bmin, p->d_bspan, pad_mode, padvals, out, ld_out, n_out, debug_flags(),
                     p->stride, (int)n_tblk, (int)p->n_dblk);
  PDD_LAUNCHED();
  return 0;
}

int64_t pdd_sweep_pattern_bytes(const pdd_sweep_plan* p, int64_t n_out) {
  PDD_REQUIRE(p && n_out >= 0, "pdd_sweep_pattern_bytes: bad arguments");
  if (!p->fx || !p->d_gtab || p->v.kind != 0) return 0;
  const int Tq = 64 * p->v.G;
  int64_t lo, hi;
  il_lohi(p, lo, hi);
  const int64_t Qs = cdiv(cdiv(std::max<int64_t>(n_out, 1), p->v.S), Tq) * Tq;
  return (int64_t)(p->n_pat + 1) * (Qs + (hi - lo) + 64) * 16;
}

int pdd_sweep_execute_stage(const pdd_sweep_plan* p, const void* x, int64_t N, int64_t ld,
                            int64_t piece, int64_t x_off, int pad_mode, const float* padvals,
                            float* out, int64_t ld_out, int64_t n_out, float out_bias,
                            void* patterns, int64_t pattern_bytes, int stage, void* stream) {
  PDD_REQUIRE(p && x && patterns && (out || stage == 1), "pdd_sweep_execute_stage: null pointer");
  PDD_REQUIRE(p->fx && p->d_gtab && p->v.kind == 0 && p->n_grp == 1,
              "pdd_sweep_execute_stage: needs a factorised single-group plan");
  PDD_REQUIRE(stage >= 1 && stage <= 3, "pdd_sweep_execute_stage: stage %d not 1, 2 or 3", stage);
  PDD_REQUIRE(N > 0 && n_out >= 0 && (stage == 1 || ld_out >= n_out) && x_off >= 0,
              "pdd_sweep_execute_stage: bad shape");
  PDD_REQUIRE(piece > 0 || ld >= N, "pdd_sweep_execute_stage: row stride %lld < N", (long long)ld);
  PDD_REQUIRE(piece == 0 || (piece & (piece - 1)) == 0, "pdd_sweep_execute_stage: piece must be 2^k");
  PDD_REQUIRE(pad_mode == PDD_PAD_ROTATE || (pad_mode == PDD_PAD_VALUE && padvals),
              "pdd_sweep_execute_stage: bad pad mode %d", pad_mode);
  if (n_out == 0) return 0;
  InLayout lay{ld, piece, 0, 0};
  if (piece) {
    while ((1ll << lay.psh) < piece) ++lay.psh;
    lay.pstride = p->C * piece;
  }
  IlExtra ex;
  ex.stages = stage;
  ex.P_ext = static_cast<uint4*>(patterns);
  ex.P_bytes = pattern_bytes;
  return execute_il(p, x, N, lay, x_off, pad_mode, padvals, out, ld_out, n_out, 0, 1, out_bias,
                    stream, ex);
}

int pdd_stream_create_cu_mask(const uint32_t* mask, int n_words, void** stream) {
  PDD_REQUIRE(mask && stream && n_words > 0, "pdd_stream_create_cu_mask: bad arguments");
  hipStream_t st = nullptr;
  PDD_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)n_words, mask));
  *stream = st;
  return 0;
}

int pdd_stream_destroy(void* stream) {
  PDD_REQUIRE(stream, "pdd_stream_destroy: null stream");
  PDD_HIP(hipStreamDestroy(as_stream(stream)));
  return 0;
}

int pdd_sweep_execute_grouped(const pdd_sweep_plan* p, const void* x, int64_t N, int64_t ld,
                              int pad_mode, const float* padvals, float* out, int64_t ld_out,
                              int64_t n_out, int64_t row_g, int64_t row_d, void* stream) {
  PDD_REQUIRE(p && x && out, "pdd_sweep_execute_grouped: null pointer");
  PDD_REQUIRE(p->v.kind == 0, "pdd_sweep_execute_grouped: plan has no grouped kernel");
  PDD_REQUIRE(N > 0 && ld >= N && n_out >= 0 && ld_out >= n_out && row_g >= 0 && row_d >= 0,
              "pdd_sweep_execute_grouped: bad shape");
  PDD_REQUIRE(pad_mode == PDD_PAD_ROTATE || (pad_mode == PDD_PAD_VALUE && padvals),
              "pdd_sweep_execute_grouped: bad pad mode %d", pad_mode);
  if (n_out == 0) return 0;
  return execute_il(p, x, N, InLayout{ld, 0, 0, 0}, 0, pad_mode, padvals, out, ld_out, n_out, row_g,
                    row_d, 0.f, stream);
}

int pdd_sweep_execute_ds(const pdd_sweep_plan* p, const uint8_t* x8, int64_t n_raw, int64_t ld,
                         int64_t ds, int pad_mode, const float* padvals, float* out,
                         int64_t ld_out, int64_t n_out, int64_t row_g, int64_t row_d,
                         void* stream) {
  PDD_REQUIRE(p && x8 && out, "pdd_sweep_execute_ds: null pointer");
  PDD_REQUIRE(p->v.kind == 0 && p->v.S == 8 && p->dtype == PDD_U16,
              "pdd_sweep_execute_ds: needs a PDD_U16 plan on the 16-bit interleaved tiling");
  PDD_REQUIRE(ds >= 2 && ds <= 4, "pdd_sweep_execute_ds: downsample factor %lld not in 2..4",
              (long long)ds);
  const int64_t N = n_raw / ds;
  PDD_REQUIRE(N >= 0 && ld >= n_raw && n_out >= 0 && n_out <= N && ld_out >= n_out && row_g >= 0 &&
                  row_d >= 0,
              "pdd_sweep_execute_ds: bad shape");
  PDD_REQUIRE(pad_mode == PDD_PAD_ROTATE || (pad_mode == PDD_PAD_VALUE && padvals),
              "pdd_sweep_execute_ds: bad pad mode %d", pad_mode);
  if (n_out == 0) return 0;
  IlExtra ex;
  ex.ds = (int)ds;
  return execute_il(p, x8, N, InLayout{ld, 0, 0, 0}, 0, pad_mode, padvals, out, ld_out, n_out,
                    p->n_grp > 1 ? row_g : 0, row_d, 0.f, stream, ex);
}

int pdd_subband_chain(const pdd_sweep_plan* p1, const void* x, int64_t n_raw, int64_t ld, int64_t ds,
                      int pad1_mode, const float* pad1vals, const pdd_sweep_plan* p2,
                      const float* pad2vals, float* out, int64_t ld_out, int64_t n_out,
                      int64_t row_g, int64_t row_d, void* stream) {
  PDD_REQUIRE(p1 && p2 && x && out && pad2vals, "pdd_subband_chain: null pointer");
  PDD_REQUIRE(p1->v.kind == 0 && p1->v.S == 8 &&
                  ((p1->dtype == PDD_U8 && ds == 1) || (p1->dtype == PDD_U16 && ds >= 2 && ds <= 4)),
              "pdd_subband_chain: stage 1 needs an 8-bit (ds 1) or 16-bit (ds 2..4) plan on the "
              "16-bit interleaved tiling");
  PDD_REQUIRE(p2->v.kind == 0 && p2->v.S == 4 && p2->dtype == PDD_F32 && p2->min_bin >= 0,
              "pdd_subband_chain: stage 2 needs a float32 interleaved plan with delays >= 0");
  PDD_REQUIRE(p2->C * p2->n_grp == p1->D * p1->n_grp,
              "pdd_subband_chain: stage-2 channels (%lld) != stage-1 rows (%lld)",
              (long long)(p2->C * p2->n_grp), (long long)(p1->D * p1->n_grp));
  PDD_REQUIRE(pad1_mode == PDD_PAD_ROTATE || (pad1_mode == PDD_PAD_VALUE && pad1vals),
              "pdd_subband_chain: bad pad mode %d", pad1_mode);
  const int64_t N1 = n_raw / ds;
  PDD_REQUIRE(N1 > 0 && ld >= n_raw && n_out >= 0 && n_out <= N1 && ld_out >= n_out &&
                  row_g >= 0 && row_d >= 0,
              "pdd_subband_chain: bad shape");
  if (n_out == 0) return 0;
  // factorised plans sweep single-group input through their pattern image:
  // they do not chain (pdd.h)
  if (p1->fx || p2->fx) {
    set_error("pdd_subband_chain: factorised plans do not chain");
    return PDD_ENOCHAIN;
  }
  // stage 1 covers N1 samples in one segment of eighth length Qs1; stage 2
  // reads quarters of length 2 Qs1 (a multiple of its 256-element tile)
  const int64_t Qs1 = cdiv(cdiv(N1, 8), 64 * p1->v.G) * (64 * p1->v.G);
  const int64_t ov = std::max(0, p2->max_bin) + 64;
  if (!(ov <= Qs1 && (2 * Qs1) % (64 * p2->v.G) == 0)) {
    set_error("pdd_subband_chain: block of %lld samples does not chain (stage-2 span %d)",
              (long long)N1, p2->max_bin);
    return PDD_ENOCHAIN;  // nothing launched: run the stages apart
  }
  const int64_t C2 = p2->C * p2->n_grp;
  const int64_t nR2 = 2 * Qs1 + ov;
  hipStream_t st = as_stream(stream);
  // stage 2's image first, THEN the one-segment check of both stages (their
  // budgets are capped by the device memory free after it): the decision is
  // made once, here, and the stages run with it (IlExtra.one_seg) instead of
  // re-deriving it from a free-memory figure that their own scratch changes
  float4* R2 = static_cast<float4*>(scratch(st, kScratchChain, (size_t)(C2 * nR2) * sizeof(float4)));
  if (!R2) return -2;
  if (!(il_seg_samples(p1, st) >= N1 && il_seg_samples(p2, st) >= n_out)) {
    set_error("pdd_subband_chain: block of %lld samples does not chain (one segment per stage "
              "needed)", (long long)N1);
    return PDD_ENOCHAIN;  // nothing launched: run the stages apart
  }
  IlExtra e1;
  e1.ds = (int)ds;
  e1.one_seg = true;
  e1.r2_pad = pad2vals;
  e1.r2_nR = nR2;
  e1.r2_ov = ov;
  // stage-1 rows (= stage-2 channels): trial d of group g -> row d * n_grp1 + g
  int rc = execute_il(p1, x, N1, InLayout{ld, 0, 0, 0}, 0, pad1_mode, pad1vals, (float*)R2, 0, N1,
                      1, p1->n_grp, 0.f, stream, e1);
  if (rc == 0) {
    IlExtra e2;
    e2.one_seg = true;
    e2.R_pre = R2;
    e2.Qs_pre = 2 * Qs1;
    e2.nR_pre = nR2;
    rc = execute_il(p2, nullptr, N1, InLayout{0, 0, 0, 0}, 0, PDD_PAD_VALUE, pad2vals, out, ld_out,
                    n_out, row_g, row_d, 0.f, stream, e2);
  }
  return rc;
}

int pdd_sweep_plan_set_input_max(pdd_sweep_plan* p, int max_value) {
  PDD_REQUIRE(p, "pdd_sweep_plan_set_input_max: null pointer");
  PDD_REQUIRE(p->dtype != PDD_F32, "pdd_sweep_plan_set_input_max: integer-input plans only");
  const int bound = p->dtype == PDD_U8 ? 255 : 1023;
  PDD_REQUIRE(max_value >= 1 && max_value <= bound,
              "pdd_sweep_plan_set_input_max: %d outside [1, %d]", max_value, bound);
  p->input_max = max_value;
  return 0;
}

int pdd_sweep_plan_set_poison(pdd_sweep_plan* p, int on) {
  PDD_REQUIRE(p, "pdd_sweep_plan_set_poison: null pointer");
  p->poison = on ? 1 : 0;
  return 0;
}

int pdd_sweep_plan_set_segment_bytes(pdd_sweep_plan* p, int64_t bytes) {
  PDD_REQUIRE(p, "pdd_sweep_plan_set_segment_bytes: null pointer");
  PDD_REQUIRE(bytes >= 0, "pdd_sweep_plan_set_segment_bytes: negative budget");
  p->seg_bytes = bytes;
  return 0;
}

int pdd_sweep_set_timing(pdd_sweep_plan* p, int on) {
  PDD_REQUIRE(p, "pdd_sweep_set_timing: null pointer");
  if (on && !p->ev) {
    p->ev = new hipEvent_t[2 * pdd_sweep_plan::kEvPairs]();
    for (int i = 0; i < 2 * pdd_sweep_plan::kEvPairs; ++i) PDD_HIP(hipEventCreate(&p->ev[i]));
  }
  p->timing = on ? 1 : 0;
  p->timed = 0;
  p->dropped = 0;
  return 0;
}

int pdd_sweep_timing_read(pdd_sweep_plan* p, float* total_ms, int64_t* launches) {
  PDD_REQUIRE(p && total_ms && launches, "pdd_sweep_timing_read: null pointer");
  PDD_REQUIRE(p->timing && p->timed, "pdd_sweep_timing_read: no timed launch (pdd_sweep_set_timing)");
  PDD_REQUIRE(!p->dropped, "pdd_sweep_timing_read: %d launches past the %d-pair event pool",
              p->dropped, pdd_sweep_plan::kEvPairs);
  PDD_HIP(hipEventSynchronize(p->ev[2 * p->timed - 1]));
  double sum = 0.0;
  for (int i = 0; i < p->timed; ++i) {
    float ms = 0.f;
    PDD_HIP(hipEventElapsedTime(&ms, p->ev[2 * i], p->ev[2 * i + 1]));
    sum += ms;
  }
  *total_ms = (float)sum;
  *launches = p->timed;
  p->timed = 0;
  return 0;
}

int pdd_sweep_kernel_ms(pdd_sweep_plan* p, float* ms) {
  int64_t n = 0;
  return pdd_sweep_timing_read(p, ms, &n);
}

int pdd_sweep_plan_destroy(pdd_sweep_plan* p) {
  if (!p) return 0;
  if (p->ev) {
    for (int i = 0; i < 2 * pdd_sweep_plan::kEvPairs; ++i)
      if (p->ev[i]) (void)hipEventDestroy(p->ev[i]);
    delete[] p->ev;
  }
  if (p->d_tab) (void)hipFree(p->d_tab);
  if (p->d_bmin) (void)hipFree(p->d_bmin);
  if (p->d_bspan) (void)hipFree(p->d_bspan);
  if (p->d_pat) (void)hipFree(p->d_pat);
  if (p->d_wt) (void)hipFree(p->d_wt);
  if (p->d_gtab) (void)hipFree(p->d_gtab);
  if (p->d_sig) (void)hipFree(p->d_sig);
  delete p;
  return 0;
}

}  // extern "C"
