// libpdd: PSRFITS search-mode subint decode on the device (SURVEY.md §8(f)
// rank 3), gfx950.  One HBM-bound pass replaces the reference's host chain
// (formats/psrfits.py):
//   unpack_4bit            psrfits.py:37-50   (low nibble first)
//   read_subint            psrfits.py:67-107  ((data*scales)+offsets)*weights,
//                                             float32, in that order
//   get_spectra            psrfits.py:140-183 (concatenate subints, transpose
//                                             to [chan, time], skip/trunc,
//                                             band flip when the band ascends)
// Input: nsub consecutive BINTABLE rows copied verbatim (row_bytes each; the
// DATA column starts data_off bytes into a row), big-endian as on disk:
// nbits 4 (two samples per byte), 8 (uint8), 16 (int16, FITS 'I'), 32
// (float32, FITS 'E').  wso: [nsub][3][nchan] float32 scale, offset, weight.
// Output: out[c'][j] for j < N, the sample g = s0 + j of the concatenated
// subints (subint g / nsblk, spectrum g % nsblk), c' = flip ? nchan-1-c : c.
// 64 x 64 (spectrum x channel) tiles through LDS: the decode reads rows
// channel-fastest (coalesced), the store writes channel rows time-fastest.
#include "pdd_internal.h"

namespace pdd {

namespace {

template <int NBITS>
__device__ __forceinline__ float decode(const uint8_t* __restrict__ data, int64_t idx) {
  if constexpr (NBITS == 8) {
    return (float)data[idx];
  } else if constexpr (NBITS == 4) {
    const uint8_t b = data[idx >> 1];
    return (float)((idx & 1) ? (b >> 4) : (b & 15));
  } else if constexpr (NBITS == 16) {
    const uint8_t* p = data + 2 * idx;
    return (float)(int16_t)(((uint16_t)p[0] << 8) | p[1]);
  } else {
    const uint8_t* p = data + 4 * idx;
    const uint32_t u = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
    return __uint_as_float(u);
  }
}

template <int NBITS>
__global__ __launch_bounds__(256) void k_psrfits_subints(
    const uint8_t* __restrict__ raw, int64_t row_bytes, int64_t data_off, int64_t nsblk,
    int64_t nchan, const float* __restrict__ wso, int64_t s0, int64_t N, int flip,
    float* __restrict__ out, int64_t ld_out, int64_t tiles_c) {
  __shared__ float tile[64][65];
  const int64_t tt = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int64_t j0 = tt * 64, c0 = tc * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t c = c0 + tx;
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int64_t j = j0 + i;
    if (j < N && c < nchan) {
      const int64_t g = s0 + j, sub = g / nsblk, s = g - sub * nsblk;
      const uint8_t* data = raw + sub * row_bytes + data_off;
      const float* p = wso + sub * 3 * nchan;
      const float v = decode<NBITS>(data, s * nchan + c);
      tile[i][tx] = ((v * p[c]) + p[nchan + c]) * p[2 * nchan + c];
    }
  }
  __syncthreads();
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int64_t cc = c0 + i, j = j0 + tx;
    if (j < N && cc < nchan) out[(flip ? nchan - 1 - cc : cc) * ld_out + j] = tile[tx][i];
  }
}

}  // namespace

}  // namespace pdd

using namespace pdd;

extern "C" {

int pdd_psrfits_subints(const uint8_t* raw, int64_t nsub, int64_t row_bytes, int64_t data_off,
                        int nbits, int64_t nsblk, int64_t nchan, const float* wso, int64_t s0,
                        int64_t N, int flip, float* out, int64_t ld_out, void* stream) {
  PDD_REQUIRE(raw && wso && out, "pdd_psrfits_subints: null pointer");
  PDD_REQUIRE(nbits == 4 || nbits == 8 || nbits == 16 || nbits == 32,
              "pdd_psrfits_subints: nbits %d not supported (4, 8, 16, 32)", nbits);
  PDD_REQUIRE(nsub >= 1 && nsblk >= 1 && nchan >= 1 && N >= 0 && s0 >= 0 && ld_out >= N,
              "pdd_psrfits_subints: bad shape");
  PDD_REQUIRE(s0 + N <= nsub * nsblk, "pdd_psrfits_subints: samples [%lld, %lld) beyond %lld",
              (long long)s0, (long long)(s0 + N), (long long)(nsub * nsblk));
  PDD_REQUIRE(data_off + (nsblk * nchan * nbits + 7) / 8 <= row_bytes,
              "pdd_psrfits_subints: DATA column exceeds the row");
  if (N == 0) return 0;
  const int64_t tiles_c = cdiv(nchan, 64);
  const int64_t blocks = cdiv(N, 64) * tiles_c;
  PDD_REQUIRE(blocks < (1ll << 31), "pdd_psrfits_subints: too large");
  hipStream_t s = as_stream(stream);
#define PF(B)                                                                                      \
  k_psrfits_subints<B><<<(unsigned)blocks, 256, 0, s>>>(raw, row_bytes, data_off, nsblk, nchan, \
                                                        wso, s0, N, flip, out, ld_out, tiles_c)
  if (nbits == 4) PF(4);
  else if (nbits == 8) PF(8);
  else if (nbits == 16) PF(16);
  else PF(32);
#undef PF
  PDD_LAUNCHED();
  return 0;
}

}  // extern "C"
