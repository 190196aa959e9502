// Internal helpers shared by the libpdd translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <string>

#include "../../include/pdd.h"

namespace pdd {

void set_error(const char* fmt, ...);

#define PDD_REQUIRE(cond, ...)               \
  do {                                       \
    if (!(cond)) {                           \
      ::pdd::set_error(__VA_ARGS__);         \
      return -1;                             \
    }                                        \
  } while (0)

#define PDD_HIP(call)                                                              \
  do {                                                                             \
    hipError_t e_ = (call);                                                        \
    if (e_ != hipSuccess) {                                                        \
      ::pdd::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),      \
                       __FILE__, __LINE__);                                        \
      return -2;                                                                   \
    }                                                                              \
  } while (0)

// Check the launch that was just enqueued.
#define PDD_LAUNCHED()                                                             \
  do {                                                                             \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ != hipSuccess) {                                                        \
      ::pdd::set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(e_),  \
                       __FILE__, __LINE__);                                        \
      return -3;                                                                   \
    }                                                                              \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Device scratch owned by the library, one buffer per (device, stream, calling
// host thread, slot), grown with hipMalloc and kept for reuse.  Work on one
// stream is ordered and one thread queues it in program order, so
// consecutive calls of a thread on the same stream share a slot safely (a
// second thread on the same stream gets its own buffers); a call that
// needs two buffers at once uses two slots.  (Replaces stream-ordered
// hipMallocAsync/hipFreeAsync, whose pool pages, released at device
// synchronisation, were seen to alias live hipMalloc buffers -- wrong sweep
// results in tests/native/abi_asan.cpp.)  Returns nullptr and sets the error
// message on failure.
enum { kScratchImage = 0, kScratchChain = 1, kScratchPartial = 2, kScratchSmall = 3, kScratchPattern = 4 };
void* scratch(hipStream_t st, int slot, size_t bytes);
// Bytes the calling thread's (stream, slot) buffer holds now (0: none): memory
// a larger request of the same slot would free before allocating.
size_t scratch_held(hipStream_t st, int slot);

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Value of channel row `row` at sample s, with the reference pad semantics
// (formats/spectra.py:80-94): inside [0,N) the data, outside the pad value,
// or the wrapped sample for rotate.  For rotate the caller has reduced the
// shift modulo N so s is in [0, 2N).
__device__ __forceinline__ float fetch_padded(const float* __restrict__ row, int64_t s, int64_t N,
                                              int pad_mode, float pad) {
  if (pad_mode == PDD_PAD_ROTATE) {
    s = (s >= N) ? s - N : s;
    return row[s];
  }
  return (s >= 0 && s < N) ? row[s] : pad;
}

}  // namespace pdd
