// Shared helpers for the bpk HIP library (gfx950 / CDNA4 only).
//
// Every exported entry point is `extern "C"`, takes raw device pointers, sizes
// and a `hipStream_t` passed as `void*`, and returns an int status (0 = ok).
// On failure the message is retrievable with bpk_last_error() (thread local),
// which the Python host turns into a RuntimeError -- mirroring the reference's
// TORCH_CHECK -> c10::Error -> RuntimeError behaviour (op/upfirdn2d.cpp:8).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/bpk.h"

namespace bpk {

void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// floor division / modulo that are correct for negative numerators
__host__ __device__ inline int floordiv(int a, int b) {
  int q = a / b;
  return (q * b > a) ? q - 1 : q;
}
__host__ __device__ inline int floormod(int a, int b) { return a - floordiv(a, b) * b; }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// XCD-aware block order for stencil kernels: blocks are observed to be dealt round-robin over
// the 8 XCDs (b and b + 8 share one, MI355X_MICROARCH.md), so neighbouring tiles b, b + 1 land
// on different L2s and each XCD fetches the other's halo rows from HBM.  This bijection on
// [0, nb) gives the blocks sharing an XCD one contiguous run of logical tiles (any nb; speed
// only -- every tile is still processed exactly once).
__device__ inline int64_t xcd_tile(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, xcd = b % 8, slot = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

}  // namespace bpk

#define BPK_REQUIRE(cond, ...)           \
  do {                                   \
    if (!(cond)) {                       \
      bpk::set_error(__VA_ARGS__);       \
      return BPK_ERR_ARG;                \
    }                                    \
  } while (0)

#define BPK_LAUNCH_CHECK(what)                                                   \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
    if (e_ != hipSuccess) {                                                      \
      bpk::set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e_)); \
      return BPK_ERR_LAUNCH;                                                     \
    }                                                                            \
  } while (0)
