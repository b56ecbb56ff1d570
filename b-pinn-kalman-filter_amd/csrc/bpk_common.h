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

// In-launch split-K combine (cdna_hip_programming.md §6 Guideline 16, counter form): each
// K-slice workgroup stores its partial slab with plain stores, then draws a ticket on its
// output tile's counter; the workgroup drawing the last ticket reads every slab and writes the
// tile -- the separate reduce launch (and its kernel boundary, ~1.5-1.9 us) is gone, the sum
// order (slab 0, 1, ..., S - 1) and with it the result are unchanged.  Correct for any
// placement of a tile's slices over CUs / XCDs: agent-scope release before the ticket,
// agent-scope acquire in the last arriver.  `flag` is a word of the kernel's own LDS array
// (a second __shared__ object can de-pipeline the main loop, ibid. item 4a), free by now.
// The last arriver resets the counter, so the tickets are zero again when the launch ends.
__device__ inline bool splitk_last(unsigned* cnt, unsigned splits, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == splits - 1;
    if (last) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// host: n zeroed tile counters for one launch (a ring over a device array that every launch
// leaves zeroed; consecutive launches take different slots, so kernels running concurrently on
// different streams do not share counters), or nullptr when the in-launch combine is off
// (BPK_SPLITK_FUSE_MAX=0) or unavailable -- callers then launch their reduce kernel
unsigned* splitk_tickets(int64_t n);
// largest split count combined in-launch (the last arriver reads S partial slabs of its tile
// serially; BPK_SPLITK_FUSE_MAX, default 16; 0 = never)
int splitk_fuse_max();

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
