// Error plumbing shared by every entry point.
#include "bpk_common.h"

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <mutex>

namespace {
thread_local char g_last_error[1024] = "";
}

// split-K tile counters (zero at load; every launch that uses some leaves them zero)
constexpr int64_t kTickets = 1 << 16;
__device__ unsigned g_splitk_tickets[kTickets];

namespace bpk {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

std::atomic<int> g_fuse_max{-1};

int splitk_fuse_max() {
  int v = g_fuse_max.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("BPK_SPLITK_FUSE_MAX");
    int want = e ? std::atoi(e) : 0;
    if (want < 0) want = 0;
    int expect = -1;
    g_fuse_max.compare_exchange_strong(expect, want);
    v = g_fuse_max.load(std::memory_order_relaxed);
  }
  return v;
}

unsigned* splitk_tickets(int64_t n) {
  static std::mutex mu;
  static unsigned* base[64] = {};
  static bool tried[64] = {};
  static int64_t cursor[64] = {};
  if (n <= 0 || n > kTickets || splitk_fuse_max() <= 0) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(mu);
  if (!tried[dev]) {  // the array's address on this device (one code object per device)
    tried[dev] = true;
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_splitk_tickets)) == hipSuccess)
      base[dev] = static_cast<unsigned*>(p);
    else
      (void)hipGetLastError();
  }
  if (!base[dev]) return nullptr;
  if (cursor[dev] + n > kTickets) cursor[dev] = 0;
  unsigned* r = base[dev] + cursor[dev];
  cursor[dev] += n;
  return r;
}
}  // namespace bpk

extern "C" const char* bpk_last_error(void) { return g_last_error; }
extern "C" int bpk_abi_version(void) { return BPK_ABI_VERSION; }

extern "C" int bpk_splitk_set_fuse_max(int max_splits) {
  const int prev = bpk::splitk_fuse_max();
  bpk::g_fuse_max.store(max_splits < 0 ? 0 : max_splits, std::memory_order_relaxed);
  return prev;
}
