// Error plumbing shared by every entry point.
#include "bpk_common.h"

#include <cstdarg>
#include <cstdio>

namespace {
thread_local char g_last_error[1024] = "";
}

namespace bpk {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}
}  // namespace bpk

extern "C" const char* bpk_last_error(void) { return g_last_error; }
extern "C" int bpk_abi_version(void) { return BPK_ABI_VERSION; }
