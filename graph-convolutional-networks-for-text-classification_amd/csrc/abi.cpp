// ABI bookkeeping for libgcnk: version and thread-local error text.
#include <cstdarg>
#include <cstdio>

#include "../../include/gcnk.h"

namespace gcnk {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

}  // namespace gcnk

extern "C" int gcnk_abi_version(void) { return GCNK_ABI_VERSION; }

extern "C" const char* gcnk_last_error(void) { return gcnk::g_err; }
