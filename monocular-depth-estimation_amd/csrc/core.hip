// Library-wide state: the thread-local error message returned by mdemi_last_error().
#include "common.h"

namespace mdemi {
static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace mdemi

extern "C" const char* mdemi_last_error(void) { return mdemi::g_err; }
extern "C" int mdemi_version(void) { return 1; }
