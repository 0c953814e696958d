// Error plumbing shared by every C-ABI entry point.
#include <cstdarg>
#include <cstdio>

#include "flamed_hip.h"

namespace fl {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char* last_error() { return g_err; }
}  // namespace fl

extern "C" {
FLAMED_API const char* flamed_last_error(void) { return fl::last_error(); }
FLAMED_API int flamed_version(void) { return 1; }
}
