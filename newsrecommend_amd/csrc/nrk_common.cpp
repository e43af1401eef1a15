// nrk_common.cpp — error state of libnrk (thread-local, re-entrant).
#include <stdarg.h>

#include "nrk_common.h"

namespace nrk {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

}  // namespace nrk

extern "C" const char* nrk_last_error(void) { return nrk::g_err; }
extern "C" int nrk_version(void) { return 1; }
