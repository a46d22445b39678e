// Thread-local error message for the C ABI (include/abcgpu.h).
#include <stdarg.h>
#include <stdio.h>
#include "abc_common.h"

namespace {
thread_local char g_err[1024] = "";
}

namespace abc {
int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
}  // namespace abc

extern "C" const char* abc_last_error(void) { return g_err; }
extern "C" int abc_version(void) { return 1; }
