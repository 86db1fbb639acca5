// Library-level C-ABI: error reporting and version.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/artsbir.h"

namespace artsbir {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
static thread_local const char* g_kernel = "";
void set_last_kernel(const char* name) { g_kernel = name; }
}  // namespace artsbir

extern "C" const char* artsbir_last_error(void) { return artsbir::g_err; }
extern "C" const char* artsbir_last_kernel(void) { return artsbir::g_kernel; }
extern "C" int artsbir_version(void) { return 1; }
