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

// A stream whose kernels may only use the CUs set in mask (bit i of word w = CU
// 32 w + i).  The training step's weight gradients (MFMA-bound) run on such a
// stream next to the HBM-bound data-gradient / BatchNorm chain, so the two share
// the chip by CUs instead of the weight gradients occupying every CU in turn.
extern "C" int artsbir_stream_create_cu_mask(const unsigned* mask, int nwords, void** out) {
  if (!mask || nwords < 1 || !out) { artsbir::set_error("stream_create_cu_mask: bad arguments"); return -1; }
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask);
  if (e != hipSuccess) {
    artsbir::set_error("hipExtStreamCreateWithCUMask: %s", hipGetErrorString(e));
    return -2;
  }
  *out = (void*)s;
  return 0;
}

extern "C" int artsbir_stream_destroy(void* stream) {
  const hipError_t e = hipStreamDestroy((hipStream_t)stream);
  if (e != hipSuccess) { artsbir::set_error("hipStreamDestroy: %s", hipGetErrorString(e)); return -2; }
  return 0;
}
