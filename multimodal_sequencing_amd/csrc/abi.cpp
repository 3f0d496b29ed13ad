// Error plumbing and version for the mmseq C ABI (include/mmseq.h).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/mmseq.h"

static thread_local char g_err[512] = "";

mmseq_status mmseq_set_error(mmseq_status code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

mmseq_status mmseq_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return mmseq_set_error(MMSEQ_EHIP, "%s: %s", what, hipGetErrorString(e));
  return MMSEQ_OK;
}

extern "C" const char* mmseq_last_error(void) { return g_err; }
extern "C" const char* mmseq_version(void) { return "mmseq 0.1 gfx950"; }
