// Error plumbing and version entry points of the C ABI (include/avr.h).
#include <stdarg.h>
#include <stdio.h>

#include "avr_common.h"

namespace avr {

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

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(AVR_E_HIP, "%s: %s", what, hipGetErrorString(e));
  return AVR_OK;
}

}  // namespace avr

extern "C" int avr_version(void) { return AVR_ABI_VERSION; }

extern "C" const char* avr_last_error_string(void) { return avr::g_err; }

extern "C" int avr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}
