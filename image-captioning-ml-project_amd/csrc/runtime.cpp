// Error state, version and device query for libcapk.
#include <stdarg.h>
#include <string.h>

#include "common.h"

namespace capk {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int hip_status(hipError_t e, const char* what) {
  set_error("%s: HIP error %d (%s)", what, (int)e, hipGetErrorString(e));
  return CAPK_EHIP;
}
}  // namespace capk

extern "C" {
const char* capk_last_error(void) { return capk::g_err; }
int capk_version(void) { return 100; }

int capk_device_arch(char* buf, int len) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return capk::hip_status(e, "hipGetDevice");
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return capk::hip_status(e, "hipGetDeviceProperties");
  snprintf(buf, (size_t)len, "%s", prop.gcnArchName);
  return CAPK_OK;
}
}
