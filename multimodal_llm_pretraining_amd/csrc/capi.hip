// C-ABI plumbing: thread-local error string, launch checks, device info.
// SURVEY.md §8b "Errors": int status, never throw across the ABI.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace mmpt {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return MMPT_OK;
}
}  // namespace mmpt

extern "C" int mmpt_abi_version(void) { return MMPT_ABI_VERSION; }

extern "C" const char* mmpt_last_error(void) { return mmpt::g_err; }

extern "C" int mmpt_device_info(int* cus, int* clock_khz, int* arch_gfx) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) {
    mmpt::set_error("hipGetDevice: %s", hipGetErrorString(e));
    return (int)e;
  }
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) {
    mmpt::set_error("hipGetDeviceProperties: %s", hipGetErrorString(e));
    return (int)e;
  }
  if (cus) *cus = prop.multiProcessorCount;
  if (clock_khz) *clock_khz = prop.clockRate;
  if (arch_gfx) {
    int v = 0;
    sscanf(prop.gcnArchName, "gfx%x", &v);
    *arch_gfx = v;
  }
  return MMPT_OK;
}
