// C-ABI plumbing of libnrse_hip.so: device check, error reporting, ABI version.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include "common.h"

namespace {
thread_local char g_err[512] = "";
}

void nrse_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int nrse_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    nrse_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return NRSE_ERR_LAUNCH;
  }
  return NRSE_OK;
}

extern "C" const char* nrse_last_error(void) { return g_err; }

extern "C" int nrse_abi_version(void) { return NRSE_ABI_VERSION; }

extern "C" int nrse_init(int device, nrse_caps* caps) {
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) {
    nrse_set_error("nrse_init: hipGetDeviceProperties(%d): %s", device, hipGetErrorString(e));
    return NRSE_ERR_ARG;
  }
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    nrse_set_error("nrse_init: device %d is %s, libnrse_hip.so is built for gfx950 only", device, prop.gcnArchName);
    return NRSE_ERR_ARCH;
  }
  if (caps) {
    caps->device = device;
    caps->cu_count = prop.multiProcessorCount;
    caps->xcd_count = 8;
    caps->lds_bytes_per_cu = (int)prop.maxSharedMemoryPerMultiProcessor;
    caps->hbm_bytes = (long long)prop.totalGlobalMem;
    strncpy(caps->arch, prop.gcnArchName, sizeof(caps->arch) - 1);
    caps->arch[sizeof(caps->arch) - 1] = 0;
  }
  return NRSE_OK;
}
