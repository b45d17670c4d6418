// Library-level C-ABI entry points: version, error string, device queries.
#include "common.hpp"
#include "../../include/everest_amd.h"

namespace evr {
static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char* last_error() { return g_err; }
}  // namespace evr

extern "C" {

int evr_version(void) { return EVR_VERSION; }

const char* evr_last_error(void) { return evr::last_error(); }

int evr_device_arch(int device, char* buf, int buflen) {
  hipDeviceProp_t p;
  EVR_HIP(hipGetDeviceProperties(&p, device));
  snprintf(buf, (size_t)buflen, "%s", p.gcnArchName);
  return 0;
}

int evr_stream_sync(void* stream) {
  EVR_HIP(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

}  // extern "C"
