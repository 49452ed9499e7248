// Error reporting for the C-ABI: every entry point returns 0 on success, a negative
// code on failure, and leaves a message readable through slx_last_error().
#include "common.h"

namespace slx {
static thread_local char g_err[512] = {0};
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

}  // namespace slx

extern "C" {
const char* slx_last_error(void) { return slx::g_err; }
int slx_abi_version(void) { return 1; }
int slx_device_sync(void) {
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    slx::set_error("hipDeviceSynchronize: %s", hipGetErrorString(e));
    return -(int)e - 1000;
  }
  return 0;
}
}
