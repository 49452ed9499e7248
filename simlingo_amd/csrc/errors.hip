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

// Fork/join helper: a side stream per (thread, device) for a launch that should run concurrently with the
// caller's stream (e.g. a GEMM's M-remainder next to its main grid). fork() makes the side stream wait for
// everything already queued on `main`; join() makes `main` wait for the side stream's work. Events come from
// a small per-thread ring (a wait captures the most recent record, so reuse after the join is safe).
struct SideStream {
  int device = -1;
  hipStream_t s = nullptr;
  hipEvent_t ev[8] = {};
  int next = 0;
};
static thread_local SideStream g_side;

static hipEvent_t side_event() {
  hipEvent_t e = g_side.ev[g_side.next];
  g_side.next = (g_side.next + 1) & 7;
  return e;
}

hipStream_t side_fork(hipStream_t main) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (g_side.s == nullptr || g_side.device != dev) {
    if (hipStreamCreateWithFlags(&g_side.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    for (auto& e : g_side.ev)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    g_side.device = dev;
  }
  hipEvent_t e = side_event();
  if (hipEventRecord(e, main) != hipSuccess || hipStreamWaitEvent(g_side.s, e, 0) != hipSuccess) return nullptr;
  return g_side.s;
}

int side_join(hipStream_t main) {
  hipEvent_t e = side_event();
  if (hipEventRecord(e, g_side.s) != hipSuccess || hipStreamWaitEvent(main, e, 0) != hipSuccess) {
    set_error("side_join: event record/wait failed");
    return -1;
  }
  return 0;
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
