// Deterministic-reduction mode (slx_set_deterministic). The training step's cross-block reductions normally end in
// f32 atomics (split-K partials of some GEMMs, the LoRA parameter gradients, column sums, norm parameter gradients,
// the gradient sum of squares), so a step's gradients differ from run to run in the last bits. With the mode on,
// every such reduction stores its per-block partials in the caller's workspace and one ordered pass adds them
// (partial 0 + partial 1 + ... in index order), GEMM split-K runs only in its in-launch slab form (split order) or
// not at all: two runs of a step on the same inputs give bitwise-equal gradients and parameters. The switch and the
// workspace are process-wide (a test / reproducibility mode; one stream at a time), the default is off.
#include "common.h"
#include "../../include/slx.h"

namespace slx {

DetMode& det_mode() {
  static DetMode m = {0, nullptr, 0};
  return m;
}

// out[i] (+)= sum_{p < nparts} part[p * stride + i], p in order
__global__ __launch_bounds__(256) void det_reduce_kernel(const float* __restrict__ part, int nparts, long n, long stride,
                                                         float* __restrict__ out, int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int p = 0; p < nparts; ++p) s += part[(long)p * stride + i];
  out[i] = accumulate ? out[i] + s : s;
}

// one output (the clip's gradient sum of squares over 2048 partials): 256 threads each sum a strided subset in a fixed
// order, then a fixed LDS tree (one serial thread over 2048 dependent loads took 125 us)
__global__ __launch_bounds__(256) void det_sum1_kernel(const float* __restrict__ part, int nparts, long stride,
                                                       float* __restrict__ out, int accumulate) {
  __shared__ float sh[256];
  float s = 0.f;
  for (int p = threadIdx.x; p < nparts; p += 256) s += part[(long)p * stride];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (threadIdx.x < h) sh[threadIdx.x] += sh[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + sh[0] : sh[0];
}

int det_reduce(const float* part, int nparts, long n, long stride, float* out, int accumulate, hipStream_t st) {
  if (n <= 0 || !out) return 0;
  if (n == 1 && nparts > 64) {
    hipLaunchKernelGGL(det_sum1_kernel, dim3(1), dim3(256), 0, st, part, nparts, stride, out, accumulate);
    SLX_LAUNCH_CHECK("det_reduce");
    return 0;
  }
  hipLaunchKernelGGL(det_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part, nparts, n, stride, out,
                     accumulate);
  SLX_LAUNCH_CHECK("det_reduce");
  return 0;
}

}  // namespace slx

extern "C" {
int slx_set_deterministic(int on, float* ws, int64_t ws_floats) {
  SLX_CHECK_ARG(!on || (ws && ws_floats >= (1 << 20)), "slx_set_deterministic: on needs a workspace of >= 2^20 floats");
  slx::DetMode& m = slx::det_mode();
  m.on = on ? 1 : 0;
  m.ws = on ? ws : nullptr;
  m.ws_floats = on ? ws_floats : 0;
  return 0;
}
int slx_get_deterministic(void) { return slx::det_mode().on; }
}
