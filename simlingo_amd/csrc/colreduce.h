// Column reduction of per-block partial sums: out[c] (+)= sum_b partial[b*ldp + c].
// 64 columns x 4 row-lanes per workgroup: coalesced 256-B row segments, LDS combine.
#pragma once
#include "common.h"
namespace slx {
static __global__ __launch_bounds__(256) void colreduce_kernel(const float* partial, int nblk, int ncols, long ldp, float* out,
                                                        int accumulate) {
  __shared__ float sh[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float s = 0.f;
  if (c < ncols)
    for (int b = ty; b < nblk; b += 4) s += partial[(long)b * ldp + c];
  sh[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < ncols) {
    const float t = sh[0][tx] + sh[1][tx] + sh[2][tx] + sh[3][tx];
    out[c] = accumulate ? out[c] + t : t;
  }
}
static inline void launch_colreduce(const float* partial, int nblk, int ncols, long ldp, float* out, int accumulate,
                                    hipStream_t st) {
  hipLaunchKernelGGL(colreduce_kernel, dim3((ncols + 63) / 64), dim3(256), 0, st, partial, nblk, ncols, ldp, out, accumulate);
}
}  // namespace slx
