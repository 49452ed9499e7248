// On-box calibration of the bf16 MFMA ceiling ("calibrate on-box ... and report both").
//
// The vendor's 2.5 PFLOP/s dense bf16 figure assumes 2.4 GHz; under a sustained bf16 load on random data the chip holds
// a lower clock (MI355X_MICROARCH.md 'DVFS give-back'), so the bench line reports, beside the spec, what a bare MFMA
// loop sustains on this box: every SIMD of every CU issues v_mfma_f32_32x32x16_bf16 back to back on register operands
// drawn from a seeded hash (random bits, not zeros: zero operands clock higher), four independent accumulators per
// wave, one wave per SIMD. No memory traffic inside the loop; the accumulators are reduced and stored once so the loop
// is not dead code.
#include "common.h"
#include "../../include/slx.h"

namespace slx {

__device__ __forceinline__ unsigned calib_hash(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(256, 1) void mfma_peak_kernel(int iters, float* out) {
  const unsigned t = blockIdx.x * 256u + threadIdx.x;
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // bf16 values in [-1, 1): sign + exponent 0x3F.. + random mantissa
    const unsigned ha = calib_hash(t * 16u + j), hb = calib_hash(t * 16u + 8u + j);
    a[j] = __builtin_bit_cast(bf16, (unsigned short)(0x3F00u | (ha & 0x80FFu)));
    b[j] = __builtin_bit_cast(bf16, (unsigned short)(0x3F00u | (hb & 0x80FFu)));
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c3, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[t] = s;
}

}  // namespace slx

extern "C" {

// grid x 256 threads (one wave per SIMD at one workgroup per CU), iters x 4 MFMAs per wave; FLOPs = grid * 4 waves *
// iters * 4 * 32 * 32 * 16 * 2. out: grid * 256 floats.
int slx_mfma_peak(int grid, int iters, float* out, slx_stream_t s) {
  SLX_CHECK_ARG(grid > 0 && iters > 0 && out, "slx_mfma_peak: grid, iters > 0 and an output buffer");
  hipLaunchKernelGGL(slx::mfma_peak_kernel, dim3(grid), dim3(256), 0, (hipStream_t)s, iters, out);
  SLX_LAUNCH_CHECK("slx_mfma_peak");
  return 0;
}

}  // extern "C"
