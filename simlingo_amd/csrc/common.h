// Shared device/host helpers for the SimLingo MI355X (gfx950) kernels.
// Every kernel in this library is written for CDNA4 wave64 directly: no CUDA shims,
// no multi-backend dispatch. Storage types on the C-ABI are plain integers
// (bf16 = uint16_t bit pattern); device code uses __bf16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace slx {

// Thread-local error string (the C-ABI's slx_last_error()).
void set_error(const char* fmt, ...);

#define SLX_CHECK_ARG(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      slx::set_error(__VA_ARGS__);          \
      return -22; /* -EINVAL */             \
    }                                       \
  } while (0)

#define SLX_LAUNCH_CHECK(name)                                              \
  do {                                                                      \
    hipError_t e__ = hipGetLastError();                                     \
    if (e__ != hipSuccess) {                                                \
      slx::set_error("%s: launch failed: %s", name, hipGetErrorString(e__)); \
      return -(int)e__ - 1000;                                              \
    }                                                                       \
  } while (0)

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 and <= 1024; `sh` needs 16 floats.
__device__ __forceinline__ float block_sum(float v, float* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = warp_sum(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += sh[i];
  return t;
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float silu_grad(float x) {
  const float s = 1.0f / (1.0f + __expf(-x));
  return s * (1.0f + x * (1.0f - s));
}

// Counter-based hash RNG (for LoRA dropout masks): deterministic in (seed, index)
// so forward and backward regenerate the identical mask without storing it.
__device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t idx) {
  uint32_t h = hash_u32((uint32_t)idx ^ hash_u32((uint32_t)seed ^ (uint32_t)(idx >> 32) * 0x9e3779b9U) ^
                        (uint32_t)(seed >> 32));
  return (h >> 8) * (1.0f / 16777216.0f);
}

}  // namespace slx
