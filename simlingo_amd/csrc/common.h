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
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace slx {

// Thread-local error string (the C-ABI's slx_last_error()).
void set_error(const char* fmt, ...);
// deterministic-reduction mode (det.hip, slx_set_deterministic): partials in ws + ordered sums instead of f32 atomics
struct DetMode { int on; float* ws; long ws_floats; };
DetMode& det_mode();
int det_reduce(const float* part, int nparts, long n, long stride, float* out, int accumulate, hipStream_t st);


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

// GELU(erf) and its derivative, branch-free, from ONE exponential: with a = |x|/sqrt2, erfc(a) = P(t) e^{-a^2},
// t = 1/(1 + p a) (Abramowitz & Stegun 7.1.26, |error of erf| <= 1.5e-7), and e^{-a^2} = e^{-x^2/2} is also the
// normal density's exponential, so Phi(x) = 0.5 erfc(-x/sqrt2) and x phi(x) share it. One rcp + one exp2 + ~10 FMA
// per element (the Numerical Recipes form used before: rcp + two exp2 + ~17): the GEMM epilogues evaluate these on
// every element of InternViT's 16400 x 4096 fc1 output and fc2 input gradient, outside the MFMA main loop.
struct GeluTerms { float cdf, e; };  // Phi(x), e^{-x^2/2}
__device__ __forceinline__ GeluTerms gelu_terms(float x) {
  const float a = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f, a, 1.0f));
  const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);  // e^{-x^2/2}
  float q = 0.5f * 1.061405429f;  // 0.5 * (a1 t + ... + a5 t^5), Horner
  q = __builtin_fmaf(q, t, 0.5f * -1.453152027f);
  q = __builtin_fmaf(q, t, 0.5f * 1.421413741f);
  q = __builtin_fmaf(q, t, 0.5f * -0.284496736f);
  q = __builtin_fmaf(q, t, 0.5f * 0.254829592f);
  const float half_erfc = q * t * e;
  return GeluTerms{x > 0.f ? 1.0f - half_erfc : half_erfc, e};
}
__device__ __forceinline__ float normal_cdf(float x) { return gelu_terms(x).cdf; }
__device__ __forceinline__ float gelu_erf(float x) { return x * gelu_terms(x).cdf; }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const GeluTerms g = gelu_terms(x);
  return __builtin_fmaf(x * 0.39894228040143268f, g.e, g.cdf);
}
// x * sigmoid(x) with the sigmoid from the hardware reciprocal (v_rcp_f32, 1 ulp) instead of an IEEE division: every
// forward and backward kernel of the bf16 engine (SwiGLU forward, its LoRA-fused forms, the backward's recomputation,
// the decode GEMV) shares this one definition, so recomputed activations still equal the forward's bit for bit
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// the derivative likewise (it only feeds gradients, bf16-rounded dgu)
__device__ __forceinline__ float silu_grad(float x) {
  const float s = __builtin_amdgcn_rcpf(1.0f + __expf(-x));
  return s * (1.0f + x * (1.0f - s));
}

// Packed A (slx_lora_pack_a / slx_pack_scaled mode 2, read by slx_lora_down): the B-operand fragments of v_mfma_f32_32x32x16_bf16 in lane
// order, Af[((2*st + hh) * 64 + lane) * 8 + j] = A[lane & 31][32*st + 16*hh + 8*(lane >> 5) + j], so a wave reads one
// contiguous KiB per fragment instead of touching 32 rows of A.
__device__ __forceinline__ long lora_frag_index(int r, int k) {
  return ((long)(2 * (k >> 5) + ((k >> 4) & 1)) * 64 + r + 32 * ((k >> 3) & 1)) * 8 + (k & 7);
}

// Packed A for the dx term of slx_lora_bwd (slx_lora_pack_a layout 1 / slx_pack_scaled mode 3): the A-operand
// fragments of the transposed tile A^T dT^T, Ax[((2*ct + kb) * 64 + lane) * 8 + i] = A[16*kb + 8*(lane >> 5) + i][32*ct +
// (lane & 31)].
__device__ __forceinline__ long lora_dxfrag_index(int r, int k) {
  return ((long)(2 * (k >> 5) + (r >> 4)) * 64 + (k & 31) + 32 * ((r >> 3) & 1)) * 8 + (r & 7);
}

// Counter-based hash RNG for the LoRA dropout masks: deterministic in (seed, index). One 32-bit hash per PAIR of
// consecutive mask indices (idx >> 1); its low / high 16 bits are the uniforms of the even / odd element, and an
// element is kept iff its uniform >= thr = round(p * 65536) (p = 0.1 -> 6554 / 65536 = 0.100006). The forward
// (slx_lora_down) evaluates it once per element and stores the keep bits; the backward reads the bits.
__host__ __device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__host__ __device__ __forceinline__ uint32_t drop_seed_mix(uint64_t seed) {
  return hash_u32((uint32_t)seed ^ hash_u32((uint32_t)(seed >> 32) ^ 0x9e3779b9U));
}
__device__ __forceinline__ uint32_t drop_thr(float p) { return (uint32_t)(p * 65536.0f + 0.5f); }
__device__ __forceinline__ uint32_t drop_pair_hash(uint32_t s1, uint64_t idx) { return hash_u32((uint32_t)(idx >> 1) ^ s1); }
__device__ __forceinline__ bool drop_keep(uint32_t s1, uint64_t idx, uint32_t thr) {
  const uint32_t h = drop_pair_hash(s1, idx);
  return ((idx & 1) ? (h >> 16) : (h & 0xFFFFu)) >= thr;
}
// keep bits of 8 consecutive indices idx0..idx0+7 (idx0 even): bit j = keep(idx0 + j); 4 hashes
__device__ __forceinline__ uint32_t drop_keep8(uint32_t s1, uint64_t idx0, uint32_t thr) {
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t h = drop_pair_hash(s1, idx0 + 2 * j);
    b |= (uint32_t)((h & 0xFFFFu) >= thr) << (2 * j);
    b |= (uint32_t)((h >> 16) >= thr) << (2 * j + 1);
  }
  return b;
}

}  // namespace slx
