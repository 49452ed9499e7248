// LoRA down-projection for the Qwen2 hot path (peft LoraLayer with lora_dropout, llm.py:106-119):
//   t_s = dropout_s(x) . A_s^T      for the S sites of a group that share x (q/k/v or gate/up)
// written as bf16 into the extra columns of the activation buffer that the fused [W | s*B] GEMM
// reads (engine.py). One launch per group; grid = (row blocks of 64, sites); the dropout mask is the
// counter hash of slx_dropout applied while staging x (regenerated bit-exactly in backward).
// N = 32 per site is far too narrow for the 128x128 GEMM (50 blocks on 256 CUs); here each block
// owns 64 rows x 32 outputs: 4 waves x (16 rows x 32 cols) = 2 v_mfma_f32_16x16x32_bf16 per k-step.
#include "common.h"
#include "../../include/slx.h"

namespace slx {

struct LoraDownArgs {
  const bf16* x; long ldx;
  int M, Kin, nsites;
  const bf16* A[4];
  unsigned long long seed[4];
  bf16* t; long ldt;
  float p;
  long ldmask;
};

__device__ __forceinline__ int kc_off(int row, int c) { return row * 128 + ((c ^ ((row >> 1) & 7)) << 4); }

__global__ __launch_bounds__(256) void lora_down_kernel(LoraDownArgs a) {
  __shared__ __attribute__((aligned(16))) char xs[64 * 128];
  __shared__ __attribute__((aligned(16))) char as[32 * 128];
  const int site = blockIdx.y;
  const int m0 = blockIdx.x * 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bf16* A = a.A[site];
  const unsigned long long seed = a.seed[site];
  const float sc = a.p > 0.f ? 1.0f / (1.0f - a.p) : 1.0f;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const int xr = tid >> 2, xc = (tid & 3) * 2;     // x: 64 rows x 8 chunks, 2 chunks per thread
  const int ar = tid >> 3, acn = tid & 7;          // A: 32 rows x 8 chunks, 1 chunk per thread
  for (int k0 = 0; k0 < a.Kin; k0 += 64) {
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
      const int c = xc + c2, gm = m0 + xr, gk = k0 + c * 8;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (gm < a.M && gk < a.Kin) {
        v = *reinterpret_cast<const uint4*>(a.x + (long)gm * a.ldx + gk);
        if (a.p > 0.f) {
          bf16x8 e = __builtin_bit_cast(bf16x8, v);
          const long base = (long)gm * a.ldmask + gk;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = (bf16)((float)e[j] * (uniform01(seed, (unsigned long long)(base + j)) >= a.p ? sc : 0.f));
          v = __builtin_bit_cast(uint4, e);
        }
      }
      *reinterpret_cast<uint4*>(xs + kc_off(xr, c)) = v;
    }
    {
      const int gk = k0 + acn * 8;
      const uint4 v = gk < a.Kin ? *reinterpret_cast<const uint4*>(A + (long)ar * a.Kin + gk) : make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4*>(as + kc_off(ar, acn)) = v;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + (lane >> 4);
      const bf16x8 fa = *reinterpret_cast<const bf16x8*>(xs + kc_off(16 * w + (lane & 15), c));
      const bf16x8 fb0 = *reinterpret_cast<const bf16x8*>(as + kc_off(lane & 15, c));
      const bf16x8 fb1 = *reinterpret_cast<const bf16x8*>(as + kc_off(16 + (lane & 15), c));
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb1, acc1, 0, 0, 0);
    }
    __syncthreads();
  }
  bf16* out = a.t + site * 32;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + 16 * w + 4 * (lane >> 4) + r;
    if (m < a.M) {
      out[(long)m * a.ldt + (lane & 15)] = (bf16)acc0[r];
      out[(long)m * a.ldt + 16 + (lane & 15)] = (bf16)acc1[r];
    }
  }
}

}  // namespace slx

using namespace slx;

extern "C" int slx_lora_down(const slx_lora_down_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d->nsites >= 1 && d->nsites <= 4 && d->r == 32, "slx_lora_down: 1..4 sites of rank 32");
  SLX_CHECK_ARG(d->Kin % 8 == 0 && d->ldx % 8 == 0, "slx_lora_down: Kin/ldx %% 8");
  SLX_CHECK_ARG(d->p >= 0.f && d->p < 1.f, "slx_lora_down: 0 <= p < 1");
  if (d->M == 0) return 0;
  LoraDownArgs a;
  a.x = (const bf16*)d->x; a.ldx = d->ldx; a.M = d->M; a.Kin = d->Kin; a.nsites = d->nsites;
  for (int i = 0; i < 4; ++i) {
    a.A[i] = (const bf16*)(i < d->nsites ? d->A[i] : d->A[0]);
    a.seed[i] = i < d->nsites ? d->seed[i] : 0;
  }
  a.t = (bf16*)d->t; a.ldt = d->ldt; a.p = d->p; a.ldmask = d->ldmask;
  dim3 grid((d->M + 63) / 64, d->nsites);
  hipLaunchKernelGGL(lora_down_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  SLX_LAUNCH_CHECK("slx_lora_down");
  return 0;
}
