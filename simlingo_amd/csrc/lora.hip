// LoRA down-projection for the Qwen2 hot path (peft LoraLayer with lora_dropout, llm.py:106-119):
//   t_s = dropout_s(x) . A_s^T      for the S sites of a group that share x (q/k/v or gate/up)
// written as bf16 into the extra columns of the activation buffer that the fused [W | s*B] GEMM
// reads (engine.py). One launch per group; grid = (row blocks of 64, sites); the dropout mask is the
// counter hash of slx_dropout applied while staging x (regenerated bit-exactly in backward).
// N = 32 per site is far too narrow for the 128x128 GEMM (50 blocks on 256 CUs), and the K = 4864 down
// projection is a pure HBM stream of x: see the kernel comment for the layout.
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

// Operand fragments of v_mfma_f32_16x16x32_bf16 are loaded straight from global memory (no LDS staging):
// lane l holds x[row l&15][k0 + 8(l>>4) .. +8] (A) and A_s[n = l&15][same k] (B). The 4 waves of a block split
// the K dimension (k32 step s goes to wave s % 4) so each wave keeps 2 steps = 16 x 16-byte loads per lane in
// flight; the partial 32x32 tiles are summed through LDS at the end. Block = 32 rows x 32 outputs of one site.
__device__ __forceinline__ bf16x8 load_masked(const bf16* p, bool ok, bool drop, unsigned long long seed, long midx,
                                             float pdrop, float sc) {
  bf16x8 e;
  if (ok) {
    e = *reinterpret_cast<const bf16x8*>(p);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = (bf16)0.f;
  }
  if (drop) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      e[j] = (bf16)((float)e[j] * (uniform01(seed, (unsigned long long)(midx + j)) >= pdrop ? sc : 0.f));
  }
  return e;
}

__global__ __launch_bounds__(256) void lora_down_kernel(LoraDownArgs a) {
  __shared__ float red[4][32][33];
  const int site = blockIdx.y;
  const int m0 = blockIdx.x * 32;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bf16* A = a.A[site];
  const unsigned long long seed = a.seed[site];
  const bool drop = a.p > 0.f;
  const float sc = drop ? 1.0f / (1.0f - a.p) : 1.0f;
  const int r0 = lane & 15, kq = 8 * (lane >> 4);
  const int gm0 = m0 + r0, gm1 = m0 + 16 + r0;
  const bool v0 = gm0 < a.M, v1 = gm1 < a.M;
  const bf16* x0 = a.x + (long)(v0 ? gm0 : 0) * a.ldx;
  const bf16* x1 = a.x + (long)(v1 ? gm1 : 0) * a.ldx;
  const long mi0 = (long)gm0 * a.ldmask, mi1 = (long)gm1 * a.ldmask;
  const bf16* b0 = A + (long)r0 * a.Kin;
  const bf16* b1 = A + (long)(16 + r0) * a.Kin;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (a.Kin + 31) / 32;
  for (int s = w; s < nk; s += 8) {
    const int ka = s * 32 + kq, kb = (s + 4) * 32 + kq;
    const bool oka = ka < a.Kin, okb = (s + 4) < nk && kb < a.Kin;
    // issue every load of two k32 steps before the first MFMA
    const bf16x8 xa0 = load_masked(x0 + ka, v0 && oka, drop, seed, mi0 + ka, a.p, sc);
    const bf16x8 xa1 = load_masked(x1 + ka, v1 && oka, drop, seed, mi1 + ka, a.p, sc);
    const bf16x8 ba0 = load_masked(b0 + ka, oka, false, 0, 0, 0.f, 1.f);
    const bf16x8 ba1 = load_masked(b1 + ka, oka, false, 0, 0, 0.f, 1.f);
    const bf16x8 xb0 = load_masked(x0 + kb, v0 && okb, drop, seed, mi0 + kb, a.p, sc);
    const bf16x8 xb1 = load_masked(x1 + kb, v1 && okb, drop, seed, mi1 + kb, a.p, sc);
    const bf16x8 bb0 = load_masked(b0 + kb, okb, false, 0, 0, 0.f, 1.f);
    const bf16x8 bb1 = load_masked(b1 + kb, okb, false, 0, 0, 0.f, 1.f);
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa0, ba0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa0, ba1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa1, ba0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa1, ba1, acc[1][1], 0, 0, 0);
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb0, bb0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb0, bb1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb1, bb0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb1, bb1, acc[1][1], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][16 * i + 4 * (lane >> 4) + r][16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int row = threadIdx.x >> 3, c0 = (threadIdx.x & 7) * 4;
  const int m = m0 + row;
  if (m < a.M) {
    bf16* out = a.t + (long)m * a.ldt + site * 32 + c0;
#pragma unroll
    for (int c = 0; c < 4; ++c) out[c] = (bf16)(red[0][row][c0 + c] + red[1][row][c0 + c] + red[2][row][c0 + c] + red[3][row][c0 + c]);
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
  dim3 grid((d->M + 31) / 32, d->nsites);
  hipLaunchKernelGGL(lora_down_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  SLX_LAUNCH_CHECK("slx_lora_down");
  return 0;
}
