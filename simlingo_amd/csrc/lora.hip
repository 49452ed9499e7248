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


// ---- dA_j += dT_j^T drop_j(x) for the sites sharing x (peft LoRA backward of lora_A, llm.py:106-119).
// One launch per group: a block owns 128 columns of x (4 waves x 32) and a range of rows; every 64-row chunk
// of x and of the group's dT is staged once in LDS and read transposed (ds_read_b64_tr_b16) as the two
// operands of v_mfma_f32_32x32x16_bf16 (reduction over rows), with each site's dropout mask applied to the
// x fragment in registers. The [32 x 128] partials leave as 2 x 128-B-segment f32 atomics per instruction.
struct LoraDaArgs {
  const bf16* x; long ldx;
  int M, Kin, nsites;
  const bf16* dT; long ldt;
  float* dA[4];
  unsigned long long seed[4];
  float p;
  long ldmask;
  int mchunk;
};

__device__ __forceinline__ int la_sw(int row, int chunk) {
  return row * 128 + ((chunk ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3))) << 4);
}
__device__ __forceinline__ bf16x8 la_tr(const char* lds, int rbase, int cbase, int lane) {
  // lane l: X[rbase + 8(j>>2) + 4(l>>5) + (j&3)][cbase + (l&31)], j = 0..7
  const int G = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3, h = lane >> 5;
  const int row = rbase + 4 * h + q;
  const int col = cbase + 16 * (G & 1) + 4 * pp;
  const int e0 = la_sw(row, col >> 3) + ((col & 7) << 1);
  const int e1 = la_sw(row + 8, col >> 3) + ((col & 7) << 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + e0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + e1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

__global__ __launch_bounds__(256) void lora_da_kernel(LoraDaArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[4 * 8192];  // x: 2 x [64][64] | dT: 2 x [64][64]
  char* xs = smem;
  char* ts = smem + 2 * 8192;
  const int k0 = blockIdx.x * 128;
  const int mb = blockIdx.y * a.mchunk, me = min(a.M, mb + a.mchunk);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kc = k0 + 32 * w;
  const bool drop = a.p > 0.f;
  const float sc = drop ? 1.0f / (1.0f - a.p) : 1.0f;
  const int tcols = 32 * a.nsites;
  f32x16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  for (int mm = mb; mm < me; mm += 64) {
    const int row = tid >> 2, gm = mm + row;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const int c = (tid & 3) * 4 + c4;  // 16-B chunk 0..15 of the 128 columns
      const int gk = k0 + 8 * c;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (gm < me && gk < a.Kin) v = *reinterpret_cast<const uint4*>(a.x + (long)gm * a.ldx + gk);
      *reinterpret_cast<uint4*>(xs + (c >> 3) * 8192 + la_sw(row, c & 7)) = v;
      uint4 u = make_uint4(0u, 0u, 0u, 0u);
      if (gm < me && 8 * c < tcols) u = *reinterpret_cast<const uint4*>(a.dT + (long)gm * a.ldt + 8 * c);
      *reinterpret_cast<uint4*>(ts + (c >> 3) * 8192 + la_sw(row, c & 7)) = u;
    }
    __syncthreads();
#pragma unroll
    for (int ms = 0; ms < 4; ++ms) {
      const bf16x8 xb = la_tr(xs + (w >> 1) * 8192, 16 * ms, 32 * (w & 1), lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < a.nsites) {
          const bf16x8 ta = la_tr(ts + ((32 * j) >> 6) * 8192, 16 * ms, (32 * j) & 63, lane);
          bf16x8 xm = xb;
          if (drop) {
            const long col = kc + (lane & 31);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const long m = mm + 16 * ms + 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3);
              const float keep = uniform01(a.seed[j], (unsigned long long)(m * a.ldmask + col)) >= a.p ? sc : 0.f;
              xm[e] = (bf16)((float)xb[e] * keep);
            }
          }
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ta, xm, acc[j], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  const int col = kc + (lane & 31);
  if (col >= a.Kin) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j < a.nsites) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int r = (g & 3) + 8 * (g >> 2) + 4 * (lane >> 5);
        atomicAdd(a.dA[j] + (long)r * a.Kin + col, acc[j][g]);
      }
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
  dim3 grid((d->M + 31) / 32, d->nsites);
  hipLaunchKernelGGL(lora_down_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  SLX_LAUNCH_CHECK("slx_lora_down");
  return 0;
}

extern "C" int slx_lora_da(const slx_lora_da_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d->nsites >= 1 && d->nsites <= 4 && d->r == 32, "slx_lora_da: 1..4 sites of rank 32");
  SLX_CHECK_ARG(d->Kin % 8 == 0 && d->ldx % 8 == 0 && d->ldt % 8 == 0, "slx_lora_da: Kin/ldx/ldt %% 8");
  SLX_CHECK_ARG(d->p >= 0.f && d->p < 1.f, "slx_lora_da: 0 <= p < 1");
  if (d->M == 0) return 0;
  LoraDaArgs a;
  a.x = (const bf16*)d->x; a.ldx = d->ldx; a.M = d->M; a.Kin = d->Kin; a.nsites = d->nsites;
  a.dT = (const bf16*)d->dT; a.ldt = d->ldt;
  for (int i = 0; i < 4; ++i) {
    a.dA[i] = i < d->nsites ? d->dA[i] : d->dA[0];
    a.seed[i] = i < d->nsites ? d->seed[i] : 0;
  }
  a.p = d->p; a.ldmask = d->ldmask;
  const int cb = (d->Kin + 127) / 128;
  int ms = (512 + cb - 1) / cb;                       // ~2 blocks per CU
  int mchunk = (int)((d->M + ms - 1) / ms);
  mchunk = ((mchunk + 63) / 64) * 64;
  if (mchunk < 64) mchunk = 64;
  a.mchunk = mchunk;
  dim3 grid(cb, (unsigned)((d->M + mchunk - 1) / mchunk));
  hipLaunchKernelGGL(lora_da_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  SLX_LAUNCH_CHECK("slx_lora_da");
  return 0;
}
