// LayerNorm (InternViT blocks eps 1e-6, mlp1 eps 1e-5) and RMSNorm (Qwen2, eps 1e-6), fwd + bwd.
// D <= 1024: one wave per row (shuffle reductions only). Wider rows (the mlp1 LayerNorm over 4096
// channels): one workgroup per row. The backward walks a strided set of rows per wave/workgroup so the
// gamma/beta column partials stay in registers and leave as one set of column atomics per workgroup. The mlp1 LayerNorm can gather its input through InternVL's
// pixel_shuffle(0.5, ps_version v2) (remote `extract_feature`, called at
// simlingo_training/models/encoder/internvl2_model.py:114), so the shuffled tensor never exists.
#include "common.h"
#include "../../include/slx.h"

namespace slx {

// Source row of pixel-shuffle output row `r`, chunk `c4` (0..3) of C channels.
// out[n, i2*G/2 + j2, c4*C + c] = x[n, 1 + (2*i2 + c4/2)*G + 2*j2 + c4%2, c]   (CLS token skipped)
__device__ __forceinline__ long ps_src_row(long r, int c4, int G, int tok_per_img) {
  const int half = G / 2;
  const long n = r / (half * half);
  const int t = r % (half * half);
  const int i2 = t / half, j2 = t % half;
  return n * tok_per_img + 1 + (long)(2 * i2 + (c4 >> 1)) * G + 2 * j2 + (c4 & 1);
}

struct NormArgs {
  const float* x; long ldx;
  const float* gamma; const float* beta;
  bf16* y; long ldy;
  float* mean; float* rstd;
  long rows; int D; float eps;
  int ps; int G; int C; int tok_per_img;  // pixel-shuffle gather
  int y_f32;                              // y holds f32 rows (CLIP pre_layrnorm feeds the f32 residual; for
                                          // RMS, the f32 parity mode: input dtype f32, no bf16 cast of x_hat)
  // bwd
  const float* dy; long lddy; int dy_bf16;  // dy_bf16: dy points to bf16 rows (slx_norm_desc.dy_bf16)
  float* dx; long lddx; int dx_accumulate;
  bf16* dxb; long lddxb;  // optional bf16 copy of dx (non-pixel-shuffle rows only)
  float* partial;   // unused (kept for ABI workspace sizing)
  float* detp;      // deterministic mode: per-block partial rows [4][gridDim.x][D] (dgamma, dbeta, dls, dlsb)
  float* dgamma; float* dbeta;
  // fused layer-scale branch backward on the updated dx (slx_norm_desc.ls*)
  const float* ls; const bf16* lsy; long ldlsy; bf16* lsg; long ldlsg; float* dls; float* dlsb;
};

// one block's column partial of parameter gradient q (0 dgamma, 1 dbeta, 2 dls, 3 dlsb) into its output: an f32 atomic,
// or (deterministic mode) a plain store into the partial rows summed in block order afterwards
__device__ __forceinline__ void norm_param_out(const NormArgs& a, int q, float* out, int c, float v) {
  if (a.detp) a.detp[((long)q * gridDim.x + blockIdx.x) * a.D + c] = v;
  else atomicAdd(out + c, v);
}

// 4 consecutive dy values of a row (f32 rows, or bf16 rows when a.dy_bf16; DYB: decided at compile time)
template <int DYB = -1>
__device__ __forceinline__ float4 load_dy4(const NormArgs& a, long row, int col) {
  if (DYB == 1 || (DYB < 0 && a.dy_bf16)) {
    const bf16x4 b = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(a.dy) + row * a.lddy + col);
    return make_float4((float)b[0], (float)b[1], (float)b[2], (float)b[3]);
  }
  return *reinterpret_cast<const float4*>(a.dy + row * a.lddy + col);
}

template <int VPT, bool RMS>
__global__ __launch_bounds__(256) void norm_fwd_kernel(NormArgs a) {
  __shared__ float sh[16];
  const long row = blockIdx.x;
  const int tid = threadIdx.x;
  float v[VPT];
#pragma unroll
  for (int i = 0; i < VPT / 4; ++i) {
    const int col = (tid + i * 256) * 4;
    if (col >= a.D) { v[4 * i] = v[4 * i + 1] = v[4 * i + 2] = v[4 * i + 3] = 0.f; continue; }
    const float* src;
    if (a.ps) {
      const int c4 = col / a.C;
      src = a.x + ps_src_row(row, c4, a.G, a.tok_per_img) * a.ldx + (col % a.C);
    } else {
      src = a.x + row * a.ldx + col;
    }
    const float4 t = *reinterpret_cast<const float4*>(src);
    v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
  }
  float mu = 0.f;
  if (!RMS) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) s += v[i];
    mu = block_sum(s, sh) / a.D;
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const float d = ((tid + (i / 4) * 256) * 4 < a.D) ? v[i] - mu : 0.f;
    ss += d * d;
  }
  const float var = block_sum(ss, sh) / a.D;
  const float rs = rsqrtf(var + a.eps);
  if (tid == 0) {
    if (a.mean) a.mean[row] = mu;
    a.rstd[row] = rs;
  }
#pragma unroll
  for (int i = 0; i < VPT / 4; ++i) {
    const int col = (tid + i * 256) * 4;
    if (col >= a.D) continue;
    float yv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (v[4 * i + e] - mu) * rs;
      if (RMS) yv[e] = (a.y_f32 ? xh : (float)(bf16)xh) * a.gamma[col + e];  // Qwen2: weight * hs.to(input_dtype)
      else yv[e] = xh * a.gamma[col + e] + a.beta[col + e];
    }
    if (a.y_f32) {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.y) + row * a.ldy + col) = make_float4(yv[0], yv[1], yv[2], yv[3]);
    } else {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)yv[e];
      *reinterpret_cast<bf16x4*>(a.y + row * a.ldy + col) = o;
    }
  }
}

// Wave-per-row variants for D <= 1024 (InternViT 1024, Qwen2 896): one 64-lane wave owns a row, lane l
// holds float4 chunks l, l+64, l+128, l+192; reductions are wave shuffles (no LDS, no barriers), so a
// 4-wave block keeps four independent rows of loads in flight instead of serialising one row behind two
// block-wide reductions.
template <bool RMS>
__global__ __launch_bounds__(256) void norm_fwd_wave_kernel(NormArgs a) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  // every load unconditional (columns past D read column 0 and are zeroed by a select): a load inside a branch makes
  // hipcc drain vmcnt(0) behind it; gamma / beta are issued with x, so the row costs one round trip
  float v[16];
  float4 gm[4], bt[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = (lane + 64 * i) * 4;
    const bool ok = col < a.D;
    const int cl = ok ? col : 0;
    const float* src = a.ps ? a.x + ps_src_row(row, cl / a.C, a.G, a.tok_per_img) * a.ldx + (cl % a.C)
                            : a.x + row * a.ldx + cl;
    float4 t = *reinterpret_cast<const float4*>(src);
    gm[i] = *reinterpret_cast<const float4*>(a.gamma + cl);
    if (!RMS) bt[i] = *reinterpret_cast<const float4*>(a.beta + cl);
    if (!ok) t = make_float4(0.f, 0.f, 0.f, 0.f);
    v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
  }
  float mu = 0.f;
  if (!RMS) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += v[i];
    mu = warp_sum(s) / a.D;
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float d = ((lane + 64 * (i / 4)) * 4 < a.D) ? v[i] - mu : 0.f;
    ss += d * d;
  }
  const float rs = rsqrtf(warp_sum(ss) / a.D + a.eps);
  if (lane == 0) {
    if (a.mean) a.mean[row] = mu;
    a.rstd[row] = rs;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = (lane + 64 * i) * 4;
    if (col >= a.D) continue;
    float yv[4];
    const float gv[4] = {gm[i].x, gm[i].y, gm[i].z, gm[i].w};
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (!RMS) { bv[0] = bt[i].x; bv[1] = bt[i].y; bv[2] = bt[i].z; bv[3] = bt[i].w; }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (v[4 * i + e] - mu) * rs;
      yv[e] = RMS ? (a.y_f32 ? xh : (float)(bf16)xh) * gv[e] : xh * gv[e] + bv[e];
    }
    if (a.y_f32) {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.y) + row * a.ldy + col) = make_float4(yv[0], yv[1], yv[2], yv[3]);
    } else {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)yv[e];
      *reinterpret_cast<bf16x4*>(a.y + row * a.ldy + col) = o;
    }
  }
}

// read-once streams of the LayerNorm backward (x, dy, the accumulated dx input, the layer-scale branch rows) as
// nontemporal loads: +0.2 % on the step (the next GEMM's operands are not evicted by them), although the isolated
// microbenchmark, which re-reads the same MALL-resident buffers every call, runs 7-13 % slower
// (profiles/round5_norm_bwd_nt_ab.txt)
typedef float nt_f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned nt_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 ldnt_f4(const float* p) {
  const nt_f32x4 t = __builtin_nontemporal_load(reinterpret_cast<const nt_f32x4*>(p));
  return make_float4(t[0], t[1], t[2], t[3]);
}
__device__ __forceinline__ bf16x4 ldnt_b4(const bf16* p) {
  const nt_u32x2 t = __builtin_nontemporal_load(reinterpret_cast<const nt_u32x2*>(p));
  return __builtin_bit_cast(bf16x4, t);
}

template <bool RMS, bool LS, bool DYB>
__global__ __launch_bounds__(256) void norm_bwd_wave_kernel(NormArgs a) {
  // column sums (dgamma, dbeta; dls, dbias of the layer-scale branch) accumulate in wave-private LDS rows: each lane
  // owns its 16 columns, so there are no conflicts and no barriers until the end, and the 64 accumulator registers go
  // to the second row in flight instead
  __shared__ __attribute__((aligned(16))) float cs[4][LS ? 4 : 2][1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int NACC = LS ? 4 : 2;
#pragma unroll
  for (int q = 0; q < NACC; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      if (col < 1024) *reinterpret_cast<float4*>(&cs[w][q][col]) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  auto acc4 = [&](int q, int col, const float (&v)[4]) {
    float4* p = reinterpret_cast<float4*>(&cs[w][q][col]);
    float4 c = *p;
    c.x += v[0]; c.y += v[1]; c.z += v[2]; c.w += v[3];
    *p = c;
  };
  // Software-pipelined rows: the next row's loads (x, dy, the accumulated dx row, the layer-scale branch row and its
  // mean / rstd) are issued before the current row's reductions and stores, so each wave keeps two rows of HBM traffic
  // in flight (the kernel is HBM-bound; gamma and ls are loaded once per wave).
  struct RowIn {
    float mu, rs;
    float4 t[4], dxo[4];
    float4 d[4];
    bf16x4 lyv[4];
  };
  // gamma / ls of this lane's columns: re-read per row (L1 hits) ahead of the next row's loads, so their wait does
  // not cover the next row's traffic (in-order vmcnt) and they hold no registers across the row
  auto load_cols = [&](float4 (&gm)[4], float4 (&lsv)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      gm[i] = col < a.D ? *reinterpret_cast<const float4*>(a.gamma + col) : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (LS) lsv[i] = col < a.D ? *reinterpret_cast<const float4*>(a.ls + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto load_row = [&](long row, RowIn& r) {
    r.mu = RMS ? 0.f : a.mean[row];
    r.rs = a.rstd[row];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      r.dxo[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      r.t[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      r.d[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (col < a.D) {
        if (a.dx_accumulate) {
          const float* dsrc = a.ps ? a.dx + ps_src_row(row, col / a.C, a.G, a.tok_per_img) * a.lddx + (col % a.C)
                                   : a.dx + row * a.lddx + col;
          r.dxo[i] = ldnt_f4(dsrc);
        }
        if constexpr (LS) r.lyv[i] = ldnt_b4(a.lsy + row * a.ldlsy + col);
        const float* src = a.ps ? a.x + ps_src_row(row, col / a.C, a.G, a.tok_per_img) * a.ldx + (col % a.C)
                                : a.x + row * a.ldx + col;
        r.t[i] = ldnt_f4(src);
        if constexpr (DYB) {
          const bf16x4 b = ldnt_b4(reinterpret_cast<const bf16*>(a.dy) + row * a.lddy + col);
          r.d[i] = make_float4((float)b[0], (float)b[1], (float)b[2], (float)b[3]);
        } else {
          r.d[i] = ldnt_f4(a.dy + row * a.lddy + col);
        }
      }
    }
  };
  const long stride = (long)gridDim.x * 4;
  long row = (long)blockIdx.x * 4 + w;
  RowIn cur;
  if (row < a.rows) load_row(row, cur);
  for (; row < a.rows; row += stride) {
    float4 gm[4], lsv[4];
    load_cols(gm, lsv);
    RowIn nxt;
    if (row + stride < a.rows) load_row(row + stride, nxt);
    const float mu = cur.mu, rs = cur.rs;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      const float4 t = cur.t[i], d = cur.d[i], g = gm[i];
      const float tv[4] = {t.x, t.y, t.z, t.w}, dv[4] = {d.x, d.y, d.z, d.w}, gv[4] = {g.x, g.y, g.z, g.w};
      float ag[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = col < a.D ? (tv[e] - mu) * rs : 0.f;
        const float gd = dv[e] * gv[e];
        s1 += gd;
        s2 += gd * xh;
        ag[e] = dv[e] * (RMS ? (float)(bf16)xh : xh);
      }
      if (col < a.D) {
        acc4(0, col, ag);
        acc4(1, col, dv);
      }
    }
    const float m1 = RMS ? 0.f : warp_sum(s1) / a.D;
    const float m2 = warp_sum(s2) / a.D;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      if (col >= a.D) continue;
      float* dst = a.ps ? a.dx + ps_src_row(row, col / a.C, a.G, a.tok_per_img) * a.lddx + (col % a.C)
                        : a.dx + row * a.lddx + col;
      float ov[4];
      {  // x_hat and g*dy recomputed from the row's registers (cheaper than keeping 32 of them live)
        const float4 t = cur.t[i], d = cur.d[i], g = gm[i];
        const float tv[4] = {t.x, t.y, t.z, t.w}, dv[4] = {d.x, d.y, d.z, d.w}, gv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (tv[e] - mu) * rs;
          const float gd = __fmul_rn(dv[e], gv[e]);  // a rounded product, as norm_bwd_row_kernel keeps it (no FMA fusion)
          ov[e] = rs * (gd - m1 - xh * m2);
        }
      }
      if (a.dx_accumulate) {
        ov[0] += cur.dxo[i].x; ov[1] += cur.dxo[i].y; ov[2] += cur.dxo[i].z; ov[3] += cur.dxo[i].w;
      }
      *reinterpret_cast<float4*>(dst) = make_float4(ov[0], ov[1], ov[2], ov[3]);
      if (a.dxb) {
        bf16x4 ob;
#pragma unroll
        for (int e = 0; e < 4; ++e) ob[e] = (bf16)ov[e];
        *reinterpret_cast<bf16x4*>(a.dxb + row * a.lddxb + col) = ob;
      }
      if constexpr (LS) {  // slx_ls_branch_bwd's per-element work on the row just produced (colsum_kernel<2>)
        const float4 l4 = lsv[i];
        const bf16x4 yy = cur.lyv[i];
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
        bf16x4 go;
        float al[4], aq[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gv = ov[e] * lv[e];
          go[e] = (bf16)gv;
          al[e] = ov[e] * (float)yy[e];
          aq[e] = gv;
        }
        acc4(LS ? 2 : 0, col, al);
        acc4(LS ? 3 : 0, col, aq);
        *reinterpret_cast<bf16x4*>(a.lsg + row * a.ldlsg + col) = go;
      }
    }
    cur = nxt;
  }
  if (a.dgamma || a.dbeta || LS) {  // 4 waves' column partials summed through LDS, then contiguous f32 atomics
    __syncthreads();
    for (int c = threadIdx.x; c < a.D; c += 256) {
      if (a.dgamma) norm_param_out(a, 0, a.dgamma, c, cs[0][0][c] + cs[1][0][c] + cs[2][0][c] + cs[3][0][c]);
      if (a.dbeta) norm_param_out(a, 1, a.dbeta, c, cs[0][1][c] + cs[1][1][c] + cs[2][1][c] + cs[3][1][c]);
      if constexpr (LS) {
        norm_param_out(a, 2, a.dls, c,
                       cs[0][LS ? 2 : 0][c] + cs[1][LS ? 2 : 0][c] + cs[2][LS ? 2 : 0][c] + cs[3][LS ? 2 : 0][c]);
        norm_param_out(a, 3, a.dlsb, c,
                       cs[0][LS ? 3 : 0][c] + cs[1][LS ? 3 : 0][c] + cs[2][LS ? 3 : 0][c] + cs[3][LS ? 3 : 0][c]);
      }
    }
  }
}

// The same backward for the InternViT / CLIP rows (D = 1024, accumulating dx, no pixel shuffle, no bf16 dx copy) with
// every load and store unconditional. In norm_bwd_wave_kernel the per-column `col < D` guards, the runtime
// accumulate / pixel-shuffle choices and the guarded next-row prefetch put each load inside a branch; hipcc then waited
// for each column chunk's dy before issuing the next chunk's loads (4 round trips per row) and drained vmcnt(0) behind
// the prefetch. Here:
//  * the next row's loads are issued for a clamped row index (a wave's last row re-reads itself), and the loop is a
//    two-row ping-pong (A / B register sets, the first row peeled) so no loop-carried copy of in-flight registers forces
//    a drain at the loop head, and the loop is entered with the same loads-then-stores pattern it repeats;
//  * gamma and the layer scale come from LDS (staged once), so no global load of them is queued behind a row's stream;
//  * dy stays in its bf16 registers until it is used; the row sums are DPP row sums + 4 readlanes.
__device__ __forceinline__ float wave_sum_dpp(float x) {
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true));   // quad_perm [1, 0, 3, 2]
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, true));   // quad_perm [2, 3, 0, 1]
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x124, 0xF, 0xF, true));  // row_ror:4
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x128, 0xF, 0xF, true));  // row_ror:8
  const auto rl = [&](int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l)); };
  return (rl(0) + rl(16)) + (rl(32) + rl(48));
}

template <bool RMS, bool LS, bool DYB>
__global__ __launch_bounds__(256) void norm_bwd_wave1024_kernel(NormArgs a) {
  constexpr int D = 1024;
  constexpr int NACC = LS ? 4 : 2;
  __shared__ __attribute__((aligned(16))) float cs[4][NACC][D];
  __shared__ __attribute__((aligned(16))) float gl[LS ? 2 : 1][D];  // gamma | layer scale
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  *reinterpret_cast<float4*>(&gl[0][threadIdx.x * 4]) = *reinterpret_cast<const float4*>(a.gamma + threadIdx.x * 4);
  if constexpr (LS) *reinterpret_cast<float4*>(&gl[LS ? 1 : 0][threadIdx.x * 4]) = *reinterpret_cast<const float4*>(a.ls + threadIdx.x * 4);
#pragma unroll
  for (int q = 0; q < NACC; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(&cs[w][q][(lane + 64 * i) * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  auto acc4 = [&](int q, int col, const float (&v)[4]) {
    float4* p = reinterpret_cast<float4*>(&cs[w][q][col]);
    float4 c = *p;
    c.x += v[0]; c.y += v[1]; c.z += v[2]; c.w += v[3];
    *p = c;
  };
  struct RowIn {
    float mu, rs;
    float4 t[4], dxo[4], df[4];
    bf16x4 db[4], lyv[4];
  };
  auto load_row = [&](long row, RowIn& r) {
    r.mu = RMS ? 0.f : a.mean[row];
    r.rs = a.rstd[row];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      r.dxo[i] = ldnt_f4(a.dx + row * a.lddx + col);
      if constexpr (LS) r.lyv[i] = ldnt_b4(a.lsy + row * a.ldlsy + col);
      r.t[i] = ldnt_f4(a.x + row * a.ldx + col);
      if constexpr (DYB) r.db[i] = ldnt_b4(reinterpret_cast<const bf16*>(a.dy) + row * a.lddy + col);
      else r.df[i] = ldnt_f4(a.dy + row * a.lddy + col);
    }
  };
  auto dy4 = [&](const RowIn& r, int i, float (&dv)[4]) {
    if constexpr (DYB) {
#pragma unroll
      for (int e = 0; e < 4; ++e) dv[e] = (float)r.db[i][e];
    } else {
      dv[0] = r.df[i].x; dv[1] = r.df[i].y; dv[2] = r.df[i].z; dv[3] = r.df[i].w;
    }
  };
  auto process = [&](const RowIn& cur, long row) {
    const float mu = cur.mu, rs = cur.rs;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      const float4 t = cur.t[i], g = *reinterpret_cast<const float4*>(&gl[0][col]);
      const float tv[4] = {t.x, t.y, t.z, t.w}, gv[4] = {g.x, g.y, g.z, g.w};
      float dv[4], ag[4];
      dy4(cur, i, dv);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = (tv[e] - mu) * rs;
        const float gd = dv[e] * gv[e];
        s1 += gd;
        s2 += gd * xh;
        ag[e] = dv[e] * (RMS ? (float)(bf16)xh : xh);
      }
      acc4(0, col, ag);
      acc4(1, col, dv);
    }
    const float m1 = RMS ? 0.f : wave_sum_dpp(s1) / D;
    const float m2 = wave_sum_dpp(s2) / D;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      float ov[4];
      {
        const float4 t = cur.t[i], g = *reinterpret_cast<const float4*>(&gl[0][col]);
        const float tv[4] = {t.x, t.y, t.z, t.w}, gv[4] = {g.x, g.y, g.z, g.w};
        float dv[4];
        dy4(cur, i, dv);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (tv[e] - mu) * rs;
          const float gd = __fmul_rn(dv[e], gv[e]);  // a rounded product, as norm_bwd_wave_kernel keeps it
          ov[e] = rs * (gd - m1 - xh * m2);
        }
      }
      ov[0] += cur.dxo[i].x; ov[1] += cur.dxo[i].y; ov[2] += cur.dxo[i].z; ov[3] += cur.dxo[i].w;
      *reinterpret_cast<float4*>(a.dx + row * a.lddx + col) = make_float4(ov[0], ov[1], ov[2], ov[3]);
      if constexpr (LS) {
        const float4 l4 = *reinterpret_cast<const float4*>(&gl[LS ? 1 : 0][col]);
        const bf16x4 yy = cur.lyv[i];
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
        bf16x4 go;
        float al[4], aq[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gv = ov[e] * lv[e];
          go[e] = (bf16)gv;
          al[e] = ov[e] * (float)yy[e];
          aq[e] = gv;
        }
        acc4(LS ? 2 : 0, col, al);
        acc4(LS ? 3 : 0, col, aq);
        *reinterpret_cast<bf16x4*>(a.lsg + row * a.ldlsg + col) = go;
      }
    }
  };
  // host guarantees rows >= 16 * gridDim.x: every wave owns at least its first row
  const long stride = (long)gridDim.x * 4;
  const auto clamp = [&](long r) { return r < a.rows ? r : a.rows - 1; };
  long row = (long)blockIdx.x * 4 + w;
  // sched_barrier after each prefetch: without it the scheduler hoists the current row's first arithmetic above the
  // next row's loads, which then wait for the current row's data (the overlap this loop exists for is lost)
  RowIn A, B;
  load_row(row, B);
  load_row(clamp(row + stride), A);
  __builtin_amdgcn_sched_barrier(0);
  process(B, row);
  row += stride;
  while (row < a.rows) {  // A holds `row`
    load_row(clamp(row + stride), B);
    __builtin_amdgcn_sched_barrier(0);
    process(A, row);
    row += stride;
    if (row >= a.rows) break;
    load_row(clamp(row + stride), A);
    __builtin_amdgcn_sched_barrier(0);
    process(B, row);
    row += stride;
  }
  __syncthreads();  // 4 waves' column partials summed through LDS, then contiguous f32 atomics
  for (int c = threadIdx.x; c < D; c += 256) {
    if (a.dgamma) norm_param_out(a, 0, a.dgamma, c, cs[0][0][c] + cs[1][0][c] + cs[2][0][c] + cs[3][0][c]);
    if (a.dbeta) norm_param_out(a, 1, a.dbeta, c, cs[0][1][c] + cs[1][1][c] + cs[2][1][c] + cs[3][1][c]);
    if constexpr (LS) {
      norm_param_out(a, 2, a.dls, c,
                     cs[0][LS ? 2 : 0][c] + cs[1][LS ? 2 : 0][c] + cs[2][LS ? 2 : 0][c] + cs[3][LS ? 2 : 0][c]);
      norm_param_out(a, 3, a.dlsb, c,
                     cs[0][LS ? 3 : 0][c] + cs[1][LS ? 3 : 0][c] + cs[2][LS ? 3 : 0][c] + cs[3][LS ? 3 : 0][c]);
    }
  }
}

// One row at a time per wave, column sums in registers: the form for few rows per wave (Qwen2 RMSNorm, 6384 rows),
// where norm_bwd_wave_kernel's second row in flight does not pay for its LDS accumulators.
template <bool RMS, bool LS, bool DYB>
__global__ __launch_bounds__(256) void norm_bwd_row_kernel(NormArgs a) {
  __shared__ float cs[4][LS ? 4 : 2][1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float pg[16], pb[16], pl[16], pq[16];  // pl/pq: layer-scale branch sums (dls, dbias), LS only
#pragma unroll
  for (int i = 0; i < 16; ++i) { pg[i] = 0.f; pb[i] = 0.f; pl[i] = 0.f; pq[i] = 0.f; }
  for (long row = (long)blockIdx.x * 4 + w; row < a.rows; row += (long)gridDim.x * 4) {
    const float mu = RMS ? 0.f : a.mean[row];
    const float rs = a.rstd[row];
    float xh[16], gd[16];
    float s1 = 0.f, s2 = 0.f;
    // every load of the row issued together and unconditionally (columns past D read column 0, a non-accumulating
    // call reads the dx row it is about to overwrite; both are zeroed by a select): a load inside a branch, or a bf16
    // dy widened right after its load, made hipcc wait for each column chunk before issuing the next one's loads
    float4 dxo[4], tt[4], gg[4], df[4], lsv[4];
    bf16x4 db[4], lyv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      const int cl = col < a.D ? col : 0;
      const long xr = a.ps ? ps_src_row(row, cl / a.C, a.G, a.tok_per_img) : row;
      const int xc = a.ps ? cl % a.C : cl;
      dxo[i] = ldnt_f4(a.dx + xr * a.lddx + xc);
      if constexpr (LS) {
        lyv[i] = *reinterpret_cast<const bf16x4*>(a.lsy + row * a.ldlsy + cl);
        lsv[i] = *reinterpret_cast<const float4*>(a.ls + cl);
      }
      tt[i] = ldnt_f4(a.x + xr * a.ldx + xc);
      if constexpr (DYB) db[i] = ldnt_b4(reinterpret_cast<const bf16*>(a.dy) + row * a.lddy + cl);
      else df[i] = ldnt_f4(a.dy + row * a.lddy + cl);
      gg[i] = *reinterpret_cast<const float4*>(a.gamma + cl);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      const bool ok = col < a.D;
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 t = ok ? tt[i] : z, g = ok ? gg[i] : z;
      float4 d = df[i];
      if constexpr (DYB) d = make_float4((float)db[i][0], (float)db[i][1], (float)db[i][2], (float)db[i][3]);
      if (!ok) d = z;
      if (!(ok && a.dx_accumulate)) dxo[i] = z;
      const float tv[4] = {t.x, t.y, t.z, t.w}, dv[4] = {d.x, d.y, d.z, d.w}, gv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * i + e;
        xh[k] = ok ? (tv[e] - mu) * rs : 0.f;
        gd[k] = dv[e] * gv[e];
        s1 += gd[k];
        s2 += gd[k] * xh[k];
        pg[k] += dv[e] * (RMS ? (float)(bf16)xh[k] : xh[k]);
        pb[k] += dv[e];
      }
    }
    const float m1 = RMS ? 0.f : warp_sum(s1) / a.D;
    const float m2 = warp_sum(s2) / a.D;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      if (col >= a.D) continue;
      float* dst = a.ps ? a.dx + ps_src_row(row, col / a.C, a.G, a.tok_per_img) * a.lddx + (col % a.C)
                        : a.dx + row * a.lddx + col;
      float ov[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) ov[e] = rs * (gd[4 * i + e] - m1 - xh[4 * i + e] * m2);
      if (a.dx_accumulate) {
        ov[0] += dxo[i].x; ov[1] += dxo[i].y; ov[2] += dxo[i].z; ov[3] += dxo[i].w;
      }
      *reinterpret_cast<float4*>(dst) = make_float4(ov[0], ov[1], ov[2], ov[3]);
      if (a.dxb) {
        bf16x4 ob;
#pragma unroll
        for (int e = 0; e < 4; ++e) ob[e] = (bf16)ov[e];
        *reinterpret_cast<bf16x4*>(a.dxb + row * a.lddxb + col) = ob;
      }
      if constexpr (LS) {  // slx_ls_branch_bwd's per-element work on the row just produced (colsum_kernel<2>)
        const float4 l4 = lsv[i];
        const bf16x4 yy = lyv[i];
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
        bf16x4 go;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gv = ov[e] * lv[e];
          go[e] = (bf16)gv;
          pl[4 * i + e] += ov[e] * (float)yy[e];
          pq[4 * i + e] += gv;
        }
        *reinterpret_cast<bf16x4*>(a.lsg + row * a.ldlsg + col) = go;
      }
    }
  }
  if (a.dgamma || a.dbeta || LS) {  // 4 waves' column partials summed through LDS, then contiguous f32 atomics
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (lane + 64 * i) * 4;
      if (col >= a.D) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        cs[w][0][col + e] = pg[4 * i + e];
        cs[w][1][col + e] = pb[4 * i + e];
        if constexpr (LS) {
          cs[w][LS ? 2 : 0][col + e] = pl[4 * i + e];
          cs[w][LS ? 3 : 0][col + e] = pq[4 * i + e];
        }
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < a.D; c += 256) {
      if (a.dgamma) norm_param_out(a, 0, a.dgamma, c, cs[0][0][c] + cs[1][0][c] + cs[2][0][c] + cs[3][0][c]);
      if (a.dbeta) norm_param_out(a, 1, a.dbeta, c, cs[0][1][c] + cs[1][1][c] + cs[2][1][c] + cs[3][1][c]);
      if constexpr (LS) {
        norm_param_out(a, 2, a.dls, c,
                       cs[0][LS ? 2 : 0][c] + cs[1][LS ? 2 : 0][c] + cs[2][LS ? 2 : 0][c] + cs[3][LS ? 2 : 0][c]);
        norm_param_out(a, 3, a.dlsb, c,
                       cs[0][LS ? 3 : 0][c] + cs[1][LS ? 3 : 0][c] + cs[2][LS ? 3 : 0][c] + cs[3][LS ? 3 : 0][c]);
      }
    }
  }
}

// Backward. dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat))      (LayerNorm)
//           dx = rstd * (g*dy - xhat * mean(g*dy*xhat))                     (RMSNorm)
// dgamma = sum dy*xhat, dbeta = sum dy -> per-block partials.
template <int VPT, bool RMS>
__global__ __launch_bounds__(256) void norm_bwd_kernel(NormArgs a) {
  __shared__ float sh[16];
  const int tid = threadIdx.x;
  float pg[VPT], pb[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  for (long row = blockIdx.x; row < a.rows; row += gridDim.x) {
    const float mu = RMS ? 0.f : a.mean[row];
    const float rs = a.rstd[row];
    float xh[VPT], gd[VPT];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPT / 4; ++i) {
      const int col = (tid + i * 256) * 4;
      if (col >= a.D) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { xh[4 * i + e] = 0.f; gd[4 * i + e] = 0.f; }
        continue;
      }
      const float* src;
      if (a.ps) src = a.x + ps_src_row(row, col / a.C, a.G, a.tok_per_img) * a.ldx + (col % a.C);
      else src = a.x + row * a.ldx + col;
      const float4 t = *reinterpret_cast<const float4*>(src);
      const float4 d = load_dy4(a, row, col);
      const float tv[4] = {t.x, t.y, t.z, t.w}, dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * i + e;
        xh[k] = (tv[e] - mu) * rs;
        gd[k] = dv[e] * a.gamma[col + e];
        s1 += gd[k];
        s2 += gd[k] * xh[k];
        pg[k] += dv[e] * (RMS ? (float)(bf16)xh[k] : xh[k]);
        pb[k] += dv[e];
      }
    }
    const float m1 = RMS ? 0.f : block_sum(s1, sh) / a.D;
    const float m2 = block_sum(s2, sh) / a.D;
#pragma unroll
    for (int i = 0; i < VPT / 4; ++i) {
      const int col = (tid + i * 256) * 4;
      if (col >= a.D) continue;
      float* dst;
      if (a.ps) dst = a.dx + ps_src_row(row, col / a.C, a.G, a.tok_per_img) * a.lddx + (col % a.C);
      else dst = a.dx + row * a.lddx + col;
      float4 o;
      float ov[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * i + e;
        ov[e] = rs * (gd[k] - m1 - xh[k] * m2);
      }
      if (a.dx_accumulate) {
        const float4 p = *reinterpret_cast<const float4*>(dst);
        ov[0] += p.x; ov[1] += p.y; ov[2] += p.z; ov[3] += p.w;
      }
      o.x = ov[0]; o.y = ov[1]; o.z = ov[2]; o.w = ov[3];
      *reinterpret_cast<float4*>(dst) = o;
      if (a.dxb) {
        bf16x4 ob;
#pragma unroll
        for (int e = 0; e < 4; ++e) ob[e] = (bf16)ov[e];
        *reinterpret_cast<bf16x4*>(a.dxb + row * a.lddxb + col) = ob;
      }
    }
  }
  // column partials -> dgamma / dbeta (pre-zeroed or accumulating) with f32 atomics, transposed
  // through LDS so that each atomic wave-instruction covers 256 contiguous bytes
  if (a.dgamma || a.dbeta) {
    __shared__ float cs[2][VPT * 256];
#pragma unroll
    for (int i = 0; i < VPT / 4; ++i) {
      const int col = (tid + i * 256) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        cs[0][col + e] = pg[4 * i + e];
        cs[1][col + e] = pb[4 * i + e];
      }
    }
    __syncthreads();
    for (int c = tid; c < a.D; c += 256) {
      if (a.dgamma) norm_param_out(a, 0, a.dgamma, c, cs[0][c]);
      if (a.dbeta) norm_param_out(a, 1, a.dbeta, c, cs[1][c]);
    }
  }
}



}  // namespace slx

using namespace slx;

static constexpr int kBwdBlocks = 512;

// SLX_NORM_W1024=0: the D = 1024 LayerNorm backward through norm_bwd_wave_kernel instead (A/B)
static bool norm_w1024() {
  static const bool on = [] {
    const char* e = getenv("SLX_NORM_W1024");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <bool RMS>
static int norm_fwd(NormArgs& a, hipStream_t st) {
  SLX_CHECK_ARG(a.D % 4 == 0 && a.D <= 4096, "norm fwd: D=%d must be a multiple of 4 and <= 4096", a.D);
  if (a.D <= 1024) hipLaunchKernelGGL((norm_fwd_wave_kernel<RMS>), dim3((a.rows + 3) / 4), dim3(256), 0, st, a);
  else if (a.D <= 2048) hipLaunchKernelGGL((norm_fwd_kernel<8, RMS>), dim3(a.rows), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((norm_fwd_kernel<16, RMS>), dim3(a.rows), dim3(256), 0, st, a);
  SLX_LAUNCH_CHECK("slx_norm_fwd");
  return 0;
}

template <bool RMS>
static int norm_bwd(NormArgs& a, float* dgamma, float* dbeta, int accumulate, hipStream_t st) {
  int nblk = (int)(a.rows < kBwdBlocks ? a.rows : kBwdBlocks);
  const DetMode& dm = det_mode();
  a.detp = nullptr;
  if (dm.on && (dgamma || dbeta || a.ls)) {  // partial rows [4][nblk][D], summed in block order below
    SLX_CHECK_ARG(dm.ws_floats >= 4L * a.D, "slx_norm_bwd: deterministic workspace too small");
    if (4L * nblk * a.D > dm.ws_floats) nblk = (int)(dm.ws_floats / (4L * a.D));
    a.detp = dm.ws;
  }
  SLX_CHECK_ARG(a.D % 4 == 0 && a.D <= 4096, "norm bwd: D=%d must be a multiple of 4 and <= 4096", a.D);
  a.dgamma = dgamma;
  a.dbeta = dbeta;
  if (!accumulate) {
    if (dgamma) hipMemsetAsync(dgamma, 0, a.D * sizeof(float), st);
    if (dbeta) hipMemsetAsync(dbeta, 0, a.D * sizeof(float), st);
  }
  const bool two_rows = a.rows >= 16 * nblk;  // >= 4 rows per wave: two rows in flight per wave pay off
  if (a.D == 1024 && two_rows && !a.ps && a.dx_accumulate && !a.dxb && norm_w1024()) {
    // (InternViT / CLIP layers) branch-free form
    if (a.ls) {
      if (a.dy_bf16) hipLaunchKernelGGL((norm_bwd_wave1024_kernel<RMS, true, true>), dim3(nblk), dim3(256), 0, st, a);
      else hipLaunchKernelGGL((norm_bwd_wave1024_kernel<RMS, true, false>), dim3(nblk), dim3(256), 0, st, a);
    } else {
      if (a.dy_bf16) hipLaunchKernelGGL((norm_bwd_wave1024_kernel<RMS, false, true>), dim3(nblk), dim3(256), 0, st, a);
      else hipLaunchKernelGGL((norm_bwd_wave1024_kernel<RMS, false, false>), dim3(nblk), dim3(256), 0, st, a);
    }
  } else if (a.D <= 1024 && a.ls && two_rows) {
    if (a.dy_bf16) hipLaunchKernelGGL((norm_bwd_wave_kernel<RMS, true, true>), dim3(nblk), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((norm_bwd_wave_kernel<RMS, true, false>), dim3(nblk), dim3(256), 0, st, a);
  } else if (a.D <= 1024 && a.ls) {
    if (a.dy_bf16) hipLaunchKernelGGL((norm_bwd_row_kernel<RMS, true, true>), dim3(nblk), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((norm_bwd_row_kernel<RMS, true, false>), dim3(nblk), dim3(256), 0, st, a);
  } else if (a.D <= 1024 && two_rows) {
    if (a.dy_bf16) hipLaunchKernelGGL((norm_bwd_wave_kernel<RMS, false, true>), dim3(nblk), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((norm_bwd_wave_kernel<RMS, false, false>), dim3(nblk), dim3(256), 0, st, a);
  } else if (a.D <= 1024) {
    if (a.dy_bf16) hipLaunchKernelGGL((norm_bwd_row_kernel<RMS, false, true>), dim3(nblk), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((norm_bwd_row_kernel<RMS, false, false>), dim3(nblk), dim3(256), 0, st, a);
  }
  else if (a.D <= 2048) hipLaunchKernelGGL((norm_bwd_kernel<8, RMS>), dim3(nblk), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((norm_bwd_kernel<16, RMS>), dim3(nblk), dim3(256), 0, st, a);
  SLX_LAUNCH_CHECK("slx_norm_bwd");
  if (a.detp) {
    float* outs[4] = {dgamma, dbeta, a.ls ? a.dls : nullptr, a.ls ? a.dlsb : nullptr};
    for (int q = 0; q < 4; ++q)
      if (outs[q] && det_reduce(a.detp + (long)q * nblk * a.D, nblk, a.D, a.D, outs[q], 1, st)) return -1000;
  }
  return 0;
}

static void fill(NormArgs& a, const slx_norm_desc* d) {
  memset(&a, 0, sizeof(a));
  a.x = d->x; a.ldx = d->ldx; a.gamma = d->gamma; a.beta = d->beta;
  a.y = (bf16*)d->y; a.ldy = d->ldy; a.mean = d->mean; a.rstd = d->rstd;
  a.rows = d->rows; a.D = d->D; a.eps = d->eps;
  a.ps = d->pixel_shuffle_grid > 0; a.G = d->pixel_shuffle_grid; a.C = d->pixel_shuffle_grid > 0 ? d->D / 4 : d->D;
  a.tok_per_img = d->tokens_per_image;
  a.y_f32 = d->y_f32;
}

extern "C" int slx_norm_fwd(const slx_norm_desc* d, slx_stream_t stream) {
  if (d->rows == 0) return 0;
  NormArgs a;
  fill(a, d);
  SLX_CHECK_ARG(d->ldx % 4 == 0 && d->ldy % 4 == 0, "slx_norm_fwd: strides must be multiples of 4");
  return d->rms ? norm_fwd<true>(a, (hipStream_t)stream) : norm_fwd<false>(a, (hipStream_t)stream);
}

extern "C" int slx_norm_bwd(const slx_norm_desc* d, const float* dy, int64_t lddy, float* dx, int64_t lddx,
                            int dx_accumulate, float* dgamma, float* dbeta, int param_accumulate, float* partial_ws,
                            slx_stream_t stream) {
  if (d->rows == 0) return 0;
  NormArgs a;
  fill(a, d);
  a.dy = dy; a.lddy = lddy; a.dx = dx; a.lddx = lddx; a.dx_accumulate = dx_accumulate;
  a.dy_bf16 = d->dy_bf16;
  SLX_CHECK_ARG(!a.dy_bf16 || lddy % 4 == 0, "slx_norm_bwd: bf16 dy needs lddy %% 4 == 0");
  a.partial = (dgamma || dbeta) ? partial_ws : nullptr;
  a.dxb = (bf16*)d->dx_bf16; a.lddxb = d->lddx_bf16;
  SLX_CHECK_ARG(!a.dxb || (!a.ps && a.lddxb % 4 == 0), "slx_norm_bwd: dx_bf16 needs plain rows and lddx_bf16 %% 4 == 0");
  a.ls = d->ls; a.lsy = (const bf16*)d->ls_y; a.ldlsy = d->ld_ls_y; a.lsg = (bf16*)d->ls_g; a.ldlsg = d->ld_ls_g;
  a.dls = d->ls_dls; a.dlsb = d->ls_dbias;
  SLX_CHECK_ARG(!a.ls || (a.lsy && a.lsg && a.dls && a.dlsb && !a.ps && d->D <= 1024 && d->D % 4 == 0 && dx_accumulate &&
                          a.ldlsy % 4 == 0 && a.ldlsg % 4 == 0),
                "slx_norm_bwd: the fused layer-scale branch needs ls_y, ls_g, ls_dls, ls_dbias, D <= 1024, plain rows, "
                "dx_accumulate and 4-element strides");

  return d->rms ? norm_bwd<true>(a, dgamma, dbeta, param_accumulate, (hipStream_t)stream)
                : norm_bwd<false>(a, dgamma, dbeta, param_accumulate, (hipStream_t)stream);
}

extern "C" int slx_norm_partial_ws_floats(int D) { return kBwdBlocks * 2 * D; }
