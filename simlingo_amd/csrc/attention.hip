// Flash attention (head_dim 64) forward + backward for gfx950, v_mfma_f32_32x32x16_bf16.
//
// Replaces flash-attn 2.7.0.post2 used inside the InternVL2-1B remote code:
//  * InternViT self-attention: non-causal, T = 1025 tokens (1024 patches + CLS), 16 heads
//    (called through internvl2_model.py:114 extract_feature);
//  * Qwen2 self-attention: causal GQA (14 q-heads / 2 kv-heads) with key-padding
//    (attention_mask = inputs_mask, simlingo_training/models/driving.py:217-223).
//
// Layout: q/k/v/o are token-major rows ([B*S, ld]) with head h occupying columns h*64..h*64+63 -
// exactly the QKV GEMM output, so no transposes are needed around the kernels.
// LSE is stored in the log2 domain: lse2 = max(s*c) + log2(sum exp2(s*c - max)), c = scale*log2(e).
//
// Forward: one workgroup = 4 waves = 128 queries of one (b, h); K/V tiles of 64 keys are
// double-buffered through LDS. Scores are computed transposed (S^T = K Q^T) so each lane owns one
// query column: the row max needs one cross-half shuffle, the P^T accumulator feeds the P.V MFMA
// directly as its B operand, and V is read with ds_read_b64_tr_b16 in the matching k order.
// Backward: one workgroup = 4 waves = 128 keys of one (b, h); loops over 64-query chunks;
// S and dP are recomputed with the key on the lane (their accumulators are the B operands of the
// dV^T and dK^T products), dS^T goes through LDS once for dQ, which is accumulated with f32
// atomics (2 x 128-B row segments per wave-instruction). For GQA each q-head's dK/dV partial is
// stored with plain 16-B stores and a finalize kernel sums the group, applies the RoPE transpose
// and converts to bf16 (row-scattered f32 atomics ran ~17x below the atomic rate here).
#include "common.h"
#include "../../include/slx.h"

namespace slx {

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Swizzled byte offset of 16-B chunk `chunk` (0..7) of row `row` in a [rows][64] bf16 tile.
// Conflict-free for ds_read_b128 row reads, ds_read_b64_tr_b16 column reads and the 16-B staging
// writes (2-way for the 8-B dS^T writes); enumeration in DESIGN.md.
__device__ __forceinline__ int sw_off(int row, int chunk) {
  return row * 128 + ((chunk ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3))) << 4);
}
__device__ __forceinline__ int sw_elem(int row, int col) { return sw_off(row, col >> 3) + ((col & 7) << 1); }

// Natural-order operand: lane l holds X[rbase + (l&31)][16kk + 8(l>>5) + j].
__device__ __forceinline__ bf16x8 row_frag(const char* lds, int rbase, int kk, int lane) {
  return *reinterpret_cast<const bf16x8*>(lds + sw_off(rbase + (lane & 31), 2 * kk + (lane >> 5)));
}
// Accumulator-order operand: lane l holds X[rbase + 8(j>>2) + 4(l>>5) + (j&3)][cbase + (l&31)].
__device__ __forceinline__ bf16x8 tr_frag(const char* lds, int rbase, int cbase, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = lane >> 5;
  const int row = rbase + 4 * h + q;
  const int col = cbase + 16 * (G & 1) + 4 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + sw_elem(row, col)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + sw_elem(row + 8, col)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}
// Registers 8s..8s+7 of an accumulator as a bf16 operand fragment (k order = accumulator order).
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& x, int s) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (bf16)x[8 * s + j];
  return v;
}

struct AttnArgs {
  const bf16* q; const bf16* k; const bf16* v; bf16* o; float* lse;
  long ldq, ldk, ldv, ldo;
  int B, S, Hq, Hkv;
  const int* seqlens;
  int causal;
  float scale;
  // backward
  const bf16* dout; long lddo;
  const float* delta;
  float* dq_acc;               // [B*S, Hq*64] f32 (zeroed)
  float* dk_acc; float* dv_acc;  // [B*S, Hq*64] f32 per-q-head partials when kv_atomic (GQA)
  bf16* dk; bf16* dv; long lddk, lddv;  // direct bf16 outputs when !kv_atomic
  int kv_atomic;
};

// Stage 64 rows x 64 cols (bf16) of a token-major matrix into a swizzled LDS tile (8 KB).
// Two 16-B chunks per thread; rows >= nrows are zero-filled.
__device__ __forceinline__ void load64(const bf16* base, long ld, int row0, int nrows, uint4 (&r)[2]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (t >> 3) + 32 * i, c = t & 7;
    r[i] = (row0 + row < nrows) ? *reinterpret_cast<const uint4*>(base + (long)(row0 + row) * ld + c * 8)
                                : make_uint4(0u, 0u, 0u, 0u);
  }
}
__device__ __forceinline__ void store64(char* lds, const uint4 (&r)[2]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (t >> 3) + 32 * i, c = t & 7;
    *reinterpret_cast<uint4*>(lds + sw_off(row, c)) = r[i];
  }
}

constexpr float LOG2E = 1.4426950408889634f;
constexpr float MASKED = -INFINITY;

__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 8192];
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int hk = h / (a.Hq / a.Hkv);
  const int S = a.S;
  const int kvlen = a.seqlens ? min(a.seqlens[b], S) : S;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hl = lane >> 5;
  const int q0 = qb * 128 + w * 32;
  const int myq = q0 + (lane & 31);
  const bool active = q0 < S;
  const float c = a.scale * LOG2E;

  const bf16* kbase = a.k + (long)b * S * a.ldk + hk * 64;
  const bf16* vbase = a.v + (long)b * S * a.ldv + hk * 64;

  bf16x8 qf[4];
  {
    const bf16* qrow = a.q + ((long)b * S + min(myq, S - 1)) * a.ldq + h * 64;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      bf16x8 z;
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
      qf[kk] = myq < S ? *reinterpret_cast<const bf16x8*>(qrow + 16 * kk + 8 * hl) : z;
    }
  }
  int kend = kvlen;
  if (a.causal) kend = min(kend, qb * 128 + 128);
  const int nt = (kend + 63) / 64;

  f32x16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
  float m = -1e30f, l = 0.f;

  uint4 rk[2], rv[2];
  load64(kbase, a.ldk, 0, S, rk);
  load64(vbase, a.ldv, 0, S, rv);
  store64(smem, rk);
  store64(smem + 8192, rv);
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const char* Kl = smem + (t & 1) * 16384;
    const char* Vl = Kl + 8192;
    if (t + 1 < nt) {
      load64(kbase, a.ldk, (t + 1) * 64, S, rk);
      load64(vbase, a.ldv, (t + 1) * 64, S, rv);
    }
    if (active) {
      f32x16 s[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) s[kb] = mfma32(row_frag(Kl, kb * 32, kk, lane), qf[kk], s[kb]);
      }
      float mx = -1e30f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = t * 64 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          float x = s[kb][r] * c;
          if (key >= kvlen || (a.causal && key > myq)) x = MASKED;
          s[kb][r] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx);
      const float alpha = exp2f(m - mnew);
      m = mnew;
      float ps = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = exp2f(s[kb][r] - m);
          s[kb][r] = p;
          ps += p;
        }
      l = l * alpha + ps;
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pb = acc_frag(s[kb], st);
          o0 = mfma32(tr_frag(Vl, kb * 32 + 16 * st, 0, lane), pb, o0);
          o1 = mfma32(tr_frag(Vl, kb * 32 + 16 * st, 32, lane), pb, o1);
        }
    }
    if (t + 1 < nt) {
      char* nx = smem + ((t + 1) & 1) * 16384;
      store64(nx, rk);
      store64(nx + 8192, rv);
    }
    __syncthreads();
  }
  if (!active || myq >= S) return;
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = 1.0f / lt;
  bf16* orow = a.o + ((long)b * S + myq) * a.ldo + h * 64;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hl;
    bf16x4 v0, v1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v0[e] = (bf16)(o0[4 * g + e] * inv);
      v1[e] = (bf16)(o1[4 * g + e] * inv);
    }
    *reinterpret_cast<bf16x4*>(orow + d) = v0;
    *reinterpret_cast<bf16x4*>(orow + 32 + d) = v1;
  }
  if (hl == 0 && a.lse) a.lse[((long)b * a.Hq + h) * S + myq] = m + __log2f(lt);
}

// delta[b,h,q] = sum_d dO[q,d] * O[q,d]   (one thread per (token, head))
__global__ void attn_bwd_delta_kernel(AttnArgs a) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)a.B * a.S * a.Hq;
  if (idx >= total) return;
  const int h = idx % a.Hq;
  const long tok = idx / a.Hq;
  const int b = tok / a.S, s = tok % a.S;
  const bf16* o = a.o + tok * a.ldo + h * 64;
  const bf16* d = a.dout + tok * a.lddo + h * 64;
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(o + 8 * i);
    const bf16x8 y = *reinterpret_cast<const bf16x8*>(d + 8 * i);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += (float)x[j] * (float)y[j];
  }
  const_cast<float*>(a.delta)[((long)b * a.Hq + h) * a.S + s] = acc;
}

__global__ __launch_bounds__(256, 2) void attn_bwd_kernel(AttnArgs a) {
  // LDS: K tile [128][64] 16 KB | Q chunk x2 (8 KB each) | dO chunk x2 | dS^T [128][64] 16 KB | lse,delta x2
  __shared__ __attribute__((aligned(16))) char smem[16384 + 2 * 8192 + 2 * 8192 + 16384 + 2 * 2 * 64 * 4];
  char* Kt = smem;
  char* Qc = smem + 16384;
  char* Dc = Qc + 2 * 8192;
  char* dSt = Dc + 2 * 8192;
  float* LD = reinterpret_cast<float*>(dSt + 16384);  // [buf][lse 64 | delta 64]

  const int kblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int hk = h / (a.Hq / a.Hkv);
  const int S = a.S;
  const int kvlen = a.seqlens ? min(a.seqlens[b], S) : S;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hl = lane >> 5;
  const int k0 = kblk * 128;
  const int mykey = k0 + 32 * w + (lane & 31);
  const float c = a.scale * LOG2E;

  const bf16* kbase = a.k + (long)b * S * a.ldk + hk * 64;
  const bf16* vbase = a.v + (long)b * S * a.ldv + hk * 64;
  const bf16* qbase = a.q + (long)b * S * a.ldq + h * 64;
  const bf16* dobase = a.dout + (long)b * S * a.lddo + h * 64;
  const float* lsebase = a.lse + ((long)b * a.Hq + h) * S;
  const float* dlbase = a.delta + ((long)b * a.Hq + h) * S;

  // K tile (128 keys) for the dQ product
  {
    uint4 r[2];
    load64(kbase, a.ldk, k0, S, r);
    store64(Kt, r);
    load64(kbase, a.ldk, k0 + 64, S, r);
    store64(Kt + 8192, r);
  }
  // K and V fragments of this wave's 32 keys (B operands of S = Q K^T and dP = dO V^T)
  bf16x8 kf[4], vf[4];
  {
    const int kr = min(mykey, S - 1);
    const bf16* kp = kbase + (long)kr * a.ldk;
    const bf16* vp = vbase + (long)kr * a.ldv;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      kf[kk] = *reinterpret_cast<const bf16x8*>(kp + 16 * kk + 8 * hl);
      vf[kk] = *reinterpret_cast<const bf16x8*>(vp + 16 * kk + 8 * hl);
    }
  }
  f32x16 dk0, dk1, dv0, dv1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { dk0[r] = dk1[r] = dv0[r] = dv1[r] = 0.f; }

  const int qstart = a.causal ? (k0 / 64) * 64 : 0;
  const int nch = qstart < S ? (S - qstart + 63) / 64 : 0;

  auto stage = [&](int ci, int buf, uint4 (&rq)[2], uint4 (&rd)[2], float& ld) {
    const int qc = qstart + ci * 64;
    load64(qbase, a.ldq, qc, S, rq);
    load64(dobase, a.lddo, qc, S, rd);
    if (tid < 128) {
      const int qi = qc + (tid & 63);
      ld = qi < S ? (tid < 64 ? lsebase[qi] : dlbase[qi]) : 0.f;
    }
  };
  auto commit = [&](int buf, const uint4 (&rq)[2], const uint4 (&rd)[2], float ld) {
    store64(Qc + buf * 8192, rq);
    store64(Dc + buf * 8192, rd);
    if (tid < 128) LD[buf * 128 + tid] = ld;
  };

  uint4 rq[2], rd[2];
  float ldv = 0.f;
  if (nch > 0) {
    stage(0, 0, rq, rd, ldv);
    commit(0, rq, rd, ldv);
  }
  __syncthreads();

  for (int ci = 0; ci < nch; ++ci) {
    const int buf = ci & 1;
    const int qc = qstart + ci * 64;
    const char* Ql = Qc + buf * 8192;
    const char* Dl = Dc + buf * 8192;
    const float* lse_l = LD + buf * 128;
    const float* del_l = lse_l + 64;
    if (ci + 1 < nch) stage(ci + 1, buf ^ 1, rq, rd, ldv);

#pragma unroll
    for (int qa = 0; qa < 2; ++qa) {
      f32x16 sp, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { sp[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        sp = mfma32(row_frag(Ql, qa * 32, kk, lane), kf[kk], sp);
        dp = mfma32(row_frag(Dl, qa * 32, kk, lane), vf[kk], dp);
      }
      // P and dS with the query on the accumulator rows
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ql = qa * 32 + 8 * g + 4 * hl;  // local query of register 4g
        const f32x4 L4 = *reinterpret_cast<const f32x4*>(lse_l + ql);
        const f32x4 D4 = *reinterpret_cast<const f32x4*>(del_l + ql);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          const int q = qc + ql + e;
          const bool ok = q < S && mykey < kvlen && !(a.causal && mykey > q);
          const float p = ok ? exp2f(sp[r] * c - L4[e]) : 0.f;
          sp[r] = p;
          dp[r] = p * (dp[r] - D4[e]);
        }
      }
      // dV^T += dO^T P ; dK^T += Q^T dS
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 pb = acc_frag(sp, st);
        const bf16x8 sb = acc_frag(dp, st);
        dv0 = mfma32(tr_frag(Dl, qa * 32 + 16 * st, 0, lane), pb, dv0);
        dv1 = mfma32(tr_frag(Dl, qa * 32 + 16 * st, 32, lane), pb, dv1);
        dk0 = mfma32(tr_frag(Ql, qa * 32 + 16 * st, 0, lane), sb, dk0);
        dk1 = mfma32(tr_frag(Ql, qa * 32 + 16 * st, 32, lane), sb, dk1);
      }
      // dS^T image row = local key, columns = local query
      const int krow = 32 * w + (lane & 31);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (bf16)dp[4 * g + e];
        *reinterpret_cast<bf16x4*>(dSt + sw_elem(krow, qa * 32 + 8 * g + 4 * hl)) = v;
      }
    }
    __syncthreads();
    {  // dQ[q][d] = sum over the block's 128 keys of dS[q][key] K[key][d]; wave -> (q half, d half)
      const int qa = w >> 1, db = w & 1;
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) acc = mfma32(tr_frag(dSt, 16 * kk, 32 * qa, lane), tr_frag(Kt, 16 * kk, 32 * db, lane), acc);
      const int d = 32 * db + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = qc + 32 * qa + (r & 3) + 8 * (r >> 2) + 4 * hl;
        if (q < S) atomicAdd(a.dq_acc + ((long)b * S + q) * (a.Hq * 64) + h * 64 + d, acc[r] * a.scale);
      }
    }
    if (ci + 1 < nch) commit(buf ^ 1, rq, rd, ldv);
    __syncthreads();
  }

  if (mykey >= S) return;
  // dK^T / dV^T accumulators: column = key (lane), rows = d
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hl;
    if (a.kv_atomic) {
      // GQA: per-q-head partials with plain 16-B stores; slx_attn_bwd's finalize sums the group
      float* kp = a.dk_acc + ((long)b * S + mykey) * (a.Hq * 64) + h * 64;
      float* vp = a.dv_acc + ((long)b * S + mykey) * (a.Hq * 64) + h * 64;
      *reinterpret_cast<float4*>(kp + d) = make_float4(dk0[4 * g] * a.scale, dk0[4 * g + 1] * a.scale, dk0[4 * g + 2] * a.scale, dk0[4 * g + 3] * a.scale);
      *reinterpret_cast<float4*>(kp + 32 + d) = make_float4(dk1[4 * g] * a.scale, dk1[4 * g + 1] * a.scale, dk1[4 * g + 2] * a.scale, dk1[4 * g + 3] * a.scale);
      *reinterpret_cast<float4*>(vp + d) = make_float4(dv0[4 * g], dv0[4 * g + 1], dv0[4 * g + 2], dv0[4 * g + 3]);
      *reinterpret_cast<float4*>(vp + 32 + d) = make_float4(dv1[4 * g], dv1[4 * g + 1], dv1[4 * g + 2], dv1[4 * g + 3]);
    } else {
      bf16* kp = a.dk + ((long)b * S + mykey) * a.lddk + hk * 64;
      bf16* vp = a.dv + ((long)b * S + mykey) * a.lddv + hk * 64;
      bf16x4 k0v, k1v, v0v, v1v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        k0v[e] = (bf16)(dk0[4 * g + e] * a.scale);
        k1v[e] = (bf16)(dk1[4 * g + e] * a.scale);
        v0v[e] = (bf16)dv0[4 * g + e];
        v1v[e] = (bf16)dv1[4 * g + e];
      }
      *reinterpret_cast<bf16x4*>(kp + d) = k0v;
      *reinterpret_cast<bf16x4*>(kp + 32 + d) = k1v;
      *reinterpret_cast<bf16x4*>(vp + d) = v0v;
      *reinterpret_cast<bf16x4*>(vp + 32 + d) = v1v;
    }
  }
}

// Rotary embedding (HF rotate_half convention, Qwen2): for i < 32
//   y[i] = x[i] cos_i - x[i+32] sin_i ;  y[i+32] = x[i+32] cos_i + x[i] sin_i
// with cos_i/sin_i of (pos * theta^(-2i/64)), pos = token index within its sequence.
// inverse != 0 applies the transpose (backward).
__device__ __forceinline__ void rope_pair(float& x0, float& x1, float cs, float sn, bool inverse) {
  const float a = x0, b = x1;
  if (!inverse) { x0 = a * cs - b * sn; x1 = b * cs + a * sn; }
  else { x0 = a * cs + b * sn; x1 = b * cs - a * sn; }
}

struct RopeArgs {
  bf16* x; long ldx; int ntok, S, nheads; const float* cos; const float* sin; int inverse;
  const float* src_f32; long ldsrc;  // optional f32 source (finalize: dq/dk accumulators)
};

// One thread per (token, head, i<32 pair-group of 4): 8 pairs per thread -> 256 threads per row
__global__ void rope_kernel(RopeArgs r) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)r.ntok * r.nheads * 4;
  if (idx >= total) return;
  const int part = idx & 3;
  const long th = idx >> 2;
  const int hh = th % r.nheads;
  const long tok = th / r.nheads;
  const int pos = tok % r.S;
  bf16* x = r.x + tok * r.ldx + hh * 64;
  const int i0 = part * 8;
  float v0[8], v1[8];
  if (r.src_f32) {
    const float* s = r.src_f32 + tok * r.ldsrc + hh * 64;
#pragma unroll
    for (int j = 0; j < 8; ++j) { v0[j] = s[i0 + j]; v1[j] = s[32 + i0 + j]; }
  } else {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(x + i0);
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(x + 32 + i0);
#pragma unroll
    for (int j = 0; j < 8; ++j) { v0[j] = (float)a[j]; v1[j] = (float)b[j]; }
  }
  bf16x8 oa, ob;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float cs = r.cos[(long)pos * 32 + i0 + j], sn = r.sin[(long)pos * 32 + i0 + j];
    rope_pair(v0[j], v1[j], cs, sn, r.inverse != 0);
    oa[j] = (bf16)v0[j];
    ob[j] = (bf16)v1[j];
  }
  *reinterpret_cast<bf16x8*>(x + i0) = oa;
  *reinterpret_cast<bf16x8*>(x + 32 + i0) = ob;
}

// GQA finalize: dst[t, hk, :] = sum_{j<G} src[t, hk*G + j, :] (f32 per-q-head partials, row stride
// Hq*64) -> optional RoPE^T -> bf16. One thread per (token, kv head, quarter of the pairs).
__global__ void gqa_reduce_kernel(const float* src, int Hq, int Hkv, bf16* dst, long ldd, long ntok, int S, const float* cos,
                                  const float* sin) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= ntok * Hkv * 4) return;
  const int part = idx & 3;
  const long th = idx >> 2;
  const int hk = th % Hkv;
  const long tok = th / Hkv;
  const int G = Hq / Hkv, i0 = part * 8;
  float v0[8], v1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { v0[j] = 0.f; v1[j] = 0.f; }
  for (int g = 0; g < G; ++g) {
    const float* sp = src + tok * (long)Hq * 64 + (hk * G + g) * 64;
#pragma unroll
    for (int j = 0; j < 8; j += 4) {
      const float4 a = *reinterpret_cast<const float4*>(sp + i0 + j);
      const float4 c = *reinterpret_cast<const float4*>(sp + 32 + i0 + j);
      v0[j] += a.x; v0[j + 1] += a.y; v0[j + 2] += a.z; v0[j + 3] += a.w;
      v1[j] += c.x; v1[j + 1] += c.y; v1[j + 2] += c.z; v1[j + 3] += c.w;
    }
  }
  bf16x8 oa, ob;
  const int pos = tok % S;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (cos) rope_pair(v0[j], v1[j], cos[(long)pos * 32 + i0 + j], sin[(long)pos * 32 + i0 + j], true);
    oa[j] = (bf16)v0[j];
    ob[j] = (bf16)v1[j];
  }
  bf16* dp = dst + tok * ldd + hk * 64;
  *reinterpret_cast<bf16x8*>(dp + i0) = oa;
  *reinterpret_cast<bf16x8*>(dp + 32 + i0) = ob;
}

// f32 [ntok, ncols] -> bf16 rows (ld) (no rope)
__global__ void f32_to_bf16_rows_kernel(const float* src, long lds, bf16* dst, long ldd, long ntok, int ncols) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = ncols / 8;
  if (idx >= ntok * per) return;
  const long t = idx / per;
  const int c = (idx % per) * 8;
  const float* s = src + t * lds + c;
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (bf16)s[j];
  *reinterpret_cast<bf16x8*>(dst + t * ldd + c) = v;
}

}  // namespace slx

using namespace slx;

static int fill_common(AttnArgs& a, const slx_attn_desc* d) {
  SLX_CHECK_ARG(d->head_dim == 64, "slx_attn: only head_dim 64 is supported (got %d)", d->head_dim);
  SLX_CHECK_ARG(d->Hq > 0 && d->Hkv > 0 && d->Hq % d->Hkv == 0, "slx_attn: Hq must be a multiple of Hkv");
  SLX_CHECK_ARG(d->ldq % 8 == 0 && d->ldk % 8 == 0 && d->ldv % 8 == 0 && d->ldo % 8 == 0, "slx_attn: row strides must be multiples of 8");
  memset(&a, 0, sizeof(a));
  a.q = (const bf16*)d->q; a.k = (const bf16*)d->k; a.v = (const bf16*)d->v; a.o = (bf16*)d->o;
  a.lse = d->lse;
  a.ldq = d->ldq; a.ldk = d->ldk; a.ldv = d->ldv; a.ldo = d->ldo;
  a.B = d->B; a.S = d->S; a.Hq = d->Hq; a.Hkv = d->Hkv;
  a.seqlens = d->seqlens; a.causal = d->causal; a.scale = d->scale;
  return 0;
}

extern "C" int slx_attn_fwd(const slx_attn_desc* d, slx_stream_t stream) {
  AttnArgs a;
  int rc = fill_common(a, d);
  if (rc) return rc;
  if (a.B == 0 || a.S == 0) return 0;
  dim3 grid((a.S + 127) / 128, a.Hq, a.B);
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  SLX_LAUNCH_CHECK("slx_attn_fwd");
  return 0;
}

extern "C" int slx_attn_bwd(const slx_attn_desc* d, const slx_attn_bwd_desc* g, slx_stream_t stream) {
  AttnArgs a;
  int rc = fill_common(a, d);
  if (rc) return rc;
  if (a.B == 0 || a.S == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  a.dout = (const bf16*)g->dout; a.lddo = g->lddo;
  a.delta = g->delta_ws;
  a.dq_acc = g->dq_acc; a.dk_acc = g->dk_acc; a.dv_acc = g->dv_acc;
  a.kv_atomic = d->Hq != d->Hkv ? 1 : 0;
  SLX_CHECK_ARG(a.lse && a.delta && a.dq_acc, "slx_attn_bwd: lse, delta_ws and dq_acc are required");
  SLX_CHECK_ARG(!a.kv_atomic || (a.dk_acc && a.dv_acc), "slx_attn_bwd: GQA needs dk_acc/dv_acc workspaces");
  const long ntok = (long)a.B * a.S;
  hipMemsetAsync(a.dq_acc, 0, ntok * a.Hq * 64 * sizeof(float), st);
  if (a.kv_atomic) {
    // per-q-head partials, fully overwritten by the kernel (no memset)
  } else {
    a.dk = (bf16*)g->dk; a.dv = (bf16*)g->dv; a.lddk = g->lddk; a.lddv = g->lddv;
  }
  {
    const long total = ntok * a.Hq;
    hipLaunchKernelGGL(attn_bwd_delta_kernel, dim3((total + 255) / 256), dim3(256), 0, st, a);
    SLX_LAUNCH_CHECK("slx_attn_bwd(delta)");
  }
  dim3 grid((a.S + 127) / 128, a.Hq, a.B);
  hipLaunchKernelGGL(attn_bwd_kernel, grid, dim3(256), 0, st, a);
  SLX_LAUNCH_CHECK("slx_attn_bwd");
  // finalize: dq (and dk/dv for GQA) -> bf16, with the RoPE transpose when tables are given
  RopeArgs r;
  memset(&r, 0, sizeof(r));
  r.ntok = ntok; r.S = a.S; r.cos = g->rope_cos; r.sin = g->rope_sin; r.inverse = 1;
  auto conv = [&](const float* src, int heads, bf16* dst, long ld, bool rope) -> int {
    if (rope && r.cos) {
      r.x = dst; r.ldx = ld; r.nheads = heads; r.src_f32 = src; r.ldsrc = (long)heads * 64;
      const long total = ntok * heads * 4;
      hipLaunchKernelGGL(rope_kernel, dim3((total + 255) / 256), dim3(256), 0, st, r);
    } else {
      const long total = ntok * heads * 8;
      hipLaunchKernelGGL(f32_to_bf16_rows_kernel, dim3((total + 255) / 256), dim3(256), 0, st, src, (long)heads * 64, dst, ld, ntok, heads * 64);
    }
    SLX_LAUNCH_CHECK("slx_attn_bwd(finalize)");
    return 0;
  };
  if ((rc = conv(a.dq_acc, a.Hq, (bf16*)g->dq, g->lddq, true))) return rc;
  if (a.kv_atomic) {
    const long total = ntok * a.Hkv * 4;
    hipLaunchKernelGGL(gqa_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, a.dk_acc, a.Hq, a.Hkv, (bf16*)g->dk,
                       (long)g->lddk, ntok, a.S, r.cos, r.sin);
    hipLaunchKernelGGL(gqa_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, a.dv_acc, a.Hq, a.Hkv, (bf16*)g->dv,
                       (long)g->lddv, ntok, a.S, (const float*)nullptr, (const float*)nullptr);
    SLX_LAUNCH_CHECK("slx_attn_bwd(gqa reduce)");
  } else if (r.cos) {
    // direct bf16 dK still needs the RoPE transpose (in place)
    r.x = (bf16*)g->dk; r.ldx = g->lddk; r.nheads = a.Hkv; r.src_f32 = nullptr;
    const long total = ntok * a.Hkv * 4;
    hipLaunchKernelGGL(rope_kernel, dim3((total + 255) / 256), dim3(256), 0, st, r);
    SLX_LAUNCH_CHECK("slx_attn_bwd(rope dk)");
  }
  return 0;
}

extern "C" int slx_rope(void* x, int64_t ldx, int64_t ntok, int S, int nheads, const float* cos_tab,
                        const float* sin_tab, int inverse, slx_stream_t stream) {
  SLX_CHECK_ARG(ldx % 8 == 0, "slx_rope: ldx must be a multiple of 8");
  if (ntok == 0 || nheads == 0) return 0;
  RopeArgs r;
  memset(&r, 0, sizeof(r));
  r.x = (bf16*)x; r.ldx = ldx; r.ntok = ntok; r.S = S; r.nheads = nheads;
  r.cos = cos_tab; r.sin = sin_tab; r.inverse = inverse;
  const long total = ntok * nheads * 4;
  hipLaunchKernelGGL(rope_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, r);
  SLX_LAUNCH_CHECK("slx_rope");
  return 0;
}
