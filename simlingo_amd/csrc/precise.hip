// fp32 parity mode of the training step (SURVEY.md §7 hard part 2, §8d parity gates): forward and backward.
//
// The product path is the bf16 MFMA build; its kernels are checked one by one against fp32 references of the
// same bf16 inputs, and the whole step against the fp32 oracle at a bf16 tolerance. To pin the step itself at
// the north-star tolerance (waypoint L2 <= 1e-4 m, LM cross-entropy <= 1e-4; BASELINE.json north_star),
// VLAEngine / BaseEngine(precise=True) run the SAME launch sequence with every activation and weight in f32:
// the kernels that already take f32 (norms with y_f32 / f32 dy and dx, ViT embeddings, gathers / scatters, heads,
// losses, f32 column sums) run unchanged, and the entry points below are the f32 twins of the ones whose operands
// are bf16-only (GEMM with the forward and activation-gradient epilogues, attention forward and backward, RoPE,
// SwiGLU forward and backward, im2col, token assembly, LLaVA-NeXT merge, CE gradient, embedding gradient, the
// layer-scale branch products). They are plain f32-FMA kernels (exact products, f32 sums): parity mode is compared
// with the oracle, never timed.
#include <cmath>

#include "common.h"
#include "../../include/slx.h"

namespace slx {

static inline dim3 pg1(long n, int bs = 256) { return dim3((unsigned)((n + bs - 1) / bs)); }

// ---- GEMM: C = alpha * op(A) op(B) (+ epilogue); 64 x 64 tile per 256 threads, 4 x 4 outputs per thread ----
struct GemmF32Args {
  const float* A;
  const float* B;
  float* C;
  long lda, ldb, ldc, sA, sB, sC;
  int M, N, K, ak, bk;
  float alpha;
  const float* bias;
  const float* ls;
  float* aux_out;
  long ldaux_out;
  const float* resid;
  long ldr;
  int accumulate;
  const float* aux;   // GELU_BWD / QGELU_BWD: the saved pre-activation
  long ldaux;
};

template <int EPI>
__device__ __forceinline__ void epi_f32(const GemmF32Args& p, float* C, int m, int n, float v) {
  v *= p.alpha;
  if (p.bias) v += p.bias[n];
  const long ci = (long)m * p.ldc + n;
  if constexpr (EPI == SLX_EPI_STORE) {
    if (p.accumulate) v += C[ci];
    C[ci] = v;
  } else if constexpr (EPI == SLX_EPI_GELU_BWD || EPI == SLX_EPI_QGELU_BWD) {  // dX = dY W times act'(pre)
    const float h = p.aux[(long)m * p.ldaux + n];
    float g;
    if constexpr (EPI == SLX_EPI_GELU_BWD) {
      g = gelu_erf_grad(h);
    } else {
      const float sg = 1.0f / (1.0f + expf(-1.702f * h));
      g = sg + 1.702f * h * sg * (1.0f - sg);
    }
    C[ci] = v * g;
  } else if constexpr (EPI == SLX_EPI_RESID_LS) {
    if (p.aux_out) p.aux_out[(long)m * p.ldaux_out + n] = v;
    C[ci] = p.resid[(long)m * p.ldr + n] + p.ls[n] * v;
  } else {  // GELU (erf) / quick_gelu: pre-activation to aux_out, activation to C
    if (p.aux_out) p.aux_out[(long)m * p.ldaux_out + n] = v;
    C[ci] = EPI == SLX_EPI_GELU ? gelu_erf(v) : v / (1.0f + expf(-1.702f * v));
  }
}

// A is [M][K] (ak) or [K][M]; B is [N][K] (bk) or [K][N]. Thread (ty, tx) owns rows ty + 16i, columns tx + 16j.
template <int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmF32Args p) {
  __shared__ float As[16][65], Bs[16][65];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const long z = blockIdx.z;
  const float* A = p.A + z * p.sA;
  const float* B = p.B + z * p.sB;
  float* C = p.C + z * p.sC;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int k0 = 0; k0 < p.K; k0 += 16) {
    for (int e = threadIdx.x; e < 1024; e += 256) {
      const int ka = p.ak ? (e & 15) : (e >> 6), ra = p.ak ? (e >> 4) : (e & 63);
      const int gm = m0 + ra, gka = k0 + ka;
      As[ka][ra] = (gm < p.M && gka < p.K) ? A[p.ak ? (long)gm * p.lda + gka : (long)gka * p.lda + gm] : 0.f;
      const int kb = p.bk ? (e & 15) : (e >> 6), cb = p.bk ? (e >> 4) : (e & 63);
      const int gn = n0 + cb, gkb = k0 + kb;
      Bs[kb][cb] = (gn < p.N && gkb < p.K) ? B[p.bk ? (long)gn * p.ldb + gkb : (long)gkb * p.ldb + gn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + ty + 16 * i, n = n0 + tx + 16 * j;
      if (m < p.M && n < p.N) epi_f32<EPI>(p, C, m, n, acc[i][j]);
    }
}

// ---- attention forward: one 256-thread block per (query, head, batch); the scores of every visible key in
// LDS, exact softmax, O = P V. Same masking as attn_fwd_kernel (causal, key padding via seqlens); LSE stored
// in the log2 domain like the bf16 kernel.
struct AttnF32Args {
  const float* q;
  const float* k;
  const float* v;
  float* o;
  float* lse;
  long ldq, ldk, ldv, ldo;
  int B, S, Hq, Hkv, causal;
  const int* seqlens;
  float scale;
};

__device__ __forceinline__ float block_max256(float v, float* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = warp_max(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
}

__global__ __launch_bounds__(256) void attn_fwd_f32_kernel(AttnF32Args a) {
  extern __shared__ float sm[];
  float* qs = sm;          // [64]
  float* po = sm + 64;     // [4][64] partial outputs
  float* red = sm + 320;   // [16]
  float* sc = sm + 336;    // [S]
  const int qi = blockIdx.x, h = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
  const int hk = h / (a.Hq / a.Hkv);
  const int kvlen = a.seqlens ? min(a.seqlens[b], a.S) : a.S;
  const int kend = a.causal ? min(kvlen, qi + 1) : kvlen;
  if (tid < 64) qs[tid] = a.q[((long)b * a.S + qi) * a.ldq + h * 64 + tid];
  __syncthreads();
  float mx = -INFINITY;
  for (int k = tid; k < kend; k += 256) {
    const float* kr = a.k + ((long)b * a.S + k) * a.ldk + hk * 64;
    float s = 0.f;
    for (int d = 0; d < 64; ++d) s = fmaf(qs[d], kr[d], s);
    s *= a.scale;
    sc[k] = s;
    mx = fmaxf(mx, s);
  }
  mx = block_max256(mx, red);
  float l = 0.f;
  for (int k = tid; k < kend; k += 256) {
    const float p = expf(sc[k] - mx);
    sc[k] = p;
    l += p;
  }
  l = block_sum(l, red);
  __syncthreads();
  const int dd = tid & 63, part = tid >> 6;
  float o = 0.f;
  for (int k = part; k < kend; k += 4) o = fmaf(sc[k], a.v[((long)b * a.S + k) * a.ldv + hk * 64 + dd], o);
  po[part * 64 + dd] = o;
  __syncthreads();
  if (tid < 64) {
    const float s = (po[tid] + po[64 + tid]) + (po[128 + tid] + po[192 + tid]);
    a.o[((long)b * a.S + qi) * a.ldo + h * 64 + tid] = kend > 0 ? s / l : 0.f;
  }
  if (tid == 0 && a.lse)
    a.lse[((long)b * a.Hq + h) * a.S + qi] = kend > 0 ? mx * 1.4426950408889634f + log2f(l) : -INFINITY;
}

// ---- elementwise twins --------------------------------------------------------------------------------
// RoPE, rotate_half pairs (i, i+32) of every head slot (rope_kernel)
__global__ void rope_f32_kernel(float* x, long ldx, long ntok, int S, int nheads, const float* cs, const float* sn,
                                int inverse) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= ntok * nheads * 32) return;
  const int i = idx & 31;
  const long th = idx >> 5;
  const int hh = th % nheads;
  const long tok = th / nheads;
  const int pos = tok % S;
  float* p = x + tok * ldx + hh * 64;
  const float c = cs[(long)pos * 32 + i], s = sn[(long)pos * 32 + i];
  const float a0 = p[i], a1 = p[32 + i];
  if (!inverse) {
    p[i] = a0 * c - a1 * s;
    p[32 + i] = a1 * c + a0 * s;
  } else {
    p[i] = a0 * c + a1 * s;
    p[32 + i] = a1 * c - a0 * s;
  }
}

// out[m, f] = silu(gu[m, f]) * gu[m, F + f]
__global__ void swiglu_f32_kernel(const float* gu, long ldgu, float* out, long ldo, long M, int F) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * F) return;
  const long m = idx / F;
  const int f = idx % F;
  const float g = gu[m * ldgu + f];
  out[m * ldo + f] = g / (1.0f + expf(-g)) * gu[m * ldgu + F + f];
}

// Conv2d(3, D, k=P, s=P) as im2col (im2col_kernel), f32 columns, zero for k >= 3P^2
__global__ void im2col_f32_kernel(const float* pix, int N, int H, int W, int P, int kpad, float* out) {
  const int gw = W / P, np = gw * (H / P);
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * np * kpad) return;
  const int k = idx % kpad;
  const long rowi = idx / kpad;
  const int n = rowi / np, p = rowi % np, py = p / gw, px = p % gw;
  float x = 0.f;
  if (k < 3 * P * P) {
    const int c = k / (P * P), r = k % (P * P), ky = r / P, kx = r % P;
    x = pix[(((long)n * 3 + c) * H + py * P + ky) * W + px * P + kx];
  }
  out[idx] = x;
}

// LLM input assembly (assemble_kernel) with an f32 embedding table and f32 image rows
__global__ void assemble_f32_kernel(const int* code, long n, int D, const float* embed, int V, const float* img,
                                    const float* wp, const float* query, float* out) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * D) return;
  const long i = idx / D;
  const int c = idx % D;
  const int cd = code[i];
  const int kind = (cd >> 28) & 0xF, ix = cd & 0x0FFFFFFF;
  const float* src = kind == 0 ? embed + (long)min(ix, V - 1) * D
                   : kind == 1 ? img + (long)ix * D
                   : kind == 2 ? wp + (long)ix * D : query + (long)ix * D;
  out[idx] = src[c];
}

// LLaVA-NeXT spatial merge (llava_merge_fwd_kernel): unpad window -> avg_pool2d(pool) -> image_newline column
__global__ void llava_merge_f32_kernel(const float* src, int C, int nph, int npw, int g, int r0, int hu, int c0,
                                       int wu, int pool, long n_img, const float* newline, float* out) {
  const int ho = hu / pool, wo = wu / pool, T = ho * (wo + 1);
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_img * T * C) return;
  const int c = idx % C;
  const long tok = idx / C;
  const long img = tok / T;
  const int t = tok % T, i = t / (wo + 1), j = t % (wo + 1);
  if (j == wo) {
    out[idx] = newline[c];
    return;
  }
  float acc = 0.f;
  for (int a = 0; a < pool; ++a)
    for (int b = 0; b < pool; ++b) {
      const int hh = r0 + i * pool + a, ww = c0 + j * pool + b;
      const long r = (img * nph * npw + (hh / g) * npw + ww / g) * (long)(g * g) + (hh % g) * g + (ww % g);
      acc += src[r * C + c];
    }
  out[idx] = acc * (1.0f / (pool * pool));
}


// ---- backward twins ----------------------------------------------------------------------------------
// attention backward, restated from the softmax derivative with the forward's saved LSE (log2 domain):
// P = exp2(S*log2e - lse), dP = dO V^T, delta = rowsum(dO * O), dS = P (dP - delta), dQ = scale dS K, dK = scale dS^T Q,
// dV = P^T dO. Same visibility as attn_fwd_f32_kernel (causal, key padding via seqlens; every query row computed).
struct AttnBwdF32Args {
  const float* q; const float* k; const float* v; const float* o; const float* lse; const float* dout;
  float* dq; float* dk; float* dv; float* delta;
  long ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv;
  int B, S, Hq, Hkv, causal;
  const int* seqlens;
  float scale;
};

__global__ void attn_delta_f32_kernel(AttnBwdF32Args a) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (b, h, q)
  if (idx >= (long)a.B * a.Hq * a.S) return;
  const int qi = idx % a.S;
  const long bh = idx / a.S;
  const int h = bh % a.Hq, b = bh / a.Hq;
  const float* o = a.o + ((long)b * a.S + qi) * a.ldo + h * 64;
  const float* g = a.dout + ((long)b * a.S + qi) * a.lddo + h * 64;
  float s = 0.f;
  for (int d = 0; d < 64; ++d) s = fmaf(o[d], g[d], s);
  a.delta[idx] = s;
}

__device__ __forceinline__ float attn_prob_f32(const AttnBwdF32Args& a, const float* qrow, const float* krow,
                                               float lse2) {
  float s = 0.f;
  for (int d = 0; d < 64; ++d) s = fmaf(qrow[d], krow[d], s);
  return exp2f(s * a.scale * 1.4426950408889634f - lse2);
}

// one 256-thread block per (query, head, batch)
__global__ __launch_bounds__(256) void attn_dq_f32_kernel(AttnBwdF32Args a) {
  extern __shared__ float sm[];
  float* qs = sm;          // [64]
  float* gs = sm + 64;     // [64] dO row
  float* po = sm + 128;    // [4][64]
  float* sc = sm + 384;    // [S] dS
  const int qi = blockIdx.x, h = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
  const int hk = h / (a.Hq / a.Hkv);
  const int kvlen = a.seqlens ? min(a.seqlens[b], a.S) : a.S;
  const int kend = a.causal ? min(kvlen, qi + 1) : kvlen;
  const long row = (long)b * a.S + qi;
  if (tid < 64) {
    qs[tid] = a.q[row * a.ldq + h * 64 + tid];
    gs[tid] = a.dout[row * a.lddo + h * 64 + tid];
  }
  __syncthreads();
  const long bhq = ((long)b * a.Hq + h) * a.S + qi;
  const float lse2 = a.lse[bhq], dl = a.delta[bhq];
  for (int k = tid; k < kend; k += 256) {
    const long kr = (long)b * a.S + k;
    const float p = attn_prob_f32(a, qs, a.k + kr * a.ldk + hk * 64, lse2);
    const float* vr = a.v + kr * a.ldv + hk * 64;
    float dp = 0.f;
    for (int d = 0; d < 64; ++d) dp = fmaf(gs[d], vr[d], dp);
    sc[k] = p * (dp - dl);
  }
  __syncthreads();
  const int dd = tid & 63, part = tid >> 6;
  float acc = 0.f;
  for (int k = part; k < kend; k += 4) acc = fmaf(sc[k], a.k[((long)b * a.S + k) * a.ldk + hk * 64 + dd], acc);
  po[part * 64 + dd] = acc;
  __syncthreads();
  if (tid < 64) a.dq[row * a.lddq + h * 64 + tid] = a.scale * ((po[tid] + po[64 + tid]) + (po[128 + tid] + po[192 + tid]));
}

// one 256-thread block per (key, kv head, batch): the G = Hq / Hkv query heads of the group and every query that sees
// the key (causal: q >= key; keys at or past seqlens[b] are seen by none)
__global__ __launch_bounds__(256) void attn_dkdv_f32_kernel(AttnBwdF32Args a) {
  extern __shared__ float sm[];
  float* ks = sm;           // [64]
  float* vs = sm + 64;      // [64]
  float* pk = sm + 128;     // [4][64] dk partials
  float* pv = sm + 384;     // [4][64] dv partials
  const int kj = blockIdx.x, hk = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
  const int G = a.Hq / a.Hkv;
  const int kvlen = a.seqlens ? min(a.seqlens[b], a.S) : a.S;
  const int q0 = a.causal ? kj : 0;
  const int nq = kj < kvlen ? a.S - q0 : 0;
  float* pp = sm + 640;              // [G * nq] P
  float* ds = pp + (long)G * (a.S);  // [G * nq] dS
  const long krow = (long)b * a.S + kj;
  if (tid < 64) {
    ks[tid] = a.k[krow * a.ldk + hk * 64 + tid];
    vs[tid] = a.v[krow * a.ldv + hk * 64 + tid];
  }
  __syncthreads();
  for (int e = tid; e < G * nq; e += 256) {
    const int h = hk * G + e / nq, qi = q0 + e % nq;
    const long row = (long)b * a.S + qi;
    const long bhq = ((long)b * a.Hq + h) * a.S + qi;
    const float p = attn_prob_f32(a, a.q + row * a.ldq + h * 64, ks, a.lse[bhq]);
    const float* g = a.dout + row * a.lddo + h * 64;
    float dp = 0.f;
    for (int d = 0; d < 64; ++d) dp = fmaf(g[d], vs[d], dp);
    pp[e] = p;
    ds[e] = p * (dp - a.delta[bhq]);
  }
  __syncthreads();
  const int dd = tid & 63, part = tid >> 6;
  float gk = 0.f, gv = 0.f;
  for (int e = part; e < G * nq; e += 4) {
    const int h = hk * G + e / nq, qi = q0 + e % nq;
    const long row = (long)b * a.S + qi;
    gk = fmaf(ds[e], a.q[row * a.ldq + h * 64 + dd], gk);
    gv = fmaf(pp[e], a.dout[row * a.lddo + h * 64 + dd], gv);
  }
  pk[part * 64 + dd] = gk;
  pv[part * 64 + dd] = gv;
  __syncthreads();
  if (tid < 64) {
    a.dk[krow * a.lddk + hk * 64 + tid] = a.scale * ((pk[tid] + pk[64 + tid]) + (pk[128 + tid] + pk[192 + tid]));
    a.dv[krow * a.lddv + hk * 64 + tid] = (pv[tid] + pv[64 + tid]) + (pv[128 + tid] + pv[192 + tid]);
  }
}

// dgu = [dact * up * silu'(gate) | dact * silu(gate)]   (swiglu_bwd_kernel)
__global__ void swiglu_bwd_f32_kernel(const float* dact, long ldd, const float* gu, long ldgu, float* dgu, long lddgu,
                                      long M, int F) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * F) return;
  const long m = idx / F;
  const int f = idx % F;
  const float g = gu[m * ldgu + f], u = gu[m * ldgu + F + f], da = dact[m * ldd + f];
  const float sg = 1.0f / (1.0f + expf(-g));
  dgu[m * lddgu + f] = da * u * sg * (1.0f + g * (1.0f - sg));
  dgu[m * lddgu + F + f] = da * g * sg;
}

// out = a * b (mode 0, elementwise rows) or a * b[col] (mode 1, a column vector)
__global__ void mul_f32_kernel(int mode, const float* x, long ldx, const float* y, long ldy, float* out, long ldo, long M,
                               int N) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  const long m = idx / N;
  const int n = idx % N;
  out[m * ldo + n] = x[m * ldx + n] * (mode ? y[n] : y[m * ldy + n]);
}

// CE gradient rows (ce_bwd_kernel) with f32 output
__global__ void ce_bwd_f32_kernel(const float* logits, long ld, const int* labels, const float* lse, int V,
                                  const float* gscale, float* dlogits, long ldd) {
  const long r = blockIdx.y;
  const float g = *gscale, l = lse[r];
  const int lab = labels[r];
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < ldd; i += (long)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (i < V && lab >= 0) v = (expf(logits[r * ld + i] - l) - (i == lab ? 1.f : 0.f)) * g;
    dlogits[r * ldd + i] = v;
  }
}

// InternViT embeddings backward (vit_embed_bwd_kernel) with f32 patch gradients
__global__ void vit_embed_bwd_f32_kernel(const float* dx, int N, int T, int D, float* dpos, float* dcls, float* dpatch) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)T * D) return;
  const int t = idx / D, c = idx % D;
  float s = 0.f;
  for (int n = 0; n < N; ++n) {
    const float g = dx[((long)n * T + t) * D + c];
    s += g;
    if (t > 0) dpatch[((long)n * (T - 1) + t - 1) * D + c] = g;
  }
  dpos[idx] = s;
  if (t == 0) dcls[c] = s;
}

}  // namespace slx

using namespace slx;

extern "C" {

int slx_gemm_f32(const slx_gemm_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d != nullptr, "slx_gemm_f32: null desc");
  SLX_CHECK_ARG(d->out_f32, "slx_gemm_f32: f32 output required");
  SLX_CHECK_ARG(d->drop_operand == 0, "slx_gemm_f32: operand dropout is not part of parity mode (p = 0)");
  const int e = d->epilogue;
  SLX_CHECK_ARG(e == SLX_EPI_STORE || e == SLX_EPI_GELU || e == SLX_EPI_QGELU || e == SLX_EPI_RESID_LS ||
                e == SLX_EPI_GELU_BWD || e == SLX_EPI_QGELU_BWD,
                "slx_gemm_f32: epilogue %d has no f32 twin (STORE, GELU, QGELU, RESID_LS, GELU_BWD, QGELU_BWD)", e);
  SLX_CHECK_ARG((e != SLX_EPI_GELU_BWD && e != SLX_EPI_QGELU_BWD) || (d->aux && !d->aux_grad),
                "slx_gemm_f32: GELU_BWD needs the saved pre-activation as aux");
  SLX_CHECK_ARG(d->colsum == nullptr, "slx_gemm_f32: no fused colsum (parity mode sums the output with slx_colsum)");
  SLX_CHECK_ARG(e != SLX_EPI_RESID_LS || (d->resid && d->ls), "slx_gemm_f32: RESID_LS needs resid and ls");
  SLX_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0, "slx_gemm_f32: negative dims");
  const int batch = d->batch < 1 ? 1 : d->batch;
  if (d->M == 0 || d->N == 0) return 0;
  GemmF32Args a;
  a.A = (const float*)d->A; a.B = (const float*)d->B; a.C = (float*)d->C;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc; a.sA = d->sA; a.sB = d->sB; a.sC = d->sC;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.ak = d->layout == SLX_GEMM_NT || d->layout == SLX_GEMM_NN;
  a.bk = d->layout == SLX_GEMM_NT || d->layout == SLX_GEMM_TT;
  a.alpha = d->alpha; a.bias = d->bias; a.ls = d->ls;
  a.aux_out = (float*)d->aux_out; a.ldaux_out = d->ldaux_out;
  a.resid = d->resid; a.ldr = d->ldr; a.accumulate = d->accumulate;
  a.aux = (const float*)d->aux; a.ldaux = d->ldaux;
  dim3 grid((d->N + 63) / 64, (d->M + 63) / 64, batch);
  hipStream_t st = (hipStream_t)stream;
  switch (e) {
    case SLX_EPI_STORE: hipLaunchKernelGGL(gemm_f32_kernel<SLX_EPI_STORE>, grid, dim3(256), 0, st, a); break;
    case SLX_EPI_GELU: hipLaunchKernelGGL(gemm_f32_kernel<SLX_EPI_GELU>, grid, dim3(256), 0, st, a); break;
    case SLX_EPI_QGELU: hipLaunchKernelGGL(gemm_f32_kernel<SLX_EPI_QGELU>, grid, dim3(256), 0, st, a); break;
    case SLX_EPI_GELU_BWD: hipLaunchKernelGGL(gemm_f32_kernel<SLX_EPI_GELU_BWD>, grid, dim3(256), 0, st, a); break;
    case SLX_EPI_QGELU_BWD: hipLaunchKernelGGL(gemm_f32_kernel<SLX_EPI_QGELU_BWD>, grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(gemm_f32_kernel<SLX_EPI_RESID_LS>, grid, dim3(256), 0, st, a); break;
  }
  SLX_LAUNCH_CHECK("slx_gemm_f32");
  return 0;
}

int slx_attn_fwd_f32(const slx_attn_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d->head_dim == 64, "slx_attn_fwd_f32: only head_dim 64 is supported (got %d)", d->head_dim);
  SLX_CHECK_ARG(d->Hq > 0 && d->Hkv > 0 && d->Hq % d->Hkv == 0, "slx_attn_fwd_f32: Hq must be a multiple of Hkv");
  SLX_CHECK_ARG(d->S <= 16384, "slx_attn_fwd_f32: S <= 16384");
  if (d->B == 0 || d->S == 0) return 0;
  AttnF32Args a;
  a.q = (const float*)d->q; a.k = (const float*)d->k; a.v = (const float*)d->v; a.o = (float*)d->o; a.lse = d->lse;
  a.ldq = d->ldq; a.ldk = d->ldk; a.ldv = d->ldv; a.ldo = d->ldo;
  a.B = d->B; a.S = d->S; a.Hq = d->Hq; a.Hkv = d->Hkv; a.causal = d->causal; a.seqlens = d->seqlens;
  a.scale = d->scale;
  const size_t lds = (size_t)(336 + d->S) * sizeof(float);
  hipLaunchKernelGGL(attn_fwd_f32_kernel, dim3(d->S, d->Hq, d->B), dim3(256), lds, (hipStream_t)stream, a);
  SLX_LAUNCH_CHECK("slx_attn_fwd_f32");
  return 0;
}

int slx_rope_f32(void* x, int64_t ldx, int64_t ntok, int S, int nheads, const float* cos_tab, const float* sin_tab,
                 int inverse, slx_stream_t stream) {
  if (ntok == 0 || nheads == 0) return 0;
  hipLaunchKernelGGL(rope_f32_kernel, pg1(ntok * nheads * 32), dim3(256), 0, (hipStream_t)stream, (float*)x, ldx, ntok,
                     S, nheads, cos_tab, sin_tab, inverse);
  SLX_LAUNCH_CHECK("slx_rope_f32");
  return 0;
}

int slx_swiglu_fwd_f32(const void* gu, int64_t ldgu, void* out, int64_t ldo, int64_t M, int F, slx_stream_t s) {
  if (M == 0 || F == 0) return 0;
  hipLaunchKernelGGL(swiglu_f32_kernel, pg1(M * F), dim3(256), 0, (hipStream_t)s, (const float*)gu, ldgu, (float*)out,
                     ldo, M, F);
  SLX_LAUNCH_CHECK("slx_swiglu_fwd_f32");
  return 0;
}

int slx_im2col_patch_f32(const float* pix, int N, int H, int W, int P, int kpad, void* out, slx_stream_t s) {
  SLX_CHECK_ARG(kpad >= 3 * P * P && H % P == 0 && W % P == 0, "slx_im2col_patch_f32: bad shape");
  const long total = (long)N * (H / P) * (W / P) * kpad;
  if (!total) return 0;
  hipLaunchKernelGGL(im2col_f32_kernel, pg1(total), dim3(256), 0, (hipStream_t)s, pix, N, H, W, P, kpad, (float*)out);
  SLX_LAUNCH_CHECK("slx_im2col_patch_f32");
  return 0;
}

int slx_assemble_tokens_f32(const int* code, int64_t n, int D, const void* embed, int V, const void* img, const float* wp,
                            const float* query, float* out, slx_stream_t s) {
  if (!n) return 0;
  hipLaunchKernelGGL(assemble_f32_kernel, pg1(n * D), dim3(256), 0, (hipStream_t)s, code, n, D, (const float*)embed, V,
                     (const float*)img, wp, query, out);
  SLX_LAUNCH_CHECK("slx_assemble_tokens_f32");
  return 0;
}

int slx_llava_merge_fwd_f32(const void* src, int C, int64_t n_img, int npatch_h, int npatch_w, int g, int r0, int hu,
                            int c0, int wu, int pool, const float* newline, void* out, slx_stream_t s) {
  SLX_CHECK_ARG(pool >= 1 && r0 >= 0 && c0 >= 0 && hu >= pool && wu >= pool && r0 + hu <= npatch_h * g &&
                c0 + wu <= npatch_w * g, "slx_llava_merge_fwd_f32: bad geometry");
  const long n = n_img * (long)((hu / pool) * (wu / pool + 1)) * C;
  if (!n) return 0;
  hipLaunchKernelGGL(llava_merge_f32_kernel, pg1(n), dim3(256), 0, (hipStream_t)s, (const float*)src, C, npatch_h,
                     npatch_w, g, r0, hu, c0, wu, pool, (long)n_img, newline, (float*)out);
  SLX_LAUNCH_CHECK("slx_llava_merge_fwd_f32");
  return 0;
}

int slx_attn_bwd_f32(const slx_attn_desc* d, const slx_attn_bwd_desc* g, slx_stream_t stream) {
  SLX_CHECK_ARG(d->head_dim == 64, "slx_attn_bwd_f32: only head_dim 64 is supported (got %d)", d->head_dim);
  SLX_CHECK_ARG(d->Hq > 0 && d->Hkv > 0 && d->Hq % d->Hkv == 0, "slx_attn_bwd_f32: Hq must be a multiple of Hkv");
  SLX_CHECK_ARG(d->S <= 16384 && (long)(d->Hq / d->Hkv) * d->S * 8 + 640 * 4 <= 160 * 1024,
                "slx_attn_bwd_f32: G * S too large for the LDS rows");
  SLX_CHECK_ARG(d->lse && g->delta_ws, "slx_attn_bwd_f32: lse and delta_ws required");
  if (d->B == 0 || d->S == 0) return 0;
  AttnBwdF32Args a;
  a.q = (const float*)d->q; a.k = (const float*)d->k; a.v = (const float*)d->v; a.o = (const float*)d->o;
  a.lse = d->lse; a.dout = (const float*)g->dout;
  a.dq = (float*)g->dq; a.dk = (float*)g->dk; a.dv = (float*)g->dv; a.delta = g->delta_ws;
  a.ldq = d->ldq; a.ldk = d->ldk; a.ldv = d->ldv; a.ldo = d->ldo; a.lddo = g->lddo;
  a.lddq = g->lddq; a.lddk = g->lddk; a.lddv = g->lddv;
  a.B = d->B; a.S = d->S; a.Hq = d->Hq; a.Hkv = d->Hkv; a.causal = d->causal; a.seqlens = d->seqlens;
  a.scale = d->scale;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(attn_delta_f32_kernel, pg1((long)d->B * d->Hq * d->S), dim3(256), 0, st, a);
  hipLaunchKernelGGL(attn_dq_f32_kernel, dim3(d->S, d->Hq, d->B), dim3(256), (size_t)(384 + d->S) * sizeof(float), st,
                     a);
  const size_t lds = (size_t)(640 + 2L * (d->Hq / d->Hkv) * d->S) * sizeof(float);
  hipLaunchKernelGGL(attn_dkdv_f32_kernel, dim3(d->S, d->Hkv, d->B), dim3(256), lds, st, a);
  SLX_LAUNCH_CHECK("slx_attn_bwd_f32");
  return 0;
}

int slx_swiglu_bwd_f32(const float* dact, int64_t ldd, const void* gu, int64_t ldgu, void* dgu, int64_t lddgu, int64_t M,
                       int F, slx_stream_t s) {
  if (M == 0 || F == 0) return 0;
  hipLaunchKernelGGL(swiglu_bwd_f32_kernel, pg1(M * F), dim3(256), 0, (hipStream_t)s, dact, ldd, (const float*)gu, ldgu,
                     (float*)dgu, lddgu, M, F);
  SLX_LAUNCH_CHECK("slx_swiglu_bwd_f32");
  return 0;
}

int slx_mul_f32(int mode, const float* x, int64_t ldx, const float* y, int64_t ldy, float* out, int64_t ldo, int64_t M,
                int N, slx_stream_t s) {
  SLX_CHECK_ARG(mode == 0 || mode == 1, "slx_mul_f32: mode 0 (rows) or 1 (column vector)");
  if (M == 0 || N == 0) return 0;
  hipLaunchKernelGGL(mul_f32_kernel, pg1(M * N), dim3(256), 0, (hipStream_t)s, mode, x, ldx, y, ldy, out, ldo, M, N);
  SLX_LAUNCH_CHECK("slx_mul_f32");
  return 0;
}

int slx_ce_bwd_f32(const float* logits, int64_t ld, const int* labels, const float* lse, int64_t R, int V,
                   const float* gscale, float* dlogits, int64_t ldd, slx_stream_t s) {
  if (!R) return 0;
  dim3 grid((unsigned)((ldd + 255) / 256 < 256 ? (ldd + 255) / 256 : 256), (unsigned)R);
  hipLaunchKernelGGL(ce_bwd_f32_kernel, grid, dim3(256), 0, (hipStream_t)s, logits, ld, labels, lse, V, gscale, dlogits,
                     ldd);
  SLX_LAUNCH_CHECK("slx_ce_bwd_f32");
  return 0;
}

int slx_vit_embed_bwd_f32(const float* dx, int N, int T, int D, float* dpos, float* dcls, float* dpatch, slx_stream_t s) {
  hipLaunchKernelGGL(vit_embed_bwd_f32_kernel, pg1((long)T * D), dim3(256), 0, (hipStream_t)s, dx, N, T, D, dpos, dcls,
                     dpatch);
  SLX_LAUNCH_CHECK("slx_vit_embed_bwd_f32");
  return 0;
}

}  // extern "C"
