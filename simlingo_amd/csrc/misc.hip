// Memory-bound glue of the SimLingo VLA step, each kernel fused to one pass over HBM:
// patch im2col, InternViT embeddings, SwiGLU, column reductions (bias / layer-scale grads),
// LLM token assembly (the sync-free restatement of AdaptorList.forward + replace_placeholder_tokens),
// row gathers, LoRA dropout, small strided GEMMs for the driving heads / waypoint encoder,
// cross-entropy over the 151655-way vocabulary, waypoint cumsum + smooth-L1, and the fused
// clip + AdamW optimizer step.
#include "common.h"
#include "../../include/slx.h"

namespace slx {

// ---------------------------------------------------------------------------------------------
// im2col for Conv2d(3, D, k=P, s=P): out[n*Np + p, k] = pix[n, c, py*P+ky, px*P+kx], k = c*P*P+ky*P+kx,
// zero for k >= 3*P*P (K padded to kpad so the GEMM gets 16-B aligned rows).
__global__ void im2col_kernel(const float* pix, int N, int H, int W, int P, int kpad, bf16* out) {
  const int gw = W / P, gh = H / P, np = gw * gh;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * np * (kpad / 8);
  if (idx >= total) return;
  const int kc = (idx % (kpad / 8)) * 8;
  const long rowi = idx / (kpad / 8);
  const int n = rowi / np, p = rowi % np, py = p / gw, px = p % gw;
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = kc + j;
    float x = 0.f;
    if (k < 3 * P * P) {
      const int c = k / (P * P), r = k % (P * P), ky = r / P, kx = r % P;
      x = pix[(((long)n * 3 + c) * H + py * P + ky) * W + px * P + kx];
    }
    v[j] = (bf16)x;
  }
  *reinterpret_cast<bf16x8*>(out + rowi * kpad + kc) = v;
}

// x0[n, 0] = cls + pos[0]; x0[n, 1+p] = patch[n*Np+p] + pos[1+p]
__global__ void vit_embed_fwd_kernel(const float* patch, const float* cls, const float* pos, float* out, int N, int T, int D) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * T * (D / 4);
  if (idx >= total) return;
  const int c = (idx % (D / 4)) * 4;
  const long row = idx / (D / 4);
  const int n = row / T, t = row % T;
  float4 p4 = *reinterpret_cast<const float4*>(pos + (long)t * D + c);
  float4 s4 = t == 0 ? *reinterpret_cast<const float4*>(cls + c)
                     : *reinterpret_cast<const float4*>(patch + ((long)n * (T - 1) + t - 1) * D + c);
  float4 o = {s4.x + p4.x, s4.y + p4.y, s4.z + p4.z, s4.w + p4.w};
  *reinterpret_cast<float4*>(out + row * D + c) = o;
}

// dpos[t] = sum_n dx[n,t]; dcls = dpos[0]; dpatch[n*Np+p] = bf16(dx[n, 1+p])
__global__ void vit_embed_bwd_kernel(const float* dx, int N, int T, int D, float* dpos, float* dcls, bf16* dpatch) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)T * D) return;
  const int t = idx / D, c = idx % D;
  float s = 0.f;
  for (int n = 0; n < N; ++n) {
    const float g = dx[((long)n * T + t) * D + c];
    s += g;
    if (t > 0) dpatch[((long)n * (T - 1) + t - 1) * D + c] = (bf16)g;
  }
  dpos[idx] = s;
  if (t == 0) dcls[c] = s;
}

// out[m, f] = silu(gu[m, f]) * gu[m, F + f]
__global__ void swiglu_fwd_kernel(const bf16* gu, long ldgu, bf16* out, long ldo, long M, int F) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * (F / 8)) return;
  const long m = idx / (F / 8);
  const int f = (idx % (F / 8)) * 8;
  const bf16x8 g = *reinterpret_cast<const bf16x8*>(gu + m * ldgu + f);
  const bf16x8 u = *reinterpret_cast<const bf16x8*>(gu + m * ldgu + F + f);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16)(silu((float)g[j]) * (float)u[j]);
  *reinterpret_cast<bf16x8*>(out + m * ldo + f) = o;
}

// Column sums over a strided set of rows, accumulated into the outputs with f32 atomics
// (outputs pre-zeroed by the host wrapper unless accumulating):
// mode 0: out0[c] += sum_r x[r,c] (x bf16) ; mode 1: same with x f32 ;
// mode 2 (layer-scale branch backward): x = dres f32, y bf16 -> g = bf16(dres*ls) written,
//   out0[c] += sum dres*y (d ls), out1[c] += sum dres*ls (d bias)
template <int MODE>
__global__ __launch_bounds__(256) void colsum_kernel(const void* xv, long ldx, long M, int N, float* out0, float* out1,
                                                     const float* ls, const bf16* y, long ldy, bf16* g, long ldg,
                                                     float* part) {
  const int c0 = (blockIdx.y * 256 + threadIdx.x) * 4;
  const bool live = c0 < N;
  float s[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  float lsv[4] = {1, 1, 1, 1};
  if (MODE == 2 && live && ls) {
#pragma unroll
    for (int e = 0; e < 4; ++e) lsv[e] = ls[c0 + e];
  }
  // 4 rows per trip, every load unconditional (rows past M read row M - 1 and are not summed; a missing y reads x's
  // bytes and is not used): a load behind `r < M` or `if (y)` made hipcc drain vmcnt(0) before the next row
  const long G = gridDim.x;
  const bf16* yb = y ? y : reinterpret_cast<const bf16*>(xv);
  const long ldyb = y ? ldy : (MODE == 0 ? ldx : 2 * ldx);
  const int cl = live ? c0 : 0;
  for (long r0 = blockIdx.x; r0 < M; r0 += 4 * G) {
    float v[4][4];
    bf16x4 yy[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long r = min(r0 + k * G, M - 1);
      if (MODE == 0) {
        const bf16x4 t = *reinterpret_cast<const bf16x4*>((const bf16*)xv + r * ldx + cl);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[k][e] = (float)t[e];
      } else {
        const float4 t = *reinterpret_cast<const float4*>((const float*)xv + r * ldx + cl);
        v[k][0] = t.x; v[k][1] = t.y; v[k][2] = t.z; v[k][3] = t.w;
      }
      if (MODE == 2) yy[k] = *reinterpret_cast<const bf16x4*>(yb + r * ldyb + cl);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long r = r0 + k * G;
      if (!live || r >= M) continue;
      if (MODE == 2) {
        bf16x4 go;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (y) s2[e] += v[k][e] * (float)yy[k][e];
          const float gv = v[k][e] * lsv[e];
          go[e] = (bf16)gv;
          s[e] += gv;
        }
        *reinterpret_cast<bf16x4*>(g + r * ldg + c0) = go;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] += v[k][e];
      }
    }
  }
  // transpose through LDS: each atomic wave-instruction then covers 256 contiguous bytes
  __shared__ float cs[2][1024];
  const int lc = threadIdx.x * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    cs[0][lc + e] = (MODE == 2) ? s2[e] : s[e];
    if (MODE == 2) cs[1][lc + e] = s[e];
  }
  __syncthreads();
  const int cb = blockIdx.y * 1024;
  for (int c = threadIdx.x; c < 1024 && cb + c < N; c += 256) {
    if (part) {  // deterministic mode: per-block partial rows, summed in block order by det_reduce
      if (out0) part[(long)blockIdx.x * N + cb + c] = cs[0][c];
      if (MODE == 2) part[((long)gridDim.x + blockIdx.x) * N + cb + c] = cs[1][c];
      continue;
    }
    if (out0) atomicAdd(out0 + cb + c, cs[0][c]);
    if (MODE == 2) atomicAdd(out1 + cb + c, cs[1][c]);
  }
}



// LLM input assembly: out[i, :] (f32) from code[i] = (kind << 28) | index
//   kind 0: token  -> embed[min(index, V-1)] (bf16 table; ids clamped like adaptors.py:256)
//   kind 1: image  -> img[index] (bf16, mlp1 output rows)
//   kind 2: waypoint encoder row -> wp[index] (f32)
//   kind 3: driving query -> query[index] (f32)
__global__ void assemble_kernel(const int* code, long n, int D, const bf16* embed, int V, const bf16* img,
                                const float* wp, const float* query, float* out) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * (D / 4)) return;
  const long i = idx / (D / 4);
  const int c = (idx % (D / 4)) * 4;
  const int cd = code[i];
  const int kind = (cd >> 28) & 0xF, ix = cd & 0x0FFFFFFF;
  float4 o;
  if (kind == 0 || kind == 1) {
    const bf16* src = kind == 0 ? embed + (long)min(ix, V - 1) * D : img + (long)ix * D;
    const bf16x4 t = *reinterpret_cast<const bf16x4*>(src + c);
    o = {(float)t[0], (float)t[1], (float)t[2], (float)t[3]};
  } else {
    const float* src = (kind == 2 ? wp : query) + (long)ix * D;
    o = *reinterpret_cast<const float4*>(src + c);
  }
  *reinterpret_cast<float4*>(out + i * D + c) = o;
}

// dst[i, :] = src[idx[i], :]  (f32 -> f32 or bf16), D % 4 == 0
template <typename OutT>
__global__ void gather_rows_kernel(const float* src, long lds, const int* idx, long n, int D, OutT* dst, long ldd) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * (D / 4)) return;
  const long i = t / (D / 4);
  const int c = (t % (D / 4)) * 4;
  const float4 v = *reinterpret_cast<const float4*>(src + (long)idx[i] * lds + c);
  OutT* d = dst + i * ldd + c;
  d[0] = (OutT)v.x; d[1] = (OutT)v.y; d[2] = (OutT)v.z; d[3] = (OutT)v.w;
}

// bf16 rows -> f32 rows gather (features for the heads / loss rows)
__global__ void gather_rows_bf16_kernel(const bf16* src, long lds, const int* idx, long n, int D, bf16* dst, long ldd) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * (D / 8)) return;
  const long i = t / (D / 8);
  const int c = (t % (D / 8)) * 8;
  *reinterpret_cast<bf16x8*>(dst + i * ldd + c) = *reinterpret_cast<const bf16x8*>(src + (long)idx[i] * lds + c);
}

// out[j, c] (+)= sum_b src[pos[b*nq + j], c]
__global__ void gather_sum_kernel(const float* src, long lds, const int* pos, int B, int nq, int D, float* out, int accumulate) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)nq * D) return;
  const int j = t / D, c = t % D;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += src[(long)pos[b * nq + j] * lds + c];
  out[t] = accumulate ? out[t] + s : s;
}

// dst = src * keep(seed, m*ldmask + n) / (1-p)  (LoRA dropout; same mask as the GEMM DROPMASK epilogue)
__global__ void dropout_kernel(const bf16* src, long lds, bf16* dst, long ldd, long M, int N, unsigned long long seed,
                               float p, long ldmask) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * (N / 8)) return;
  const long m = t / (N / 8);
  const int n0 = (t % (N / 8)) * 8;
  const bf16x8 x = *reinterpret_cast<const bf16x8*>(src + m * lds + n0);
  bf16x8 o;
  const float sc = 1.0f / (1.0f - p);
  const uint32_t s1 = drop_seed_mix(seed), thr = drop_thr(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float keep = drop_keep(s1, (unsigned long long)m * ldmask + n0 + j, thr) ? sc : 0.f;
    o[j] = (bf16)((float)x[j] * keep);
  }
  *reinterpret_cast<bf16x8*>(dst + m * ldd + n0) = o;
}

// Small strided f32 GEMM for the driving heads / waypoint encoder (M <= a few hundred rows):
// C[m,n] (+)= act(alpha * sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn] + bias[n]); pre-act optional.
__global__ __launch_bounds__(256) void sgemm_kernel(slx_sgemm_desc d) {
  __shared__ float As[16][17], Bs[16][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m = blockIdx.y * 16 + ty, n = blockIdx.x * 16 + tx;
  float acc = 0.f;
  for (int k0 = 0; k0 < d.K; k0 += 16) {
    const int ka = k0 + tx, kb = k0 + ty;
    const int am = blockIdx.y * 16 + ty, bn = blockIdx.x * 16 + tx;
    As[ty][tx] = (am < d.M && ka < d.K) ? d.A[(long)am * d.sam + (long)ka * d.sak] : 0.f;
    Bs[ty][tx] = (bn < d.N && kb < d.K) ? d.B[(long)kb * d.sbk + (long)bn * d.sbn] : 0.f;
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) acc += As[ty][kk] * Bs[kk][tx];
    __syncthreads();
  }
  if (m >= d.M || n >= d.N) return;
  float v = acc * d.alpha;
  if (d.bias) v += d.bias[n];
  const long ci = (long)m * d.scm + (long)n * d.scn;
  if (d.pre) d.pre[(long)m * d.ldpre + n] = v;
  if (d.act == SLX_ACT_RELU) v = fmaxf(v, 0.f);
  else if (d.act == SLX_ACT_SILU) v = silu(v);
  if (d.accumulate) v += d.C[ci];
  d.C[ci] = v;
}

// d_pre = d_act * act'(pre)
__global__ void act_bwd_kernel(const float* dact, const float* pre, float* dpre, long n, int act) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = pre[i];
  const float g = act == SLX_ACT_RELU ? (x > 0.f ? 1.f : 0.f) : act == SLX_ACT_SILU ? silu_grad(x) : 1.f;
  dpre[i] = dact[i] * g;
}

// ---------------------------------------------------------------------------------------------
// Cross-entropy over the vocabulary for the gathered loss rows (adaptors.py:259-274).
// fwd: loss[r] = logsumexp(logits[r]) - logits[r, label[r]]; lse[r] kept for bwd.
__global__ __launch_bounds__(1024) void ce_fwd_kernel(const float* logits, long ld, const int* labels, int V, float* loss, float* lse) {
  __shared__ float sh[16];
  const long r = blockIdx.x;
  const float* x = logits + r * ld;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < V; i += blockDim.x) mx = fmaxf(mx, x[i]);
  mx = warp_max(mx);
  {
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = mx;
    __syncthreads();
    float t = -INFINITY;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t = fmaxf(t, sh[i]);
    mx = t;
  }
  float s = 0.f;
  for (int i = threadIdx.x; i < V; i += blockDim.x) s += __expf(x[i] - mx);
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    const float l = mx + __logf(s);
    lse[r] = l;
    const int lab = labels[r];
    loss[r] = (lab >= 0 && lab < V) ? l - x[lab] : 0.f;  // ignore_index (-1) rows: loss 0, as F.cross_entropy
  }
}
// bwd: dlogits[r, v] = (softmax - onehot) * (*gscale); padded columns [V, ldd) zeroed.
__global__ void ce_bwd_kernel(const float* logits, long ld, const int* labels, const float* lse, int V, const float* gscale,
                              bf16* dlogits, long ldd) {
  const long r = blockIdx.y;
  const float g = *gscale, l = lse[r];
  const int lab = labels[r];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ldd; i += gridDim.x * blockDim.x) {
    float v = 0.f;
    if (i < V && lab >= 0) v = (__expf(logits[r * ld + i] - l) - (i == lab ? 1.f : 0.f)) * g;  // ignored rows: 0
    dlogits[r * ldd + i] = (bf16)v;
  }
}

// Driving heads (adaptors.py:183-221): pred[b, i] = sum_{j<=i} out[b, j]  (cumsum over points),
// loss[b, i] = sum_xy smooth_l1(pred - label, beta=1). Backward: d_out = reverse-cumsum of
// d_pred, d_pred = smooth_l1'(pred - label) * gscale.
// kind 0: smooth_l1(beta 1).sum(-1) (simlingo_training adaptors.py:205-213);
// kind 1: mse.sum(-1) (simlingo_base_training adaptors.py:226, .mean(-1) = the per-point average downstream)
__global__ void wp_loss_fwd_kernel(const float* out, const float* label, int B, int n, int dims, int kind, float* pred,
                                   float* loss) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float run[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    float l = 0.f;
    for (int c = 0; c < dims; ++c) {
      run[c] += out[((long)b * n + i) * dims + c];
      pred[((long)b * n + i) * dims + c] = run[c];
      const float d = run[c] - label[((long)b * n + i) * dims + c];
      const float ad = fabsf(d);
      l += kind ? d * d : (ad < 1.f ? 0.5f * d * d : ad - 0.5f);
    }
    loss[(long)b * n + i] = l;
  }
}
__global__ void wp_loss_bwd_kernel(const float* pred, const float* label, int B, int n, int dims, int kind,
                                   const float* gscale, float* dout) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float g = *gscale;
  float run[4] = {0, 0, 0, 0};
  for (int i = n - 1; i >= 0; --i) {
    for (int c = 0; c < dims; ++c) {
      const long k = ((long)b * n + i) * dims + c;
      const float d = pred[k] - label[k];
      const float gd = (kind ? 2.f * d : (fabsf(d) < 1.f ? d : (d > 0.f ? 1.f : -1.f))) * g;
      run[c] += gd;
      dout[k] = run[c];
    }
  }
}

// summarise_losses (simlingo_training/models/utils.py:7-41) on device:
// out[0] = total, out[1..3] = lang, route, speed averages; gs[0..2] = d(total)/d(per-item) scales
// given the upstream gradient dtotal (device scalar, may be NULL in forward).
__global__ void loss_finalize_kernel(const float* lang, int nl, const float* route, int nr, const float* speed, int ns, float* out) {
  __shared__ float sh[16];
  float a = 0.f, b = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < nl; i += blockDim.x) a += lang[i];
  for (int i = threadIdx.x; i < nr; i += blockDim.x) b += route[i];
  for (int i = threadIdx.x; i < ns; i += blockDim.x) c += speed[i];
  a = block_sum(a, sh);
  b = block_sum(b, sh);
  c = block_sum(c, sh);
  if (threadIdx.x == 0) {
    const float la = nl > 0 ? a / nl : 0.f, ra = nr > 0 ? b / nr : 0.f, sa = ns > 0 ? c / ns : 0.f;
    out[0] = la + ra + sa;
    out[1] = la; out[2] = ra; out[3] = sa;
  }
}
__global__ void loss_gscale_kernel(const float* dl, int nl, int nr, int ns, float* gs) {
  // dl = d(out)/d[total, lang, route, speed]; every average feeds the total with weight 1
  const float t = dl ? dl[0] : 1.f;
  gs[0] = nl > 0 ? (t + (dl ? dl[1] : 0.f)) / nl : 0.f;
  gs[1] = nr > 0 ? (t + (dl ? dl[2] : 0.f)) / nr : 0.f;
  gs[2] = ns > 0 ? (t + (dl ? dl[3] : 0.f)) / ns : 0.f;
}

// ---------------------------------------------------------------------------------------------
// Optimizer: global grad-norm (sum of squares, partials + atomics) and fused clip + AdamW
// (torch.optim.AdamW semantics, decoupled weight decay; driving.py:718-724, clip train.py:206).
// GT = float, or bf16: the summed data-parallel gradients straight from the bf16 all-reduce wire (ddp.py wire="bf16")
template <typename GT>
__device__ __forceinline__ float4 load_g4(const GT* g, long i) {
  if constexpr (sizeof(GT) == 4) {
    return reinterpret_cast<const float4*>(g)[i];
  } else {
    const bf16x4 b = reinterpret_cast<const bf16x4*>(g)[i];
    return make_float4((float)b[0], (float)b[1], (float)b[2], (float)b[3]);
  }
}

template <typename GT>
__global__ __launch_bounds__(256) void sumsq_kernel(const GT* g, long n, float* out, float* part) {
  __shared__ float sh[16];
  float s = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = load_g4(g, i);
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0)
    for (long i = (n / 4) * 4 + threadIdx.x; i < n; i += blockDim.x) s += (float)g[i] * (float)g[i];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    if (part) part[blockIdx.x] = s;  // deterministic mode: summed in block order by det_reduce
    else atomicAdd(out, s);
  }
}

template <typename GT>
__global__ __launch_bounds__(256) void adamw_kernel(float* p, const GT* g, float* m, float* v, bf16* pbf, long n,
                                                    float lr, float b1, float b2, float eps, float wd, float bc1,
                                                    float bc2s, const float* sumsq, float max_norm, float gscale) {
  // gscale: 1/world for summed data-parallel gradients; clip on the averaged gradient's norm
  float coef = gscale;
  if (sumsq && max_norm > 0.f) {
    const float tn = sqrtf(*sumsq) * gscale;
    coef = gscale * fminf(1.f, max_norm / (tn + 1e-6f));
  }
  const float step = lr / bc1;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = (float)g[i] * coef;
    float pi = p[i] * (1.f - lr * wd);
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    const float den = sqrtf(vi) / bc2s + eps;
    pi -= step * mi / den;
    p[i] = pi; m[i] = mi; v[i] = vi;
    if (pbf) pbf[i] = (bf16)pi;
  }
}

// The same update four parameters per lane (16-B loads and stores of p / g / m / v, 8-B bf16 stores): n4 quads from
// 16-B aligned p / g / m / v and an 8-B aligned pbf; the launcher runs the scalar kernel on the tail.
typedef float f32x4nt __attribute__((ext_vector_type(4)));
// NT: p / m / v (and an f32 g) streamed with nontemporal loads and stores (each touched once per step; SLX_ADAMW_NT)
template <bool NT>
__device__ __forceinline__ float4 ld4(const float4* q) {
  if constexpr (NT) {
    const f32x4nt t = __builtin_nontemporal_load(reinterpret_cast<const f32x4nt*>(q));
    return make_float4(t[0], t[1], t[2], t[3]);
  } else {
    return *q;
  }
}
template <bool NT>
__device__ __forceinline__ void st4(float4* q, float a, float b, float c, float d) {
  if constexpr (NT) {
    const f32x4nt t = {a, b, c, d};
    __builtin_nontemporal_store(t, reinterpret_cast<f32x4nt*>(q));
  } else {
    *q = {a, b, c, d};
  }
}
template <typename GT, bool NT>
__device__ __forceinline__ float4 load_g4n(const GT* g, long i) {
  if constexpr (sizeof(GT) == 4) return ld4<NT>(reinterpret_cast<const float4*>(g) + i);
  else return load_g4(g, i);
}

template <typename GT, bool NT>
__global__ __launch_bounds__(256) void adamw_kernel_x4(float4* p, const GT* g, float4* m, float4* v, bf16x4* pbf,
                                                     long n4, float lr, float b1, float b2, float eps, float wd, float bc1,
                                                     float bc2s, const float* sumsq, float max_norm, float gscale) {
  float coef = gscale;
  if (sumsq && max_norm > 0.f) {
    const float tn = sqrtf(*sumsq) * gscale;
    coef = gscale * fminf(1.f, max_norm / (tn + 1e-6f));
  }
  const float step = lr / bc1;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 g4 = load_g4n<GT, NT>(g, i), p4 = ld4<NT>(p + i), m4 = ld4<NT>(m + i), v4 = ld4<NT>(v + i);
    float gi[4] = {g4.x, g4.y, g4.z, g4.w}, pi[4] = {p4.x, p4.y, p4.z, p4.w};
    float mi[4] = {m4.x, m4.y, m4.z, m4.w}, vi[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = gi[j] * coef;
      pi[j] = pi[j] * (1.f - lr * wd);
      mi[j] = mi[j] + (1.f - b1) * (gj - mi[j]);
      vi[j] = vi[j] * b2 + (1.f - b2) * gj * gj;
      const float den = sqrtf(vi[j]) / bc2s + eps;
      pi[j] -= step * mi[j] / den;
    }
    st4<NT>(p + i, pi[0], pi[1], pi[2], pi[3]);
    st4<NT>(m + i, mi[0], mi[1], mi[2], mi[3]);
    st4<NT>(v + i, vi[0], vi[1], vi[2], vi[3]);
    if (pbf) pbf[i] = {(bf16)pi[0], (bf16)pi[1], (bf16)pi[2], (bf16)pi[3]};
  }
}

// dst[idx[i], :] (+)= src[i, :]   (f32 rows; idx unique)
__global__ void scatter_rows_kernel(const float* src, long lds, const int* idx, long n, int D, float* dst, long ldd, int accumulate) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * (D / 4)) return;
  const long i = t / (D / 4);
  const int c = (t % (D / 4)) * 4;
  const float4 v = *reinterpret_cast<const float4*>(src + i * lds + c);
  float4* d = reinterpret_cast<float4*>(dst + (long)idx[i] * ldd + c);
  if (accumulate) { const float4 o = *d; *d = {o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w}; }
  else *d = v;
}

// bf16 rows gathered into f32 rows
__global__ void gather_rows_b2f_kernel(const bf16* src, long lds, const int* idx, long n, int D, float* dst, long ldd) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * (D / 8)) return;
  const long i = t / (D / 8);
  const int c = (t % (D / 8)) * 8;
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + (long)idx[i] * lds + c);
#pragma unroll
  for (int j = 0; j < 8; ++j) dst[i * ldd + c + j] = (float)v[j];
}

// SwiGLU backward from an f32 d(act): dgu[m, f] = d*u*silu'(g), dgu[m, F+f] = d*silu(g)
__global__ void swiglu_bwd_kernel(const float* dact, long ldd, const bf16* gu, long ldgu, bf16* dgu, long lddgu, long M, int F) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * (F / 8)) return;
  const long m = idx / (F / 8);
  const int f = (idx % (F / 8)) * 8;
  const bf16x8 g = *reinterpret_cast<const bf16x8*>(gu + m * ldgu + f);
  const bf16x8 u = *reinterpret_cast<const bf16x8*>(gu + m * ldgu + F + f);
  bf16x8 og, ou;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float d = dact[m * ldd + f + j], gv = (float)g[j], uv = (float)u[j];
    og[j] = (bf16)(d * uv * silu_grad(gv));
    ou[j] = (bf16)(d * silu(gv));
  }
  *reinterpret_cast<bf16x8*>(dgu + m * lddgu + f) = og;
  *reinterpret_cast<bf16x8*>(dgu + m * lddgu + F + f) = ou;
}

// f32 rows -> bf16 rows (row strides), cols % 4 == 0
__global__ void cast_rows_kernel(const float* src, long lds, bf16* dst, long ldd, long M, int N) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * (N / 4)) return;
  const long m = t / (N / 4);
  const int c = (t % (N / 4)) * 4;
  const float4 v = *reinterpret_cast<const float4*>(src + m * lds + c);
  bf16x4 o = {(bf16)v.x, (bf16)v.y, (bf16)v.z, (bf16)v.w};
  *reinterpret_cast<bf16x4*>(dst + m * ldd + c) = o;
}

// Batched 2-D scaled copy f32 -> bf16 (or f32, parity mode): entry e of `tab` =
// {src, lds, dst, ldd, rows, cols, scale(bits), mode}, mode 0 bf16 [rows][ldd], 1 f32 [rows][ldd], 2 / 3 bf16 in the
// packed LoRA-A fragment orders of slx_lora_down / slx_lora_bwd's dx term (rows == 32, ldd unused). Packs every LoRA B (times alpha/r) into the
// fused [W | s*B] GEMM operands and every LoRA A into its fragment copy in one launch.
// destination index d of a pack entry -> source (r, c) and destination offset (the loop walks the DESTINATION in order,
// so every mode's stores are contiguous; the transposed (4) and fragment-ordered (2, 3) modes used to walk the source
// and scatter 2-byte stores). 32-bit index arithmetic: the host (engine._build_lora_cat) refuses an entry of 2^31
// elements or more, and modes 2 / 3 need rows == 32 (the packed-fragment layouts of common.h).
__device__ __forceinline__ void pack_at(int mode, int i, int nrow, int ncol, long ldd, int& r, int& c, long& dst) {
  if (mode == 2) {  // inverse of lora_frag_index
    const int lane = (i >> 3) & 63, q = i >> 9;
    r = lane & 31;
    c = 32 * (q >> 1) + 16 * (q & 1) + 8 * (lane >> 5) + (i & 7);
    dst = i;
  } else if (mode == 3) {  // inverse of lora_dxfrag_index
    const int lane = (i >> 3) & 63, q = i >> 9;
    r = 16 * (q & 1) + 8 * (lane >> 5) + (i & 7);
    c = 32 * (q >> 1) + (lane & 31);
    dst = i;
  } else if (mode == 4) {  // transposed: dst[c][r]
    c = i / nrow;
    r = i - c * nrow;
    dst = (long)c * ldd + r;
  } else {
    r = i / ncol;
    c = i - r * ncol;
    dst = (long)r * ldd + c;
  }
}

__global__ void pack_scaled_kernel(const long long* tab, int n) {
  const int e = blockIdx.x;
  const long long* t = tab + 8 * (long)e;
  const float* src = reinterpret_cast<const float*>(t[0]);
  const long lds = t[1];
  const long ldd = t[3];
  const int nrow = (int)t[4], ncol = (int)t[5];
  const float sc = __int_as_float((int)t[6]);
  const int mode = (int)t[7];
  const int nel = nrow * ncol;
  for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < nel; i += gridDim.y * blockDim.x) {
    int r, c;
    long dst;
    pack_at(mode, i, nrow, ncol, ldd, r, c, dst);
    const float v = src[(long)r * lds + c] * sc;
    if (mode == 1) reinterpret_cast<float*>(t[2])[dst] = v;
    else reinterpret_cast<bf16*>(t[2])[dst] = (bf16)v;
  }
}

// flat grid (slx_pack_scaled_flat): block b packs chunk block_map[b] >> 16 (SLX_PACK_CHUNK elements, 8 per thread: 8
// loads in flight per thread, one round trip per block) of entry block_map[b] & 0xFFFF
__global__ __launch_bounds__(256) void pack_scaled_flat_kernel(const long long* tab, int n, const int* bmap) {
  const int bm = bmap[blockIdx.x];
  const int lo = bm & 0xFFFF, chunk = bm >> 16;
  const long long* t = tab + 8 * (long)lo;
  const float* src = reinterpret_cast<const float*>(t[0]);
  const long lds = t[1];
  const long ldd = t[3];
  const int nrow = (int)t[4], ncol = (int)t[5];
  const float sc = __int_as_float((int)t[6]);
  const int mode = (int)t[7];
  const int nel = nrow * ncol;
  const int i0 = chunk * SLX_PACK_CHUNK + threadIdx.x;
  constexpr int PER = SLX_PACK_CHUNK / 256;
  float v[PER];
  long dst[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = min(i0 + 256 * u, nel - 1);
    int r, c;
    pack_at(mode, i, nrow, ncol, ldd, r, c, dst[u]);
    v[u] = src[(long)r * lds + c] * sc;
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    if (i0 + 256 * u < nel) {
      if (mode == 1) reinterpret_cast<float*>(t[2])[dst[u]] = v[u];
      else reinterpret_cast<bf16*>(t[2])[dst[u]] = (bf16)v[u];
    }
  }
}

// Batched bf16 transpose dst[c][r] = src[r][c]: entry y of `tab` = {src, lds, dst, ldd, rows, cols}, block x = one
// 64 x 64 tile (blocks past the entry's tile count exit). Whole, aligned tiles move as 16-B row pieces through a
// padded LDS tile (one read and one write of every byte, coalesced on both sides); ragged edges go element-wise.
// Keeps the [in][out] copies of the weights whose data-gradient GEMM dX = dY W would otherwise run NN (slower main
// loop than NT on gfx950: tools/nn_vs_nt.py) in step with the optimizer.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const long long* tab) {
  const long long* t = tab + 6 * (long)blockIdx.y;
  const unsigned short* src = reinterpret_cast<const unsigned short*>(t[0]);
  const long lds = t[1];
  unsigned short* dst = reinterpret_cast<unsigned short*>(t[2]);
  const long ldd = t[3];
  const long rows = t[4], cols = t[5];
  const long tc = (cols + 63) / 64;
  const long tile = blockIdx.x;
  if (tile >= ((rows + 63) / 64) * tc) return;
  const long r0 = (tile / tc) * 64, c0 = (tile % tc) * 64;
  __shared__ __attribute__((aligned(16))) unsigned short s[64][72];
  const int tid = threadIdx.x;
  const bool vec = ((lds | ldd) & 7) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0 && r0 + 64 <= rows &&
                   c0 + 64 <= cols;
  if (vec) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = (tid >> 3) + 32 * h, c = (tid & 7) * 8;
      *reinterpret_cast<uint4*>(&s[r][c]) = *reinterpret_cast<const uint4*>(src + (r0 + r) * lds + c0 + c);
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int oc = (tid >> 3) + 32 * h, orr = (tid & 7) * 8;
      unsigned short o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = s[orr + j][oc];
      *reinterpret_cast<uint4*>(dst + (c0 + oc) * ldd + r0 + orr) = *reinterpret_cast<const uint4*>(o);
    }
  } else {
    for (int i = tid; i < 4096; i += 256) {
      const long r = r0 + i / 64, c = c0 + i % 64;
      if (r < rows && c < cols) s[i / 64][i % 64] = src[r * lds + c];
    }
    __syncthreads();
    for (int i = tid; i < 4096; i += 256) {
      const long c = c0 + i / 64, r = r0 + i % 64;
      if (r < rows && c < cols) dst[c * ldd + r] = s[i % 64][i / 64];
    }
  }
}

__global__ void cast_kernel(const float* src, bf16* dst, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (bf16)src[i];
}

}  // namespace slx

using namespace slx;

// out = a + b + c (the projection bias folded with temporal_encoding + camera_encoding, llavanext.py:98-110)
__global__ void vec_sum3_kernel(const float* a, const float* b, const float* c, long n, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i] + c[i];
}

// out = x * scale + shift (NormZeroOne, simlingo_base_training/models/driving.py:89-103)
__global__ void affine_kernel(const float* x, long n, float scale, float shift, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = x[i] * scale + shift;
}

// LLaVA-NeXT spatial merge (LingoLlavaNextModel.forward_image, llavanext_model.py:128-157, spatial_unpad):
// per image the npatch_h x npatch_w patches of g x g features form an (npatch_h*g) x (npatch_w*g) grid;
// unpad_image keeps rows [r0, r0+hu) and cols [c0, c0+wu); avg_pool2d(pool) (floor); then one
// image_newline column -> tokens (i, j), j <= wo, row-major: T = ho * (wo + 1).
struct MergeGeom { int npatch_h, npatch_w, g, r0, hu, c0, wu, pool; };
__device__ __forceinline__ long merge_src_row(const MergeGeom& m, long img, int h, int w) {
  const int ph = h / m.g, pw = w / m.g;
  return (img * m.npatch_h * m.npatch_w + ph * m.npatch_w + pw) * (long)(m.g * m.g) + (h % m.g) * m.g + (w % m.g);
}
__global__ void llava_merge_fwd_kernel(const bf16* src, int C, MergeGeom m, long n_img, const float* newline, bf16* out) {
  const int ho = m.hu / m.pool, wo = m.wu / m.pool, T = ho * (wo + 1);
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c8 = C / 8;
  if (idx >= n_img * T * c8) return;
  const int c = (idx % c8) * 8;
  const long tok = idx / c8;
  const long img = tok / T;
  const int t = tok % T, i = t / (wo + 1), j = t % (wo + 1);
  bf16x8 o;
  if (j == wo) {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)newline[c + e];
  } else {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int a = 0; a < m.pool; ++a)
      for (int b = 0; b < m.pool; ++b) {
        const long r = merge_src_row(m, img, m.r0 + i * m.pool + a, m.c0 + j * m.pool + b);
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + r * C + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += (float)v[e];
      }
    const float inv = 1.0f / (m.pool * m.pool);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)(acc[e] * inv);
  }
  *reinterpret_cast<bf16x8*>(out + tok * C + c) = o;
}
// backward: every source feature row gathers 1/pool^2 of its window's output gradient (0 outside)
__global__ void llava_merge_bwd_kernel(const float* dout, int C, MergeGeom m, long n_img, bf16* dsrc) {
  const int ho = m.hu / m.pool, wo = m.wu / m.pool, T = ho * (wo + 1);
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c8 = C / 8;
  const long rows_per_img = (long)m.npatch_h * m.npatch_w * m.g * m.g;
  if (idx >= n_img * rows_per_img * c8) return;
  const int c = (idx % c8) * 8;
  const long r = idx / c8;
  const long img = r / rows_per_img;
  const int q = r % rows_per_img, p = q / (m.g * m.g), y = (q % (m.g * m.g)) / m.g, x = q % m.g;
  const int h = (p / m.npatch_w) * m.g + y - m.r0, w = (p % m.npatch_w) * m.g + x - m.c0;
  bf16x8 o;
  if (h >= 0 && w >= 0 && h < ho * m.pool && w < wo * m.pool) {
    const long tok = img * T + (h / m.pool) * (wo + 1) + w / m.pool;
    const float inv = 1.0f / (m.pool * m.pool);
    const float4 a = *reinterpret_cast<const float4*>(dout + tok * C + c);
    const float4 b = *reinterpret_cast<const float4*>(dout + tok * C + c + 4);
    o[0] = (bf16)(a.x * inv); o[1] = (bf16)(a.y * inv); o[2] = (bf16)(a.z * inv); o[3] = (bf16)(a.w * inv);
    o[4] = (bf16)(b.x * inv); o[5] = (bf16)(b.y * inv); o[6] = (bf16)(b.z * inv); o[7] = (bf16)(b.w * inv);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)0.f;
  }
  *reinterpret_cast<bf16x8*>(dsrc + r * C + c) = o;
}

static inline dim3 g1(long n, int bs = 256) { return dim3((unsigned)((n + bs - 1) / bs)); }

extern "C" {

int slx_im2col_patch(const float* pix, int N, int H, int W, int P, int kpad, void* out, slx_stream_t s) {
  SLX_CHECK_ARG(kpad % 8 == 0 && kpad >= 3 * P * P && H % P == 0 && W % P == 0, "slx_im2col_patch: bad shape");
  const long total = (long)N * (H / P) * (W / P) * (kpad / 8);
  if (!total) return 0;
  hipLaunchKernelGGL(im2col_kernel, g1(total), dim3(256), 0, (hipStream_t)s, pix, N, H, W, P, kpad, (bf16*)out);
  SLX_LAUNCH_CHECK("slx_im2col_patch");
  return 0;
}

int slx_vit_embed_fwd(const float* patch, const float* cls, const float* pos, float* out, int N, int T, int D, slx_stream_t s) {
  SLX_CHECK_ARG(D % 4 == 0, "slx_vit_embed_fwd: D %% 4");
  const long total = (long)N * T * (D / 4);
  hipLaunchKernelGGL(vit_embed_fwd_kernel, g1(total), dim3(256), 0, (hipStream_t)s, patch, cls, pos, out, N, T, D);
  SLX_LAUNCH_CHECK("slx_vit_embed_fwd");
  return 0;
}

int slx_vit_embed_bwd(const float* dx, int N, int T, int D, float* dpos, float* dcls, void* dpatch, slx_stream_t s) {
  hipLaunchKernelGGL(vit_embed_bwd_kernel, g1((long)T * D), dim3(256), 0, (hipStream_t)s, dx, N, T, D, dpos, dcls, (bf16*)dpatch);
  SLX_LAUNCH_CHECK("slx_vit_embed_bwd");
  return 0;
}

int slx_swiglu_fwd(const void* gu, int64_t ldgu, void* out, int64_t ldo, int64_t M, int F, slx_stream_t s) {
  SLX_CHECK_ARG(F % 8 == 0 && ldgu % 8 == 0 && ldo % 8 == 0, "slx_swiglu_fwd: F/ld must be multiples of 8");
  hipLaunchKernelGGL(swiglu_fwd_kernel, g1(M * (F / 8)), dim3(256), 0, (hipStream_t)s, (const bf16*)gu, ldgu, (bf16*)out, ldo, M, F);
  SLX_LAUNCH_CHECK("slx_swiglu_fwd");
  return 0;
}

int slx_colsum_ws_floats(int N) { return 256 * 2 * N; }

// mode 0: x bf16, 1: x f32 -> out[c] (+)= sum_r x[r,c]
int slx_colsum(int mode, const void* x, int64_t ldx, int64_t M, int N, float* out, int accumulate, float* ws, slx_stream_t s) {
  SLX_CHECK_ARG(N % 4 == 0 && (mode == 0 || mode == 1), "slx_colsum: N %% 4 / mode");
  (void)ws;
  hipStream_t st = (hipStream_t)s;
  if (!accumulate) hipMemsetAsync(out, 0, (size_t)N * sizeof(float), st);
  int nblk = (int)(M < 512 ? (M > 0 ? M : 1) : 512);
  const DetMode& dm = det_mode();
  float* part = nullptr;
  if (dm.on) {
    SLX_CHECK_ARG(dm.ws_floats >= N, "slx_colsum: deterministic workspace too small");
    if ((long)nblk * N > dm.ws_floats) nblk = (int)(dm.ws_floats / N);
    part = dm.ws;
  }
  dim3 grid(nblk, (N / 4 + 255) / 256);
  if (mode == 0) hipLaunchKernelGGL((colsum_kernel<0>), grid, dim3(256), 0, st, x, ldx, M, N, out, (float*)nullptr, nullptr, nullptr, 0L, nullptr, 0L, part);
  else hipLaunchKernelGGL((colsum_kernel<1>), grid, dim3(256), 0, st, x, ldx, M, N, out, (float*)nullptr, nullptr, nullptr, 0L, nullptr, 0L, part);
  SLX_LAUNCH_CHECK("slx_colsum");
  if (part) return det_reduce(part, nblk, N, N, out, 1, st);
  return 0;
}

// Layer-scale residual branch backward: g = bf16(dres*ls), dls = sum dres*y, dbias = sum g
int slx_ls_branch_bwd(const float* dres, int64_t ldr, const float* ls, const void* y, int64_t ldy, void* g, int64_t ldg,
                      int64_t M, int N, float* dls, float* dbias, int accumulate, float* ws, slx_stream_t s) {
  SLX_CHECK_ARG(N % 4 == 0, "slx_ls_branch_bwd: N %% 4");
  (void)ws;
  hipStream_t st = (hipStream_t)s;
  SLX_CHECK_ARG((dls == nullptr) == (y == nullptr) && dbias, "slx_ls_branch_bwd: dls iff y; dbias required");
  if (!accumulate) {
    if (dls) hipMemsetAsync(dls, 0, (size_t)N * sizeof(float), st);
    hipMemsetAsync(dbias, 0, (size_t)N * sizeof(float), st);
  }
  int nblk = (int)(M < 512 ? (M > 0 ? M : 1) : 512);
  const DetMode& dm = det_mode();
  float* part = nullptr;
  if (dm.on) {
    SLX_CHECK_ARG(dm.ws_floats >= 2L * N, "slx_ls_branch_bwd: deterministic workspace too small");
    if (2L * nblk * N > dm.ws_floats) nblk = (int)(dm.ws_floats / (2L * N));
    part = dm.ws;
  }
  dim3 grid(nblk, (N / 4 + 255) / 256);
  hipLaunchKernelGGL((colsum_kernel<2>), grid, dim3(256), 0, st, (const void*)dres, ldr, M, N, dls, dbias, ls, (const bf16*)y, ldy, (bf16*)g, ldg, part);
  SLX_LAUNCH_CHECK("slx_ls_branch_bwd");
  if (part) {
    if (dls && det_reduce(part, nblk, N, N, dls, 1, st)) return -1000;
    return det_reduce(part + (long)nblk * N, nblk, N, N, dbias, 1, st);
  }
  return 0;
}

int slx_assemble_tokens(const int* code, int64_t n, int D, const void* embed, int V, const void* img, const float* wp,
                        const float* query, float* out, slx_stream_t s) {
  SLX_CHECK_ARG(D % 4 == 0, "slx_assemble_tokens: D %% 4");
  hipLaunchKernelGGL(assemble_kernel, g1(n * (D / 4)), dim3(256), 0, (hipStream_t)s, code, n, D, (const bf16*)embed, V,
                     (const bf16*)img, wp, query, out);
  SLX_LAUNCH_CHECK("slx_assemble_tokens");
  return 0;
}

int slx_gather_rows(const float* src, int64_t lds, const int* idx, int64_t n, int D, void* dst, int64_t ldd, int dst_bf16, slx_stream_t s) {
  SLX_CHECK_ARG(D % 4 == 0, "slx_gather_rows: D %% 4");
  if (!n) return 0;
  if (dst_bf16) hipLaunchKernelGGL(gather_rows_kernel<bf16>, g1(n * (D / 4)), dim3(256), 0, (hipStream_t)s, src, lds, idx, n, D, (bf16*)dst, ldd);
  else hipLaunchKernelGGL(gather_rows_kernel<float>, g1(n * (D / 4)), dim3(256), 0, (hipStream_t)s, src, lds, idx, n, D, (float*)dst, ldd);
  SLX_LAUNCH_CHECK("slx_gather_rows");
  return 0;
}

int slx_gather_rows_bf16(const void* src, int64_t lds, const int* idx, int64_t n, int D, void* dst, int64_t ldd, slx_stream_t s) {
  SLX_CHECK_ARG(D % 8 == 0 && lds % 8 == 0 && ldd % 8 == 0, "slx_gather_rows_bf16: D/ld %% 8");
  if (!n) return 0;
  hipLaunchKernelGGL(gather_rows_bf16_kernel, g1(n * (D / 8)), dim3(256), 0, (hipStream_t)s, (const bf16*)src, lds, idx, n, D, (bf16*)dst, ldd);
  SLX_LAUNCH_CHECK("slx_gather_rows_bf16");
  return 0;
}

int slx_gather_sum(const float* src, int64_t lds, const int* pos, int B, int nq, int D, float* out, int accumulate, slx_stream_t s) {
  hipLaunchKernelGGL(gather_sum_kernel, g1((long)nq * D), dim3(256), 0, (hipStream_t)s, src, lds, pos, B, nq, D, out, accumulate);
  SLX_LAUNCH_CHECK("slx_gather_sum");
  return 0;
}

int slx_dropout(const void* src, int64_t lds, void* dst, int64_t ldd, int64_t M, int N, uint64_t seed, float p, int64_t ldmask, slx_stream_t s) {
  SLX_CHECK_ARG(N % 8 == 0 && p >= 0.f && p < 1.f, "slx_dropout: N %% 8, 0 <= p < 1");
  hipLaunchKernelGGL(dropout_kernel, g1(M * (N / 8)), dim3(256), 0, (hipStream_t)s, (const bf16*)src, lds, (bf16*)dst, ldd, M, N, seed, p, ldmask);
  SLX_LAUNCH_CHECK("slx_dropout");
  return 0;
}

int slx_sgemm(const slx_sgemm_desc* d, slx_stream_t s) {
  if (d->M == 0 || d->N == 0) return 0;
  dim3 grid((d->N + 15) / 16, (d->M + 15) / 16);
  hipLaunchKernelGGL(sgemm_kernel, grid, dim3(256), 0, (hipStream_t)s, *d);
  SLX_LAUNCH_CHECK("slx_sgemm");
  return 0;
}

int slx_act_bwd(const float* dact, const float* pre, float* dpre, int64_t n, int act, slx_stream_t s) {
  hipLaunchKernelGGL(act_bwd_kernel, g1(n), dim3(256), 0, (hipStream_t)s, dact, pre, dpre, n, act);
  SLX_LAUNCH_CHECK("slx_act_bwd");
  return 0;
}

int slx_ce_fwd(const float* logits, int64_t ld, const int* labels, int64_t R, int V, float* loss, float* lse, slx_stream_t s) {
  if (!R) return 0;
  hipLaunchKernelGGL(ce_fwd_kernel, dim3((unsigned)R), dim3(1024), 0, (hipStream_t)s, logits, ld, labels, V, loss, lse);
  SLX_LAUNCH_CHECK("slx_ce_fwd");
  return 0;
}

int slx_ce_bwd(const float* logits, int64_t ld, const int* labels, const float* lse, int64_t R, int V, const float* gscale,
               void* dlogits, int64_t ldd, slx_stream_t s) {
  if (!R) return 0;
  dim3 grid((unsigned)((ldd + 1023) / 1024 < 64 ? (ldd + 1023) / 1024 : 64), (unsigned)R);
  hipLaunchKernelGGL(ce_bwd_kernel, grid, dim3(1024), 0, (hipStream_t)s, logits, ld, labels, lse, V, gscale, (bf16*)dlogits, ldd);
  SLX_LAUNCH_CHECK("slx_ce_bwd");
  return 0;
}

int slx_wp_loss_fwd(const float* out, const float* label, int B, int n, int dims, int kind, float* pred, float* loss,
                    slx_stream_t s) {
  SLX_CHECK_ARG(dims <= 4 && (kind == 0 || kind == 1), "slx_wp_loss_fwd: dims <= 4, kind 0/1");
  hipLaunchKernelGGL(wp_loss_fwd_kernel, g1(B, 64), dim3(64), 0, (hipStream_t)s, out, label, B, n, dims, kind, pred, loss);
  SLX_LAUNCH_CHECK("slx_wp_loss_fwd");
  return 0;
}

int slx_wp_loss_bwd(const float* pred, const float* label, int B, int n, int dims, int kind, const float* gscale,
                    float* dout, slx_stream_t s) {
  SLX_CHECK_ARG(dims <= 4 && (kind == 0 || kind == 1), "slx_wp_loss_bwd: dims <= 4, kind 0/1");
  hipLaunchKernelGGL(wp_loss_bwd_kernel, g1(B, 64), dim3(64), 0, (hipStream_t)s, pred, label, B, n, dims, kind, gscale, dout);
  SLX_LAUNCH_CHECK("slx_wp_loss_bwd");
  return 0;
}

int slx_loss_finalize(const float* lang, int nl, const float* route, int nr, const float* speed, int ns, float* out, slx_stream_t s) {
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)s, lang, nl, route, nr, speed, ns, out);
  SLX_LAUNCH_CHECK("slx_loss_finalize");
  return 0;
}

int slx_loss_gscale(const float* dtotal, int nl, int nr, int ns, float* gs, slx_stream_t s) {
  hipLaunchKernelGGL(loss_gscale_kernel, dim3(1), dim3(1), 0, (hipStream_t)s, dtotal, nl, nr, ns, gs);
  SLX_LAUNCH_CHECK("slx_loss_gscale");
  return 0;
}

extern "C++" {
template <typename GT>
static int sumsq_impl(const GT* g, int64_t n, float* out, int zero_first, slx_stream_t s, float* ws = nullptr,
                      int64_t ws_floats = 0) {  // out (+)= sum g^2
  hipStream_t st = (hipStream_t)s;
  if (zero_first) hipMemsetAsync(out, 0, sizeof(float), st);
  if (!n) return 0;
  long blocks = (n / 4 + 255) / 256;
  if (blocks > SLX_SUMSQ_PARTS) blocks = SLX_SUMSQ_PARTS;
  if (blocks < 1) blocks = 1;
  const DetMode& dm = det_mode();
  // ordered partial sums: the caller's workspace (slx_sumsq_ws), else the deterministic mode's
  float* part = ws ? ws : (dm.on ? dm.ws : nullptr);
  if (ws) SLX_CHECK_ARG(ws_floats >= blocks, "slx_sumsq_ws: workspace of at least SLX_SUMSQ_PARTS floats");
  hipLaunchKernelGGL(sumsq_kernel<GT>, dim3((unsigned)blocks), dim3(256), 0, st, g, n, out, part);
  SLX_LAUNCH_CHECK("slx_sumsq");
  if (part) return det_reduce(part, (int)blocks, 1, 1, out, 1, st);
  return 0;
}
}  // extern "C++"

int slx_sumsq(const float* g, int64_t n, float* out, int zero_first, slx_stream_t s) {
  return sumsq_impl(g, n, out, zero_first, s);
}

int slx_sumsq_ws(const float* g, int64_t n, float* out, int zero_first, float* ws, int64_t ws_floats, slx_stream_t s) {
  SLX_CHECK_ARG(ws != nullptr, "slx_sumsq_ws: workspace");
  return sumsq_impl(g, n, out, zero_first, s, ws, ws_floats);
}

int slx_sumsq_bf16_ws(const void* g, int64_t n, float* out, int zero_first, float* ws, int64_t ws_floats,
                      slx_stream_t s) {
  SLX_CHECK_ARG(((uintptr_t)g & 7) == 0, "slx_sumsq_bf16_ws: 8-B aligned gradients");
  SLX_CHECK_ARG(ws != nullptr, "slx_sumsq_bf16_ws: workspace");
  return sumsq_impl((const bf16*)g, n, out, zero_first, s, ws, ws_floats);
}

int slx_sumsq_bf16(const void* g, int64_t n, float* out, int zero_first, slx_stream_t s) {
  SLX_CHECK_ARG(((uintptr_t)g & 7) == 0, "slx_sumsq_bf16: 8-B aligned gradients");
  return sumsq_impl((const bf16*)g, n, out, zero_first, s);
}

extern "C++" {
template <typename GT>
static int adamw_impl(float* p, const GT* g, float* m, float* v, void* p_bf16, int64_t n, float lr, float beta1,
                      float beta2, float eps, float weight_decay, int step, const float* sumsq, float max_norm,
                      float grad_scale, slx_stream_t s) {
  SLX_CHECK_ARG(step >= 1, "slx_adamw: step >= 1");
  if (!n) return 0;
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2s = sqrtf(1.f - powf(beta2, (float)step));
  const bool vec = ((((uintptr_t)p | (uintptr_t)m | (uintptr_t)v) & 15) == 0) &&
                   (((uintptr_t)g & (sizeof(GT) == 4 ? 15 : 7)) == 0) && (((uintptr_t)p_bf16 & 7) == 0);
  long done = 0;
  if (vec && n >= 4) {
    const long n4 = n / 4;
    // one quad per lane, no grid-stride loop: 1730 us at 315M parameters vs 1.83-2.03 ms with the grid capped at
    // 65536-1024 blocks and 1.94 ms for the scalar kernel (tools/adamw_bench.py, profiles/round3_adamw_grid.txt);
    // SLX_ADAMW_BLOCKS caps it (A/B hook)
    static const long cap = [] { const char* e = getenv("SLX_ADAMW_BLOCKS"); return e ? atol(e) : 0L; }();
    long blocks = (n4 + 255) / 256;
    if (cap > 0 && blocks > cap) blocks = cap;
    if (blocks > 0x7fffffffL) blocks = 0x7fffffffL;
    // nontemporal p / m / v streams (SLX_ADAMW_NT, default 1): 1675 vs 1733 us at 315M parameters
    // (tools/adamw_bench.py, profiles/round5_adamw_nt_ab.txt), the same arithmetic
    static const bool nt = [] { const char* e = getenv("SLX_ADAMW_NT"); return !e || atoi(e) != 0; }();
    if (nt)
      hipLaunchKernelGGL((adamw_kernel_x4<GT, true>), dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)s, (float4*)p,
                         g, (float4*)m, (float4*)v, (bf16x4*)p_bf16, n4, lr, beta1, beta2, eps, weight_decay, bc1, bc2s,
                         sumsq, max_norm, grad_scale);
    else
      hipLaunchKernelGGL((adamw_kernel_x4<GT, false>), dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)s, (float4*)p,
                         g, (float4*)m, (float4*)v, (bf16x4*)p_bf16, n4, lr, beta1, beta2, eps, weight_decay, bc1, bc2s,
                         sumsq, max_norm, grad_scale);
    SLX_LAUNCH_CHECK("slx_adamw");
    done = n4 * 4;
  }
  if (done < n) {
    const long rest = n - done;
    long blocks = (rest + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(adamw_kernel<GT>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)s, p + done, g + done, m + done,
                       v + done, p_bf16 ? (bf16*)p_bf16 + done : nullptr, rest, lr, beta1, beta2, eps, weight_decay, bc1,
                       bc2s, sumsq, max_norm, grad_scale);
    SLX_LAUNCH_CHECK("slx_adamw");
  }
  return 0;
}
}  // extern "C++"

int slx_adamw(float* p, const float* g, float* m, float* v, void* p_bf16, int64_t n, float lr, float beta1, float beta2,
              float eps, float weight_decay, int step, const float* sumsq, float max_norm, float grad_scale, slx_stream_t s) {
  return adamw_impl(p, g, m, v, p_bf16, n, lr, beta1, beta2, eps, weight_decay, step, sumsq, max_norm, grad_scale, s);
}

int slx_adamw_bf16g(float* p, const void* g, float* m, float* v, void* p_bf16, int64_t n, float lr, float beta1,
                    float beta2, float eps, float weight_decay, int step, const float* sumsq, float max_norm,
                    float grad_scale, slx_stream_t s) {
  return adamw_impl(p, (const bf16*)g, m, v, p_bf16, n, lr, beta1, beta2, eps, weight_decay, step, sumsq, max_norm,
                    grad_scale, s);
}

int slx_scatter_rows(const float* src, int64_t lds, const int* idx, int64_t n, int D, float* dst, int64_t ldd, int accumulate, slx_stream_t s) {
  SLX_CHECK_ARG(D % 4 == 0, "slx_scatter_rows: D %% 4");
  if (!n) return 0;
  hipLaunchKernelGGL(scatter_rows_kernel, g1(n * (D / 4)), dim3(256), 0, (hipStream_t)s, src, lds, idx, n, D, dst, ldd, accumulate);
  SLX_LAUNCH_CHECK("slx_scatter_rows");
  return 0;
}

int slx_gather_rows_b2f(const void* src, int64_t lds, const int* idx, int64_t n, int D, float* dst, int64_t ldd, slx_stream_t s) {
  SLX_CHECK_ARG(D % 8 == 0 && lds % 8 == 0, "slx_gather_rows_b2f: D/lds %% 8");
  if (!n) return 0;
  hipLaunchKernelGGL(gather_rows_b2f_kernel, g1(n * (D / 8)), dim3(256), 0, (hipStream_t)s, (const bf16*)src, lds, idx, n, D, dst, ldd);
  SLX_LAUNCH_CHECK("slx_gather_rows_b2f");
  return 0;
}

int slx_swiglu_bwd(const float* dact, int64_t ldd, const void* gu, int64_t ldgu, void* dgu, int64_t lddgu, int64_t M, int F, slx_stream_t s) {
  SLX_CHECK_ARG(F % 8 == 0 && ldgu % 8 == 0 && lddgu % 8 == 0, "slx_swiglu_bwd: F/ld %% 8");
  hipLaunchKernelGGL(swiglu_bwd_kernel, g1(M * (F / 8)), dim3(256), 0, (hipStream_t)s, dact, ldd, (const bf16*)gu, ldgu, (bf16*)dgu, lddgu, M, F);
  SLX_LAUNCH_CHECK("slx_swiglu_bwd");
  return 0;
}

int slx_cast_rows(const float* src, int64_t lds, void* dst, int64_t ldd, int64_t M, int N, slx_stream_t s) {
  SLX_CHECK_ARG(N % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0, "slx_cast_rows: N/ld %% 4");
  if (!M) return 0;
  hipLaunchKernelGGL(cast_rows_kernel, g1(M * (N / 4)), dim3(256), 0, (hipStream_t)s, src, lds, (bf16*)dst, ldd, M, N);
  SLX_LAUNCH_CHECK("slx_cast_rows");
  return 0;
}

int slx_pack_scaled(const int64_t* table, int n, slx_stream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(pack_scaled_kernel, dim3(n, 32), dim3(256), 0, (hipStream_t)s, (const long long*)table, n);
  SLX_LAUNCH_CHECK("slx_pack_scaled");
  return 0;
}

int slx_pack_scaled_flat(const int64_t* table, int n, const int* block_map, int nblocks, slx_stream_t s) {
  SLX_CHECK_ARG(n >= 0 && n <= 65536 && nblocks >= 0 && (n == 0 || (table && block_map)),
                "slx_pack_scaled_flat: table, block_map, n <= 65536");
  if (n <= 0 || nblocks == 0) return 0;
  hipLaunchKernelGGL(pack_scaled_flat_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)s, (const long long*)table, n,
                     block_map);
  SLX_LAUNCH_CHECK("slx_pack_scaled_flat");
  return 0;
}

int slx_transpose_bf16(const int64_t* table, int n, int64_t max_tiles, slx_stream_t s) {
  SLX_CHECK_ARG(n >= 0 && n <= 65535 && max_tiles >= 0 && max_tiles <= 0x7fffffff, "slx_transpose_bf16: bad n / max_tiles");
  if (n == 0 || max_tiles == 0) return 0;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((unsigned)max_tiles, n), dim3(256), 0, (hipStream_t)s,
                     (const long long*)table);
  SLX_LAUNCH_CHECK("slx_transpose_bf16");
  return 0;
}

int slx_affine(const float* x, int64_t n, float scale, float shift, float* out, slx_stream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(affine_kernel, g1(n), dim3(256), 0, (hipStream_t)s, x, n, scale, shift, out);
  SLX_LAUNCH_CHECK("slx_affine");
  return 0;
}

int slx_vec_sum3(const float* a, const float* b, const float* c, int64_t n, float* out, slx_stream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(vec_sum3_kernel, g1(n), dim3(256), 0, (hipStream_t)s, a, b, c, n, out);
  SLX_LAUNCH_CHECK("slx_vec_sum3");
  return 0;
}

static int merge_geom(MergeGeom& m, int npatch_h, int npatch_w, int g, int r0, int hu, int c0, int wu, int pool) {
  m = MergeGeom{npatch_h, npatch_w, g, r0, hu, c0, wu, pool};
  SLX_CHECK_ARG(pool >= 1 && r0 >= 0 && c0 >= 0 && hu >= pool && wu >= pool && r0 + hu <= npatch_h * g &&
                c0 + wu <= npatch_w * g, "slx_llava_merge: bad geometry");
  return 0;
}

int slx_llava_merge_tokens(int hu, int wu, int pool) { return (hu / pool) * (wu / pool + 1); }

int slx_llava_merge_fwd(const void* src, int C, int64_t n_img, int npatch_h, int npatch_w, int g, int r0, int hu, int c0,
                        int wu, int pool, const float* newline, void* out, slx_stream_t s) {
  SLX_CHECK_ARG(C % 8 == 0, "slx_llava_merge_fwd: C %% 8");
  MergeGeom m;
  int rc = merge_geom(m, npatch_h, npatch_w, g, r0, hu, c0, wu, pool);
  if (rc) return rc;
  const long n = n_img * slx_llava_merge_tokens(hu, wu, pool) * (C / 8);
  if (n == 0) return 0;
  hipLaunchKernelGGL(llava_merge_fwd_kernel, g1(n), dim3(256), 0, (hipStream_t)s, (const bf16*)src, C, m, (long)n_img,
                     newline, (bf16*)out);
  SLX_LAUNCH_CHECK("slx_llava_merge_fwd");
  return 0;
}

int slx_llava_merge_bwd(const float* dout, int C, int64_t n_img, int npatch_h, int npatch_w, int g, int r0, int hu, int c0,
                        int wu, int pool, void* dsrc, slx_stream_t s) {
  SLX_CHECK_ARG(C % 8 == 0, "slx_llava_merge_bwd: C %% 8");
  MergeGeom m;
  int rc = merge_geom(m, npatch_h, npatch_w, g, r0, hu, c0, wu, pool);
  if (rc) return rc;
  const long n = n_img * (long)npatch_h * npatch_w * g * g * (C / 8);
  if (n == 0) return 0;
  hipLaunchKernelGGL(llava_merge_bwd_kernel, g1(n), dim3(256), 0, (hipStream_t)s, dout, C, m, (long)n_img, (bf16*)dsrc);
  SLX_LAUNCH_CHECK("slx_llava_merge_bwd");
  return 0;
}

int slx_cast_f32_bf16(const float* src, void* dst, int64_t n, slx_stream_t s) {
  if (!n) return 0;
  hipLaunchKernelGGL(cast_kernel, g1(n), dim3(256), 0, (hipStream_t)s, src, (bf16*)dst, n);
  SLX_LAUNCH_CHECK("slx_cast_f32_bf16");
  return 0;
}

}  // extern "C"
