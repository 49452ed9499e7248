// bf16 MFMA GEMM for gfx950 (CDNA4): C[M,N] = alpha * op(A) * op(B) with fused epilogues.
//
// Replaces every cuBLAS GEMM behind nn.Linear / Conv2d(patch) in the reference hot path
// (SURVEY.md 2.N3/2.N4): InternViT qkv/proj/fc1/fc2 (remote InternVisionEncoderLayer, called at
// simlingo_training/models/encoder/internvl2_model.py:114), mlp1, Qwen2 q/k/v/o/gate/up/down
// (+ LoRA A/B, simlingo_training/models/language_model/llm.py:106-119) and the LM head
// (simlingo_training/models/adaptors/adaptors.py:265-273).
//
// Design (MI355X-first):
//  * 128x128 output tile, BK=64, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 tiles of
//    v_mfma_f32_16x16x32_bf16 (the gfx950 double-K bf16 MFMA).
//  * Both operands may be K-contiguous ("row" storage, e.g. nn.Linear weight [N][K]) or
//    MN-contiguous (e.g. activations read as X^T in the weight-gradient GEMM). K-contiguous tiles
//    live in LDS as [rows][64] with a (row>>1)&7 XOR swizzle of the 16-B chunk (conflict-free
//    ds_read_b128); MN-contiguous tiles live as [64][rows] with a (k&3 | k>>3&1) XOR swizzle and
//    are read with ds_read_b64_tr_b16 (hardware transpose) - conflict-free for both the
//    tr-reads and the 16-B staging writes (verified by enumeration).
//  * Register-staged double buffer: tile k+1 is loaded to VGPRs before the MFMAs of tile k and
//    written to the other LDS buffer after them; one barrier per K-step.
//  * Bijective XCD-aware block remap + GROUP_M=8 tile ordering so neighbouring tiles that share
//    operand panels sit in one XCD's L2.
#include <cmath>

#include <cstdlib>

#include "common.h"
#include "../../include/slx.h"

namespace slx {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;

enum { EPI_STORE = 0, EPI_GELU = 1, EPI_RESID_LS = 2, EPI_GELU_BWD = 3, EPI_SWIGLU_BWD = 4, EPI_DROPMASK = 5,
       EPI_DROPMASK_SWIGLU = 6, EPI_QGELU = 7, EPI_QGELU_BWD = 8,
       EPI_DROPMASK_SWIGLU_B = 9 /* internal: DROPMASK_SWIGLU with a bf16 resid (slx_gemm_desc.resid_bf16) */,
       EPI_CE_PART = 10,  /* internal (slx_lmhead_ce_fwd): per-row (max, sum exp) over each 64-column sub-tile + label logit */
       EPI_CE_GRAD = 11   /* internal (slx_lmhead_ce_bwd): bf16 (softmax - onehot) * gscale from recomputed logits */ };

// CLIP quick_gelu x*sigmoid(1.702x) (transformers ACT2FN["quick_gelu"], the LLaVA-NeXT vision tower)
__device__ __forceinline__ float qgelu(float x) { return x / (1.0f + __expf(-1.702f * x)); }
__device__ __forceinline__ float qgelu_grad(float x) {
  const float s = 1.0f / (1.0f + __expf(-1.702f * x));
  return s * (1.0f + 1.702f * x * (1.0f - s));
}
// act(h) and, with p.aux_grad, the value stored as aux: the derivative act'(h) instead of h
template <int EPI>
__device__ __forceinline__ float act_fwd(float h, bool aux_grad, float& aux) {
  if constexpr (EPI == EPI_GELU) {
    const GeluTerms g = gelu_terms(h);
    aux = aux_grad ? __builtin_fmaf(h * 0.39894228040143268f, g.e, g.cdf) : h;
    return h * g.cdf;
  } else {
    aux = aux_grad ? qgelu_grad(h) : h;
    return qgelu(h);
  }
}
template <int EPI>
__device__ __forceinline__ float act_bwd(float aux, bool aux_grad) {
  if (aux_grad) return aux;
  if constexpr (EPI == EPI_GELU_BWD) return gelu_erf_grad(aux);
  else return qgelu_grad(aux);
}

struct GemmArgs {
  const bf16* A;
  const bf16* B;
  void* C;
  long lda, ldb, ldc;
  long sA, sB, sC;
  int M, N, K;
  float alpha;
  const float* bias;
  const float* ls;
  const bf16* aux;
  long ldaux;
  bf16* aux_out;
  long ldaux_out;
  const float* resid;
  long ldr;
  int resid_bf16;  // DROPMASK_SWIGLU: resid points to bf16 rows
  int accumulate;
  unsigned long long seed;
  float drop_p;
  long ldmask;
  int tilesM, tilesN;
  int ksplit;        // > 1: split-K, f32 atomic accumulation into a pre-zeroed / accumulating C
  int kchunk;        // K range per split (multiple of BK)
  int vec_ok;        // 16-B aligned rows for C / aux / resid -> vectorised epilogue
  int drop_operand;  // 0 none, 1 = dropout on A while loading, 2 = on B (v1 main loop only)
  int mshift_last;   // v3: the last M tile starts at M - 256 (overlaps its neighbour; idempotent epilogues only)
  float* colsum;     // optional [N]: += column sums of the f32 epilogue output (vector epilogue path only)
  float* colsum_ws;  // [ceil(M/64) + colsum_row0][N] partials, one row per 64-row output subtile
  int colsum_row0;   // subtile-row offset of this launch (the M-remainder launch continues the main grid's rows)
  long split_stride; // split-K: 0 = f32 atomics into C; > 0 = split y stores its partial to C + y * split_stride
  const uint32_t* maskbits;  // DROPMASK epilogues: keep bits [M][ldbits] (slx_lora_down), else the hash
  long ldbits;
  // v3 with the M-remainder folded in (rows [rem_r0, M), at most 64): split-K partials + last-arriver epilogue
  int rem_r0;        // 0 = no folded remainder
  int rem_nsplit;    // K splits per 256-column group
  int rem_kc;        // K per split (multiple of 32)
  float* rem_part;   // [rem_nsplit][M - rem_r0][N] f32 partials
  int* rem_cnt;      // [ceil(N / 256)] arrival counters, zero on entry, reset by each group's last arriver
  // v3 split-K reduced inside the launch (f32 STORE): per tile one [ksplit][256*256] f32 slab set + 2 counters
  float* split_ws;   // null = split-K partials go to C with f32 atomics
  int* split_cnt;    // [2 * tiles] arrival / published counters, zero on entry, reset by each tile's last arriver
  int split_tile0;   // tile-index offset of this GEMM in the shared workspace (slx_gemm_bf16_pair's second GEMM)
  int xcd_split;     // slx_gemm_bf16_pair: 1-D grid of 256, XCD x takes K split x % ksplit (gemm_bf16_v3_pair_kernel)
  // fused LM head + cross entropy (EPI_CE_PART / EPI_CE_GRAD)
  const int* ce_labels;  // [M] next-token label per row (-1 = ignored)
  float* ce_part;        // [M][ce_ldpart] (max, sumexp) pairs, one per 64-column sub-tile
  float* ce_lab;         // [M] the label's logit
  const float* ce_lse;   // [M] log-sum-exp (backward)
  const float* ce_gscale;  // d loss / d (per-row CE): one scalar (the LM loss weight / count)
  int ce_ldpart;
  // RoPE fused into a bf16 STORE epilogue (slx_gemm_desc.rope_*): columns < rope_ncols, position = row % rope_S
  const float* rope_cos;
  const float* rope_sin;
  int rope_S, rope_ncols;
  // GELU / QGELU store the derivative at h as aux; GELU_BWD / QGELU_BWD multiply the aux in directly
  int aux_grad;
};

// Dropout applied while loading an operand (LoRA dropout, regenerated bit-exactly in backward):
// element at STORAGE coordinates (srow, scol) is kept with probability 1-p and scaled by 1/(1-p),
// keep = uniform01(seed, srow*ldmask + scol) >= p  (same hash as slx_dropout / EPI_DROPMASK).
struct LoadMask {
  unsigned long long seed;
  float p;
  long ldmask;
};

__device__ __forceinline__ uint4 mask8(uint4 v, const LoadMask& mk, long base) {
  bf16x8 x = __builtin_bit_cast(bf16x8, v);
  const float sc = 1.0f / (1.0f - mk.p);
  const uint32_t s1 = drop_seed_mix(mk.seed), thr = drop_thr(mk.p);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (bf16)((float)x[j] * (drop_keep(s1, (unsigned long long)(base + j), thr) ? sc : 0.f));
  return __builtin_bit_cast(uint4, x);
}

// keep factor of element (m, n) of a DROPMASK epilogue: the stored keep bits when given, else the hash
__device__ __forceinline__ float epi_keep(const GemmArgs& p, int m, int n) {
  const float sc = 1.0f / (1.0f - p.drop_p);
  if (p.maskbits) return (p.maskbits[(long)m * p.ldbits + (n >> 5)] >> (n & 31)) & 1u ? sc : 0.f;
  return drop_keep(drop_seed_mix(p.seed), (unsigned long long)m * p.ldmask + n, drop_thr(p.drop_p)) ? sc : 0.f;
}
// keep bits of columns n..n+7 (n % 8 == 0) of row m
__device__ __forceinline__ uint32_t epi_keep8(const GemmArgs& p, int m, int n) {
  if (p.maskbits) return (p.maskbits[(long)m * p.ldbits + (n >> 5)] >> (n & 31)) & 0xFFu;
  const unsigned long long i0 = (unsigned long long)m * p.ldmask + n;
  const uint32_t s1 = drop_seed_mix(p.seed), thr = drop_thr(p.drop_p);
  if ((i0 & 1) == 0) return drop_keep8(s1, i0, thr);
  uint32_t b = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) b |= (uint32_t)drop_keep(s1, i0 + e, thr) << e;
  return b;
}

template <bool KC>
__device__ __forceinline__ void load_tile(const bf16* __restrict__ X, long ld, int row0, int rows_total, int k0,
                                          int K, uint4 (&r)[4], const LoadMask* mk = nullptr) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + NT * i;
    int row, kk;
    if (KC) {
      row = id >> 3;
      kk = (id & 7) * 8;
    } else {
      kk = id >> 4;
      row = (id & 15) * 8;
    }
    const int grow = row0 + row, gk = k0 + kk;
    if (grow < rows_total && gk < K) {
      const bf16* ptr = KC ? X + (long)grow * ld + gk : X + (long)gk * ld + grow;
      r[i] = *reinterpret_cast<const uint4*>(ptr);
      if (mk) r[i] = mask8(r[i], *mk, KC ? (long)grow * mk->ldmask + gk : (long)gk * mk->ldmask + grow);
    } else {
      r[i] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
}

template <bool KC>
__device__ __forceinline__ void store_tile(char* lds, const uint4 (&r)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + NT * i;
    int off;
    if (KC) {
      const int row = id >> 3, c = id & 7;
      off = row * 128 + ((c ^ ((row >> 1) & 7)) << 4);
    } else {
      const int kr = id >> 4, c = id & 15;
      const int x = (kr & 3) | (((kr >> 3) & 1) << 2);
      off = kr * 256 + ((c ^ (2 * x)) << 4);
    }
    *reinterpret_cast<uint4*>(lds + off) = r[i];
  }
}

// Fragment of a 16-row x 32-k operand block for v_mfma_f32_16x16x32_bf16:
// lane l holds X[row = rb + (l&15)][k = 32s + 8(l>>4) + j], j = 0..7.
template <bool KC>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int rb, int s, int lane) {
  if (KC) {
    const int row = rb + (lane & 15);
    const int c = 4 * s + (lane >> 4);
    const int off = row * 128 + ((c ^ ((row >> 1) & 7)) << 4);
    return *reinterpret_cast<const bf16x8*>(lds + off);
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k1 = 32 * s + 8 * g + q;
    const int m = rb + 4 * p;
    const int c = m >> 3;
    const int x = (k1 & 3) | (((k1 >> 3) & 1) << 2);
    const int off1 = k1 * 256 + ((c ^ (2 * x)) << 4) + (p & 1) * 8;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + off1));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + off1 + 4 * 256));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v;
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <int EPI, typename OutT>
__device__ __forceinline__ void epilogue_elem(const GemmArgs& p, OutT* __restrict__ C, int m, int n, float acc,
                                              bool reduced = false) {
  float v = acc * p.alpha;
  const long ci = (long)m * p.ldc + n;
  if constexpr (EPI == EPI_STORE) {
    if (p.ksplit > 1 && !reduced) {  // split-K: every split adds its partial; split 0 adds the bias
      if (p.bias && blockIdx.y == 0) v += p.bias[n];
      atomicAdd(reinterpret_cast<float*>(C) + ci, v);
      return;
    }
    if (p.bias) v += p.bias[n];
    if (p.accumulate) v += (float)C[ci];
    C[ci] = (OutT)v;
  } else if constexpr (EPI == EPI_GELU) {
    if (p.bias) v += p.bias[n];
    const bf16 hb = (bf16)v;
    float ax;
    const float y = act_fwd<EPI_GELU>((float)hb, p.aux_grad, ax);
    p.aux_out[(long)m * p.ldaux_out + n] = (bf16)ax;
    C[ci] = (OutT)y;
  } else if constexpr (EPI == EPI_RESID_LS) {
    if (p.bias) v += p.bias[n];
    const bf16 yb = (bf16)v;
    if (p.aux_out) p.aux_out[(long)m * p.ldaux_out + n] = yb;
    C[ci] = (OutT)(p.resid[(long)m * p.ldr + n] + p.ls[n] * v);
  } else if constexpr (EPI == EPI_QGELU) {
    if (p.bias) v += p.bias[n];
    const bf16 hb = (bf16)v;
    float ax;
    const float y = act_fwd<EPI_QGELU>((float)hb, p.aux_grad, ax);
    p.aux_out[(long)m * p.ldaux_out + n] = (bf16)ax;
    C[ci] = (OutT)y;
  } else if constexpr (EPI == EPI_QGELU_BWD) {
    const float h = (float)p.aux[(long)m * p.ldaux + n];
    C[ci] = (OutT)(v * act_bwd<EPI_QGELU_BWD>(h, p.aux_grad));
  } else if constexpr (EPI == EPI_GELU_BWD) {
    const float h = (float)p.aux[(long)m * p.ldaux + n];
    C[ci] = (OutT)(v * act_bwd<EPI_GELU_BWD>(h, p.aux_grad));
  } else if constexpr (EPI == EPI_SWIGLU_BWD) {
    const long ai = (long)m * p.ldaux + n;
    const float g = (float)p.aux[ai], u = (float)p.aux[ai + p.N];
    C[ci] = (OutT)(v * u * silu_grad(g));
    C[ci + p.N] = (OutT)(v * silu(g));
  } else if constexpr (EPI == EPI_DROPMASK) {
    v *= epi_keep(p, m, n);
    if (p.accumulate) v += (float)C[ci];
    C[ci] = (OutT)v;
  } else if constexpr (EPI == EPI_DROPMASK_SWIGLU || EPI == EPI_DROPMASK_SWIGLU_B) {
    if (p.drop_p > 0.f) v *= epi_keep(p, m, n);
    const long ri = (long)m * p.ldr + n;
    float d = v;
    if constexpr (EPI == EPI_DROPMASK_SWIGLU_B) d += (float)reinterpret_cast<const bf16*>(p.resid)[ri];
    else d += p.resid[ri];
    const long ai = (long)m * p.ldaux + n;
    const float g = (float)p.aux[ai], u = (float)p.aux[ai + p.N];
    C[ci] = (OutT)(d * u * silu_grad(g));
    C[ci + p.N] = (OutT)(d * silu(g));
  }
}


// 8 consecutive columns n..n+7 of row m (vector path: caller guarantees n+8 <= N and 16-B alignment)
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 x;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = (bf16)v[e];
    *reinterpret_cast<bf16x8*>(p) = x;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

template <int EPI, typename OutT>
__device__ __forceinline__ void epilogue_vec8(const GemmArgs& p, OutT* __restrict__ C, int m, int n, float (&v)[8],
                                              bool reduced = false) {
  const long ci = (long)m * p.ldc + n;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] *= p.alpha;
  if constexpr (EPI == EPI_STORE) {
    if (p.ksplit > 1 && !reduced) {
      if (p.bias && blockIdx.y == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += p.bias[n + e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(reinterpret_cast<float*>(C) + ci + e, v[e]);
      return;
    }
    if (p.bias) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += p.bias[n + e];
    }
    if (p.accumulate) {
      float c[8];
      ld8(C + ci, c);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += c[e];
    }
    st8(C + ci, v);
  } else if constexpr (EPI == EPI_GELU) {
    float h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = (float)(bf16)(v[e] + (p.bias ? p.bias[n + e] : 0.f));
    float ax[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = act_fwd<EPI_GELU>(h[e], p.aux_grad, ax[e]);
    st8(p.aux_out + (long)m * p.ldaux_out + n, ax);
    st8(C + ci, h);
  } else if constexpr (EPI == EPI_RESID_LS) {
    if (p.bias) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += p.bias[n + e];
    }
    if (p.aux_out) st8(p.aux_out + (long)m * p.ldaux_out + n, v);
    float r[8];
    ld8(p.resid + (long)m * p.ldr + n, r);
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] += p.ls[n + e] * v[e];
    st8(C + ci, r);
  } else if constexpr (EPI == EPI_QGELU) {
    float h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = (float)(bf16)(v[e] + (p.bias ? p.bias[n + e] : 0.f));
    float ax[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = act_fwd<EPI_QGELU>(h[e], p.aux_grad, ax[e]);
    st8(p.aux_out + (long)m * p.ldaux_out + n, ax);
    st8(C + ci, h);
  } else if constexpr (EPI == EPI_QGELU_BWD) {
    float h[8];
    ld8(p.aux + (long)m * p.ldaux + n, h);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= act_bwd<EPI_QGELU_BWD>(h[e], p.aux_grad);
    st8(C + ci, v);
  } else if constexpr (EPI == EPI_GELU_BWD) {
    float h[8];
    ld8(p.aux + (long)m * p.ldaux + n, h);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= act_bwd<EPI_GELU_BWD>(h[e], p.aux_grad);
    st8(C + ci, v);
  } else if constexpr (EPI == EPI_SWIGLU_BWD) {
    float g[8], u[8], o[8];
    ld8(p.aux + (long)m * p.ldaux + n, g);
    ld8(p.aux + (long)m * p.ldaux + p.N + n, u);
#pragma unroll
    for (int e = 0; e < 8; ++e) { o[e] = v[e] * u[e] * silu_grad(g[e]); u[e] = v[e] * silu(g[e]); }
    st8(C + ci, o);
    st8(C + ci + p.N, u);
  } else if constexpr (EPI == EPI_DROPMASK_SWIGLU || EPI == EPI_DROPMASK_SWIGLU_B) {
    if (p.drop_p > 0.f) {
      const uint32_t kb = epi_keep8(p, m, n);
      const float sc = 1.0f / (1.0f - p.drop_p);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= (kb >> e) & 1u ? sc : 0.f;
    }
    float r[8], g[8], u[8];
    if constexpr (EPI == EPI_DROPMASK_SWIGLU_B) ld8(reinterpret_cast<const bf16*>(p.resid) + (long)m * p.ldr + n, r);
    else ld8(p.resid + (long)m * p.ldr + n, r);
    ld8(p.aux + (long)m * p.ldaux + n, g);
    ld8(p.aux + (long)m * p.ldaux + p.N + n, u);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[e] + r[e];
      r[e] = d * u[e] * silu_grad(g[e]);
      u[e] = d * silu(g[e]);
    }
    st8(C + ci, r);
    st8(C + ci + p.N, u);
  } else if constexpr (EPI == EPI_DROPMASK) {
    {
      const uint32_t kb = epi_keep8(p, m, n);
      const float sc = 1.0f / (1.0f - p.drop_p);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= (kb >> e) & 1u ? sc : 0.f;
    }
    if (p.accumulate) {
      float c[8];
      ld8(C + ci, c);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += c[e];
    }
    st8(C + ci, v);
  }
}

template <bool AK, bool BKc, int EPI, typename OutT>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * (BM * BK * 2 + BN * BK * 2)];
  const int nwg = p.tilesM * p.tilesN;
  int bid = blockIdx.x;
  {  // bijective XCD remap: blocks b and b+8 share an XCD; give each XCD a contiguous range
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  constexpr int GROUP = 8;
  const int npg = GROUP * p.tilesN;
  const int gid = bid / npg;
  const int fm = gid * GROUP;
  const int gs = min(p.tilesM - fm, GROUP);
  const int tm = fm + (bid % npg) % gs;
  const int tn = (bid % npg) / gs;
  const int m0 = tm * BM, n0 = tn * BN;

  const long z = blockIdx.z;
  const bf16* __restrict__ A = p.A + z * p.sA;
  const bf16* __restrict__ B = p.B + z * p.sB;
  OutT* __restrict__ C = reinterpret_cast<OutT*>(p.C) + z * p.sC;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int kbeg = 0, kend = p.K;
  if (p.ksplit > 1) {
    kbeg = blockIdx.y * p.kchunk;
    kend = min(p.K, kbeg + p.kchunk);
  }
  const int nk = (kend - kbeg + BK - 1) / BK;
  char* As0 = smem;
  char* Bs0 = smem + BM * BK * 2;
  constexpr int STAGE = BM * BK * 2 + BN * BK * 2;

  uint4 ra[4], rb[4];
  LoadMask mk{p.seed, p.drop_p, p.ldmask};
  const LoadMask* mka = p.drop_operand == 1 ? &mk : nullptr;
  const LoadMask* mkb = p.drop_operand == 2 ? &mk : nullptr;
  load_tile<AK>(A, p.lda, m0, p.M, kbeg, kend, ra, mka);
  load_tile<BKc>(B, p.ldb, n0, p.N, kbeg, kend, rb, mkb);
  store_tile<AK>(As0, ra);
  store_tile<BKc>(Bs0, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const char* As = As0 + cur * STAGE;
    const char* Bs = Bs0 + cur * STAGE;
    if (kt + 1 < nk) {
      load_tile<AK>(A, p.lda, m0, p.M, kbeg + (kt + 1) * BK, kend, ra, mka);
      load_tile<BKc>(B, p.ldb, n0, p.N, kbeg + (kt + 1) * BK, kend, rb, mkb);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<AK>(As, wm * 64 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<BKc>(Bs, wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      store_tile<AK>(As0 + (cur ^ 1) * STAGE, ra);
      store_tile<BKc>(Bs0 + (cur ^ 1) * STAGE, rb);
    }
    __syncthreads();
  }

  // C/D layout of 16x16x32: col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wn * 64 + j * 16 + (lane & 15);
        if (m < p.M && n < p.N) epilogue_elem<EPI, OutT>(p, C, m, n, acc[i][j][r]);
      }
}

// ---------------------------------------------------------------------------------------------
// v2 main loop: LDS-DMA (buffer_load_dwordx4 ... lds) ring of NS stages, counted vmcnt, one raw
// s_barrier per K-step. Each wave-instruction writes 1 KiB of LDS lane-linearly, so the XOR
// swizzles of v1 are applied to the per-lane SOURCE address (the LDS images are identical to v1's,
// and so are the fragment reads). Rows outside the matrix get a sentinel offset beyond the buffer
// descriptor's num_records -> the hardware returns zeros. Tile BM x 128 (BM = 128 or 256), waves
// (BM/64) x 2, each 64x64. Requirements: K-contiguous operands need K % 64 == 0 (else v1).
constexpr unsigned kSent = 0x7FFFFFF0u;
constexpr int EP_LD = 68;  // epilogue staging row stride (floats)

template <bool KC, int ROWS>
struct DmaOperand {
  // per-lane precomputed element offsets of the LOADS this wave issues for one stage
  static constexpr int BYTES = ROWS * BK * 2;       // per stage
  static constexpr int INSTR = BYTES / 1024;         // wave-instructions per stage (whole block)
};

template <bool KC, int ROWS, int NW>
__device__ __forceinline__ void dma_setup(int lane, int wave, int r0, int rows_total, long ld, long (&base)[ROWS * BK * 2 / 1024 / NW],
                                          int (&kr)[ROWS * BK * 2 / 1024 / NW], bool (&ok)[ROWS * BK * 2 / 1024 / NW]) {
  constexpr int PER = ROWS * BK * 2 / 1024 / NW;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int o = (wave * PER + i) * 1024 + lane * 16;
    if (KC) {
      const int row = o >> 7, pc = (o >> 4) & 7;
      const int c = pc ^ ((row >> 1) & 7);
      ok[i] = r0 + row < rows_total;
      base[i] = (long)(r0 + row) * ld + 8 * c;
      kr[i] = 0;
    } else {
      const int panel = o >> 14, o2 = o & 16383;
      const int k = o2 >> 8, pc = (o2 >> 4) & 15;
      const int x = (k & 3) | (((k >> 3) & 1) << 2);
      const int c = pc ^ (2 * x);
      const int col = r0 + panel * 128 + 8 * c;
      ok[i] = col < rows_total;
      base[i] = (long)k * ld + col;
      kr[i] = k;
    }
  }
}

template <bool KC, int ROWS, int NW>
__device__ __forceinline__ void dma_issue(__amdgpu_buffer_rsrc_t rs, char* lds_tile, int wave, int k0, int K, long ld,
                                          const long (&base)[ROWS * BK * 2 / 1024 / NW],
                                          const int (&kr)[ROWS * BK * 2 / 1024 / NW],
                                          const bool (&ok)[ROWS * BK * 2 / 1024 / NW]) {
  constexpr int PER = ROWS * BK * 2 / 1024 / NW;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    unsigned off;
    if (KC) off = ok[i] ? (unsigned)((base[i] + k0) * 2) : kSent;
    else off = (ok[i] && k0 + kr[i] < K) ? (unsigned)((base[i] + (long)k0 * ld) * 2) : kSent;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds_tile + (wave * PER + i) * 1024),
                                             16, off, 0, 0, 0);
  }
}

// fragment read from a tile made of 128-row panels
template <bool KC>
__device__ __forceinline__ bf16x8 read_frag_p(const char* lds, int rb, int s, int lane) {
  if (KC) return read_frag<true>(lds, rb, s, lane);
  return read_frag<false>(lds + (rb >> 7) * 16384, rb & 127, s, lane);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 18) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}

// LDS-staged epilogue of one 64x64 f32 sub-tile held in `ep` (row stride EP_LD), rows m_base.., cols n_base..
// Fused LM head + CE epilogues on one 64 x 64 f32 sub-tile of logits (rows = loss rows, columns = vocabulary).
// Lane: 8 columns (lane & 7) of row (lane >> 3) + 8 pass. CE_PART: the row's (max, sum exp(x - max)) over the
// sub-tile's valid columns, combined over the 8 lanes of a row with xor shuffles, and the label logit where the
// label falls; CE_GRAD: dlogits = (exp(x - lse) - [n == label]) * gscale in bf16, zero for ignored rows and for
// the padded columns past V (the dgrad GEMM reads them).
template <int EPI>
__device__ __forceinline__ void ce_tile64(const GemmArgs& p, const float* ep, int lane, int m_base, int n_base) {
  const int cc = (lane & 7) * 8, n = n_base + cc;
  const float g = EPI == EPI_CE_GRAD ? *p.ce_gscale : 0.f;
#pragma unroll 2
  for (int pass = 0; pass < 8; ++pass) {
    const int row = pass * 8 + (lane >> 3);
    const int m = m_base + row;
    const bool mok = m < p.M;
    const int lab = mok ? p.ce_labels[m] : -1;
    float v[8];
    const float4 a0 = *reinterpret_cast<const float4*>(ep + row * EP_LD + cc);
    const float4 a1 = *reinterpret_cast<const float4*>(ep + row * EP_LD + cc + 4);
    v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
    if constexpr (EPI == EPI_CE_PART) {
      float mx = -INFINITY;
#pragma unroll
      for (int e = 0; e < 8; ++e) mx = n + e < p.N ? fmaxf(mx, v[e]) : mx;
      float sm = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) sm += n + e < p.N ? __expf(v[e] - mx) : 0.f;
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {
        const float m2 = __shfl_xor(mx, o, 64), s2 = __shfl_xor(sm, o, 64);
        const float mm = fmaxf(mx, m2);
        sm = (mx == -INFINITY ? 0.f : sm * __expf(mx - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
        mx = mm;
      }
      if (mok && (lane & 7) == 0)
        *reinterpret_cast<float2*>(p.ce_part + ((long)m * p.ce_ldpart + n_base / 64) * 2) = make_float2(mx, sm);
      if (mok && lab >= n && lab < n + 8) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (lab == n + e) p.ce_lab[m] = v[e];
      }
    } else {
      if (!mok) continue;
      const float lse = p.ce_lse[m];
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = (lab >= 0 && n + e < p.N) ? (__expf(v[e] - lse) - (n + e == lab ? 1.f : 0.f)) * g : 0.f;
        o[e] = (bf16)t;
      }
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(p.C) + (long)m * p.ldc + n) = o;
    }
  }
}

template <int EPI, typename OutT>
__device__ __forceinline__ void epilogue_tile64(const GemmArgs& p, OutT* __restrict__ C, const float* ep, int lane,
                                                int m_base, int n_base, bool reduced = false) {
  if constexpr (EPI == EPI_CE_PART || EPI == EPI_CE_GRAD) {
    ce_tile64<EPI>(p, ep, lane, m_base, n_base);
    return;
  }
  if constexpr (EPI == EPI_STORE) {
    if (p.ksplit > 1 && !reduced) {  // split-K partials: one 64-float row (256 contiguous bytes) per atomic wave-instruction
      const int n1 = n_base + lane;
      const float bv = (p.bias && blockIdx.y == 0 && n1 < p.N) ? p.bias[n1] : 0.f;
      float* Cf = reinterpret_cast<float*>(C);
      if (p.split_stride) {  // partials mode: plain stores, summed by the caller's next kernel
        float* Cy = Cf + (long)blockIdx.y * p.split_stride;
        for (int row = 0; row < 64; ++row) {
          const int m = m_base + row;
          if (m < p.M && n1 < p.N) Cy[(long)m * p.ldc + n1] = ep[row * EP_LD + lane] * p.alpha + bv;
        }
        return;
      }
      for (int row = 0; row < 64; ++row) {
        const int m = m_base + row;
        if (m < p.M && n1 < p.N) atomicAdd(Cf + (long)m * p.ldc + n1, ep[row * EP_LD + lane] * p.alpha + bv);
      }
      return;
    }
  }
  const int cc = (lane & 7) * 8;
  const int n = n_base + cc;
  const bool vec_ok = p.vec_ok && n + 8 <= p.N;
  if constexpr (EPI == EPI_STORE && sizeof(OutT) == 2) {
    if (p.rope_cos && n_base < p.rope_ncols && p.vec_ok && n_base + 64 <= p.N) {  // wave-uniform: one 64-wide head
      // y = alpha*acc + bias, then the head's dims d / d + 32 rotated as a pair: lane octet (lane & 7) holds 8
      // consecutive columns, the partner half is lane ^ 4 of the same row (rope_pair of slx_rope, forward)
      const int d32 = cc & 31;
      const float sg = cc < 32 ? -1.f : 1.f;
      float bv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[e] = p.bias ? p.bias[n + e] : 0.f;
#pragma unroll 2
      for (int pass = 0; pass < 8; ++pass) {
        const int row = pass * 8 + (lane >> 3);
        const int m = min(m_base + row, p.M - 1);  // (rows past M: computed, not stored - the shuffles need the lanes)
        float v[8], w[8];
        const float4 a0 = *reinterpret_cast<const float4*>(ep + row * EP_LD + cc);
        const float4 a1 = *reinterpret_cast<const float4*>(ep + row * EP_LD + cc + 4);
        v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = v[e] * p.alpha + bv[e];
#pragma unroll
        for (int e = 0; e < 8; ++e) w[e] = __shfl_xor(v[e], 4, 64);
        const long tb = (long)(m % p.rope_S) * 32 + d32;
        const float4 c0 = *reinterpret_cast<const float4*>(p.rope_cos + tb), c1 = *reinterpret_cast<const float4*>(p.rope_cos + tb + 4);
        const float4 s0 = *reinterpret_cast<const float4*>(p.rope_sin + tb), s1 = *reinterpret_cast<const float4*>(p.rope_sin + tb + 4);
        const float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = v[e] * cv[e] + sg * w[e] * sv[e];
        if (m_base + row < p.M) st8(C + (long)m * p.ldc + n, o);
      }
      return;
    }
  }
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int pass = 0; pass < 8; ++pass) {
    const int row = pass * 8 + (lane >> 3);
    const int m = m_base + row;
    if (m >= p.M) continue;
    float v[8];
    const float4 a0 = *reinterpret_cast<const float4*>(ep + row * EP_LD + cc);
    const float4 a1 = *reinterpret_cast<const float4*>(ep + row * EP_LD + cc + 4);
    v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
    if (vec_ok) {
      epilogue_vec8<EPI, OutT>(p, C, m, n, v, reduced);
      if constexpr (EPI == EPI_STORE || EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[e] += v[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (n + e < p.N) epilogue_elem<EPI, OutT>(p, C, m, n + e, v[e], reduced);
    }
  }
  if constexpr (EPI == EPI_STORE || EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
    // bias gradient: the 8 lanes sharing columns (lane & 7) hold partials of 8 rows each -> 3 xor-shuffles
    if (p.colsum) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[e] += __shfl_xor(cs[e], 8, 64);
        cs[e] += __shfl_xor(cs[e], 16, 64);
        cs[e] += __shfl_xor(cs[e], 32, 64);
      }
      if (lane < 8 && vec_ok && m_base < p.M) {  // partial row of this 64-row subtile (reduced after the GEMM)
        float* w = p.colsum_ws + (long)(p.colsum_row0 + m_base / 64) * p.N + n;
        *reinterpret_cast<float4*>(w) = make_float4(cs[0], cs[1], cs[2], cs[3]);
        *reinterpret_cast<float4*>(w + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
      }
    }
  }
}

// ---- prefetching vector epilogue ------------------------------------------------------------------------------
// The row loop above finishes one row per lane-octet at a time (2 unrolled), so an epilogue that reads global data
// (the GELU'/SwiGLU' aux, the layer-scale residual, an accumulated C) pays one dependent load round trip per 2 rows:
// 4 round trips per 64x64 sub-tile while the CU's MFMAs idle. Here every global load of a batch of rows (all 8 rows
// of the lane, or 4 when a row needs more than 2 x 16 B) is issued first, then the rows are finished. Invalid rows
// (past M) load a clamped row and are never stored, so the loads need no branch (a branch around each load makes
// hipcc wait vmcnt(0) per row, cdna_hip_programming.md §5 'Three .s-level traps' (c)).
template <int EPI, typename OutT> struct EpiLd { static constexpr int N = 0; };
template <typename OutT> struct EpiLd<EPI_STORE, OutT> { static constexpr int N = sizeof(OutT) == 4 ? 2 : 1; };  // accumulate
template <typename OutT> struct EpiLd<EPI_RESID_LS, OutT> { static constexpr int N = 2; };
template <typename OutT> struct EpiLd<EPI_GELU_BWD, OutT> { static constexpr int N = 1; };
template <typename OutT> struct EpiLd<EPI_QGELU_BWD, OutT> { static constexpr int N = 1; };
template <typename OutT> struct EpiLd<EPI_SWIGLU_BWD, OutT> { static constexpr int N = 2; };
template <typename OutT> struct EpiLd<EPI_DROPMASK_SWIGLU, OutT> { static constexpr int N = 5; };    // resid f32 x2, g, u, bits
template <typename OutT> struct EpiLd<EPI_DROPMASK_SWIGLU_B, OutT> { static constexpr int N = 4; };  // resid bf16, g, u, bits

__device__ __forceinline__ void unpack_bf8(uint4 u, float (&f)[8]) {
  const bf16x8 x = __builtin_bit_cast(bf16x8, u);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = (float)x[e];
}
__device__ __forceinline__ void unpack_f8(uint4 a, uint4 b, float (&f)[8]) {
  f[0] = __uint_as_float(a.x); f[1] = __uint_as_float(a.y); f[2] = __uint_as_float(a.z); f[3] = __uint_as_float(a.w);
  f[4] = __uint_as_float(b.x); f[5] = __uint_as_float(b.y); f[6] = __uint_as_float(b.z); f[7] = __uint_as_float(b.w);
}

template <int EPI, typename OutT, int NL>
__device__ __forceinline__ void epi_issue(const GemmArgs& p, const OutT* C, int m, int n, uint4 (&L)[NL]) {
  if constexpr (EPI == EPI_STORE) {
    const uint4* q = reinterpret_cast<const uint4*>(C + (long)m * p.ldc + n);
    L[0] = q[0];
    if constexpr (NL == 2) L[1] = q[1];
  } else if constexpr (EPI == EPI_RESID_LS) {
    const uint4* q = reinterpret_cast<const uint4*>(p.resid + (long)m * p.ldr + n);
    L[0] = q[0];
    L[1] = q[1];
  } else if constexpr (EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
    L[0] = *reinterpret_cast<const uint4*>(p.aux + (long)m * p.ldaux + n);
  } else if constexpr (EPI == EPI_SWIGLU_BWD) {
    L[0] = *reinterpret_cast<const uint4*>(p.aux + (long)m * p.ldaux + n);
    L[1] = *reinterpret_cast<const uint4*>(p.aux + (long)m * p.ldaux + p.N + n);
  } else if constexpr (EPI == EPI_DROPMASK_SWIGLU || EPI == EPI_DROPMASK_SWIGLU_B) {
    constexpr int R = EPI == EPI_DROPMASK_SWIGLU ? 2 : 1;  // resid words
    if constexpr (R == 2) {
      const uint4* q = reinterpret_cast<const uint4*>(p.resid + (long)m * p.ldr + n);
      L[0] = q[0];
      L[1] = q[1];
    } else {
      L[0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p.resid) + (long)m * p.ldr + n);
    }
    L[R] = *reinterpret_cast<const uint4*>(p.aux + (long)m * p.ldaux + n);
    L[R + 1] = *reinterpret_cast<const uint4*>(p.aux + (long)m * p.ldaux + p.N + n);
    // the keep-bit word (stored bits) - loaded unconditionally from a valid address, used only with maskbits
    const uint32_t* bw = p.maskbits ? p.maskbits + (long)m * p.ldbits + (n >> 5) : reinterpret_cast<const uint32_t*>(p.aux);
    L[R + 2].x = *bw;
  }
}

// epilogue_vec8 with the row's global inputs already in L (same arithmetic, same rounding points)
template <int EPI, typename OutT, int NL, bool LD>
__device__ __forceinline__ void epi_finish(const GemmArgs& p, OutT* __restrict__ C, int m, int n, float (&v)[8],
                                           const uint4 (&L)[NL]) {
  const long ci = (long)m * p.ldc + n;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] *= p.alpha;
  if constexpr (EPI == EPI_STORE) {
    if (p.bias) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += p.bias[n + e];
    }
    if constexpr (LD) {
      float c[8];
      if constexpr (NL == 2) unpack_f8(L[0], L[1], c);
      else unpack_bf8(L[0], c);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += c[e];
    }
    st8(C + ci, v);
  } else if constexpr (EPI == EPI_GELU || EPI == EPI_QGELU) {
    float h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = (float)(bf16)(v[e] + (p.bias ? p.bias[n + e] : 0.f));
    float ax[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = act_fwd<EPI>(h[e], p.aux_grad, ax[e]);
    st8(p.aux_out + (long)m * p.ldaux_out + n, ax);
    st8(C + ci, h);
  } else if constexpr (EPI == EPI_RESID_LS) {
    if (p.bias) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += p.bias[n + e];
    }
    if (p.aux_out) st8(p.aux_out + (long)m * p.ldaux_out + n, v);
    float r[8];
    unpack_f8(L[0], L[1], r);
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] += p.ls[n + e] * v[e];
    st8(C + ci, r);
  } else if constexpr (EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
    float h[8];
    unpack_bf8(L[0], h);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= act_bwd<EPI>(h[e], p.aux_grad);
    st8(C + ci, v);
  } else if constexpr (EPI == EPI_SWIGLU_BWD) {
    float g[8], u[8], o[8];
    unpack_bf8(L[0], g);
    unpack_bf8(L[1], u);
#pragma unroll
    for (int e = 0; e < 8; ++e) { o[e] = v[e] * u[e] * silu_grad(g[e]); u[e] = v[e] * silu(g[e]); }
    st8(C + ci, o);
    st8(C + ci + p.N, u);
  } else if constexpr (EPI == EPI_DROPMASK_SWIGLU || EPI == EPI_DROPMASK_SWIGLU_B) {
    constexpr int R = EPI == EPI_DROPMASK_SWIGLU ? 2 : 1;
    if (p.drop_p > 0.f) {
      const uint32_t kb = p.maskbits ? (L[R + 2].x >> (n & 31)) & 0xFFu : epi_keep8(p, m, n);
      const float sc = 1.0f / (1.0f - p.drop_p);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= (kb >> e) & 1u ? sc : 0.f;
    }
    float r[8], g[8], u[8];
    if constexpr (R == 2) unpack_f8(L[0], L[1], r);
    else unpack_bf8(L[0], r);
    unpack_bf8(L[R], g);
    unpack_bf8(L[R + 1], u);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[e] + r[e];
      r[e] = d * u[e] * silu_grad(g[e]);
      u[e] = d * silu(g[e]);
    }
    st8(C + ci, r);
    st8(C + ci + p.N, u);
  }
}

template <int EPI, typename OutT, bool LD>
__device__ __forceinline__ void epilogue_tile64_pf_impl(const GemmArgs& p, OutT* __restrict__ C, const float* ep, int lane,
                                                        int m_base, int n_base) {
  constexpr int NL = LD ? EpiLd<EPI, OutT>::N : 1;
  constexpr int PF = NL <= 2 ? 8 : 4;
  const int cc = (lane & 7) * 8;
  const int n = n_base + cc;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < 8; b += PF) {
    uint4 L[PF][NL];
    if constexpr (LD) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int m = m_base + (b + q) * 8 + (lane >> 3);
        epi_issue<EPI, OutT, NL>(p, C, m < p.M ? m : p.M - 1, n, L[q]);
      }
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int row = (b + q) * 8 + (lane >> 3);
      const int m = m_base + row;
      float v[8];
      const float4 a0 = *reinterpret_cast<const float4*>(ep + row * EP_LD + cc);
      const float4 a1 = *reinterpret_cast<const float4*>(ep + row * EP_LD + cc + 4);
      v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
      if (m < p.M) {
        epi_finish<EPI, OutT, NL, LD>(p, C, m, n, v, L[q]);
        if constexpr (EPI == EPI_STORE || EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[e] += v[e];
        }
      }
    }
  }
  if constexpr (EPI == EPI_STORE || EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
    if (p.colsum) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[e] += __shfl_xor(cs[e], 8, 64);
        cs[e] += __shfl_xor(cs[e], 16, 64);
        cs[e] += __shfl_xor(cs[e], 32, 64);
      }
      if (lane < 8 && m_base < p.M) {
        float* w = p.colsum_ws + (long)(p.colsum_row0 + m_base / 64) * p.N + n;
        *reinterpret_cast<float4*>(w) = make_float4(cs[0], cs[1], cs[2], cs[3]);
        *reinterpret_cast<float4*>(w + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
      }
    }
  }
}

// The 64x64 sub-tile epilogue with batched global loads where the epilogue kind allows it, else epilogue_tile64.
template <int EPI, typename OutT>
__device__ __forceinline__ void epilogue_tile64_pf(const GemmArgs& p, OutT* __restrict__ C, const float* ep, int lane,
                                                   int m_base, int n_base, bool reduced = false) {
  constexpr bool kPf = EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_QGELU || EPI == EPI_RESID_LS ||
                       EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD || EPI == EPI_SWIGLU_BWD ||
                       EPI == EPI_DROPMASK_SWIGLU || EPI == EPI_DROPMASK_SWIGLU_B;
  if constexpr (kPf) {
    const bool whole = p.vec_ok && n_base + 64 <= p.N && !(EPI == EPI_STORE && p.ksplit > 1 && !reduced) &&
                       !(EPI == EPI_STORE && p.rope_cos);  // wave-uniform (RoPE: epilogue_tile64's row loop)
    if (whole) {
      if constexpr (EPI == EPI_GELU || EPI == EPI_QGELU) {
        epilogue_tile64_pf_impl<EPI, OutT, false>(p, C, ep, lane, m_base, n_base);
      } else if constexpr (EPI == EPI_STORE) {
        if (p.accumulate) epilogue_tile64_pf_impl<EPI, OutT, true>(p, C, ep, lane, m_base, n_base);
        else epilogue_tile64_pf_impl<EPI, OutT, false>(p, C, ep, lane, m_base, n_base);
      } else {
        epilogue_tile64_pf_impl<EPI, OutT, true>(p, C, ep, lane, m_base, n_base);
      }
      return;
    }
  }
  epilogue_tile64<EPI, OutT>(p, C, ep, lane, m_base, n_base, reduced);
}

// The staged-tile epilogue of the v2 / v3 kernels: the batched-load form for the residual and SwiGLU' kinds (their
// per-row load round trips were the tail of the single-round residual GEMMs: +0.35 % on the VLA step), the row loop for
// the others. Through the batched form the Qwen2 down / gate-up data-gradient GEMMs (plain STORE) ran 4-15 % slower and
// SimLingo-Base's accumulating f32 weight-gradient GEMMs 22 % slower (profiles/round5_gemm_pf_epilogue_ab.txt).
template <int EPI, typename OutT>
__device__ __forceinline__ void epilogue_tile64_auto(const GemmArgs& p, OutT* __restrict__ C, const float* ep, int lane,
                                                     int m_base, int n_base, bool reduced = false) {
  if constexpr (EPI == EPI_RESID_LS || EPI == EPI_SWIGLU_BWD || EPI == EPI_DROPMASK_SWIGLU ||
                EPI == EPI_DROPMASK_SWIGLU_B)
    epilogue_tile64_pf<EPI, OutT>(p, C, ep, lane, m_base, n_base, reduced);
  else
    epilogue_tile64<EPI, OutT>(p, C, ep, lane, m_base, n_base, reduced);
}

template <bool AK, bool BKc, int EPI, typename OutT, int BMv, int NS>
__global__ __launch_bounds__(BMv * 2, 1) void gemm_bf16_dma_kernel(GemmArgs p) {
  constexpr int NW = BMv / 32;                 // waves: (BM/64) x 2
  constexpr int A_BYTES = BMv * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int LPW = (A_BYTES + B_BYTES) / 1024 / NW;   // DMA instructions per wave per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tilesM = p.tilesM, tilesN = p.tilesN;
  const int nwg = tilesM * tilesN;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  constexpr int GROUP = 8;
  const int npg = GROUP * tilesN;
  const int gid = bid / npg;
  const int fm = gid * GROUP;
  const int gs = min(tilesM - fm, GROUP);
  const int tm = fm + (bid % npg) % gs;
  const int tn = (bid % npg) / gs;
  const int m0 = tm * BMv, n0 = tn * BN;
  const long z = blockIdx.z;
  const bf16* A = p.A + z * p.sA;
  const bf16* B = p.B + z * p.sB;
  OutT* __restrict__ C = reinterpret_cast<OutT*>(p.C) + z * p.sC;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  int kbeg = 0, kend = p.K;
  if (p.ksplit > 1) {
    kbeg = blockIdx.y * p.kchunk;
    kend = min(p.K, kbeg + p.kchunk);
  }
  const int nk = (kend - kbeg + BK - 1) / BK;
  // buffer descriptors over each operand's exact extent (OOB -> 0)
  const long extA = AK ? ((long)(p.M - 1) * p.lda + p.K) : ((long)(p.K - 1) * p.lda + p.M);
  const long extB = BKc ? ((long)(p.N - 1) * p.ldb + p.K) : ((long)(p.K - 1) * p.ldb + p.N);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)(extA * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)(extB * 2), 0x00020000);
  constexpr int PA = A_BYTES / 1024 / NW, PB = B_BYTES / 1024 / NW;
  long baseA[PA], baseB[PB];
  int krA[PA], krB[PB];
  bool okA[PA], okB[PB];
  dma_setup<AK, BMv, NW>(lane, wave, m0, p.M, p.lda, baseA, krA, okA);
  dma_setup<BKc, BN, NW>(lane, wave, n0, p.N, p.ldb, baseB, krB, okB);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int st = 0; st < NS - 1; ++st) {
    if (st < nk) {
      char* sl = smem + st * STAGE;
      dma_issue<AK, BMv, NW>(ra, sl, wave, kbeg + st * BK, kend, p.lda, baseA, krA, okA);
      dma_issue<BKc, BN, NW>(rb, sl + A_BYTES, wave, kbeg + st * BK, kend, p.ldb, baseB, krB, okB);
    }
  }
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed for this wave: newer stages may stay in flight
    const int newer = min(NS - 2, nk - 1 - kt);
    if constexpr (NS >= 3) {
      if (newer >= 1) wait_vm<LPW * (NS - 2)>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NS - 1 < nk) {
      char* sl = smem + ((kt + NS - 1) % NS) * STAGE;
      dma_issue<AK, BMv, NW>(ra, sl, wave, kbeg + (kt + NS - 1) * BK, kend, p.lda, baseA, krA, okA);
      dma_issue<BKc, BN, NW>(rb, sl + A_BYTES, wave, kbeg + (kt + NS - 1) * BK, kend, p.ldb, baseB, krB, okB);
    }
    const char* As = smem + (kt % NS) * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag_p<AK>(As, wm * 64 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag_p<BKc>(Bs, wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  // ---- epilogue: stage the wave's 64x64 f32 tile in LDS (row stride 68 floats: conflict-free
  // writes), then every lane finishes 8 consecutive columns of a row with 16-B loads/stores.
  __syncthreads();
  float* ep = reinterpret_cast<float*>(smem) + wave * (64 * EP_LD);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) ep[(i * 16 + (lane >> 4) * 4 + r) * EP_LD + j * 16 + (lane & 15)] = acc[i][j][r];
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done (wave-private region)
  // the batched-load epilogue where the epilogue reads global data (the Qwen2 o / down residual GEMMs' per-row load
  // round trips were the tail of their single round)
  epilogue_tile64_auto<EPI, OutT>(p, C, ep, lane, m0 + wm * 64, n0 + wn * 64);
}

// ---------------------------------------------------------------------------------------------
// v3 main loop: 256x256 tile, BK=64, 512 threads = 8 waves as 2 (M) x 4 (N), each wave 128x64
// (8x4 tiles of v_mfma_f32_16x16x32_bf16). LDS = 2 stages x (A 32 KiB + B 32 KiB), filled by LDS-DMA.
// The per-wave tile halves the LDS read bytes per MFMA of v2 (64x64 waves), which is what caps v2.
//
// Ping-pong: waves 0-3 (M half 0) and 4-7 (M half 1) are offset by one s_barrier, so one SIMD's two
// waves alternate between a LOAD section (ds_reads of the next fragments + a slice of the DMA
// prefetch) and an MFMA section (16 MFMAs = one 64x32 quadrant of the wave tile x K=64, at raised
// priority). Every K-tile t is 4 phases:
//   q0: read A[rows 0-63], B[cols 0-31] of tile t  | issue B pieces 0,1 of tile t+1 | MFMA (lo,lo)
//   q1: read A[rows 64-127], B[cols 32-63]         | issue B pieces 2,3 of tile t+1 | MFMA (lo,hi)
//   q2:                                            | issue A pieces 0,1 of tile t+2 | MFMA (hi,lo)
//   q3:                           vmcnt(tile t+1)  | issue A pieces 2,3 of tile t+2 | MFMA (hi,hi)
// Stage t&1 is last read in q1 (the load sections end with lgkmcnt(0) before their barrier, so the
// reads are retired before the other group can pass that barrier and issue its q2 DMA into the same
// stage). The wait for tile t+1 sits at the end of q3's load section, before the barrier that
// precedes the leading group's first read of it; only tile t+2's 4 newest pieces stay in flight.
constexpr int V3_BM = 256, V3_BN = 256;

template <bool KC, int ROWS, int NW, int I0, int CNT>
__device__ __forceinline__ void dma_issue_range(__amdgpu_buffer_rsrc_t rs, char* lds_tile, int wave, int k0, int K,
                                                long ld, const long (&base)[ROWS * BK * 2 / 1024 / NW],
                                                const int (&kr)[ROWS * BK * 2 / 1024 / NW],
                                                const bool (&ok)[ROWS * BK * 2 / 1024 / NW]) {
  constexpr int PER = ROWS * BK * 2 / 1024 / NW;
#pragma unroll
  for (int i = I0; i < I0 + CNT; ++i) {
    unsigned off;
    if (KC) off = ok[i] ? (unsigned)((base[i] + k0) * 2) : kSent;
    else off = (ok[i] && k0 + kr[i] < K) ? (unsigned)((base[i] + (long)k0 * ld) * 2) : kSent;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds_tile + (wave * PER + i) * 1024),
                                             16, off, 0, 0, 0);
  }
}

__device__ __forceinline__ void v3_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <bool AK, bool BKc>
__device__ __forceinline__ void v3_read(const char* As, const char* Bs, int arow, int bcol, int lane, bf16x8 (&af)[4][2],
                                        bf16x8 (&bfr)[2][2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[j][s] = read_frag_p<BKc>(Bs, bcol + 16 * j, s, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i][s] = read_frag_p<AK>(As, arow + 16 * i, s, lane);
  }
}

// SW: operands swapped (B fragment as the MFMA's A), so each 16x16 accumulator holds C^T: lane l has
// C[m = l & 15][n = 4 (l >> 4) + r], four consecutive columns of one row (one 16-B LDS store per block).
template <bool SW>
__device__ __forceinline__ void v3_mfma(f32x4 (&acc)[8][4], int mh, int nh, const bf16x8 (&af)[4][2],
                                        const bf16x8 (&bfr)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (SW)
          acc[4 * mh + i][2 * nh + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][s], af[i][s], acc[4 * mh + i][2 * nh + j], 0, 0, 0);
        else
          acc[4 * mh + i][2 * nh + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bfr[j][s], acc[4 * mh + i][2 * nh + j], 0, 0, 0);
      }
  __builtin_amdgcn_s_setprio(0);
}

// XCD-bijective block order: blocks dealt round-robin over the 8 XCDs get contiguous tile ranges per XCD
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// In-launch split-K reduction of one v3 tile (f32 STORE, ksplit = S > 1), replacing S x 256 KiB of f32 atomics per
// tile: with every block of a weight-gradient launch reaching its epilogue together, the atomics ran as one burst at
// the ~1.3 TB/s chip-wide atomic rate (MI355X_MICROARCH.md 'Global float atomics': ~52 us per InternViT fc pair).
// Arrive-first protocol (cdna_hip_programming.md §5 'In-launch split-K reduction', Guideline 16): a block first
// takes an arrival ticket; the first S - 1 arrivals store their partial as a slab (plain 16-B stores in register
// order: one KiB per wave-instruction), then release (agent fence) and bump the tile's published counter; the LAST
// arrival waits on that counter - only for blocks that have already arrived, so the wait cannot deadlock whatever
// the residency - acquires (agent fence), adds the slabs to its own accumulators in split order (bit-identical
// for any arrival order) and runs the ordinary epilogue once. It also resets both counters for the next launch.
// Returns false for the blocks whose partial went to a slab (their tile is done).
template <int S>
__device__ __forceinline__ void v3_split_sum(const float* slabs, int y, f32x4 (&acc)[8][4], int wave, int lane) {
  // total = ((part_0 + part_1) + part_2) + ... with this block's own partial (part_y) in its place; every slot is
  // loaded (this block's own slot holds stale data and is never selected): no branch around a load
  constexpr int CH = S == 2 ? 4 : 2;  // 16-B chunks in flight per slab (<= 32 VGPRs of loads: the accumulators are live)
#pragma unroll
  for (int c0 = 0; c0 < 32; c0 += CH) {
    f32x4 sl[CH][S];
#pragma unroll
    for (int u = 0; u < CH; ++u)
#pragma unroll
      for (int yy = 0; yy < S; ++yy)
        sl[u][yy] = *reinterpret_cast<const f32x4*>(slabs + (long)yy * 65536 + (((c0 + u) * 8 + wave) * 64 + lane) * 4);
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      f32x4& a = acc[(c0 + u) >> 2][(c0 + u) & 3];
      f32x4 r = y == 0 ? a : sl[u][0];
#pragma unroll
      for (int yy = 1; yy < S; ++yy) r = r + (yy == y ? a : sl[u][yy]);
      a = r;
    }
  }
}

__device__ __forceinline__ bool v3_split_reduce(const GemmArgs& p, int tile, f32x4 (&acc)[8][4], int* role_lds,
                                                int wave, int lane, int y) {
  const int S = p.ksplit;
  const int t = p.split_tile0 + tile;
  int* arrive = p.split_cnt + 2 * t;
  int* pub = arrive + 1;
  float* slabs = p.split_ws + (long)t * S * 65536;
  if (threadIdx.x == 0) *role_lds = __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int role = *reinterpret_cast<volatile int*>(role_lds);
  if (role < S - 1) {
    float* slab = slabs + (long)y * 65536;
#pragma unroll
    for (int c = 0; c < 32; ++c)
      *reinterpret_cast<f32x4*>(slab + ((c * 8 + wave) * 64 + lane) * 4) = acc[c >> 2][c & 3];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keep: ROCm 7.2 can drop the fence's own wait
      __hip_atomic_fetch_add(pub, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return false;
  }
  if (threadIdx.x == 0) {
    // every other split has arrived (this block drew the last ticket), so each of them is resident and already past
    // its ticket: all S - 1 publish unconditionally and this wait ends without a bound. A bounded wait that fell
    // through would sum unwritten slabs and leave a nonzero counter for the next launch on this workspace.
    while (__hip_atomic_load(pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < S - 1) __builtin_amdgcn_s_sleep(2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(pub, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (S == 2) v3_split_sum<2>(slabs, y, acc, wave, lane);
  else if (S == 3) v3_split_sum<3>(slabs, y, acc, wave, lane);
  else v3_split_sum<4>(slabs, y, acc, wave, lane);
  return true;
}

// Tile origin of tile index bid (after the XCD remap): GROUP = 4 row tiles x all column tiles per group.
// mshift_last: the partial last M tile is shifted up to end at M, so every tile is full; the rows it shares with
// the previous tile are recomputed bit-identically (same K order) and stored twice with the same values.
__device__ __forceinline__ void v3_origin(const GemmArgs& p, int bid, int& m0, int& n0) {
  constexpr int GROUP = 4;
  const int npg = GROUP * p.tilesN;
  const int fm = (bid / npg) * GROUP;
  const int gs = min(p.tilesM - fm, GROUP);
  const int tm = fm + (bid % npg) % gs;
  const int tn = (bid % npg) / gs;
  m0 = (p.mshift_last && tm == p.tilesM - 1) ? p.M - V3_BM : tm * V3_BM;
  n0 = tn * V3_BN;
}

template <int N>
__device__ __forceinline__ void wait_vm_n() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- FE: register-direct epilogue of the swapped-operand (SW) accumulator layout, with the next tile's first two
// K-steps already in flight ----
// The LDS-staged epilogue runs while the whole CU's matrix pipes idle, and every CU of a round stores its tile at the
// same moment: in the K-sweep of tools/gemm_ksweep.py the fixed cost per 256 x 256 tile is 11-14 us with bf16 output
// and 21 us with f32 output against ~1.4 us per 64-deep K-step - a third of an InternViT K = 1024 GEMM. Here the
// epilogue needs no LDS, so the next tile's stages 0 and 1 (A and B) are issued by LDS-DMA before the first store:
// the next tile's first wait then covers only its own loads (gfx950 counts stores in vmcnt, in issue order), and the
// stores drain under the epilogue arithmetic and the first two K-steps instead of in front of them.
// Lane l of a wave holds, in acc[a][b], rows 16a + (l & 15) and columns 16b + 4(l >> 4) + r (r = 0..3) of the wave's
// 128 x 64 sub-tile. bf16 rows leave as 16-B stores after one v_permlane16_swap per packed dword pair (blocks b, b+1):
// row-group g = l >> 4 then holds 8 consecutive columns, 16(b + (g & 1)) + 8(g >> 1) .. + 7.
// Eligible (host side, fe_ok): ksplit 1, batch 1, N % 256 == 0, 16-B aligned rows, no accumulation, K >= 192,
// epilogues STORE / GELU / QGELU / RESID_LS / GELU_BWD / QGELU_BWD (colsum with the GELU' pair); whole tiles (M % 256
// == 0, folded remainder or shifted last tile), or a partial last tile for STORE / GELU / QGELU (rows past M dropped
// by the stores' range check).
template <int EPI, typename OutT> struct FeStores { static constexpr int N = sizeof(OutT) == 2 ? 16 : 32; };
template <typename OutT> struct FeStores<EPI_GELU, OutT> { static constexpr int N = 32; };
template <typename OutT> struct FeStores<EPI_QGELU, OutT> { static constexpr int N = 32; };
template <typename OutT> struct FeStores<EPI_RESID_LS, OutT> { static constexpr int N = 32; };  // (+ 16 with aux_out)

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  bf16x2 v;
  v[0] = (bf16)a;
  v[1] = (bf16)b;
  return __builtin_bit_cast(uint32_t, v);
}
// sum over the 16 lanes of a row group (every lane gets the sum): quad swaps, half-row mirror, row mirror
__device__ __forceinline__ float row16_sum(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xF, 0xF, false));
  return x;
}
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

// A 16-B buffer store whose data VGPRs the next instructions may overwrite. Measured on gfx950 / ROCm 7.2: when the
// compiler reuses a dwordx4 store's data registers in the very next VALU instruction (v_pk_fma_f32 into v[22:23]
// right after buffer_store_dwordx4 v[22:25]), lanes 12-15 of each 16-lane row stored the NEW value of dword 1
// (tools/fe_dbg.py: rows 4-7 / 12-15, columns 2-3 of the second chunk wrong). Two wait states after the store, with
// scheduling barriers so nothing is moved in between, keep the data read ahead of the overwrite.
__device__ __forceinline__ void bst16(__amdgpu_buffer_rsrc_t r, uint4 d, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b128(u32x4v{d.x, d.y, d.z, d.w}, r, voff, soff, 0);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Stores of one 16-row block of the wave's sub-tile (y[b][r] in the register layout: row rr, columns 16b + 4g + r)
// as 8-row x 128-B store instructions (whole lines; 16 rows x 64 B per instruction measured slower than the
// LDS-staged epilogue). The block goes through the wave's private LDS scratch (rows of 16-B chunks XOR-swizzled by
// the row: conflict-free 16-B writes and reads, 2-way for the bf16 8-B writes) and comes back one 16-B chunk per
// lane in row order. LDS rather than cross-lane permutes: lgkmcnt, not vmcnt, so the stores in flight are never
// waited for. Buffer stores: voffL = the lane's byte offset in the block's first row group, the block row and the
// further row groups in soffset (wave-uniform); no 64-bit address arithmetic.
__device__ __forceinline__ void fe_st_bf16(char* scr, __amdgpu_buffer_rsrc_t r, int voffL, int soff, int sgrp, int lane,
                                           const float (&y)[4][4]) {
  const int rr = lane & 15, g = lane >> 4;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    bf16x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (bf16)y[b][e];
    const int c = 2 * b + (g >> 1);
    *reinterpret_cast<bf16x4*>(scr + rr * 128 + ((c ^ (rr & 7)) << 4) + (g & 1) * 8) = v;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // rows 8h .. 8h + 7
    const int row = (lane >> 3) + 8 * h, c = lane & 7;
    const uint4 d = *reinterpret_cast<const uint4*>(scr + row * 128 + ((c ^ (row & 7)) << 4));
    bst16(r, d, voffL, soff + h * sgrp);
  }
}
__device__ __forceinline__ void fe_st_f32(char* scr, __amdgpu_buffer_rsrc_t r, int voffL, int soff, int sgrp, int lane,
                                          const float (&y)[4][4]) {
  const int rr = lane & 15, g = lane >> 4;
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {  // blocks 2hb, 2hb + 1: 16 rows x 128 B per pass (2 KiB of scratch)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      const int c = 4 * bb + g;
      const float* v = y[2 * hb + bb];
      *reinterpret_cast<f32x4*>(scr + rr * 128 + ((c ^ (rr & 7)) << 4)) = f32x4{v[0], v[1], v[2], v[3]};
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // rows 8h .. 8h + 7
      const int row = (lane >> 3) + 8 * h, c = lane & 7;
      const uint4 d = *reinterpret_cast<const uint4*>(scr + row * 128 + ((c ^ (row & 7)) << 4));
      bst16(r, d, voffL + 128 * hb, soff + h * sgrp);
    }
  }
}
// the lane's byte offset in a block's first row group (8 rows x 8 16-B chunks: bf16 the whole 64 columns, f32 the
// first 32) of a [rows][ld] matrix of sz-byte elements whose sub-tile starts at (mw, nw)
__device__ __forceinline__ int fe_voff(int mw, int nw, long ld, int sz, int lane) {
  return (int)(((long)(mw + (lane >> 3)) * ld + nw + (lane & 7) * (16 / sz)) * sz);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t fe_rsrc(const void* base, long rows, long ld, int sz) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)(rows * ld * sz), 0x00020000);
}
constexpr int FE_SCR = 2048;  // LDS scratch per wave (16 rows x 128 B), past the ring

template <int EPI, typename OutT, typename NextFn>
__device__ __forceinline__ void fe_epilogue(const GemmArgs& p, OutT* __restrict__ C, const f32x4 (&acc)[8][4], int mw,
                                            int nw, int lane, char* scr, NextFn issue_next) {
  const int rr = lane & 15, g = lane >> 4;
  const int nc = nw + 4 * g;  // column of register 0 of block 0
  constexpr bool kAux = EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD;
  constexpr bool kResid = EPI == EPI_RESID_LS;
  constexpr bool kBias = EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_QGELU || EPI == EPI_RESID_LS;
  constexpr int csz = sizeof(OutT);
  const __amdgpu_buffer_rsrc_t rc = fe_rsrc(C, p.M, p.ldc, csz);
  const int vc = fe_voff(mw, nw, p.ldc, csz, lane);
  const int sc = 16 * (int)p.ldc * csz;  // one 16-row block
  __amdgpu_buffer_rsrc_t ra = rc;
  int va = 0, sa = 0;
  if constexpr (EPI == EPI_GELU || EPI == EPI_QGELU || EPI == EPI_RESID_LS) {
    if (p.aux_out) {
      ra = fe_rsrc(p.aux_out, p.M, p.ldaux_out, 2);
      va = fe_voff(mw, nw, p.ldaux_out, 2, lane);
      sa = 16 * (int)p.ldaux_out * 2;
    }
  }
  // Every global load of the epilogue is issued before the next tile's DMA: a load issued after it (or after a
  // store) could only be waited for behind them (vmcnt counts in issue order).
  f32x4 bias[4], lsv[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    bias[b] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (kBias) {
      if (p.bias) bias[b] = *reinterpret_cast<const f32x4*>(p.bias + nc + 16 * b);
    }
    if constexpr (kResid) lsv[b] = *reinterpret_cast<const f32x4*>(p.ls + nc + 16 * b);
  }
  uint2 ax[4][4];  // bf16 pre-activations (GELU' epilogues), half the sub-tile at a time: 32 VGPRs
  f32x4 rv[4][4];  // f32 residual rows, half the sub-tile at a time (RESID_LS): 64 VGPRs
  if constexpr (kAux) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) ax[a][b] = *reinterpret_cast<const uint2*>(p.aux + (long)(mw + 16 * a + rr) * p.ldaux + nc + 16 * b);
  }
  if constexpr (kResid) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) rv[a][b] = *reinterpret_cast<const f32x4*>(p.resid + (long)(mw + 16 * a + rr) * p.ldr + nc + 16 * b);
  }
  __builtin_amdgcn_sched_barrier(0);
  issue_next();
  __builtin_amdgcn_sched_barrier(0);
  float cs[4][4];
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[b][r] = 0.f;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    if (a == 4) {  // second half of the row inputs
      if constexpr (kResid) {
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
          for (int b = 0; b < 4; ++b)
            rv[a2][b] = *reinterpret_cast<const f32x4*>(p.resid + (long)(mw + 16 * (4 + a2) + rr) * p.ldr + nc + 16 * b);
      }
      if constexpr (kAux) {
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
          for (int b = 0; b < 4; ++b)
            ax[a2][b] = *reinterpret_cast<const uint2*>(p.aux + (long)(mw + 16 * (4 + a2) + rr) * p.ldaux + nc + 16 * b);
      }
    }
    float y[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) y[b][r] = acc[a][b][r] * p.alpha + bias[b][r];
    if constexpr (EPI == EPI_STORE) {
      if constexpr (csz == 2) fe_st_bf16(scr, rc, vc, a * sc, sc / 2, lane, y);
      else fe_st_f32(scr, rc, vc, a * sc, sc / 2, lane, y);
    } else if constexpr (EPI == EPI_GELU || EPI == EPI_QGELU) {
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) y[b][r] = (float)(bf16)y[b][r];
      if (p.aux_grad) {  // aux = act'(h): the derivative replaces h in y for the aux store, act(h) kept aside
        float g[4][4];
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float ax;
            g[b][r] = act_fwd<EPI>(y[b][r], true, ax);
            y[b][r] = ax;
          }
        fe_st_bf16(scr, ra, va, a * sa, sa / 2, lane, y);
        fe_st_bf16(scr, rc, vc, a * sc, sc / 2, lane, g);
      } else {
        fe_st_bf16(scr, ra, va, a * sa, sa / 2, lane, y);
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) y[b][r] = EPI == EPI_GELU ? gelu_erf(y[b][r]) : qgelu(y[b][r]);
        fe_st_bf16(scr, rc, vc, a * sc, sc / 2, lane, y);
      }
    } else if constexpr (EPI == EPI_RESID_LS) {
      if (p.aux_out) fe_st_bf16(scr, ra, va, a * sa, sa / 2, lane, y);
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) y[b][r] = rv[a & 3][b][r] + lsv[b][r] * y[b][r];
      fe_st_f32(scr, rc, vc, a * sc, sc / 2, lane, y);
    } else if constexpr (kAux) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const bf16x4 hv = __builtin_bit_cast(bf16x4, ax[a & 3][b]);
#pragma unroll
        for (int r = 0; r < 4; ++r) y[b][r] *= act_bwd<EPI>((float)hv[r], p.aux_grad);
      }
      fe_st_bf16(scr, rc, vc, a * sc, sc / 2, lane, y);
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[b][r] += y[b][r];
    }
  }
  if constexpr (kAux) {
    if (p.colsum) {  // the wave's 128 rows summed into the partial row of its first 64-row subtile, zeros in the second
      float* w0 = p.colsum_ws + (long)(p.colsum_row0 + mw / 64) * p.N + nc;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        f32x4 t;
#pragma unroll
        for (int r = 0; r < 4; ++r) t[r] = row16_sum(cs[b][r]);
        if (rr == 0) {
          *reinterpret_cast<f32x4*>(w0 + 16 * b) = t;
          *reinterpret_cast<f32x4*>(w0 + p.N + 16 * b) = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  }
}

// One 256x256 output tile (tile index bid of p's grid after the XCD remap), K range of split blockIdx.y, batch z.
// FE (with SW): register-direct epilogue; `pre` = this tile's stages 0 and 1 were issued by the previous tile's
// epilogue; next_bid >= 0 = issue the next tile's stages 0 and 1 inside this tile's epilogue.
template <bool AK, bool BKc, int EPI, typename OutT, bool SW, bool FE = false>
__device__ __forceinline__ void v3_tile(const GemmArgs& p, int bid, long z, char* smem, bool pre = false,
                                        int next_bid = -1, int ysplit = -1) {
  const int ys = ysplit >= 0 ? ysplit : (int)blockIdx.y;  // this block's K split
  static_assert(!FE || SW, "the register-direct epilogue needs the swapped-operand accumulator layout");
  constexpr int NW = 8;
  constexpr int A_BYTES = V3_BM * BK * 2, B_BYTES = V3_BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  int m0, n0;
  v3_origin(p, bid, m0, n0);
  const bf16* A = p.A + z * p.sA;
  const bf16* B = p.B + z * p.sB;
  OutT* __restrict__ C = reinterpret_cast<OutT*>(p.C) + z * p.sC;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  int kbeg = 0, kend = p.K;
  if (p.ksplit > 1) {
    kbeg = ys * p.kchunk;
    kend = min(p.K, kbeg + p.kchunk);
  }
  const int nk = (kend - kbeg + BK - 1) / BK;
  const long extA = AK ? ((long)(p.M - 1) * p.lda + p.K) : ((long)(p.K - 1) * p.lda + p.M);
  const long extB = BKc ? ((long)(p.N - 1) * p.ldb + p.K) : ((long)(p.K - 1) * p.ldb + p.N);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)(extA * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)(extB * 2), 0x00020000);
  constexpr int PA = A_BYTES / 1024 / NW, PB = B_BYTES / 1024 / NW;  // 4 + 4 pieces per wave per tile
  static_assert(PA == 4 && PB == 4, "v3 piece schedule assumes 4+4 pieces per wave");
  long baseA[PA], baseB[PB];
  int krA[PA], krB[PB];
  bool okA[PA], okB[PB];
  dma_setup<AK, V3_BM, NW>(lane, wave, m0, p.M, p.lda, baseA, krA, okA);
  dma_setup<BKc, V3_BN, NW>(lane, wave, n0, p.N, p.ldb, baseB, krB, okB);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // FE: stores the previous tile's epilogue issued after this tile's stages 0 and 1 (a lower bound: waiting for
  // fewer younger ops only waits longer)
  constexpr int FES = FE ? FeStores<EPI, OutT>::N : 0;
  if (FE && pre) {
    wait_vm_n<8 + FES>();  // stage 0 landed; stage 1 (8 pieces) and the stores may still be in flight
  } else {
    // prologue: tile 0 (A and B) and tile 1's A pieces
    dma_issue_range<AK, V3_BM, NW, 0, 4>(ra, smem, wave, kbeg, kend, p.lda, baseA, krA, okA);
    dma_issue_range<BKc, V3_BN, NW, 0, 4>(rb, smem + A_BYTES, wave, kbeg, kend, p.ldb, baseB, krB, okB);
    if (nk > 1) {
      dma_issue_range<AK, V3_BM, NW, 0, 4>(ra, smem + STAGE, wave, kbeg + BK, kend, p.lda, baseA, krA, okA);
      wait_vm<4>();
    } else {
      wait_vm<0>();
    }
  }
  v3_barrier();
  if (wr == 1) v3_barrier();  // the M-half-1 waves run one barrier behind

  const int arow = wr * 128, bcol = wc * 64;
  bf16x8 alo[4][2], ahi[4][2], blo[2][2], bhi[2][2];
  for (int t = 0; t < nk; ++t) {
    const char* As = smem + (t & 1) * STAGE;
    const char* Bs = As + A_BYTES;
    char* st1 = smem + ((t + 1) & 1) * STAGE;  // tile t+1
    char* st2 = smem + (t & 1) * STAGE;        // tile t+2 (this stage, free after q1)
    const bool has2 = t + 2 < nk;
    const bool has1 = t + 1 < nk && !(FE && pre && t == 0);  // (FE pre: stage 1's B came with the prefetch)
    const int k1 = kbeg + (t + 1) * BK, k2 = kbeg + (t + 2) * BK;
    // ---- q0
    v3_read<AK, BKc>(As, Bs, arow, bcol, lane, alo, blo);
    if (has1) dma_issue_range<BKc, V3_BN, NW, 0, 2>(rb, st1 + A_BYTES, wave, k1, kend, p.ldb, baseB, krB, okB);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    v3_barrier();
    v3_mfma<SW>(acc, 0, 0, alo, blo);
    v3_barrier();
    // ---- q1
    v3_read<AK, BKc>(As, Bs, arow + 64, bcol + 32, lane, ahi, bhi);
    if (has1) dma_issue_range<BKc, V3_BN, NW, 2, 2>(rb, st1 + A_BYTES, wave, k1, kend, p.ldb, baseB, krB, okB);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    v3_barrier();
    v3_mfma<SW>(acc, 0, 1, alo, bhi);
    v3_barrier();
    // ---- q2
    if (has2) dma_issue_range<AK, V3_BM, NW, 0, 2>(ra, st2, wave, k2, kend, p.lda, baseA, krA, okA);
    v3_barrier();
    v3_mfma<SW>(acc, 1, 0, ahi, blo);
    v3_barrier();
    // ---- q3
    if (has2) {
      dma_issue_range<AK, V3_BM, NW, 2, 2>(ra, st2, wave, k2, kend, p.lda, baseA, krA, okA);
      if (FE && pre && t == 0) wait_vm_n<4 + FES>();  // stage 1 landed; the previous tile's stores may still drain
      else wait_vm<4>();
    } else {
      wait_vm<0>();
    }
    v3_barrier();
    v3_mfma<SW>(acc, 1, 1, ahi, bhi);
    v3_barrier();
  }
  if (wr == 0) v3_barrier();  // re-align the barrier counts of the two wave groups

  if constexpr (FE) {
    auto issue_next = [&]() {
      if (next_bid < 0) return;
      int mn, nn;
      v3_origin(p, next_bid, mn, nn);
      long bA[PA], bB[PB];
      int kA[PA], kB[PB];
      bool oA[PA], oB[PB];
      dma_setup<AK, V3_BM, NW>(lane, wave, mn, p.M, p.lda, bA, kA, oA);
      dma_setup<BKc, V3_BN, NW>(lane, wave, nn, p.N, p.ldb, bB, kB, oB);
      dma_issue_range<AK, V3_BM, NW, 0, 4>(ra, smem, wave, kbeg, kend, p.lda, bA, kA, oA);
      dma_issue_range<BKc, V3_BN, NW, 0, 4>(rb, smem + A_BYTES, wave, kbeg, kend, p.ldb, bB, kB, oB);
      dma_issue_range<AK, V3_BM, NW, 0, 4>(ra, smem + STAGE, wave, kbeg + BK, kend, p.lda, bA, kA, oA);
      dma_issue_range<BKc, V3_BN, NW, 0, 4>(rb, smem + STAGE + A_BYTES, wave, kbeg + BK, kend, p.ldb, bB, kB, oB);
    };
    fe_epilogue<EPI, OutT>(p, C, acc, m0 + arow, n0 + bcol, lane, smem + 2 * STAGE + wave * FE_SCR, issue_next);
    return;
  }
  bool reduced = false;
  if constexpr (EPI == EPI_STORE) {
    if (p.ksplit > 1 && p.split_ws) {
      __syncthreads();  // every wave is done reading the ring (the role word sits past the epilogue region)
      if (!v3_split_reduce(p, bid, acc, reinterpret_cast<int*>(smem + 8 * 64 * EP_LD * 4), wave, lane, ys)) return;
      reduced = true;
    }
  }
  // ---- epilogue: two 64x64 passes per wave through a wave-private LDS region
  __syncthreads();
  float* ep = reinterpret_cast<float*>(smem) + wave * (64 * EP_LD);
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
    if constexpr (SW) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<f32x4*>(ep + (i * 16 + (lane & 15)) * EP_LD + j * 16 + 4 * (lane >> 4)) = acc[4 * mh + i][j];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) ep[(i * 16 + (lane >> 4) * 4 + r) * EP_LD + j * 16 + (lane & 15)] = acc[4 * mh + i][j][r];
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): wave-private region written
    // the staged image is row-major in both layouts, so the batched-load epilogue serves SW = false too (InternViT
    // proj / fc2 residual GEMMs: +0.35 % on the step, profiles/round5_gemm_pf_epilogue_ab.txt)
    if constexpr (SW) epilogue_tile64_pf<EPI, OutT>(p, C, ep, lane, m0 + arow + 64 * mh, n0 + bcol, reduced);
    else epilogue_tile64_auto<EPI, OutT>(p, C, ep, lane, m0 + arow + 64 * mh, n0 + bcol, reduced);
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
}

// The M remainder (rows [rem_r0, M) past the last whole 256-row tile: InternViT's 16 class-token rows of 16 x 1025,
// CLIP's 64 of 64 x 577) inside the v3 launch instead of two extra launches. Work unit u (one block, before its tiles)
// = 256-column group u % ncg x K split u / ncg: 8 waves x 32 columns, 16-row MFMA blocks, operands straight from
// global (A K-contiguous). The partial is published with agent-scope stores; the group's last arriver sums the splits
// with agent-scope loads and runs the real epilogue (and the colsum partial row) on those rows, then resets the
// counter (MI355X_MICROARCH.md inter-workgroup visibility, table row 1). No block ever waits on another.
template <bool BKc, int EPI, typename OutT, int NTH = 512>
__device__ __forceinline__ void v3_remainder(const GemmArgs& p, int u) {
  constexpr int CG = NTH / 2;  // columns per work unit: 32 per wave
  __shared__ int last_s;
  __shared__ float csred[CG];
  const int rem = p.M - p.rem_r0, r0 = p.rem_r0;
  const int ncg = (p.N + CG - 1) / CG, cg = u % ncg, sp = u / ncg;
  const int n0 = cg * CG, k0 = sp * p.rem_kc, k1 = min(p.K, k0 + p.rem_kc);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nrb = (rem + 15) >> 4;
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = k0; k < k1; k += 32) {
    const int kk = k + 8 * (lane >> 4);
    bf16x8 af[4], bfr[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + 16 * i + (lane & 15);
      bf16x8 z = {};
      if (i < nrb && m < p.M && kk < k1) z = *reinterpret_cast<const bf16x8*>(p.A + (long)m * p.lda + kk);
      af[i] = z;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 32 * w + 16 * j + (lane & 15);
      bf16x8 z = {};
      if (n < p.N && kk < k1) {
        if (BKc) {
          z = *reinterpret_cast<const bf16x8*>(p.B + (long)n * p.ldb + kk);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) z[e] = p.B[(long)(kk + e) * p.ldb + n];
        }
      }
      bfr[j] = z;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < nrb)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }
  // publish: C layout of 16x16x32 is col = lane & 15, row = 4 (lane >> 4) + r
  float* part = p.rem_part + (long)sp * rem * p.N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + 4 * (lane >> 4) + r, n = n0 + 32 * w + 16 * j + (lane & 15);
        if (m < rem && n < p.N)
          __hip_atomic_store(part + (long)m * p.N + n, acc[i][j][r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {  // release (cumulative over the barrier) the group's partials, then arrive
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    last_s = __hip_atomic_fetch_add(p.rem_cnt + cg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p.rem_nsplit - 1;
  }
  __syncthreads();
  if (!last_s) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the last arriver sees every split's partials
  // last arriver: column n0 + (tid % CG), rows tid / CG, + 2, ...; four rows x up to 16 splits (64 agent-scope loads)
  // in flight per thread, so the group's epilogue costs a round trip or two, not one per split
  OutT* C = reinterpret_cast<OutT*>(p.C);
  const int n = n0 + (tid % CG);
  float cs = 0.f;
  if (n < p.N) {
    const long ss = (long)rem * p.N;
    for (int mb = tid / CG; mb < rem; mb += 8) {
      float v[4][16];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = mb + 2 * i;
#pragma unroll
        for (int y = 0; y < 16; ++y)
          v[i][y] = (m < rem && y < p.rem_nsplit)
                        ? __hip_atomic_load(p.rem_part + y * ss + (long)m * p.N + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = mb + 2 * i;
        if (m >= rem) continue;
        float a8[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) a8[y] = v[i][y] + v[i][y + 8];
        const float a = ((a8[0] + a8[1]) + (a8[2] + a8[3])) + ((a8[4] + a8[5]) + (a8[6] + a8[7]));
        epilogue_elem<EPI, OutT>(p, C, r0 + m, n, a);
        if constexpr (EPI == EPI_STORE) cs += a * p.alpha + (p.bias ? p.bias[n] : 0.f);
        else if constexpr (EPI == EPI_GELU_BWD) cs += a * p.alpha * act_bwd<EPI_GELU_BWD>((float)p.aux[(long)(r0 + m) * p.ldaux + n], p.aux_grad);
        else if constexpr (EPI == EPI_QGELU_BWD) cs += a * p.alpha * act_bwd<EPI_QGELU_BWD>((float)p.aux[(long)(r0 + m) * p.ldaux + n], p.aux_grad);
      }
    }
  }
  if (p.colsum) {  // the colsum partial row of these rows (row r0 / 64 of colsum_ws, as the remainder kernel wrote it)
    if (tid >= CG) csred[tid - CG] = cs;
    __syncthreads();
    if (tid < CG && n < p.N) p.colsum_ws[(long)(r0 / 64) * p.N + n] = cs + csred[tid];
  }
  if (tid == 0) __hip_atomic_store(p.rem_cnt + cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// gridDim.x < tiles: a persistent grid, each block walks tiles blockIdx.x, + gridDim.x, ... (gridDim.x a multiple of 8,
// so a block keeps its XCD's tile range); the epilogue stores of one tile drain while the next tile's loads start.
template <bool AK, bool BKc, int EPI, typename OutT, bool SW>
__global__ __launch_bounds__(512, 1) void gemm_bf16_v3_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if constexpr (AK) {
    if (p.rem_r0 > 0 && (int)blockIdx.x < p.rem_nsplit * ((p.N + 255) / 256)) {
      v3_remainder<BKc, EPI, OutT>(p, blockIdx.x);
      __syncthreads();
    }
  }
  const int nwg = p.tilesM * p.tilesN;
  for (int t = blockIdx.x; t < nwg; t += gridDim.x) {
    if (t != (int)blockIdx.x) __syncthreads();  // the previous tile's epilogue is done with the LDS
    v3_tile<AK, BKc, EPI, OutT, SW>(p, xcd_remap(t, nwg), blockIdx.z, smem);
  }
}

// FE persistent kernel: each block walks its tiles with the next tile's first two K-steps issued inside the previous
// tile's register-direct epilogue (no barrier between tiles: the epilogue uses no LDS).
template <bool AK, bool BKc, int EPI, typename OutT>
__global__ __launch_bounds__(512, 1) void gemm_bf16_v3fe_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if constexpr (AK) {
    if (p.rem_r0 > 0 && (int)blockIdx.x < p.rem_nsplit * ((p.N + 255) / 256)) {
      v3_remainder<BKc, EPI, OutT>(p, blockIdx.x);
      __syncthreads();
    }
  }
  const int nwg = p.tilesM * p.tilesN;
  bool pre = false;
  for (int t = blockIdx.x; t < nwg; t += gridDim.x) {
    const int tn = t + (int)gridDim.x;
    v3_tile<AK, BKc, EPI, OutT, true, true>(p, xcd_remap(t, nwg), 0, smem, pre, tn < nwg ? xcd_remap(tn, nwg) : -1);
    pre = tn < nwg;
  }
}

// Two independent GEMMs of one layout (f32 outputs accumulated, same K and split count) in one launch: grid.x
// covers both tile sets, so two under-filled weight-gradient grids (InternViT fc2 + fc1, proj + qkv) fill the chip
// together instead of leaving CUs idle one after the other.
template <bool AK, bool BKc, bool SW>
__global__ __launch_bounds__(512, 1) void gemm_bf16_v3_pair_kernel(GemmArgs p, GemmArgs q) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n1 = p.tilesM * p.tilesN;
  const int nt = n1 + q.tilesM * q.tilesN;
  if (p.xcd_split) {
    // one round of 8 x 32 blocks (tiles x splits = 256): blocks dealt round-robin over the XCDs, so XCD x = L & 7 takes
    // K split x % S of the tile range [region * nt / R, +nt / R), R = 8 / S regions: every XCD streams ONE K range of
    // a contiguous run of tiles (the 4 x 8 / 8 x 4 regions of v3_origin's tile order) instead of both splits of a 4 x 4
    // region, which cuts the operand panels each XCD's L2 fills (placement only decides speed, never correctness)
    const int L = blockIdx.x, x = L & 7, S = p.ksplit, R = 8 / S;
    const int tile = (x / S) * (nt / R) + (L >> 3);
    if (tile < n1) v3_tile<AK, BKc, EPI_STORE, float, SW>(p, tile, 0, smem, false, -1, x % S);
    else v3_tile<AK, BKc, EPI_STORE, float, SW>(q, tile - n1, 0, smem, false, -1, x % S);
    return;
  }
  const int bid = xcd_remap(blockIdx.x, nt);
  if (bid < n1) v3_tile<AK, BKc, EPI_STORE, float, SW>(p, bid, 0, smem);
  else v3_tile<AK, BKc, EPI_STORE, float, SW>(q, bid - n1, 0, smem);
}

// ---------------------------------------------------------------------------------------------
// v4: TWO workgroups per CU, so one workgroup's epilogue (LDS staging, GELU/GELU' VALU, the output stores and the
// aux / residual loads) runs while the other's MFMAs keep the matrix pipes busy - v3 holds one 256-thread-pair
// block per CU and serialises every tile's epilogue behind its main loop (gemm_epi_bench: fc1 GELU 204 us vs 134 us
// for the same main loop with plain stores). Each workgroup's vmcnt only counts its own stores, so a tile's
// stores no longer hold the next tile's DMA waits of the whole CU.
//   tile 256 x 128, BK = 32, 4 waves (2 M x 2 N, each 128 x 64 = 8 x 4 v_mfma_f32_16x16x32_bf16 blocks: v3's
//   per-wave tile and LDS-read-per-MFMA ratio), 3-stage LDS-DMA ring of 24 KiB (72 KiB per workgroup; two fit
//   the 160 KiB LDS), counted vmcnt, one raw s_barrier per K-step, persistent grid of 2 x 256 blocks.
//   K-contiguous operands live in LDS as [rows][32] (64-B rows) with the 16-B chunk XOR-swizzled by
//   h((row >> 2) & 3), h = {0, 2, 3, 1}: ds_read_b128 of a 16 x 32 fragment is conflict-free in every lane group
//   (enumerated); MN-contiguous operands keep v2/v3's [k][128-column panel] image (8 KiB panels) and tr-reads.
constexpr int V4_BM = 256, V4_BN = 128, V4_BK = 32, V4_NS = 3;
constexpr int V4_ABYTES = V4_BM * V4_BK * 2, V4_BBYTES = V4_BN * V4_BK * 2, V4_STAGE = V4_ABYTES + V4_BBYTES;

__device__ __forceinline__ int v4_h(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

// per-lane source offsets (elements) of the LDS-DMA pieces this wave issues for one stage of an operand
template <bool KC, int ROWS>
__device__ __forceinline__ void v4_dma_setup(int lane, int wave, int r0, int rows_total, long ld, long (&base)[ROWS / 64],
                                             int (&kr)[ROWS / 64], bool (&ok)[ROWS / 64]) {
  constexpr int PER = ROWS * V4_BK * 2 / 1024 / 4;  // = ROWS / 64
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int o = (wave * PER + i) * 1024 + lane * 16;
    if (KC) {  // [rows][32]: 64-B rows, chunk swizzle h
      const int row = o >> 6, pc = (o >> 4) & 3;
      const int c = pc ^ v4_h(row);
      ok[i] = r0 + row < rows_total;
      base[i] = (long)(r0 + row) * ld + 8 * c;
      kr[i] = 0;
    } else {   // [panel][32 k][128]: 256-B k-rows, v2's (k & 3 | k >> 3 & 1) swizzle
      const int panel = o >> 13, o2 = o & 8191;
      const int k = o2 >> 8, pc = (o2 >> 4) & 15;
      const int x = (k & 3) | (((k >> 3) & 1) << 2);
      const int c = pc ^ (2 * x);
      const int col = r0 + panel * 128 + 8 * c;
      ok[i] = col < rows_total;
      base[i] = (long)k * ld + col;
      kr[i] = k;
    }
  }
}

template <bool KC, int ROWS>
__device__ __forceinline__ void v4_dma_issue(__amdgpu_buffer_rsrc_t rs, char* lds_tile, int wave, int k0, int K, long ld,
                                             const long (&base)[ROWS / 64], const int (&kr)[ROWS / 64],
                                             const bool (&ok)[ROWS / 64]) {
  constexpr int PER = ROWS / 64;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    unsigned off;
    if (KC) off = ok[i] ? (unsigned)((base[i] + k0) * 2) : kSent;
    else off = (ok[i] && k0 + kr[i] < K) ? (unsigned)((base[i] + (long)k0 * ld) * 2) : kSent;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds_tile + (wave * PER + i) * 1024),
                                             16, off, 0, 0, 0);
  }
}

template <bool KC>
__device__ __forceinline__ bf16x8 v4_read_frag(const char* lds, int rb, int lane) {
  if (KC) {
    const int row = rb + (lane & 15), c = lane >> 4;
    return *reinterpret_cast<const bf16x8*>(lds + row * 64 + ((c ^ v4_h(row)) << 4));
  }
  return read_frag<false>(lds + (rb >> 7) * 8192, rb & 127, 0, lane);
}

template <int N>
__device__ __forceinline__ void wait_vm_v4() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}

// One 256 x 128 output tile of p's grid (tile index after the XCD remap), K split blockIdx.y, batch z.
template <bool AK, bool BKc, int EPI, typename OutT, bool SW>
__device__ __forceinline__ void v4_tile(const GemmArgs& p, int bid, long z, char* smem) {
  const int tilesM = p.tilesM, tilesN = p.tilesN;
  constexpr int GROUP = 4;
  const int npg = GROUP * tilesN;
  const int gid = bid / npg;
  const int fm = gid * GROUP;
  const int gs = min(tilesM - fm, GROUP);
  const int tm = fm + (bid % npg) % gs;
  const int tn = (bid % npg) / gs;
  const int m0 = (p.mshift_last && tm == tilesM - 1) ? p.M - V4_BM : tm * V4_BM, n0 = tn * V4_BN;
  const bf16* A = p.A + z * p.sA;
  const bf16* B = p.B + z * p.sB;
  OutT* __restrict__ C = reinterpret_cast<OutT*>(p.C) + z * p.sC;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  int kbeg = 0, kend = p.K;
  if (p.ksplit > 1) {
    kbeg = blockIdx.y * p.kchunk;
    kend = min(p.K, kbeg + p.kchunk);
  }
  const int nk = (kend - kbeg + V4_BK - 1) / V4_BK;
  const long extA = AK ? ((long)(p.M - 1) * p.lda + p.K) : ((long)(p.K - 1) * p.lda + p.M);
  const long extB = BKc ? ((long)(p.N - 1) * p.ldb + p.K) : ((long)(p.K - 1) * p.ldb + p.N);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)(extA * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)(extB * 2), 0x00020000);
  long baseA[V4_BM / 64], baseB[V4_BN / 64];
  int krA[V4_BM / 64], krB[V4_BN / 64];
  bool okA[V4_BM / 64], okB[V4_BN / 64];
  v4_dma_setup<AK, V4_BM>(lane, wave, m0, p.M, p.lda, baseA, krA, okA);
  v4_dma_setup<BKc, V4_BN>(lane, wave, n0, p.N, p.ldb, baseB, krB, okB);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int st = 0; st < V4_NS - 1; ++st) {
    if (st < nk) {
      char* sl = smem + st * V4_STAGE;
      v4_dma_issue<AK, V4_BM>(ra, sl, wave, kbeg + st * V4_BK, kend, p.lda, baseA, krA, okA);
      v4_dma_issue<BKc, V4_BN>(rb, sl + V4_ABYTES, wave, kbeg + st * V4_BK, kend, p.ldb, baseB, krB, okB);
    }
  }
  const int arow = wr * 128, bcol = wc * 64;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) wait_vm_v4<6>();  // stage kt landed; stage kt+1 (6 pieces per wave) may stay in flight
    else wait_vm_v4<0>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // every wave's stage-kt pieces landed; every wave finished reading stage kt-1
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < nk) {
      char* sl = smem + ((kt + 2) % V4_NS) * V4_STAGE;
      v4_dma_issue<AK, V4_BM>(ra, sl, wave, kbeg + (kt + 2) * V4_BK, kend, p.lda, baseA, krA, okA);
      v4_dma_issue<BKc, V4_BN>(rb, sl + V4_ABYTES, wave, kbeg + (kt + 2) * V4_BK, kend, p.ldb, baseB, krB, okB);
    }
    const char* As = smem + (kt % V4_NS) * V4_STAGE;
    const char* Bs = As + V4_ABYTES;
    bf16x8 af[8], bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = v4_read_frag<BKc>(Bs, bcol + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = v4_read_frag<AK>(As, arow + 16 * i, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (SW) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
  }
  // ---- epilogue: two 64x64 passes per wave through a wave-private LDS region (4 x 17 KiB <= the 72 KiB ring)
  __syncthreads();
  float* ep = reinterpret_cast<float*>(smem) + wave * (64 * EP_LD);
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
    if constexpr (SW) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<f32x4*>(ep + (i * 16 + (lane & 15)) * EP_LD + j * 16 + 4 * (lane >> 4)) = acc[4 * mh + i][j];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) ep[(i * 16 + (lane >> 4) * 4 + r) * EP_LD + j * 16 + (lane & 15)] = acc[4 * mh + i][j][r];
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): wave-private region written
    if constexpr (SW) epilogue_tile64_pf<EPI, OutT>(p, C, ep, lane, m0 + arow + 64 * mh, n0 + bcol);
    else epilogue_tile64<EPI, OutT>(p, C, ep, lane, m0 + arow + 64 * mh, n0 + bcol);
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
}

// Persistent: gridDim.x = 2 x 256 (two resident blocks per CU) walking tiles blockIdx.x + k * gridDim.x in the XCD
// remapped order; the folded M remainder (as v3, 128-column work units) runs first.
template <bool AK, bool BKc, int EPI, typename OutT, bool SW>
__global__ __launch_bounds__(256, 2) void gemm_bf16_v4_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if constexpr (AK) {
    if (p.rem_r0 > 0 && (int)blockIdx.x < p.rem_nsplit * ((p.N + 127) / 128)) {
      v3_remainder<BKc, EPI, OutT, 256>(p, blockIdx.x);
      __syncthreads();
    }
  }
  const int nwg = p.tilesM * p.tilesN;
  for (int t = blockIdx.x; t < nwg; t += gridDim.x) {
    if (t != (int)blockIdx.x) __syncthreads();  // the previous tile's epilogue is done with the LDS
    v4_tile<AK, BKc, EPI, OutT, SW>(p, xcd_remap(t, nwg), blockIdx.z, smem);
  }
}

template <bool AK, bool BKc, int EPI, typename OutT, bool SW>
static int launch_v4(GemmArgs a, int batch, hipStream_t st) {
  constexpr int LDS_RING = V4_NS * V4_STAGE;
  constexpr int LDS_EP = 4 * 64 * EP_LD * 4;
  constexpr int LDS = LDS_RING > LDS_EP ? LDS_RING : LDS_EP;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemm_bf16_v4_kernel<AK, BKc, EPI, OutT, SW>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  a.tilesM = a.rem_r0 > 0 ? a.rem_r0 / V4_BM : (a.M + V4_BM - 1) / V4_BM;
  a.tilesN = (a.N + V4_BN - 1) / V4_BN;
  static const int persist = [] { const char* e = getenv("SLX_GEMM_V4_PERSIST"); return e ? atoi(e) : 2; }();
  int gx = a.tilesM * a.tilesN;
  if (persist > 0 && a.ksplit <= 1 && batch == 1 && gx > 256 * persist) gx = 256 * persist;
  if (a.rem_r0 > 0) {
    const int ncg = (a.N + 127) / 128, k32 = (a.K + 31) / 32;
    int sp = gx / ncg;
    sp = sp < k32 / 2 ? sp : k32 / 2;
    sp = sp < 16 ? sp : 16;
    sp = sp < 1 ? 1 : sp;
    a.rem_kc = ((k32 + sp - 1) / sp) * 32;
    a.rem_nsplit = (a.K + a.rem_kc - 1) / a.rem_kc;
    if (a.rem_nsplit * ncg > gx) gx = a.rem_nsplit * ncg;
  }
  dim3 grid(gx, a.ksplit > 1 ? a.ksplit : 1, batch);
  hipLaunchKernelGGL((gemm_bf16_v4_kernel<AK, BKc, EPI, OutT, SW>), grid, dim3(256), LDS, st, a);
  SLX_LAUNCH_CHECK("slx_gemm_bf16(v4)");
  return 0;
}

template <bool AK, bool BKc, int EPI, typename OutT, bool SW, bool FE = false>
static int launch_v3(GemmArgs a, int batch, hipStream_t st) {
  constexpr int LDS_RING = 2 * (V3_BM * BK * 2 + V3_BN * BK * 2);
  constexpr int LDS_EP = FE ? LDS_RING + 8 * FE_SCR : 8 * 64 * EP_LD * 4 + 16;  // + the split-K role word
  constexpr int LDS = LDS_RING > LDS_EP ? LDS_RING : LDS_EP;
  const void* fn;
  if constexpr (FE) fn = (const void*)gemm_bf16_v3fe_kernel<AK, BKc, EPI, OutT>;
  else fn = (const void*)gemm_bf16_v3_kernel<AK, BKc, EPI, OutT, SW>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  a.tilesM = a.rem_r0 > 0 ? a.rem_r0 / V3_BM : (a.M + V3_BM - 1) / V3_BM;  // folded remainder rows are not tiles
  a.tilesN = (a.N + V3_BN - 1) / V3_BN;
  // persistent grid (one round of 256 blocks walking the tiles) by default: +0.3 % on the VLA step
  // (profiles/round2_s3_persist_ab.txt); SLX_GEMM_PERSIST=0 launches one block per tile
  static const int persist = [] { const char* e = getenv("SLX_GEMM_PERSIST"); return e ? atoi(e) : 1; }();
  int gx = a.tilesM * a.tilesN;
  if (persist > 0 && a.ksplit <= 1 && batch == 1 && gx > 256 * persist) gx = 256 * persist;
  if (a.rem_r0 > 0) {  // the folded remainder's work units (one per block, ahead of its tiles)
    const int ncg = (a.N + 255) / 256, k32 = (a.K + 31) / 32;
    int sp = gx / ncg;
    sp = sp < k32 / 2 ? sp : k32 / 2;  // >= 2 MFMA K-steps per split
    static const int smax = [] { const char* e = getenv("SLX_GEMM_FOLD_SPLIT"); const int v = e ? atoi(e) : 16;
                                 return v >= 1 && v <= 16 ? v : 16; }();
    sp = sp < smax ? sp : smax;  // <= 16 splits: the last arriver sums them with one batch of loads per 4 rows
    sp = sp < 1 ? 1 : sp;
    a.rem_kc = ((k32 + sp - 1) / sp) * 32;
    a.rem_nsplit = (a.K + a.rem_kc - 1) / a.rem_kc;
    if (a.rem_nsplit * ncg > gx) gx = a.rem_nsplit * ncg;
  }
  dim3 grid(gx, a.ksplit > 1 ? a.ksplit : 1, batch);
  if constexpr (FE) hipLaunchKernelGGL((gemm_bf16_v3fe_kernel<AK, BKc, EPI, OutT>), grid, dim3(512), LDS, st, a);
  else hipLaunchKernelGGL((gemm_bf16_v3_kernel<AK, BKc, EPI, OutT, SW>), grid, dim3(512), LDS, st, a);
  SLX_LAUNCH_CHECK("slx_gemm_bf16(v3)");
  return 0;
}

// The FE member's eligibility (see fe_epilogue): whole 256 x 256 tiles, one K range, no accumulation, an epilogue it
// implements. Anything else launches plain v3 (variant 7).
template <int EPI, typename OutT>
static bool fe_ok(const GemmArgs& a, int batch) {
  constexpr bool epi = EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_QGELU || EPI == EPI_RESID_LS ||
                       EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD;
  if (!epi || batch != 1 || a.ksplit > 1 || !a.vec_ok || a.accumulate || a.N % V3_BN != 0 || a.K % BK != 0 ||
      a.K < 3 * BK)
    return false;
  // the FE stores address the output through a buffer descriptor with 32-bit byte offsets and num_records
  if ((long long)a.M * a.ldc * (long long)sizeof(OutT) >= (1LL << 31)) return false;
  if (EPI == EPI_STORE && (a.split_stride || a.colsum || a.rope_cos)) return false;
  const int main_rows = a.rem_r0 > 0 ? a.rem_r0 : a.M;
  if (main_rows % V3_BM == 0 || (a.mshift_last && a.M >= V3_BM)) return true;
  // a partial last M tile (Qwen2: 6384 = 24 * 256 + 240 rows): the buffer stores drop the rows past M (range check
  // of the descriptor, num_records = M rows); only epilogues without per-row loads and without column sums
  return a.rem_r0 == 0 && (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_QGELU);
}

template <bool AK, bool BKc, int EPI, typename OutT>
static int launch(GemmArgs& a, int batch, hipStream_t st) {
  dim3 grid(a.tilesM * a.tilesN, a.ksplit > 1 ? a.ksplit : 1, batch);
  hipLaunchKernelGGL((gemm_bf16_kernel<AK, BKc, EPI, OutT>), grid, dim3(NT), 0, st, a);
  SLX_LAUNCH_CHECK("slx_gemm_bf16");
  return 0;
}

template <bool AK, bool BKc, int EPI, typename OutT, int BMv, int NS>
static int launch_v2(GemmArgs a, int batch, hipStream_t st) {
  constexpr int LDS_RING = NS * (BMv * BK * 2 + BN * BK * 2);
  constexpr int LDS_EP = (BMv / 32) * 64 * EP_LD * 4;
  constexpr int LDS = LDS_RING > LDS_EP ? LDS_RING : LDS_EP;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemm_bf16_dma_kernel<AK, BKc, EPI, OutT, BMv, NS>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  a.tilesM = (a.M + BMv - 1) / BMv;
  dim3 grid(a.tilesM * a.tilesN, a.ksplit > 1 ? a.ksplit : 1, batch);
  hipLaunchKernelGGL((gemm_bf16_dma_kernel<AK, BKc, EPI, OutT, BMv, NS>), grid, dim3(BMv * 2), LDS, st, a);
  SLX_LAUNCH_CHECK("slx_gemm_bf16(dma)");
  return 0;
}

// variant: 1 = v1 register-staged 128x128; 2 = DMA 128x128 NS2; 3 = DMA 128x128 NS3; 4 = DMA 128x128 NS4;
//          5 = DMA 256x128 NS2; 6 = DMA 256x128 NS3; 7 = v3 256x256 ping-pong; 8 = v3 with swapped operands
//          (row-contiguous accumulators, 16-B LDS staging) and the batched-load epilogue; 0 = automatic
template <bool AK, bool BKc, int EPI, typename OutT>
static int launch_any(GemmArgs& a, int batch, hipStream_t st, int variant) {
  const bool dma_ok = (!AK || a.K % BK == 0) && (!BKc || a.K % BK == 0) && (a.ksplit <= 1 || a.kchunk % BK == 0) &&
                      a.drop_operand == 0;
  if (variant == 0) variant = dma_ok ? 2 : 1;
  if (variant != 1 && !dma_ok) variant = 1;
  switch (variant) {
    case 2: return launch_v2<AK, BKc, EPI, OutT, 128, 2>(a, batch, st);
    case 3: return launch_v2<AK, BKc, EPI, OutT, 128, 3>(a, batch, st);
    case 4: return launch_v2<AK, BKc, EPI, OutT, 128, 4>(a, batch, st);
    case 5: return launch_v2<AK, BKc, EPI, OutT, 256, 2>(a, batch, st);
    case 6: return launch_v2<AK, BKc, EPI, OutT, 256, 3>(a, batch, st);
    case 7: return launch_v3<AK, BKc, EPI, OutT, false>(a, batch, st);
    case 8: return launch_v3<AK, BKc, EPI, OutT, true>(a, batch, st);
    case 11:
      if constexpr (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_QGELU || EPI == EPI_RESID_LS ||
                    EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
        if (fe_ok<EPI, OutT>(a, batch)) return launch_v3<AK, BKc, EPI, OutT, true, true>(a, batch, st);
      }
      return launch_v3<AK, BKc, EPI, OutT, false>(a, batch, st);
    case 9: return launch_v4<AK, BKc, EPI, OutT, false>(a, batch, st);
    case 10: return launch_v4<AK, BKc, EPI, OutT, true>(a, batch, st);
    default: return launch<AK, BKc, EPI, OutT>(a, batch, st);
  }
}

template <int EPI, typename OutT>
static int dispatch_layout(int layout, GemmArgs& a, int batch, hipStream_t st, int variant) {
  switch (layout) {
    case SLX_GEMM_NT: return launch_any<true, true, EPI, OutT>(a, batch, st, variant);
    case SLX_GEMM_NN: return launch_any<true, false, EPI, OutT>(a, batch, st, variant);
    case SLX_GEMM_TN: return launch_any<false, false, EPI, OutT>(a, batch, st, variant);
    case SLX_GEMM_TT: return launch_any<false, true, EPI, OutT>(a, batch, st, variant);
  }
  set_error("slx_gemm_bf16: bad layout %d", layout);
  return -22;
}


// ---- host side ------------------------------------------------------------------------------
// Variant choice: per launch the chip holds 512 blocks of the 128x128 kernels (2 per CU) or 256 of v3
// (one 512-thread block with 139 KB LDS per CU). The cost of a variant is its number of block rounds
// x the work of one round at that kernel's rate (v3's per-CU rate ~1.26x v2's, measured at 8192^3), so
// partially filled last rounds are priced in. For v3, a small M remainder (M % 256 <= 64, e.g. the 16
// class tokens of 16 InternViT tiles: 16400 = 64*256 + 16) is peeled into a v2 launch so the main grid
// is whole rounds.
constexpr long kSplitCntInts = 16384;  // arrival / published counters at the end of split_ws (2 per tile)
constexpr long kSlabFloats = 65536;    // one 256 x 256 f32 partial

// The in-launch split-K reduction applies when the caller gave a workspace big enough for every tile's slabs, at
// 2 splits: the InternViT fc2.w + fc1.w pair, 302 -> 295 us against f32 atomics; at 4 splits (proj.w + qkv.w) the
// last arriver's serial read of three 256 KiB slabs made it slower than the atomics (178 vs 164 us,
// tools/wgrad_group_bench.py SPLIT_AB=1, profiles/round3_split_ab.txt). SLX_SPLIT_REDUCE_MAX raises the cap (A/B).
static bool split_ws_fits(const slx_gemm_desc* d, long tiles, int sp) {
  static const int smax_env = [] { const char* e = getenv("SLX_SPLIT_REDUCE_MAX"); const int v = e ? atoi(e) : 2;
                                   return v >= 2 && v <= 4 ? v : 2; }();
  const int smax = det_mode().on ? 4 : smax_env;  // deterministic mode: every split count the slab sum supports
  return d->split_ws && sp > 1 && sp <= smax && 2 * tiles <= kSplitCntInts &&
         tiles * sp * kSlabFloats <= d->split_ws_floats - kSplitCntInts;
}

static int v_tile_m(int v) { return v == 7 ? 256 : (v == 5 || v == 6) ? 256 : 128; }
static int v_tile_n(int v) { return v == 7 ? 256 : 128; }
static int v_slots(int v) { return v == 7 ? 256 : 512; }

static int split_for(const slx_gemm_desc* d, int v, int M, int batch) {
  const int tiles = ((M + v_tile_m(v) - 1) / v_tile_m(v)) * ((d->N + v_tile_n(v) - 1) / v_tile_n(v)) * batch;
  const int ksteps = (d->K + BK - 1) / BK;
  const int slots = v_slots(v);
  // (batched launches split too when they accumulate into C: no per-batch pre-zeroing needed; grid z = batch)
  if (!(d->epilogue == SLX_EPI_STORE && d->out_f32 && (batch == 1 || d->accumulate) && tiles <= slots / 2 &&
        ksteps >= 8)) return 1;
  if (d->ksplit_max < 0 || d->colsum) return 1;
  int sp = slots / tiles;  // floor: never more blocks than one round holds
  sp = sp < ksteps / 4 ? sp : ksteps / 4;
  if (v == 7 && sp > 4) sp = 4;  // beyond 4 the f32 atomic traffic (sp x M x N x 4 B) dominates
  if (d->ksplit_max > 0 && sp > d->ksplit_max) sp = d->ksplit_max;
  return sp < 1 ? 1 : sp;
}

// Estimated seconds: block rounds x one block's time at its kernel's per-CU rate (v2 blocks share a CU two
// at a time, so a lone v2 block is credited ~1.4x its shared rate), plus split-K atomic traffic.
static double v_cost(const slx_gemm_desc* d, int v, int M, int batch) {
  const double tiles = (double)((M + v_tile_m(v) - 1) / v_tile_m(v)) * ((d->N + v_tile_n(v) - 1) / v_tile_n(v)) * batch;
  const int sp = split_for(d, v, M, batch);
  const double blocks = tiles * sp;
  const double rounds = std::ceil(blocks / v_slots(v));
  const double block_flop = 2.0 * v_tile_m(v) * v_tile_n(v) * ((double)d->K / sp);
  double block_rate = v == 7 ? 1.35e15 / 256 : 1.1e15 / 512;
  if (v != 7 && blocks <= 256) block_rate *= 1.4;
  double t = rounds * block_flop / block_rate;
  if (sp > 1) {
    if (v == 7 && batch == 1 && d->epilogue == SLX_EPI_STORE && d->out_f32 && split_ws_fits(d, (long)tiles, sp))
      t += 5e-6;  // in-launch reduction: one 256 KiB slab per tile read by its last arriver
    else
      t += (double)sp * M * d->N * 4.0 / 1.3e12;  // f32 atomics: ~1.3 TB/s chip-wide
  }
  if (v == 7 && blocks < 192) t *= 1.5;  // an under-filled 256x256 grid leaves whole CUs idle
  return t;
}

// ---- M remainder (rows past the last whole 256-row tile, e.g. InternViT's 16 class-token rows of 16400) ----
// Instead of a 16-row tile walking the whole K on a few CUs (latency-bound, 15-85 us), the remainder is a split-K
// GEMM over ~all CUs writing f32 partials (plain stores, split-major), then one kernel that sums the splits and runs
// the real epilogue on the rem x N accumulators. One thread per output column walks the rem rows, so the colsum
// partial row of these rows comes out of the same pass.
template <int EPI, typename OutT>
__global__ __launch_bounds__(256) void rows_epilogue_kernel(GemmArgs p, const float* __restrict__ part, int nsplit,
                                                            long split_stride, int colsum_row) {
  // block = 64 columns x 4 row lanes over rows [blockIdx.y * rpb, +rpb) (rpb = M when the colsum partial row is
  // needed, else 4: one row per thread); each thread sums its rows' split partials, 8 loads in flight
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + tx;
  const int rpb = p.colsum ? p.M : 4;
  const int mend = min(p.M, (int)(blockIdx.y + 1) * rpb);
  float cs = 0.f;
  if (n < p.N) {
    OutT* C = reinterpret_cast<OutT*>(p.C);
    for (int m = blockIdx.y * rpb + ty; m < mend; m += 4) {
      const float* q = part + (long)m * p.N + n;
      float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int y = 0;
      for (; y + 8 <= nsplit; y += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] += q[(long)(y + u) * split_stride];
      }
      for (; y < nsplit; ++y) a[0] += q[(long)y * split_stride];
      const float acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
      epilogue_elem<EPI, OutT>(p, C, m, n, acc);
      if constexpr (EPI == EPI_STORE) cs += acc * p.alpha + (p.bias ? p.bias[n] : 0.f);
      else if constexpr (EPI == EPI_GELU_BWD) cs += acc * p.alpha * act_bwd<EPI_GELU_BWD>((float)p.aux[(long)m * p.ldaux + n], p.aux_grad);
      else if constexpr (EPI == EPI_QGELU_BWD) cs += acc * p.alpha * act_bwd<EPI_QGELU_BWD>((float)p.aux[(long)m * p.ldaux + n], p.aux_grad);
    }
  }
  if (p.colsum) {
    red[ty][tx] = cs;
    __syncthreads();
    if (ty == 0 && n < p.N) p.colsum_ws[(long)colsum_row * p.N + n] = red[0][tx] + red[1][tx] + red[2][tx] + red[3][tx];
  }
}

// colsum partials: out[n] += sum over rows r < nrows of ws[r][n]; 32 rows per thread, one atomic per (column, 32 rows)
__global__ __launch_bounds__(256) void colsum_reduce_kernel(const float* __restrict__ ws, int nrows, int N,
                                                            float* __restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int r0 = blockIdx.y * 32, r1 = min(nrows, r0 + 32);
  float s = 0.f;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) s += ws[(long)r * N + n];
  atomicAdd(out + n, s);
}

static int colsum_reduce(const slx_gemm_desc* d, hipStream_t st) {
  const int nrows = (d->M + 63) / 64;
  if (det_mode().on)  // deterministic mode: every column summed by one thread in row order (no atomics)
    return det_reduce(d->colsum_ws, nrows, d->N, d->N, d->colsum, 1, st);
  hipLaunchKernelGGL(colsum_reduce_kernel, dim3((d->N + 255) / 256, (nrows + 31) / 32), dim3(256), 0, st,
                     (const float*)d->colsum_ws, nrows, d->N, d->colsum);
  SLX_LAUNCH_CHECK("slx_gemm_bf16(colsum reduce)");
  return 0;
}

constexpr long kRemCntInts = 4096;  // arrival counters at the end of rem_ws (zeroed once by the caller)
// SLX_GEMM_FOLD_REM=0: the M remainder as its own split-K launch + epilogue launch (A/B)
static bool fold_off() {
  static const bool off = [] { const char* e = getenv("SLX_GEMM_FOLD_REM"); return e && atoi(e) == 0; }();
  return off;
}

static int gemm_launch(const slx_gemm_desc* d, int v, hipStream_t st, int mshift_last = 0, int colsum_row0 = 0,
                       int force_split = 0, long split_stride = 0, int rem_r0 = 0) {
  GemmArgs a;
  a.split_stride = split_stride;
  a.rem_r0 = rem_r0; a.rem_nsplit = 0; a.rem_kc = 0;
  a.rem_part = rem_r0 ? d->rem_ws : nullptr;
  a.rem_cnt = rem_r0 ? reinterpret_cast<int*>(d->rem_ws + d->rem_ws_floats - kRemCntInts) : nullptr;
  a.A = (const bf16*)d->A; a.B = (const bf16*)d->B; a.C = d->C;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.sA = d->sA; a.sB = d->sB; a.sC = d->sC;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.alpha = d->alpha;
  a.bias = d->bias; a.ls = d->ls;
  a.aux = (const bf16*)d->aux; a.ldaux = d->ldaux;
  a.aux_out = (bf16*)d->aux_out; a.ldaux_out = d->ldaux_out;
  a.resid = d->resid; a.ldr = d->ldr; a.resid_bf16 = d->resid_bf16;
  a.accumulate = d->accumulate;
  a.seed = d->seed; a.drop_p = d->drop_p; a.ldmask = d->ldmask;
  a.drop_operand = d->drop_operand;
  a.colsum = d->colsum;
  a.colsum_ws = d->colsum_ws;
  a.maskbits = d->maskbits; a.ldbits = d->ldbits;
  a.colsum_row0 = colsum_row0;
  a.split_ws = nullptr; a.split_cnt = nullptr; a.split_tile0 = 0;
  a.rope_cos = d->rope_cos; a.rope_sin = d->rope_sin; a.rope_S = d->rope_S; a.rope_ncols = d->rope_ncols;
  a.aux_grad = d->aux_grad;
  a.mshift_last = 0;
  a.tilesM = (d->M + BM - 1) / BM;
  a.tilesN = (d->N + BN - 1) / BN;
  {
    bool ok = d->ldc % 8 == 0 && ((uintptr_t)d->C % 16) == 0 && (d->batch <= 1 || d->sC % 8 == 0);
    if (d->aux) ok = ok && d->ldaux % 8 == 0 && ((uintptr_t)d->aux % 16) == 0;
    if (d->aux_out) ok = ok && d->ldaux_out % 8 == 0 && ((uintptr_t)d->aux_out % 16) == 0;
    if (d->resid) ok = ok && d->ldr % 8 == 0 && ((uintptr_t)d->resid % 16) == 0;
    if (d->epilogue == SLX_EPI_SWIGLU_BWD || d->epilogue == SLX_EPI_DROPMASK_SWIGLU) ok = ok && d->N % 8 == 0;
    a.vec_ok = ok ? 1 : 0;
  }
  const int batch = d->batch < 1 ? 1 : d->batch;
  a.mshift_last = (v >= 7 && v <= 11) ? mshift_last : 0;
  a.ksplit = 1;
  a.kchunk = d->K;
  {  // split-K for under-filled grids (weight gradients): f32 atomics, >= 4 K-steps per split
    int sp = (rem_r0 || d->rope_cos) ? 1 : force_split > 0 ? force_split : split_for(d, (v >= 7 && v <= 11) ? 7 : v, d->M, batch);  // (no split-K with a fold)
    const int ksteps = (d->K + BK - 1) / BK;
    if (sp > 1) {
      const int per = ((ksteps + sp - 1) / sp) * BK;
      sp = (d->K + per - 1) / per;
    }
    if (sp > 1) {
      a.ksplit = sp;
      a.kchunk = ((ksteps + sp - 1) / sp) * BK;
      const long v3tiles = (long)((d->M + V3_BM - 1) / V3_BM) * ((d->N + V3_BN - 1) / V3_BN);
      if ((v == 7 || v == 8 || v >= 11) && batch == 1 && !split_stride && d->epilogue == SLX_EPI_STORE && d->out_f32 &&
          split_ws_fits(d, v3tiles, sp)) {  // reduced inside the launch: plain stores, no pre-zeroed C
        a.split_ws = d->split_ws;
        a.split_cnt = reinterpret_cast<int*>(d->split_ws + d->split_ws_floats - kSplitCntInts);
      }
      if (det_mode().on && !a.split_ws && !split_stride) {  // deterministic mode: no f32-atomic split-K
        sp = 1;
        a.ksplit = 1;
        a.kchunk = d->K;
      }
    }
    if (sp > 1) {
      if (!d->accumulate && !split_stride && !a.split_ws) {
        hipError_t e = hipMemset2DAsync(d->C, d->ldc * sizeof(float), 0, (size_t)d->N * sizeof(float), d->M, st);
        if (e != hipSuccess) { set_error("slx_gemm_bf16: memset2D failed: %s", hipGetErrorString(e)); return -1000 - (int)e; }
      }
    }
  }
  {  // more than one round of 256^2 tiles: the FE member (the next tile's loads overlap this tile's epilogue; on a
     // single round there is no next tile and the LDS-staged epilogue is as fast or faster: gemm_epi_bench proj)
    // Single-round launches too with the plain STORE epilogue (SLX_GEMM_FE1=1, default): register-direct stores
    // measured 824 vs 711 TF on the InternViT proj dgrad shape and 1247 vs 1176 on the fc1 dgrad shape
    // (tools/gemm_bench.py), +0.7 % on the step (profiles/round4_fe1_ab.txt); SLX_GEMM_FE1=2 adds every epilogue
    static const bool fe_on = [] { const char* e = getenv("SLX_GEMM_FE"); return !e || atoi(e) != 0; }();
    static const int fe1 = [] { const char* e = getenv("SLX_GEMM_FE1"); return e ? atoi(e) : 1; }();
    const long t3 = (long)(((rem_r0 > 0 ? rem_r0 : d->M) + V3_BM - 1) / V3_BM) * ((d->N + V3_BN - 1) / V3_BN);
    const bool single_ok = fe1 >= 2 || (fe1 == 1 && d->epilogue == SLX_EPI_STORE);
    if (v == 7 && fe_on && batch == 1 && (t3 > 256 || single_ok) && !d->rope_cos) v = 11;
  }
  SLX_CHECK_ARG(!d->colsum || (d->colsum_ws && a.vec_ok && a.ksplit == 1 && v != 1 && d->N % 8 == 0 &&
                                (d->epilogue == SLX_EPI_STORE || d->epilogue == SLX_EPI_GELU_BWD ||
                                 d->epilogue == SLX_EPI_QGELU_BWD)),
                "slx_gemm_bf16: colsum needs the vector epilogue (16-B aligned rows, N %% 8 == 0), no split-K, a "
                "DMA/v3 main loop and a STORE / GELU_BWD / QGELU_BWD epilogue");
  switch (d->epilogue) {
    case SLX_EPI_STORE:
      return d->out_f32 ? dispatch_layout<EPI_STORE, float>(d->layout, a, batch, st, v)
                        : dispatch_layout<EPI_STORE, bf16>(d->layout, a, batch, st, v);
    case SLX_EPI_GELU:
      SLX_CHECK_ARG(!d->out_f32 && d->layout == SLX_GEMM_NT && d->aux_out, "slx_gemm_bf16: GELU needs NT, bf16 out, aux_out");
      return launch_any<true, true, EPI_GELU, bf16>(a, batch, st, v);
    case SLX_EPI_RESID_LS:
      SLX_CHECK_ARG(d->out_f32 && d->layout == SLX_GEMM_NT && d->resid && d->ls, "slx_gemm_bf16: RESID_LS needs NT, f32 out, resid, ls");
      return launch_any<true, true, EPI_RESID_LS, float>(a, batch, st, v);
    case SLX_EPI_GELU_BWD:
      SLX_CHECK_ARG(!d->out_f32 && (d->layout == SLX_GEMM_NN || d->layout == SLX_GEMM_NT) && d->aux,
                    "slx_gemm_bf16: GELU_BWD needs NN or NT, bf16 out, aux");
      if (d->layout == SLX_GEMM_NT) return launch_any<true, true, EPI_GELU_BWD, bf16>(a, batch, st, v);
      return launch_any<true, false, EPI_GELU_BWD, bf16>(a, batch, st, v);
    case SLX_EPI_QGELU:
      SLX_CHECK_ARG(!d->out_f32 && d->layout == SLX_GEMM_NT && d->aux_out, "slx_gemm_bf16: QGELU needs NT, bf16 out, aux_out");
      return launch_any<true, true, EPI_QGELU, bf16>(a, batch, st, v);
    case SLX_EPI_QGELU_BWD:
      SLX_CHECK_ARG(!d->out_f32 && (d->layout == SLX_GEMM_NN || d->layout == SLX_GEMM_NT) && d->aux,
                    "slx_gemm_bf16: QGELU_BWD needs NN or NT, bf16 out, aux");
      if (d->layout == SLX_GEMM_NT) return launch_any<true, true, EPI_QGELU_BWD, bf16>(a, batch, st, v);
      return launch_any<true, false, EPI_QGELU_BWD, bf16>(a, batch, st, v);
    case SLX_EPI_SWIGLU_BWD:
      SLX_CHECK_ARG(!d->out_f32 && d->layout == SLX_GEMM_NN && d->aux, "slx_gemm_bf16: SWIGLU_BWD needs NN, bf16 out, aux");
      return launch_any<true, false, EPI_SWIGLU_BWD, bf16>(a, batch, st, v);
    case SLX_EPI_DROPMASK:
      SLX_CHECK_ARG(d->out_f32 && d->layout == SLX_GEMM_NN, "slx_gemm_bf16: DROPMASK needs NN, f32 out");
      return launch_any<true, false, EPI_DROPMASK, float>(a, batch, st, v);
    case SLX_EPI_DROPMASK_SWIGLU:
      SLX_CHECK_ARG(!d->out_f32 && d->layout == SLX_GEMM_NN && d->aux && d->resid,
                    "slx_gemm_bf16: DROPMASK_SWIGLU needs NN, bf16 out, aux (gate|up), resid (f32 or bf16 base grad)");
      SLX_CHECK_ARG(!d->resid_bf16 || d->epilogue == SLX_EPI_DROPMASK_SWIGLU, "slx_gemm_bf16: resid_bf16 is for DROPMASK_SWIGLU");
      if (d->resid_bf16) return launch_any<true, false, EPI_DROPMASK_SWIGLU_B, bf16>(a, batch, st, v);
      return launch_any<true, false, EPI_DROPMASK_SWIGLU, bf16>(a, batch, st, v);
  }
  set_error("slx_gemm_bf16: bad epilogue %d", d->epilogue);
  return -22;
}

template <int EPI, typename OutT>
static int launch_rows(GemmArgs& a, const float* part, int nsplit, long split_stride, int colsum_row, hipStream_t st) {
  const unsigned gy = a.colsum ? 1u : (unsigned)((a.M + 3) / 4);
  hipLaunchKernelGGL((rows_epilogue_kernel<EPI, OutT>), dim3((a.N + 63) / 64, gy), dim3(256), 0, st, a, part, nsplit,
                     split_stride, colsum_row);
  SLX_LAUNCH_CHECK("slx_gemm_bf16(remainder epilogue)");
  return 0;
}

// Rows [r0, M) of d (fewer than 256): split-K partials over the whole chip, then the epilogue kernel. Returns 1 (and
// launches nothing) when the caller's remainder workspace is missing or too small.
static int gemm_remainder(const slx_gemm_desc* d, int r0, hipStream_t st) {
  const int rem = d->M - r0;
  const bool ak = d->layout == SLX_GEMM_NT || d->layout == SLX_GEMM_NN;
  const int ksteps = (d->K + BK - 1) / BK;
  const int tilesN = (d->N + BN - 1) / BN;
  int sp = 512 / tilesN;                 // ~2 blocks per CU
  sp = sp < ksteps / 2 ? sp : ksteps / 2;  // >= 2 K-steps per split
  sp = sp < 1 ? 1 : (sp > 32 ? 32 : sp);
  const int kchunk = ((ksteps + sp - 1) / sp);
  sp = (ksteps + kchunk - 1) / kchunk;
  const long stride = (long)rem * d->N;
  if (!d->rem_ws || d->rem_ws_floats - kRemCntInts < stride * sp) return 1;
  slx_gemm_desc t = *d;
  t.M = rem;
  t.A = ak ? (const void*)((const bf16*)d->A + (long)r0 * d->lda) : (const void*)((const bf16*)d->A + r0);
  t.C = d->rem_ws; t.ldc = d->N; t.out_f32 = 1;
  t.epilogue = SLX_EPI_STORE; t.alpha = 1.f; t.bias = nullptr; t.ls = nullptr; t.accumulate = 0;
  t.aux = nullptr; t.aux_out = nullptr; t.resid = nullptr; t.colsum = nullptr; t.batch = 1;
  int rc = gemm_launch(&t, 2, st, 0, 0, sp, stride);
  if (rc) return rc;
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  const size_t csz = d->out_f32 ? 4 : 2;
  a.C = (void*)((char*)d->C + (size_t)r0 * d->ldc * csz);
  a.ldc = d->ldc;
  a.M = rem; a.N = d->N; a.K = d->K;
  a.alpha = d->alpha;
  a.bias = d->bias; a.ls = d->ls;
  a.aux = d->aux ? (const bf16*)d->aux + (long)r0 * d->ldaux : nullptr; a.ldaux = d->ldaux;
  a.aux_out = d->aux_out ? (bf16*)d->aux_out + (long)r0 * d->ldaux_out : nullptr; a.ldaux_out = d->ldaux_out;
  a.resid = d->resid ? d->resid + (long)r0 * d->ldr : nullptr; a.ldr = d->ldr;
  a.accumulate = d->accumulate;
  a.ksplit = 1;
  a.colsum = d->colsum; a.colsum_ws = d->colsum_ws;
  const float* part = d->rem_ws;
  const int crow = r0 / 64;
  switch (d->epilogue) {
    case SLX_EPI_STORE:
      return d->out_f32 ? launch_rows<EPI_STORE, float>(a, part, sp, stride, crow, st)
                        : launch_rows<EPI_STORE, bf16>(a, part, sp, stride, crow, st);
    case SLX_EPI_GELU: return launch_rows<EPI_GELU, bf16>(a, part, sp, stride, crow, st);
    case SLX_EPI_RESID_LS: return launch_rows<EPI_RESID_LS, float>(a, part, sp, stride, crow, st);
    case SLX_EPI_GELU_BWD: return launch_rows<EPI_GELU_BWD, bf16>(a, part, sp, stride, crow, st);
    case SLX_EPI_QGELU: return launch_rows<EPI_QGELU, bf16>(a, part, sp, stride, crow, st);
    case SLX_EPI_QGELU_BWD: return launch_rows<EPI_QGELU_BWD, bf16>(a, part, sp, stride, crow, st);
    case SLX_EPI_SWIGLU_BWD: return launch_rows<EPI_SWIGLU_BWD, bf16>(a, part, sp, stride, crow, st);
  }
  return 1;  // DROPMASK epilogues index the mask by absolute row: not handled here
}

}  // namespace slx

using namespace slx;

extern "C" int slx_gemm_bf16(const slx_gemm_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d != nullptr, "slx_gemm_bf16: null desc");
  SLX_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0, "slx_gemm_bf16: negative dims");
  if (d->M == 0 || d->N == 0 || d->batch == 0) return 0;
  const bool ak = d->layout == SLX_GEMM_NT || d->layout == SLX_GEMM_NN;
  const bool bk = d->layout == SLX_GEMM_NT || d->layout == SLX_GEMM_TT;
  // contiguous dimension of every operand must allow 16-byte vector loads
  SLX_CHECK_ARG((ak ? d->K : d->M) % 8 == 0, "slx_gemm_bf16: A contiguous dim (%d) must be a multiple of 8",
                ak ? d->K : d->M);
  SLX_CHECK_ARG((bk ? d->K : d->N) % 8 == 0, "slx_gemm_bf16: B contiguous dim (%d) must be a multiple of 8",
                bk ? d->K : d->N);
  SLX_CHECK_ARG(d->lda % 8 == 0 && d->ldb % 8 == 0, "slx_gemm_bf16: lda/ldb must be multiples of 8");
  SLX_CHECK_ARG(((uintptr_t)d->A & 15) == 0 && ((uintptr_t)d->B & 15) == 0, "slx_gemm_bf16: A/B must be 16B aligned");
  SLX_CHECK_ARG(d->batch == 1 || (d->sA % 8 == 0 && d->sB % 8 == 0), "slx_gemm_bf16: batch strides must be multiples of 8");
  SLX_CHECK_ARG(d->drop_operand == 0 || (d->epilogue == SLX_EPI_STORE && d->drop_p >= 0.f && d->drop_p < 1.f),
                "slx_gemm_bf16: operand dropout needs EPI_STORE and 0 <= p < 1");
  hipStream_t st = (hipStream_t)stream;
  const int batch = d->batch < 1 ? 1 : d->batch;
  const bool dma_ok = (!ak || d->K % BK == 0) && (!bk || d->K % BK == 0) && d->drop_operand == 0;
  int v = d->variant;
  // The 256-row family shares the remainder handling (fold / overlapped last tile / peel): 7 = v3, 8 = v3 with
  // swapped operands + batched-load epilogue, 9 / 10 = v4 (two workgroups per CU) without / with the swap.
  // SLX_V3_KIND picks the member the automatic choice launches (A/B hook).
  static const int kind_default = [] { const char* e = getenv("SLX_V3_KIND"); const int k = e ? atoi(e) : 7;
                                       return k >= 7 && k <= 11 ? k : 7; }();
  int v3k = kind_default;
  if (v >= 8 && v <= 11) { v3k = v; v = 7; }
  else if (v == 7) v3k = 7;
  SLX_CHECK_ARG(!d->rope_cos || (d->rope_sin && d->epilogue == SLX_EPI_STORE && !d->out_f32 && !d->accumulate &&
                                  batch == 1 && !d->colsum && d->rope_S > 0 && d->rope_ncols % 64 == 0 &&
                                  d->K % BK == 0 && d->drop_operand == 0 && d->variant != 1 &&
                                  d->rope_ncols <= d->N && d->ldc % 8 == 0 && ((uintptr_t)d->C & 15) == 0 &&
                                  ((uintptr_t)d->rope_cos & 15) == 0 && ((uintptr_t)d->rope_sin & 15) == 0),
                "slx_gemm_bf16: RoPE needs a bf16 STORE epilogue without accumulate / colsum / batch, K %% 64 == 0 (the "
                "LDS-staged main loops), 16-B aligned C rows and tables, rope_S > 0 and rope_ncols a multiple of 64 not "
                "past N");
  const int rem = d->M % V3_BM;
  const bool peel_ok = batch == 1 && d->epilogue != SLX_EPI_DROPMASK && d->epilogue != SLX_EPI_DROPMASK_SWIGLU &&
                       d->M > V3_BM && rem > 0 && rem <= 64 && !d->rope_cos;  // (RoPE: partial last tile instead)
  if (v == 0) {
    v = dma_ok ? 2 : 1;
    if (dma_ok) {
      const int Mmain = peel_ok ? d->M - rem : d->M;
      double c3 = v_cost(d, 7, Mmain, batch);
      if (peel_ok) c3 += v_cost(d, 2, rem, batch);  // (the overlapped last tile costs less than this peel)
      if (c3 < v_cost(d, 2, d->M, batch)) v = 7;
    }
  }
  // A write-once epilogue (no accumulation into C, no split-K atomics) tolerates two blocks storing the same
  // rows: the last M tile is shifted to end at M instead of peeling the remainder into a second, latency-bound
  // launch (16 extra rows cost 1/65 of the grid; the peel cost ~8% of an InternViT FC1).
  const bool overlap_ok = peel_ok && !d->accumulate && !d->colsum && split_for(d, 7, d->M, batch) == 1 &&
                          !(d->resid && d->resid == (const float*)d->C) && d->aux != (const void*)d->C;
  // ... but only when the extra tile row does not cost a whole extra block round (measured: InternViT FC1's
  // 64x16 main grid is exactly 4 rounds of 256, the overlap makes it 5 and the step 5% slower than the peel)
  if (v == 7 && dma_ok && overlap_ok &&
      v_cost(d, 7, d->M, batch) < v_cost(d, 7, d->M - rem, batch) + v_cost(d, 2, rem, batch))
    return gemm_launch(d, v3k, st, 1);  // (overlap_ok excludes colsum: shifted rows would be summed twice)
  if (v == 7 && dma_ok && peel_ok) {
    // main block rows on v3, the M remainder on v2 (same stream, same epilogue)
    slx_gemm_desc m = *d, t = *d;
    m.M = d->M - rem;
    t.M = rem;
    const long r0 = m.M;
    const size_t csz = d->out_f32 ? 4 : 2;
    t.A = ak ? (const void*)((const bf16*)d->A + r0 * d->lda) : (const void*)((const bf16*)d->A + r0);
    t.C = (void*)((char*)d->C + (size_t)r0 * d->ldc * csz);
    if (d->aux) t.aux = (const void*)((const bf16*)d->aux + r0 * d->ldaux);
    if (d->aux_out) t.aux_out = (void*)((bf16*)d->aux_out + r0 * d->ldaux_out);
    if (d->resid) t.resid = d->resid + r0 * d->ldr;
    // The peel is a handful of blocks walking the whole K: latency-bound, so give it the 4-stage ring and run it on
    // a side stream next to the main grid (it writes disjoint rows of C); the caller's stream joins it after.
    const int row0 = m.M / 64;  // the remainder's colsum partial rows follow the main grid's
    // Remainder rows: split-K over the whole chip + epilogue kernel (workspace permitting), else the classic peel
    // (a few latency-bound blocks walking all of K on the 4-stage ring). Serial on the caller's stream: running
    // them next to the main grid (side stream) measured slower - v3 holds one 139 KB block per CU and whole rounds
    // of 256 blocks, so any CU taken by a side kernel delays a main block.
    // A K-contiguous (the activation-row GEMMs that have a remainder): fold the remainder rows into the v3 launch
    const int ncg = (d->N + 255) / 256;
    if (ak && !fold_off() && d->rem_ws && d->rem_ws_floats - kRemCntInts >= 16L * rem * d->N && ncg <= kRemCntInts) {
      const int rc = gemm_launch(d, v3k, st, 0, 0, 0, 0, m.M);
      if (rc) return rc;
      return d->colsum ? colsum_reduce(d, st) : 0;
    }
    int rc = gemm_launch(&m, v3k, st);
    if (!rc) rc = gemm_remainder(d, m.M, st);
    if (rc == 1) rc = gemm_launch(&t, 4, st, 0, row0);
    if (rc) return rc;
    return d->colsum ? colsum_reduce(d, st) : 0;
  }
  const int rc = gemm_launch(d, v == 7 ? v3k : v, st);
  if (rc) return rc;
  return d->colsum ? colsum_reduce(d, st) : 0;
}

// ---- fused LM head + cross entropy (LanguageAdaptor.compute_loss, adaptors.py:259-274, on the gathered loss rows) ----
// Forward: the LM-head GEMM (NT, feat [R][D] x W [V][D]^T) keeps its logits in registers / LDS; its epilogue
// writes one (max, sum exp) pair per row and 64-column sub-tile plus the label logit, and ce_combine_kernel folds
// the pairs into lse and the loss. Backward: the same GEMM recomputed with the softmax-gradient epilogue writing
// bf16 dlogits [R][ldd] (the operand of the dlogits x W dgrad). No f32 [R, V] logits buffer exists.
__global__ __launch_bounds__(256) void ce_combine_kernel(const float* __restrict__ part, int ntile, const float* __restrict__ lab_logit,
                                                         const int* __restrict__ labels, int V, float* loss, float* lse) {
  __shared__ float sh[16];
  const long r = blockIdx.x;
  const float2* pr = reinterpret_cast<const float2*>(part) + r * ntile;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < ntile; i += blockDim.x) mx = fmaxf(mx, pr[i].x);
  mx = warp_max(mx);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  float s = 0.f;
  for (int i = threadIdx.x; i < ntile; i += blockDim.x) {
    const float2 q = pr[i];
    s += q.x == -INFINITY ? 0.f : q.y * __expf(q.x - mx);
  }
  __syncthreads();
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    const float l = mx + __logf(s);
    lse[r] = l;
    const int lab = labels[r];
    loss[r] = (lab >= 0 && lab < V) ? l - lab_logit[r] : 0.f;  // ignore_index (-1): 0, as F.cross_entropy
  }
}

static void ce_args(GemmArgs& a, const void* feat, int64_t ldf, const void* W, int64_t ldw, int64_t R, int V, int D) {
  memset(&a, 0, sizeof(a));
  a.A = (const bf16*)feat; a.lda = ldf;
  a.B = (const bf16*)W; a.ldb = ldw;
  a.M = (int)R; a.N = V; a.K = D;
  a.alpha = 1.f;
  a.ksplit = 1; a.kchunk = D;
  a.tilesN = (V + BN - 1) / BN;
}

// one (max, sumexp) pair per row and 64-column sub-tile of the 128-column GEMM tiles, + the label logits
static int ce_ntile(int V) { return 2 * ((V + BN - 1) / BN); }
extern "C" int slx_lmhead_ce_ws_floats(int64_t R, int V) { return (int)(R * 2 * ce_ntile(V) + R); }

extern "C" int slx_lmhead_ce_fwd(const void* feat, int64_t ldf, const void* W, int64_t ldw, const int* labels, int64_t R,
                                 int V, int D, float* loss, float* lse, float* ws, int64_t ws_floats, slx_stream_t stream) {
  if (R <= 0) return 0;
  SLX_CHECK_ARG(feat && W && labels && loss && lse && ws, "slx_lmhead_ce_fwd: null pointer");
  SLX_CHECK_ARG(D % BK == 0 && ldf % 8 == 0 && ldw % 8 == 0 && ((uintptr_t)feat & 15) == 0 && ((uintptr_t)W & 15) == 0,
                "slx_lmhead_ce_fwd: D %% %d == 0, 16-B aligned operands, leading dims multiples of 8", BK);
  const int nt = ce_ntile(V);
  SLX_CHECK_ARG(ws_floats >= R * 2 * nt + R, "slx_lmhead_ce_fwd: workspace %lld < %lld floats", (long long)ws_floats,
                (long long)(R * 2 * nt + R));
  GemmArgs a;
  ce_args(a, feat, ldf, W, ldw, R, V, D);
  a.ce_labels = labels; a.ce_part = ws; a.ce_lab = ws + R * 2 * nt; a.ce_ldpart = nt;
  hipStream_t st = (hipStream_t)stream;
  const int rc = launch_v2<true, true, EPI_CE_PART, float, 128, 2>(a, 1, st);
  if (rc) return rc;
  hipLaunchKernelGGL(ce_combine_kernel, dim3((unsigned)R), dim3(256), 0, st, (const float*)ws, nt, (const float*)a.ce_lab,
                     labels, V, loss, lse);
  SLX_LAUNCH_CHECK("slx_lmhead_ce_fwd(combine)");
  return 0;
}

extern "C" int slx_lmhead_ce_bwd(const void* feat, int64_t ldf, const void* W, int64_t ldw, const int* labels,
                                 const float* lse, int64_t R, int V, int D, const float* gscale, void* dlogits, int64_t ldd,
                                 slx_stream_t stream) {
  if (R <= 0) return 0;
  SLX_CHECK_ARG(feat && W && labels && lse && gscale && dlogits, "slx_lmhead_ce_bwd: null pointer");
  SLX_CHECK_ARG(D % BK == 0 && ldf % 8 == 0 && ldw % 8 == 0 && ldd % 8 == 0 && ldd >= ((V + 127) / 128) * 128 &&
                ((uintptr_t)feat & 15) == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)dlogits & 15) == 0,
                "slx_lmhead_ce_bwd: D %% %d == 0, ldd >= V rounded up to 128, 16-B aligned operands", BK);
  GemmArgs a;
  ce_args(a, feat, ldf, W, ldw, R, V, D);
  a.C = dlogits; a.ldc = ldd;
  a.ce_labels = labels; a.ce_lse = lse; a.ce_gscale = gscale;
  return launch_v2<true, true, EPI_CE_GRAD, float, 128, 2>(a, 1, (hipStream_t)stream);
}

// Two accumulating f32-output GEMMs of one layout and one K in a single v3 launch (gemm_bf16_v3_pair_kernel): the
// InternViT weight gradients come in pairs whose separate grids under-fill the chip (fc1/fc2: 64 tiles of 256^2
// each, qkv/proj: 48 + 16 tiles, K = 16400 tokens); together they split K over one full round of 256 blocks.
static void pair_args(const slx_gemm_desc* d, GemmArgs& a) {
  memset(&a, 0, sizeof(a));
  a.split_ws = nullptr; a.split_cnt = nullptr; a.split_tile0 = 0;
  a.A = (const bf16*)d->A; a.B = (const bf16*)d->B; a.C = d->C;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.alpha = d->alpha;
  a.accumulate = 1;
  a.vec_ok = d->ldc % 8 == 0 && ((uintptr_t)d->C % 16) == 0;
  a.tilesM = (d->M + V3_BM - 1) / V3_BM;
  a.tilesN = (d->N + V3_BN - 1) / V3_BN;
}

template <bool AK, bool BKc, bool SW>
static int launch_pair(GemmArgs& a, GemmArgs& b, hipStream_t st) {
  constexpr int LDS_RING = 2 * (V3_BM * BK * 2 + V3_BN * BK * 2);
  constexpr int LDS_EP = 8 * 64 * EP_LD * 4 + 16;  // + the split-K role word
  constexpr int LDS = LDS_RING > LDS_EP ? LDS_RING : LDS_EP;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemm_bf16_v3_pair_kernel<AK, BKc, SW>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const int nt = a.tilesM * a.tilesN + b.tilesM * b.tilesN, sp = a.ksplit;
  static const bool xs_env = [] { const char* e = getenv("SLX_PAIR_XCD_SPLIT"); return e ? atoi(e) != 0 : true; }();
  const bool xs = xs_env && nt * sp == 256 && (sp == 1 || sp == 2 || sp == 4 || sp == 8) && nt % (8 / sp) == 0;
  a.xcd_split = b.xcd_split = xs ? 1 : 0;
  dim3 grid = xs ? dim3(256) : dim3(nt, sp);
  hipLaunchKernelGGL((gemm_bf16_v3_pair_kernel<AK, BKc, SW>), grid, dim3(512), LDS, st, a, b);
  SLX_LAUNCH_CHECK("slx_gemm_bf16_pair");
  return 0;
}

extern "C" int slx_gemm_bf16_pair(const slx_gemm_desc* d1, const slx_gemm_desc* d2, slx_stream_t stream) {
  SLX_CHECK_ARG(d1 && d2, "slx_gemm_bf16_pair: null desc");
  SLX_CHECK_ARG(d1->layout == d2->layout && d1->K == d2->K, "slx_gemm_bf16_pair: the two GEMMs need one layout and one K");
  for (const slx_gemm_desc* d : {d1, d2}) {
    SLX_CHECK_ARG(d->M > 0 && d->N > 0 && d->K > 0 && d->batch <= 1, "slx_gemm_bf16_pair: positive dims, no batch");
    SLX_CHECK_ARG(d->epilogue == SLX_EPI_STORE && d->out_f32 && d->accumulate && !d->colsum && !d->bias &&
                  d->drop_operand == 0, "slx_gemm_bf16_pair: f32 accumulate STORE only (no bias / colsum / dropout)");
    const bool ak = d->layout == SLX_GEMM_NT || d->layout == SLX_GEMM_NN;
    const bool bk = d->layout == SLX_GEMM_NT || d->layout == SLX_GEMM_TT;
    SLX_CHECK_ARG((ak ? d->K : d->M) % 8 == 0 && (bk ? d->K : d->N) % 8 == 0 && d->lda % 8 == 0 && d->ldb % 8 == 0 &&
                  ((uintptr_t)d->A & 15) == 0 && ((uintptr_t)d->B & 15) == 0,
                  "slx_gemm_bf16_pair: 16-B aligned operands with contiguous dims and leading dims multiples of 8");
    SLX_CHECK_ARG((!ak || d->K % BK == 0) && (!bk || d->K % BK == 0), "slx_gemm_bf16_pair: K-contiguous operands need K %% %d == 0", BK);
  }
  GemmArgs a, b;
  pair_args(d1, a);
  pair_args(d2, b);
  const int tiles = a.tilesM * a.tilesN + b.tilesM * b.tilesN;
  const int ksteps = (d1->K + BK - 1) / BK;
  int sp = 256 / tiles;  // one round of 256 blocks
  if (sp > ksteps / 4) sp = ksteps / 4;
  if (d1->ksplit_max > 0 && sp > d1->ksplit_max) sp = d1->ksplit_max;
  if (sp < 1) sp = 1;
  // in-launch reduction (slabs in d1's split_ws) when split_ws_fits allows it, else f32 atomics
  const int per = ((ksteps + sp - 1) / sp) * BK;
  sp = (d1->K + per - 1) / per;
  bool red = split_ws_fits(d1, tiles, sp);
  if (det_mode().on && sp > 1 && !red) {  // deterministic mode: one split (no f32-atomic partials)
    sp = 1;
    red = false;
  }
  a.ksplit = b.ksplit = sp;
  a.kchunk = b.kchunk = sp > 1 ? per : d1->K;
  if (red && sp > 1) {
    a.split_ws = b.split_ws = d1->split_ws;
    a.split_cnt = b.split_cnt = reinterpret_cast<int*>(d1->split_ws + d1->split_ws_floats - kSplitCntInts);
    b.split_tile0 = a.tilesM * a.tilesN;
  }
  hipStream_t st = (hipStream_t)stream;
  static const bool sw_default = [] { const char* e = getenv("SLX_V3_KIND"); return e && atoi(e) == 8; }();
  const bool sw = d1->variant == 8 || (d1->variant == 0 && sw_default);
  switch (d1->layout) {
    case SLX_GEMM_NT: return sw ? launch_pair<true, true, true>(a, b, st) : launch_pair<true, true, false>(a, b, st);
    case SLX_GEMM_NN: return sw ? launch_pair<true, false, true>(a, b, st) : launch_pair<true, false, false>(a, b, st);
    case SLX_GEMM_TN: return sw ? launch_pair<false, false, true>(a, b, st) : launch_pair<false, false, false>(a, b, st);
    case SLX_GEMM_TT: return sw ? launch_pair<false, true, true>(a, b, st) : launch_pair<false, true, false>(a, b, st);
  }
  set_error("slx_gemm_bf16_pair: bad layout %d", d1->layout);
  return -22;
}
