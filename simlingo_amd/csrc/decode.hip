// KV-cached greedy decode for the SimLingo agent call (BASELINE.json configs[4]):
// DrivingModel.forward -> LLM.greedy_sample (simlingo_training/models/driving.py:131-176,
// simlingo_training/models/language_model/llm.py:178-250). The reference recomputes the whole prefix
// for every generated token; here the prefix is run once (batched MFMA kernels, the training
// forward's GEMMs) and each new token is one pass of the kernels below over a per-layer cache that is
// simply the fused q|k|v projection output [S_max, (Hq + 2 Hkv) * 64] (k already rotated).
//
// Decode is weight-streaming (M = 1): every GEMV reads its bf16 weight rows once with 16-B loads and
// reduces with wave shuffles; RMSNorm is recomputed per block from the f32 residual row (896 floats)
// instead of being its own launch; RoPE of the new q/k row is fused into the attention kernel; the
// LM-head GEMV keeps no logits and folds the argmax into 64-bit atomicMax keys (64 shards, reduced by
// the next step's begin kernel). All per-step scalars (position, #generated, done) live in a device
// slx_dec_state so one decode step can be captured once in a hipGraph and replayed; a step after
// the EOS token early-exits in every kernel.
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "../../include/slx.h"

namespace slx {

constexpr int kKeyShards = 64;
// attention.hip: the split MFMA form whose partials the O GEMV merges (slx_dec_attn_o_split), and the
// single-workgroup-per-kv-head MFMA form for caches of <= 1024 rows
int dec_attn_split_launch(void* cache, long ld, int Hq, int Hkv, const float* cos_tab, const float* sin_tab,
                          float* ws, int ns, const void* st, hipStream_t s);
int dec_attn_mfma_launch(void* cache, long ld, int Hq, int Hkv, const float* cos_tab, const float* sin_tab, void* out,
                         const void* st, hipStream_t s);
static long long* g_dec_trace = nullptr;  // tools only (slx_dec_attn_set_trace)
static int g_dec_force_split = 0;         // tests / tools only (slx_dec_attn_force_split)

// float -> order-preserving u32; key = value << 32 | (0xFFFFFFFF - index): max key = max value, then the
// smallest index (torch.argmax returns the first maximal element)
__device__ __forceinline__ unsigned long long argmax_key(float v, unsigned idx) {
  unsigned u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (unsigned long long)(0xFFFFFFFFu - idx);
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// streamed-once weight rows: nontemporal 16-B loads (the decode layer reads ~1 GB per token)
__device__ __forceinline__ uint4 ldnt16(const bf16* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ float dot8(const uint4 w, const bf16x8 x) {
  const bf16x8 wv = __builtin_bit_cast(bf16x8, w);
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) s = __builtin_fmaf((float)wv[e], (float)x[e], s);
  return s;
}

// ---- begin: take the token chosen by the previous step, record it, embed it ---------------------
__global__ __launch_bounds__(256) void dec_begin_kernel(slx_dec_state* st, unsigned long long* keys, const bf16* embed,
                                                        int D, float* X, int* tokens) {
  __shared__ int tok_s, run_s;
  if (threadIdx.x == 0) {
    unsigned long long k = 0;
    for (int i = 0; i < kKeyShards; ++i) {
      const unsigned long long v = keys[i];
      k = v > k ? v : k;
      keys[i] = 0ull;
    }
    const int tok = (int)(0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull));
    int run = 0;
    if (!st->done) {
      tokens[st->n_gen] = tok;
      st->n_gen += 1;
      st->pos += 1;
      // greedy_sample stops after recording EOS or max_new_tokens tokens (llm.py:225-248)
      if (tok == st->eos || st->n_gen >= st->max_new) st->done = 1;
      else run = 1;
    }
    tok_s = tok;
    run_s = run;
  }
  __syncthreads();
  if (!run_s) return;
  const bf16* src = embed + (long)tok_s * D;
  for (int j = threadIdx.x; j < D; j += blockDim.x) X[j] = (float)src[j];
}

// ---- GEMV y = W x (W [N][K] bf16 rows, x bf16 [K]) ------------------------------------------------
enum { GV_STORE_ROW = 0, GV_RESID = 1, GV_SWIGLU = 2, GV_ARGMAX = 3 };

struct GemvArgs {
  const bf16* W; long ldw; int N; int K;
  const float* X; const float* gamma; float eps;  // x = bf16(bf16(X * rstd) * gamma)  (Qwen2RMSNorm)
  const bf16* xb;                                  // or x given (bf16 [K])
  const float* bias;
  bf16* out; long out_ld;                          // STORE_ROW: out + pos * out_ld; SWIGLU: out[n]
  float* resid;                                    // RESID: resid[n] += y
  unsigned long long* keys;                        // ARGMAX
  int F;                                           // SWIGLU: up rows start at F (= N)
  const slx_dec_state* st;                         // may be null (prefill)
  long long* trace;                                // tools only (slx_dec_attn_set_trace): workgroup 0's phases
  // MG (slx_dec_attn_o_split): x = the attention output merged from the split partials of dec_attn_mfma_split_kernel,
  // part + (g*pns + s) * pG*66 = m[pG], l[pG], o[pG][64] of kv head g's split s; pout (optional) receives x (block 0)
  const float* part; int pns; int pG; bf16* pout;
};
constexpr int kMergeMaxNs = 8;

// One wave owns R output rows (SWIGLU: R gate + R up rows) of a row group; lane l holds 16-B chunks
// l, l+64, ... (CPL per row) of each row. Load order is the latency schedule of a batch-1 layer: the
// x vector (f32 residual row for the fused RMSNorm, or the bf16 input) first, then the first row
// group's weight stream, and only then the scalar done-flag check, so the norm waits for x alone
// (in-order vmcnt) and the flag / x / weight round trips all overlap.
constexpr int kGemvXPer = 8;  // x elements per thread held in registers (K <= 2048 with X, K <= 8192 with xb)
template <int MODE, int R, int CPL, bool MG = false>
__global__ __launch_bounds__(256) void dec_gemv_kernel(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* xs = reinterpret_cast<bf16*>(smem_raw);
  __shared__ float red[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = a.K, nch = K >> 3;
  float xv[kGemvXPer], gv[kGemvXPer];
  uint4 xq[kGemvXPer / 2];
  float pm[MG ? 4 : 1][kMergeMaxNs], pl[MG ? 4 : 1][kMergeMaxNs], po[MG ? 4 : 1][kMergeMaxNs];
  if constexpr (MG) {  // every split's (m, l, o) of this thread's 4 elements e = tid + 256 i (head e / 64), loaded at once
    const int stride = a.pG * 66;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, h = e >> 6, d = e & 63;
      const int g = h / a.pG, hh = h - g * a.pG;
      const float* base = a.part + (long)g * a.pns * stride;
#pragma unroll
      for (int sp = 0; sp < kMergeMaxNs; ++sp) {
        const bool ok = e < K && sp < a.pns;
        pm[i][sp] = ok ? base[sp * stride + hh] : -INFINITY;
        pl[i][sp] = ok ? base[sp * stride + a.pG + hh] : 0.f;
        po[i][sp] = ok ? base[sp * stride + 2 * a.pG + hh * 64 + d] : 0.f;
      }
    }
  } else if (a.X) {
#pragma unroll
    for (int i = 0; i < kGemvXPer; ++i) {
      const int j = tid + 256 * i;
      xv[i] = j < K ? a.X[j] : 0.f;
      gv[i] = j < K ? a.gamma[j] : 0.f;
    }
  } else {
#pragma unroll
    for (int i = 0; i < kGemvXPer / 2; ++i) {
      const int j = (tid + 256 * i) * 8;
      xq[i] = j < K ? *reinterpret_cast<const uint4*>(a.xb + j) : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  constexpr int NR = MODE == GV_SWIGLU ? 2 * R : R;
  const int nrg = (a.N + 4 * R - 1) / (4 * R);
  uint4 w[NR][CPL];
  int n0 = 0;
  bool ok[NR];
  auto issue = [&](int rg) {
    n0 = (rg * 4 + wave) * R;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int n = n0 + (r % R);
      ok[r] = n < a.N;
      const int wr = (MODE == GV_SWIGLU && r >= R) ? a.F + n : n;
      const bf16* rowp = a.W + (ok[r] ? (long)wr * a.ldw : 0);
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int ch = lane + 64 * c;
        w[r][c] = (ok[r] && ch < nch) ? ldnt16(rowp + 8 * ch) : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };
  const bool t0 = a.trace && blockIdx.x == 0 && threadIdx.x == 0;
  if (a.trace && threadIdx.x == 0) a.trace[128 + blockIdx.x] = (long long)wall_clock64();
  int rg = blockIdx.x;
  if (rg < nrg) issue(rg);
  if (t0) a.trace[32] = (long long)wall_clock64();
  if (a.st && a.st->done) return;
  if constexpr (MG) {  // flash-decoding merge in the log2 domain of the split kernel's scores
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i;
      float M = -INFINITY;
#pragma unroll
      for (int sp = 0; sp < kMergeMaxNs; ++sp) M = fmaxf(M, pm[i][sp]);
      float den = 0.f, num = 0.f;
#pragma unroll
      for (int sp = 0; sp < kMergeMaxNs; ++sp) {
        const float wgt = __builtin_amdgcn_exp2f(pm[i][sp] - M);
        den = __builtin_fmaf(wgt, pl[i][sp], den);
        num = __builtin_fmaf(wgt, po[i][sp], num);
      }
      if (e < K) {
        const bf16 x = (bf16)(num / den);
        xs[e] = x;
        if (a.pout && blockIdx.x == 0) a.pout[e] = x;
      }
    }
  } else if (a.X) {
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < kGemvXPer; ++i) ss += xv[i] * xv[i];
    const float rs = rsqrtf(block_sum(ss, red) / K + a.eps);
#pragma unroll
    for (int i = 0; i < kGemvXPer; ++i) {
      const int j = tid + 256 * i;
      if (j < K) xs[j] = (bf16)((float)(bf16)(xv[i] * rs) * gv[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < kGemvXPer / 2; ++i) {
      const int j = (tid + 256 * i) * 8;
      if (j < K) *reinterpret_cast<uint4*>(xs + j) = xq[i];
    }
  }
  __syncthreads();
  if (t0) a.trace[33] = (long long)wall_clock64();
  unsigned long long best = 0ull;  // ARGMAX: running best of this wave over its row groups
  for (; rg < nrg; rg += gridDim.x) {
    float acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int ch = lane + 64 * c;
      const bf16x8 x = ch < nch ? *reinterpret_cast<const bf16x8*>(xs + 8 * ch) : bf16x8{};
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[r] += dot8(w[r][c], x);
    }
    const int cur_n0 = n0;
    bool cur_ok[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) cur_ok[r] = ok[r];
    if (rg + (int)gridDim.x < nrg) issue(rg + gridDim.x);  // next row group's loads fly during the reduction
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = warp_sum(acc[r]);
    if (cur_n0 >= a.N) continue;
    if constexpr (MODE == GV_ARGMAX) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (cur_ok[r]) {
          const unsigned long long k = argmax_key(acc[r], (unsigned)(cur_n0 + r));
          best = k > best ? k : best;
        }
    } else {
      if (lane >= R) continue;
      float y = 0.f, u = 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (lane == r) { y = acc[r]; if (MODE == GV_SWIGLU) u = acc[R + r]; }
      const int n = cur_n0 + lane;
      if (n >= a.N) continue;
      if constexpr (MODE == GV_STORE_ROW) {
        if (a.bias) y += a.bias[n];
        const long row = a.st ? a.st->pos : 0;
        a.out[row * a.out_ld + n] = (bf16)y;
      } else if constexpr (MODE == GV_RESID) {
        a.resid[n] += y;
      } else {  // SwiGLU on the bf16-rounded gate/up projections (as swiglu_fwd_kernel does)
        const float g = (float)(bf16)y, uu = (float)(bf16)u;
        a.out[n] = (bf16)(silu(g) * uu);
      }
    }
  }
  if (t0) a.trace[34] = (long long)wall_clock64();
  if constexpr (MODE == GV_ARGMAX) {
    if (lane == 0 && best) atomicMax(a.keys + ((blockIdx.x * 4 + wave) & (kKeyShards - 1)), best);
  }
}

// ---- attention of the new token over the cache: split over keys, combined in the same launch -------
// cache row layout: [q (Hq*64) | k (Hkv*64) | v (Hkv*64)]; rows 0..pos-1 hold rotated k; row pos holds
// the fresh q/k/v of this token. Grid (Hkv, nsplit): workgroup (g, s) takes keys [s*c, (s+1)*c) of kv
// head g (c = ceil((pos+1)/nsplit) <= 128) for the G = Hq/Hkv query heads sharing it and publishes its
// partial softmax state (max, sum, unnormalised output) to a workspace; the workgroup whose arrival on
// kv head g's counter comes last merges the nsplit partials (flash-decoding) and resets the counter, so
// the split and the merge cost one launch. Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility,
// table row 1): partials stored and loaded with agent-scope (sc1) accesses, every storing wave waits
// vmcnt(0) before the workgroup barrier, one lane adds to the counter, the last adder's workgroup reads
// behind an LDS flag. The workgroup holding row pos rotates that k row and writes it back for the
// following steps; every workgroup rotates the q rows it needs itself.
constexpr int kAttnChunk = 128;
constexpr int kAttnCntStride = 32;  // one counter per kv head, 128 B apart, after the partials

struct DecAttnArgs {
  bf16* cache; long ld; int Hq, Hkv;
  const float* cos; const float* sin;  // [S_max, 32]
  float* ws;                           // [Hkv][nsplit][G * (2 + 64)] partials, then Hkv counters
  bf16* out;                           // [Hq*64]
  const slx_dec_state* st;
  float scale;
  long long* trace;  // tools only (slx_dec_attn_set_trace): phase timestamps of workgroup (0, 0) and the merger
};

__device__ __forceinline__ void tr(const DecAttnArgs& a, int slot) {
  if (a.trace && threadIdx.x == 0) a.trace[slot] = (long long)wall_clock64();
}

__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave-wide max / sum through DPP (within 16-lane rows) + readlane of the 4 row results (no LDS round trips)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <bool MAX>
__device__ __forceinline__ float wave_reduce(float x) {
  auto op = [](float u, float v) { return MAX ? fmaxf(u, v) : u + v; };
  x = op(x, dpp_f<0xB1>(x));   // quad_perm [1,0,3,2]
  x = op(x, dpp_f<0x4E>(x));   // quad_perm [2,3,0,1]
  x = op(x, dpp_f<0x141>(x));  // row_half_mirror
  x = op(x, dpp_f<0x140>(x));  // row_mirror
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 48));
  return op(op(r0, r1), op(r2, r3));
}

// Latency schedule (phase timestamps measured with tools/dec_attn_trace.py): one round trip for the cache rows
// (K and V of this split staged in LDS, q of the G heads rotated into LDS), scores spread over all 256 threads as
// (head, key) pairs, the partial softmax per head on one wave with DPP reductions, P.V with lane = output dim, the
// partial published with agent-scope stores, then one arrival; the last arriver loads every split's (m, l, o) for
// its lanes in one round trip and merges in registers.
__global__ __launch_bounds__(256) void dec_attn_kernel(DecAttnArgs a) {
  __shared__ __attribute__((aligned(16))) float ps[8][kAttnChunk];
  __shared__ __attribute__((aligned(16))) float qs[8 * 64];
  __shared__ float mh[8], lh[8];
  __shared__ __attribute__((aligned(16))) bf16 ksm[kAttnChunk * 64];  // this split's K rows (rotated)
  __shared__ __attribute__((aligned(16))) bf16 vs[kAttnChunk * 64];   // this split's V rows
  __shared__ int last_s;
  const bool t0 = a.trace && blockIdx.x == 0 && blockIdx.y == 0;
  if (a.trace && threadIdx.x == 0) a.trace[64 + blockIdx.y * gridDim.x + blockIdx.x] = (long long)wall_clock64();
  if (t0) tr(a, 0);
  if (a.st->done) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pos = a.st->pos, L = pos + 1;
  const int g = blockIdx.x, sp = blockIdx.y, ns = gridDim.y, G = a.Hq / a.Hkv;
  if (t0) tr(a, 1);
  const int c = (L + ns - 1) / ns;
  const int j0 = sp * c, j1 = min(L, j0 + c), n = max(0, j1 - j0);
  const int qn = a.Hq * 64, kn = a.Hkv * 64;
  float* part = a.ws + ((long)g * ns + sp) * (G * 66);
  int* cnt = reinterpret_cast<int*>(a.ws + (long)a.Hkv * ns * (G * 66)) + g * kAttnCntStride;
  if (n > 0) {
    bf16* row = a.cache + (long)pos * a.ld;
    const float* cs = a.cos + (long)pos * 32;
    const float* sn = a.sin + (long)pos * 32;
    // every global read is issued up front (one latency round trip): 16-B chunks of the K and V rows of the
    // split (key t = tid/8 + 32 i, chunk tid%8), the q rows and the RoPE row
    const int d8 = lane & 7, jj = tid >> 3;
    const bf16* kb = a.cache + qn + g * 64 + 8 * d8;
    const bf16* vb = a.cache + qn + kn + g * 64 + 8 * d8;
    bf16x8 kt[kAttnChunk / 32], vt[kAttnChunk / 32];
#pragma unroll
    for (int i = 0; i < kAttnChunk / 32; ++i) {
      const int t = jj + 32 * i;
      if (t < n) {
        kt[i] = *reinterpret_cast<const bf16x8*>(kb + (long)(j0 + t) * a.ld);
        vt[i] = *reinterpret_cast<const bf16x8*>(vb + (long)(j0 + t) * a.ld);
      }
    }
    if (tid < 32 * G) {  // rotate_half RoPE of the G query heads (bf16-rounded like the stored rows)
      const int h = tid >> 5, j = tid & 31;
      const bf16* q = row + (g * G + h) * 64;
      const float q0 = (float)q[j], q1 = (float)q[j + 32];
      qs[h * 64 + j] = (float)(bf16)(q0 * cs[j] - q1 * sn[j]);
      qs[h * 64 + j + 32] = (float)(bf16)(q1 * cs[j] + q0 * sn[j]);
    }
    if (tid < 32 && j1 == L) {  // k of this token: rotated, written back once (and into this split's K tile)
      const int j = tid;
      bf16* k = row + qn + g * 64;
      const float k0 = (float)k[j], k1 = (float)k[j + 32];
      const bf16 r0 = (bf16)(k0 * cs[j] - k1 * sn[j]), r1 = (bf16)(k1 * cs[j] + k0 * sn[j]);
      k[j] = r0;
      k[j + 32] = r1;
      const int tp = pos - j0, sw = tp & 7;  // K tile chunks XOR-swizzled by row (conflict-free score reads)
      ksm[tp * 64 + 8 * ((j >> 3) ^ sw) + (j & 7)] = r0;
      ksm[tp * 64 + 8 * (((j + 32) >> 3) ^ sw) + (j & 7)] = r1;
    }
#pragma unroll
    for (int i = 0; i < kAttnChunk / 32; ++i) {
      const int t = jj + 32 * i;
      if (t < n) {
        if (j0 + t != pos) *reinterpret_cast<bf16x8*>(ksm + t * 64 + 8 * (d8 ^ (t & 7))) = kt[i];
        *reinterpret_cast<bf16x8*>(vs + t * 64 + 8 * d8) = vt[i];
      }
    }
    __syncthreads();
    if (t0) tr(a, 2);
    // scores: (head, key) pairs over all threads
    for (int i = tid; i < G * n; i += 256) {
      const int h = i / n, t = i - h * n;
      const float4* q4 = reinterpret_cast<const float4*>(qs + h * 64);
      const bf16x8* k8 = reinterpret_cast<const bf16x8*>(ksm + t * 64);
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c8 = 0; c8 < 8; ++c8) {
        const bf16x8 kv = k8[c8 ^ (t & 7)];
        const float4 qa = q4[2 * c8], qb = q4[2 * c8 + 1];
        acc[0] = __builtin_fmaf(qa.x, (float)kv[0], acc[0]);
        acc[1] = __builtin_fmaf(qa.y, (float)kv[1], acc[1]);
        acc[2] = __builtin_fmaf(qa.z, (float)kv[2], acc[2]);
        acc[3] = __builtin_fmaf(qa.w, (float)kv[3], acc[3]);
        acc[0] = __builtin_fmaf(qb.x, (float)kv[4], acc[0]);
        acc[1] = __builtin_fmaf(qb.y, (float)kv[5], acc[1]);
        acc[2] = __builtin_fmaf(qb.z, (float)kv[6], acc[2]);
        acc[3] = __builtin_fmaf(qb.w, (float)kv[7], acc[3]);
      }
      ps[h][t] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) * a.scale;
    }
    __syncthreads();
    if (t0) tr(a, 3);
    // partial softmax: wave w takes heads w and w + 4 (n <= 128: two keys per lane)
    for (int h = wave; h < G; h += 4) {
      const float x0 = lane < n ? ps[h][lane] : -INFINITY;
      const float x1 = lane + 64 < n ? ps[h][lane + 64] : -INFINITY;
      const float m = wave_reduce<true>(fmaxf(x0, x1));
      const float e0 = lane < n ? __expf(x0 - m) : 0.f;
      const float e1 = lane + 64 < n ? __expf(x1 - m) : 0.f;
      if (lane < n) ps[h][lane] = e0;
      if (lane + 64 < n) ps[h][lane + 64] = e1;
      const float l = wave_reduce<false>(e0 + e1);
      if (lane == 0) { mh[h] = m; lh[h] = l; }
    }
    __syncthreads();
    if (t0) tr(a, 4);
    // unnormalised P V: lanes 0-31 of wave w take head w, lanes 32-63 head w + 4, two output dims per lane
    // (8 keys per step, LDS reads of a step issued together)
    {
      const int h = wave + 4 * (lane >> 5), dd = 2 * (lane & 31);
      if (h < G) {
        float ax[2] = {0.f, 0.f}, ay[2] = {0.f, 0.f};
        int t = 0;
        for (; t + 8 <= n; t += 8) {
          const float4 p0 = *reinterpret_cast<const float4*>(&ps[h][t]);
          const float4 p1 = *reinterpret_cast<const float4*>(&ps[h][t + 4]);
          const float pp[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
          uint32_t v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const uint32_t*>(vs + (t + u) * 64 + dd);
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            ax[u & 1] = __builtin_fmaf(pp[u], __uint_as_float(v[u] << 16), ax[u & 1]);
            ay[u & 1] = __builtin_fmaf(pp[u], __uint_as_float(v[u] & 0xFFFF0000u), ay[u & 1]);
          }
        }
        for (; t < n; ++t) {
          const uint32_t v = *reinterpret_cast<const uint32_t*>(vs + t * 64 + dd);
          ax[0] = __builtin_fmaf(ps[h][t], __uint_as_float(v << 16), ax[0]);
          ay[0] = __builtin_fmaf(ps[h][t], __uint_as_float(v & 0xFFFF0000u), ay[0]);
        }
        st_agent(part + 2 * G + h * 64 + dd, ax[0] + ax[1]);
        st_agent(part + 2 * G + h * 64 + dd + 1, ay[0] + ay[1]);
      }
    }
  } else {  // empty split: neutral partial
    for (int i = tid; i < G * 64; i += 256) st_agent(part + 2 * G + i, 0.f);
    if (tid < G) { mh[tid] = -INFINITY; lh[tid] = 0.f; }
    __syncthreads();
  }
  if (tid < G) { st_agent(part + tid, mh[tid]); st_agent(part + G + tid, lh[tid]); }
  // publish, then arrive (one lane, after every storing wave's vmcnt(0) and a workgroup barrier)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t0) tr(a, 5);
  if (tid == 0) {  // release (cumulative over the barrier) this split's partials, then arrive
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    last_s = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ns - 1;
  }
  __syncthreads();
  if (t0) tr(a, 6);
  if (!last_s) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (a.trace) tr(a, 8);
  // the last arriver merges the ns partials of kv head g: lane = dim of heads wave, wave + 4; every (m, l, o)
  // of its splits is loaded at once (kMergeBatch splits per round trip), the weights computed per lane
  float* base = a.ws + (long)g * ns * (G * 66);
  constexpr int kMergeBatch = 16;
  for (int h = wave; h < G; h += 4) {
    float M = -INFINITY, den = 0.f, num = 0.f;
    for (int s0 = 0; s0 < ns; s0 += kMergeBatch) {
      float m[kMergeBatch], l[kMergeBatch], o[kMergeBatch];
#pragma unroll
      for (int u = 0; u < kMergeBatch; ++u) {
        float* p = base + (s0 + u) * (G * 66);
        const bool ok = s0 + u < ns;
        m[u] = ok ? ld_agent(p + h) : -INFINITY;
        l[u] = ok ? ld_agent(p + G + h) : 0.f;
        o[u] = ok ? ld_agent(p + 2 * G + h * 64 + lane) : 0.f;
      }
      float Mb = M;
#pragma unroll
      for (int u = 0; u < kMergeBatch; ++u) Mb = fmaxf(Mb, m[u]);
      const float r = M == -INFINITY ? 0.f : __expf(M - Mb);  // rescale the running sums to the new max
      den *= r;
      num *= r;
#pragma unroll
      for (int u = 0; u < kMergeBatch; ++u) {
        const float w = m[u] == -INFINITY ? 0.f : __expf(m[u] - Mb);
        den = __builtin_fmaf(w, l[u], den);
        num = __builtin_fmaf(w, o[u], num);
      }
      M = Mb;
    }
    a.out[(g * G + h) * 64 + lane] = (bf16)(num / den);
  }
  if (a.trace) tr(a, 9);
  if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.trace) { __syncthreads(); tr(a, 10); }
}

template <int MODE, int R>
static void gemv_cpl(GemvArgs& a, dim3 grid, size_t lds, hipStream_t st) {
  const int cpl = (a.K / 8 + 63) / 64;
  if (cpl <= 1) hipLaunchKernelGGL((dec_gemv_kernel<MODE, R, 1>), grid, dim3(256), lds, st, a);
  else if (cpl <= 2) hipLaunchKernelGGL((dec_gemv_kernel<MODE, R, 2>), grid, dim3(256), lds, st, a);
  else if (cpl <= 4) hipLaunchKernelGGL((dec_gemv_kernel<MODE, R, 4>), grid, dim3(256), lds, st, a);
  else if (cpl <= 10) hipLaunchKernelGGL((dec_gemv_kernel<MODE, R, 10>), grid, dim3(256), lds, st, a);
  else hipLaunchKernelGGL((dec_gemv_kernel<MODE, R, 16>), grid, dim3(256), lds, st, a);
}

static int gemv_launch(int mode, GemvArgs& a, hipStream_t st) {
  // rows per wave: 4 for the LM head (argmax) and the q|k|v row GEMV (0.5 us faster than 1: a quarter of the
  // workgroups to dispatch, tools/gemv_ab.sh), else 1: the 896-row residual GEMVs and gate|up (1 gate + 1 up row per
  // wave: 0.795 vs 0.805 ms/token with 2, profiles/round2_s3_tail_swiglu_ab.txt) measured fastest with more
  // workgroups in flight
  static const int r_env = [] { const char* e = getenv("SLX_DEC_GEMV_R"); return e ? atoi(e) : 0; }();  // tools: A/B
  int R = mode == GV_ARGMAX || mode == GV_STORE_ROW ? 4 : (mode != GV_SWIGLU && a.N >= 4096) ? 2 : 1;
  if (r_env == 1 || r_env == 2 || r_env == 4) R = mode == GV_ARGMAX ? 4 : (mode == GV_SWIGLU ? 2 : r_env);
  static const int rsw_env = [] { const char* e = getenv("SLX_DEC_GEMV_RSW"); return e ? atoi(e) : 0; }();  // A/B
  if (mode == GV_SWIGLU && (rsw_env == 1 || rsw_env == 2 || rsw_env == 4)) R = rsw_env;
  const int rows_per_block = 4 * R;
  const int groups = (a.N + rows_per_block - 1) / rows_per_block;
  const dim3 grid(groups < 2048 ? groups : 2048);  // grid-stride over row groups: the norm prologue amortised
  const size_t lds = (size_t)a.K * 2;
  switch (mode) {
    case GV_STORE_ROW:
      if (R == 4) gemv_cpl<GV_STORE_ROW, 4>(a, grid, lds, st);
      else if (R == 2) gemv_cpl<GV_STORE_ROW, 2>(a, grid, lds, st);
      else gemv_cpl<GV_STORE_ROW, 1>(a, grid, lds, st);
      break;
    case GV_RESID:
      if (R == 4) gemv_cpl<GV_RESID, 4>(a, grid, lds, st);
      else if (R == 2) gemv_cpl<GV_RESID, 2>(a, grid, lds, st);
      else gemv_cpl<GV_RESID, 1>(a, grid, lds, st);
      break;
    case GV_SWIGLU:
      if (R == 4) gemv_cpl<GV_SWIGLU, 4>(a, grid, lds, st);
      else if (R == 1) gemv_cpl<GV_SWIGLU, 1>(a, grid, lds, st);
      else gemv_cpl<GV_SWIGLU, 2>(a, grid, lds, st);
      break;
    case GV_ARGMAX: gemv_cpl<GV_ARGMAX, 4>(a, grid, lds, st); break;
  }
  SLX_LAUNCH_CHECK("slx_dec_gemv");
  return 0;
}

}  // namespace slx

using namespace slx;

extern "C" {

int slx_dec_key_shards(void) { return kKeyShards; }

int slx_dec_begin(slx_dec_state* st, unsigned long long* keys, const void* embed, int D, float* X, int* tokens,
                  slx_stream_t s) {
  SLX_CHECK_ARG(st && keys && embed && X && tokens && D > 0, "slx_dec_begin: null argument");
  hipLaunchKernelGGL(dec_begin_kernel, dim3(1), dim3(256), 0, (hipStream_t)s, st, keys, (const bf16*)embed, D, X, tokens);
  SLX_LAUNCH_CHECK("slx_dec_begin");
  return 0;
}

int slx_dec_gemv(const slx_dec_gemv_desc* d, slx_stream_t s) {
  SLX_CHECK_ARG(d && d->W, "slx_dec_gemv: null desc/W");
  SLX_CHECK_ARG(d->K % 8 == 0 && d->ldw % 8 == 0 && ((uintptr_t)d->W & 15) == 0, "slx_dec_gemv: K, ldw %% 8, W 16-B aligned");
  SLX_CHECK_ARG(d->K <= 8192, "slx_dec_gemv: K <= 8192 (16 chunks of 16 B per lane)");
  SLX_CHECK_ARG(!d->X || d->K <= 256 * kGemvXPer, "slx_dec_gemv: K <= %d with the fused RMSNorm", 256 * kGemvXPer);
  SLX_CHECK_ARG((d->X && d->gamma) || (d->xb && ((uintptr_t)d->xb & 15) == 0), "slx_dec_gemv: need X+gamma or 16-B aligned xb");
  GemvArgs a;
  a.W = (const bf16*)d->W; a.ldw = d->ldw; a.N = d->N; a.K = d->K;
  a.X = d->X; a.gamma = d->gamma; a.eps = d->eps; a.xb = (const bf16*)d->xb; a.bias = d->bias;
  a.out = (bf16*)d->out; a.out_ld = d->out_ld; a.resid = d->resid; a.keys = d->keys; a.F = d->N;
  a.st = d->state;
  a.trace = g_dec_trace;
  switch (d->mode) {
    case SLX_DEC_STORE_ROW: SLX_CHECK_ARG(d->out != nullptr, "slx_dec_gemv: out"); return gemv_launch(GV_STORE_ROW, a, (hipStream_t)s);
    case SLX_DEC_RESID: SLX_CHECK_ARG(d->resid != nullptr, "slx_dec_gemv: resid"); return gemv_launch(GV_RESID, a, (hipStream_t)s);
    case SLX_DEC_SWIGLU: SLX_CHECK_ARG(d->out != nullptr, "slx_dec_gemv: out"); return gemv_launch(GV_SWIGLU, a, (hipStream_t)s);
    case SLX_DEC_ARGMAX: SLX_CHECK_ARG(d->keys != nullptr, "slx_dec_gemv: keys"); return gemv_launch(GV_ARGMAX, a, (hipStream_t)s);
  }
  set_error("slx_dec_gemv: bad mode %d", d->mode);
  return -22;
}

// tools only: phase timestamps (wall_clock64 ticks) of the next slx_dec_attn / slx_dec_gemv launches; NULL = off
void slx_dec_attn_set_trace(long long* buf) { g_dec_trace = buf; }
// tests / tools only: 1 = always use the split-K form (the path for caches of more than 1024 rows)
void slx_dec_attn_force_split(int on) { g_dec_force_split = on; }

int slx_dec_attn_nsplit(int lmax) { return (lmax + kAttnChunk - 1) / kAttnChunk > 8 ? (lmax + kAttnChunk - 1) / kAttnChunk : 8; }

int slx_dec_attn_ws_floats(int Hq, int Hkv, int lmax) {
  return Hkv > 0 ? Hkv * slx_dec_attn_nsplit(lmax) * (Hq / Hkv) * 66 + Hkv * kAttnCntStride : 0;
}

int slx_dec_attn(void* cache, int64_t ld, int Hq, int Hkv, const float* cos_tab, const float* sin_tab, int lmax,
                 float* ws, void* out, const slx_dec_state* st, slx_stream_t s) {
  SLX_CHECK_ARG(cache && cos_tab && sin_tab && ws && out && st, "slx_dec_attn: null argument");
  SLX_CHECK_ARG(Hkv > 0 && Hq % Hkv == 0 && Hq / Hkv <= 8, "slx_dec_attn: Hq/Hkv must be an integer <= 8");
  SLX_CHECK_ARG(ld % 8 == 0 && ((uintptr_t)cache & 15) == 0, "slx_dec_attn: cache rows must be 16-B aligned");
  SLX_CHECK_ARG(lmax > 0 && lmax <= 64 * kAttnChunk, "slx_dec_attn: lmax <= 8192");  // ns <= 64: ns * G <= 512
  if (lmax <= 1024 && !g_dec_trace && !g_dec_force_split)  // one workgroup per kv head: no split partials, no merge
    return dec_attn_mfma_launch(cache, ld, Hq, Hkv, cos_tab, sin_tab, out, st, (hipStream_t)s);
  const int ns = slx_dec_attn_nsplit(lmax);
  DecAttnArgs a{(bf16*)cache, ld, Hq, Hkv, cos_tab, sin_tab, ws, (bf16*)out, st, 0.125f, g_dec_trace};
  SLX_CHECK_ARG(((uintptr_t)ws & 3) == 0, "slx_dec_attn: ws must be 4-B aligned (and zeroed once: it holds the counters)");
  hipLaunchKernelGGL(dec_attn_kernel, dim3(Hkv, ns), dim3(256), 0, (hipStream_t)s, a);
  SLX_LAUNCH_CHECK("slx_dec_attn");
  return 0;
}

// split attention + O projection: dec_attn_mfma_split_kernel (Hkv x ns workgroups, partials in ws), then the O GEMV
// (+ residual) merging the partials in its prologue (dec_gemv_kernel MG); ns = SLX_DEC_SPLIT_NS (default 8)
static int dec_split_ns() {
  static const int ns_env = [] { const char* e = getenv("SLX_DEC_SPLIT_NS"); return e ? atoi(e) : 8; }();
  return ns_env;
}

int slx_dec_attn_o_split_ok(int lmax) {
  const int ns = dec_split_ns();
  return ns >= 1 && ns <= kMergeMaxNs && lmax > 0 && lmax <= 256 * ns && ns <= slx_dec_attn_nsplit(lmax);
}

int slx_dec_attn_o_split(void* cache, int64_t ld, int Hq, int Hkv, const float* cos_tab, const float* sin_tab,
                         int lmax, float* ws, void* out, const slx_dec_state* st, const void* Wo, int64_t ldwo, int N,
                         int K, float* X, slx_stream_t s) {
  const int ns = dec_split_ns();
  SLX_CHECK_ARG(cache && cos_tab && sin_tab && ws && st && Wo && X, "slx_dec_attn_o_split: null argument");
  SLX_CHECK_ARG(slx_dec_attn_o_split_ok(lmax),
                "slx_dec_attn_o_split: 1 <= ns <= %d splits of at most 8 key blocks (lmax %d, ns %d)", kMergeMaxNs,
                lmax, ns);
  SLX_CHECK_ARG(Hkv > 0 && Hq % Hkv == 0 && Hq / Hkv <= 32 && K == Hq * 64 && K <= 1024 && K % 8 == 0,
                "slx_dec_attn_o_split: K == Hq * 64 <= 1024, Hq/Hkv <= 32");
  SLX_CHECK_ARG(ld % 8 == 0 && ((uintptr_t)cache & 15) == 0 && ldwo % 8 == 0 && ((uintptr_t)Wo & 15) == 0 &&
                ((uintptr_t)ws & 3) == 0, "slx_dec_attn_o_split: 16-B aligned cache and W_o rows");
  int rc = dec_attn_split_launch(cache, ld, Hq, Hkv, cos_tab, sin_tab, ws, ns, st, (hipStream_t)s);
  if (rc) return rc;
  GemvArgs a;
  memset(&a, 0, sizeof(a));
  a.W = (const bf16*)Wo; a.ldw = ldwo; a.N = N; a.K = K; a.resid = X; a.st = st; a.F = N;
  a.part = ws; a.pns = ns; a.pG = Hq / Hkv; a.pout = (bf16*)out;
  const int groups = (N + 3) / 4;
  hipLaunchKernelGGL((dec_gemv_kernel<GV_RESID, 1, 2, true>), dim3(groups < 2048 ? groups : 2048), dim3(256),
                     (size_t)K * 2, (hipStream_t)s, a);
  SLX_LAUNCH_CHECK("slx_dec_attn_o_split(O GEMV)");
  return 0;
}

}  // extern "C"
