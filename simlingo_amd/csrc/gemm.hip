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
#include "common.h"
#include "../../include/slx.h"

namespace slx {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;

enum { EPI_STORE = 0, EPI_GELU = 1, EPI_RESID_LS = 2, EPI_GELU_BWD = 3, EPI_SWIGLU_BWD = 4, EPI_DROPMASK = 5 };

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
  int accumulate;
  unsigned long long seed;
  float drop_p;
  long ldmask;
  int tilesM, tilesN;
  int ksplit;        // > 1: split-K, f32 atomic accumulation into a pre-zeroed / accumulating C
  int kchunk;        // K range per split (multiple of BK)
};

template <bool KC>
__device__ __forceinline__ void load_tile(const bf16* __restrict__ X, long ld, int row0, int rows_total, int k0,
                                          int K, uint4 (&r)[4]) {
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
__device__ __forceinline__ void epilogue_elem(const GemmArgs& p, OutT* __restrict__ C, int m, int n, float acc) {
  float v = acc * p.alpha;
  const long ci = (long)m * p.ldc + n;
  if constexpr (EPI == EPI_STORE) {
    if (p.ksplit > 1) {  // split-K: every split adds its partial; split 0 adds the bias
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
    p.aux_out[(long)m * p.ldaux_out + n] = hb;
    C[ci] = (OutT)gelu_erf((float)hb);
  } else if constexpr (EPI == EPI_RESID_LS) {
    if (p.bias) v += p.bias[n];
    const bf16 yb = (bf16)v;
    if (p.aux_out) p.aux_out[(long)m * p.ldaux_out + n] = yb;
    C[ci] = (OutT)(p.resid[(long)m * p.ldr + n] + p.ls[n] * v);
  } else if constexpr (EPI == EPI_GELU_BWD) {
    const float h = (float)p.aux[(long)m * p.ldaux + n];
    C[ci] = (OutT)(v * gelu_erf_grad(h));
  } else if constexpr (EPI == EPI_SWIGLU_BWD) {
    const long ai = (long)m * p.ldaux + n;
    const float g = (float)p.aux[ai], u = (float)p.aux[ai + p.N];
    C[ci] = (OutT)(v * u * silu_grad(g));
    C[ci + p.N] = (OutT)(v * silu(g));
  } else if constexpr (EPI == EPI_DROPMASK) {
    const float keep = uniform01(p.seed, (unsigned long long)m * p.ldmask + n) >= p.drop_p ? 1.0f / (1.0f - p.drop_p) : 0.0f;
    v *= keep;
    if (p.accumulate) v += (float)C[ci];
    C[ci] = (OutT)v;
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
  load_tile<AK>(A, p.lda, m0, p.M, kbeg, kend, ra);
  load_tile<BKc>(B, p.ldb, n0, p.N, kbeg, kend, rb);
  store_tile<AK>(As0, ra);
  store_tile<BKc>(Bs0, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const char* As = As0 + cur * STAGE;
    const char* Bs = Bs0 + cur * STAGE;
    if (kt + 1 < nk) {
      load_tile<AK>(A, p.lda, m0, p.M, kbeg + (kt + 1) * BK, kend, ra);
      load_tile<BKc>(B, p.ldb, n0, p.N, kbeg + (kt + 1) * BK, kend, rb);
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

template <bool AK, bool BKc, int EPI, typename OutT>
static int launch(GemmArgs& a, int batch, hipStream_t st) {
  dim3 grid(a.tilesM * a.tilesN, a.ksplit > 1 ? a.ksplit : 1, batch);
  hipLaunchKernelGGL((gemm_bf16_kernel<AK, BKc, EPI, OutT>), grid, dim3(NT), 0, st, a);
  SLX_LAUNCH_CHECK("slx_gemm_bf16");
  return 0;
}

template <int EPI, typename OutT>
static int dispatch_layout(int layout, GemmArgs& a, int batch, hipStream_t st) {
  switch (layout) {
    case SLX_GEMM_NT: return launch<true, true, EPI, OutT>(a, batch, st);
    case SLX_GEMM_NN: return launch<true, false, EPI, OutT>(a, batch, st);
    case SLX_GEMM_TN: return launch<false, false, EPI, OutT>(a, batch, st);
    case SLX_GEMM_TT: return launch<false, true, EPI, OutT>(a, batch, st);
  }
  set_error("slx_gemm_bf16: bad layout %d", layout);
  return -22;
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
  GemmArgs a;
  a.A = (const bf16*)d->A; a.B = (const bf16*)d->B; a.C = d->C;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.sA = d->sA; a.sB = d->sB; a.sC = d->sC;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.alpha = d->alpha;
  a.bias = d->bias; a.ls = d->ls;
  a.aux = (const bf16*)d->aux; a.ldaux = d->ldaux;
  a.aux_out = (bf16*)d->aux_out; a.ldaux_out = d->ldaux_out;
  a.resid = d->resid; a.ldr = d->ldr;
  a.accumulate = d->accumulate;
  a.seed = d->seed; a.drop_p = d->drop_p; a.ldmask = d->ldmask;
  a.tilesM = (d->M + BM - 1) / BM;
  a.tilesN = (d->N + BN - 1) / BN;
  const int batch = d->batch < 1 ? 1 : d->batch;
  hipStream_t st = (hipStream_t)stream;
  a.ksplit = 1;
  a.kchunk = d->K;
  {  // split-K for under-filled grids (weight gradients of skinny / LoRA GEMMs): >= 4 K-steps per split
    const int tiles = a.tilesM * a.tilesN * batch;
    const int ksteps = (d->K + BK - 1) / BK;
    if (d->epilogue == SLX_EPI_STORE && d->out_f32 && tiles < 256 && ksteps >= 8) {
      int want = (512 + tiles - 1) / tiles;
      int maxs = ksteps / 4;
      int sp = want < maxs ? want : maxs;
      if (d->ksplit_max > 0 && sp > d->ksplit_max) sp = d->ksplit_max;
      if (d->ksplit_max < 0) sp = 1;
      if (sp > 1) {
        const int per = ((ksteps + sp - 1) / sp) * BK;
        sp = (d->K + per - 1) / per;
        a.ksplit = sp;
        a.kchunk = per;
        if (!d->accumulate) {
          hipError_t e = hipMemset2DAsync(d->C, d->ldc * sizeof(float), 0, (size_t)d->N * sizeof(float), d->M, st);
          if (e != hipSuccess) { set_error("slx_gemm_bf16: memset2D failed: %s", hipGetErrorString(e)); return -1000 - (int)e; }
        }
        SLX_CHECK_ARG(batch == 1, "slx_gemm_bf16: split-K with batch > 1 unsupported");
      }
    }
  }
  switch (d->epilogue) {
    case SLX_EPI_STORE:
      return d->out_f32 ? dispatch_layout<EPI_STORE, float>(d->layout, a, batch, st)
                        : dispatch_layout<EPI_STORE, bf16>(d->layout, a, batch, st);
    case SLX_EPI_GELU:
      SLX_CHECK_ARG(!d->out_f32 && d->layout == SLX_GEMM_NT && d->aux_out, "slx_gemm_bf16: GELU needs NT, bf16 out, aux_out");
      return launch<true, true, EPI_GELU, bf16>(a, batch, st);
    case SLX_EPI_RESID_LS:
      SLX_CHECK_ARG(d->out_f32 && d->layout == SLX_GEMM_NT && d->resid && d->ls, "slx_gemm_bf16: RESID_LS needs NT, f32 out, resid, ls");
      return launch<true, true, EPI_RESID_LS, float>(a, batch, st);
    case SLX_EPI_GELU_BWD:
      SLX_CHECK_ARG(!d->out_f32 && d->layout == SLX_GEMM_NN && d->aux, "slx_gemm_bf16: GELU_BWD needs NN, bf16 out, aux");
      return launch<true, false, EPI_GELU_BWD, bf16>(a, batch, st);
    case SLX_EPI_SWIGLU_BWD:
      SLX_CHECK_ARG(!d->out_f32 && d->layout == SLX_GEMM_NN && d->aux, "slx_gemm_bf16: SWIGLU_BWD needs NN, bf16 out, aux");
      return launch<true, false, EPI_SWIGLU_BWD, bf16>(a, batch, st);
    case SLX_EPI_DROPMASK:
      SLX_CHECK_ARG(d->out_f32 && d->layout == SLX_GEMM_NN, "slx_gemm_bf16: DROPMASK needs NN, f32 out");
      return launch<true, false, EPI_DROPMASK, float>(a, batch, st);
  }
  set_error("slx_gemm_bf16: bad epilogue %d", d->epilogue);
  return -22;
}
