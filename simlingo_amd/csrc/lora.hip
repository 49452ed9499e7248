// LoRA with dropout for the Qwen2 hot path (peft LoraLayer with lora_dropout, llm.py:106-119):
//   forward   t_s  = drop_s(x) . A_s^T                          (slx_lora_down, one launch per group of sites sharing x)
//   backward  dA_s += dT_s^T . drop_s(x)                         (slx_lora_bwd, one launch per group)
//             dx   += sum_s drop_s'(dT_s . A_s)                  (same launch; f32 in place, or bf16 out)
// where drop_s(x) = x * keep_s / (1 - p), keep_s a counter-hash mask (common.h drop_keep). The forward evaluates the
// hash once per element and stores the keep bits ([M][Kin/32] uint32 per site); the backward and the GEMM DROPMASK
// epilogues read the bits instead of re-hashing (the hash, ~20 VALU ops per element and site, bounded the old
// backward kernels). t is written as bf16 into the extra columns of the activation buffer that the fused [W | s*B]
// GEMM reads (engine.py); dT comes as f32 from the extra columns of the fused dgrad GEMM's output.
#include "common.h"
#include "../../include/slx.h"

namespace slx {

__device__ __forceinline__ f32x16 mfma32x32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

struct LoraDownArgs {
  const bf16* x; long ldx;
  int M, Kin, nsites;
  const bf16* A[4];
  const uint32_t* bits[4];  // keep bits per site (p > 0)
  long ldbits;
  bf16* t; long ldt;
  float p;
  uint32_t thr;
  long ldmask;
  uint32_t s1[4];  // gen: drop_seed_mix(seed) per site
  int gen;         // generate the keep bits (and write them to bits[s]) instead of reading them
};

// keep word of 32 consecutive mask indices i0 .. i0 + 31 (i0 even): bit c = drop_keep(s1, i0 + c, thr), 16 pair hashes
__device__ __forceinline__ uint32_t keep_word(uint32_t s1, unsigned long long i0, uint32_t thr) {
  uint32_t wd = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) wd |= drop_keep8(s1, i0 + 8 * q, thr) << (8 * q);
  return wd;
}

// Block = 32 rows x every site, 8 waves; wave w takes the step pairs (64 k = one 128-B line per row) w, w+8, ...
// Per pair: x [32 x 64] is read with coalesced 16-B loads (8 rows x 128 B per instruction), scaled to
// bf16(x / (1-p)) once and staged in a wave-private LDS tile (16-B chunks XOR-swizzled by row & 7: conflict-free
// writes and fragment reads); each site then ANDs its keep bits into the fragments (2 ops per element) and runs
// v_mfma_f32_32x32x16_bf16 against the packed A fragments. The next pair's global loads are issued before the
// current pair's MFMAs. The 8 waves' [32 x 32] partials are summed through per-wave LDS slices.
template <int NS>
struct DownRegs {  // one pair's x pieces and keep words (double-buffered across pairs)
  uint4 x[4];
  uint32_t kw[NS][2];
};

template <int NS>
__global__ __launch_bounds__(512) void lora_down_kernel(LoraDownArgs a) {
  __shared__ __attribute__((aligned(16))) char xs[8][32 * 128];
  __shared__ float red[8][32][33];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, r = lane & 31;
  const int m0 = blockIdx.x * 32;
  const bool drop = a.p > 0.f;
  const float sc = drop ? 1.0f / (1.0f - a.p) : 1.0f;
  const int nk = a.Kin / 32, npair = (nk + 1) / 2;
  const int srow = lane >> 3, sch = lane & 7;  // staging: row 8i + srow, 16-B chunk sch of the pair
  char* xw = xs[w];
  f32x16 acc[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[s][i] = 0.f;
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
  bf16x8 av[NS][2][2];  // A fragments of the current pair; site s is reloaded for the next pair after its MFMAs

  auto load_x = [&](int pi, DownRegs<NS>& R) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gm = m0 + 8 * i + srow, k = 64 * pi + 8 * sch;
      R.x[i] = (gm < a.M && k < a.Kin) ? *reinterpret_cast<const uint4*>(a.x + (long)gm * a.ldx + k)
                                       : make_uint4(0u, 0u, 0u, 0u);
    }
    const int gm = m0 + r;
    if (drop && a.gen) {  // keep words generated here: lane half h hashes word 2 pi + h of its row, the halves swap
      const int st = 2 * pi + h;
      const bool ok = st < nk && gm < a.M;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const uint32_t wd = ok ? keep_word(a.s1[s], (unsigned long long)gm * a.ldmask + 32 * st, a.thr) : 0u;
        if (ok) const_cast<uint32_t*>(a.bits[s])[(long)gm * a.ldbits + st] = wd;  // for the backward's consumers
        const auto sw = __builtin_amdgcn_permlane32_swap(wd, wd, false, false);
        const uint32_t other = sw[0] ^ sw[1] ^ wd;  // one of the pair is the lane's own word
        R.kw[s][0] = h ? other : wd;
        R.kw[s][1] = h ? wd : other;
      }
      return;
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const int st = 2 * pi + ss;
#pragma unroll
      for (int s = 0; s < NS; ++s)
        R.kw[s][ss] = (drop && st < nk && gm < a.M) ? a.bits[s][(long)gm * a.ldbits + st] : 0u;
    }
  };
  auto load_a = [&](int pi, int s) {
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const int st = 2 * pi + ss;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
        av[s][ss][hh] = st < nk ? *reinterpret_cast<const bf16x8*>(a.A[s] + ((long)(2 * st + hh) * 64 + lane) * 8) : z;
    }
  };
  auto process = [&](const DownRegs<NS>& R, int next) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint4 v = R.x[i];
      if (drop) {  // bf16(x * sc), the rounding of peft's dropout output
        uint32_t* u = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const float lo = __uint_as_float(u[d] << 16) * sc, hi = __uint_as_float(u[d] & 0xFFFF0000u) * sc;
          bf16x2 o;
          o[0] = (bf16)lo;
          o[1] = (bf16)hi;
          u[d] = __builtin_bit_cast(uint32_t, o);
        }
      }
      const int row = 8 * i + srow;
      *reinterpret_cast<uint4*>(xw + row * 128 + ((sch ^ (row & 7)) << 4)) = v;
    }
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private tile written (LDS is in order per wave)
    bf16x8 xf[2][2];
#pragma unroll
    for (int ss = 0; ss < 2; ++ss)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
        xf[ss][hh] = *reinterpret_cast<const bf16x8*>(xw + r * 128 + (((4 * ss + 2 * hh + h) ^ (r & 7)) << 4));
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // fragments read before the next pair overwrites the tile
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          bf16x8 xm = xf[ss][hh];
          if (drop) {
            const uint32_t b = R.kw[s][ss] >> (16 * hh + 8 * h);
            uint32_t* u = reinterpret_cast<uint32_t*>(&xm);
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              const uint32_t lo = (uint32_t)__builtin_amdgcn_sbfe((int)b, 2 * d, 1);
              const uint32_t hi = (uint32_t)__builtin_amdgcn_sbfe((int)b, 2 * d + 1, 1);
              u[d] &= (lo & 0xFFFFu) | (hi & 0xFFFF0000u);
            }
          }
          acc[s] = mfma32x32(xm, av[s][ss][hh], acc[s]);
        }
      if (next >= 0) load_a(next, s);
    }
  };

  DownRegs<NS> R0, R1;
  if (w < npair) {
    load_x(w, R0);
#pragma unroll
    for (int s = 0; s < NS; ++s) load_a(w, s);
  }
  for (int pi = w; pi < npair; pi += 16) {
    const bool more = pi + 8 < npair;
    if (more) load_x(pi + 8, R1);
    process(R0, more ? pi + 8 : -1);
    if (!more) break;
    const bool more2 = pi + 16 < npair;
    if (more2) load_x(pi + 16, R0);
    process(R1, more2 ? pi + 16 : -1);
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
#pragma unroll
    for (int i = 0; i < 16; ++i) red[w][8 * (i >> 2) + 4 * h + (i & 3)][r] = acc[s][i];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o = threadIdx.x + 512 * q, row = o >> 5, c = o & 31;
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) v += red[ww][row][c];
      if (m0 + row < a.M) a.t[(long)(m0 + row) * a.ldt + 32 * s + c] = (bf16)v;
    }
    __syncthreads();
  }
}

// A [32][Kin] bf16 (row stride lda) -> packed fragment order: layout 0 = slx_lora_down's (lora_frag_index),
// 1 = the dx kernel's (lora_dxfrag_index)
__global__ __launch_bounds__(256) void lora_pack_a_kernel(const bf16* __restrict__ A, long lda, int Kin, int layout,
                                                          bf16* __restrict__ Af) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= 32L * Kin) return;
  const int rr = (int)(i / Kin), k = (int)(i % Kin);
  Af[layout ? lora_dxfrag_index(rr, k) : lora_frag_index(rr, k)] = A[(long)rr * lda + k];
}

// ---- keep bits ---------------------------------------------------------------------------------------------------
// bits[row][w] bit c = drop_keep(seed, row*ldmask + 32w + c, thr): one thread per 32-bit word (16 pair hashes). The
// words of one row of every job (the 7 LoRA sites of a layer) lie end to end; grid (ceil(words / 64), ceil(rows / 4)),
// wave w of a block takes row 4 * blockIdx.y + w and lane l its word 64 * blockIdx.x + l, so no thread divides (the
// flat-index form spent as many instructions on a 64-bit division as on its 16 hashes: 19.6 us per layer).
struct DropBitsArgs {
  int njobs;
  uint32_t thr;
  long rows;
  int wpre[9];  // prefix sums of the jobs' words per row
  uint32_t s1[8];
  uint32_t* bits[8];
  long ldbits[8];
  long ldmask[8];
};

__global__ __launch_bounds__(256) void dropout_bits_kernel(DropBitsArgs a) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.y * 4 + (threadIdx.x >> 6);
  const int wa = (int)blockIdx.x * 64 + lane;
  if (row >= a.rows || wa >= a.wpre[a.njobs]) return;
  int j = 0;
#pragma unroll
  for (int q = 1; q < 8; ++q) j += (q < a.njobs && wa >= a.wpre[q]) ? 1 : 0;
  const int w = wa - a.wpre[j];
  const unsigned long long i0 = (unsigned long long)(row * a.ldmask[j] + 32 * w);
  uint32_t word = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) word |= drop_keep8(a.s1[j], i0 + 8 * q, a.thr) << (8 * q);
  a.bits[j][row * a.ldbits[j] + w] = word;
}

// ---- backward ---------------------------------------------------------------------------------------------------
struct LoraBwdArgs {
  const bf16* x; long ldx;
  int M, Kin, nsites;
  const float* dt; long lddt;
  const bf16* A[4];
  const uint32_t* bits[4]; long ldbits;
  float* dA[4];
  float* dx; long lddx;
  bf16* dxb; long lddxb;
  float sc;       // 1 / (1 - p)
  int mchunk;
  int dt_bf16;    // dt holds bf16 rows
  float* dA_part; // non-null: per-row-chunk partials [nchunk][nsites][32][Kin] (plain stores) instead of atomics
  bf16* dtb; long lddtb;  // non-null: the dx kernel also writes the bf16 dT rows it converts (slx_lora_grad's operand)
};

__device__ __forceinline__ int la_sw(int row, int chunk) {
  return row * 128 + ((chunk ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3))) << 4);
}
// accumulator-order operand from a swizzled [64][64] bf16 tile: lane l holds X[rbase + 8(j>>2) + 4(l>>5) + (j&3)][cbase + (l&31)]
__device__ __forceinline__ bf16x8 la_tr(const char* lds, int rbase, int cbase, int lane) {
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

// dA_j += dT_j^T drop_j(x): block = 128 columns of x (4 waves x 32) x a chunk of rows walked in 64-row sub-chunks.
// Each staging thread holds 32 consecutive columns of one row, i.e. exactly one keep word per site, so the masks are
// applied while the sub-chunk is committed to LDS: one tile per site of bf16(x / (1-p)) & keep_j (the rounding of
// peft's dropout output), plus dT [64 x 32*NS] (f32 -> bf16), all [64][64] panels with the la_sw swizzle. The inner
// loop is then transposed tile reads + v_mfma_f32_32x32x16_bf16 only (dT^T x masked x per 16-row slice), accumulated
// in registers over the chunk, one set of f32 atomics per block at the end. The next sub-chunk's global loads are
// issued into registers before the current one is multiplied.
template <int NS, bool DTB>  // DTB: dt rows are bf16
__global__ __launch_bounds__(256, 2) void lora_da_kernel(LoraBwdArgs a) {
  constexpr int TP = (32 * NS + 63) / 64;                     // dT panels
  __shared__ __attribute__((aligned(16))) char smem[(2 * NS + TP) * 8192];  // x_j: NS x 2 panels | dT: TP panels
  char* ts = smem + 2 * NS * 8192;
  const int c0 = blockIdx.x * 128;
  const int mb = blockIdx.y * a.mchunk, me = min(a.M, mb + a.mchunk);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int mycol = c0 + 32 * w + (lane & 31);
  const bool drop = a.bits[0] != nullptr;
  f32x16 acc[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  const int srow = tid >> 2;  // staging: this thread's row of the sub-chunk, 16-B chunks (tid & 3) * 4 + c4
  uint4 rx[4];
  float4 rt[4][2];
  uint32_t rm[NS];
  auto load = [&](int mm) {
    const int gm = mm + srow;
    const bool ok = gm < me;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const int c = (tid & 3) * 4 + c4;
      rx[c4] = ok ? *reinterpret_cast<const uint4*>(a.x + (long)gm * a.ldx + c0 + 8 * c) : make_uint4(0u, 0u, 0u, 0u);
      if (8 * c < 32 * NS) {
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (DTB) {  // 8 bf16 in the bits of rt[c4][0]
          const uint4 u = ok ? *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.dt) + (long)gm * a.lddt + 8 * c)
                             : make_uint4(0u, 0u, 0u, 0u);
          rt[c4][0] = __builtin_bit_cast(float4, u);
        } else {
          rt[c4][0] = ok ? *reinterpret_cast<const float4*>(a.dt + (long)gm * a.lddt + 8 * c) : z;
          rt[c4][1] = ok ? *reinterpret_cast<const float4*>(a.dt + (long)gm * a.lddt + 8 * c + 4) : z;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NS; ++j)  // keep word (row srow, columns 32 (tid & 3) ..) of site j
      rm[j] = drop ? (ok ? a.bits[j][(long)gm * a.ldbits + (c0 >> 5) + (tid & 3)] : 0u) : 0xFFFFFFFFu;
  };
  auto commit = [&]() {
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const int c = (tid & 3) * 4 + c4;
      uint4 v = rx[c4];
      uint32_t* u = reinterpret_cast<uint32_t*>(&v);
      if (drop) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          bf16x2 o;
          o[0] = (bf16)(__uint_as_float(u[d] << 16) * a.sc);
          o[1] = (bf16)(__uint_as_float(u[d] & 0xFFFF0000u) * a.sc);
          u[d] = __builtin_bit_cast(uint32_t, o);
        }
      }
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        uint4 m = v;
        if (drop) {
          uint32_t* mu = reinterpret_cast<uint32_t*>(&m);
#pragma unroll
          for (int d = 0; d < 4; ++d) {  // columns 8 c4 + 2d, +1 of this thread's 32 -> bits of rm[j]
            const uint32_t lo = (uint32_t)__builtin_amdgcn_sbfe((int)rm[j], 8 * c4 + 2 * d, 1);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_sbfe((int)rm[j], 8 * c4 + 2 * d + 1, 1);
            mu[d] &= (lo & 0xFFFFu) | (hi & 0xFFFF0000u);
          }
        }
        *reinterpret_cast<uint4*>(smem + (2 * j + (c >> 3)) * 8192 + la_sw(srow, c & 7)) = m;
      }
      if (8 * c < 32 * NS) {
        bf16x8 t;
        if constexpr (DTB) {
          t = __builtin_bit_cast(bf16x8, rt[c4][0]);
        } else {
          t[0] = (bf16)rt[c4][0].x; t[1] = (bf16)rt[c4][0].y; t[2] = (bf16)rt[c4][0].z; t[3] = (bf16)rt[c4][0].w;
          t[4] = (bf16)rt[c4][1].x; t[5] = (bf16)rt[c4][1].y; t[6] = (bf16)rt[c4][1].z; t[7] = (bf16)rt[c4][1].w;
        }
        *reinterpret_cast<bf16x8*>(ts + (c >> 3) * 8192 + la_sw(srow, c & 7)) = t;
      }
    }
  };
  if (mb < me) {
    load(mb);
    commit();
  }
  __syncthreads();
  for (int mm = mb; mm < me; mm += 64) {
    const bool more = mm + 64 < me;
    if (more) load(mm + 64);
#pragma unroll
    for (int ms = 0; ms < 4; ++ms)
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const bf16x8 xm = la_tr(smem + (2 * j + (w >> 1)) * 8192, 16 * ms, 32 * (w & 1), lane);
        const bf16x8 ta = la_tr(ts + ((32 * j) >> 6) * 8192, 16 * ms, (32 * j) & 63, lane);
        acc[j] = mfma32x32(ta, xm, acc[j]);
      }
    __syncthreads();
    if (more) {
      commit();
      __syncthreads();
    }
  }
  if (a.dA_part) {  // this row chunk's partial, summed in chunk order by lora_da_reduce_kernel
    float* part = a.dA_part + (long)blockIdx.y * NS * 32 * a.Kin;
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int rr = (g & 3) + 8 * (g >> 2) + 4 * h;
        part[((long)j * 32 + rr) * a.Kin + mycol] = acc[j][g];
      }
    return;
  }
#pragma unroll
  for (int j = 0; j < NS; ++j)
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int rr = (g & 3) + 8 * (g >> 2) + 4 * h;
      atomicAdd(a.dA[j] + (long)rr * a.Kin + mycol, acc[j][g]);
    }
}

// dA_j[r][k] += sum over the row chunks c of part[c][j][r][k]: 16 lanes per 4 consecutive k, lane t loading chunks
// t, t + 16, ... (at most kDaRedPer, all issued before the first add) and summing them in chunk order, then a fixed
// xor-butterfly over the 16 lanes (a + b == b + a, so every lane ends with the same total): deterministic, and one load
// round trip instead of nchunk dependent ones
constexpr int kDaRedLanes = 16, kDaRedPer = 12;
__global__ __launch_bounds__(256) void lora_da_reduce_kernel(LoraBwdArgs a, int nchunk) {
  const long per = (long)a.nsites * 32 * a.Kin;
  const long i4 = ((long)blockIdx.x * (256 / kDaRedLanes) + (threadIdx.x / kDaRedLanes)) * 4;
  const int t = threadIdx.x % kDaRedLanes;
  const bool ok = i4 < per;
  float4 v[kDaRedPer];
#pragma unroll
  for (int k = 0; k < kDaRedPer; ++k) {
    const int c = t + kDaRedLanes * k;
    v[k] = (ok && c < nchunk) ? *reinterpret_cast<const float4*>(a.dA_part + c * per + i4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 s = v[0];
#pragma unroll
  for (int k = 1; k < kDaRedPer; ++k) { s.x += v[k].x; s.y += v[k].y; s.z += v[k].z; s.w += v[k].w; }
#pragma unroll
  for (int m = 1; m < kDaRedLanes; m <<= 1) {
    s.x += __shfl_xor(s.x, m); s.y += __shfl_xor(s.y, m); s.z += __shfl_xor(s.z, m); s.w += __shfl_xor(s.w, m);
  }
  if (!ok || t != 0) return;
  const int j = (int)(i4 / (32L * a.Kin));
  float* d = a.dA[j] + (i4 - (long)j * 32 * a.Kin);
  float4 o = *reinterpret_cast<float4*>(d);
  o.x += s.x; o.y += s.y; o.z += s.z; o.w += s.w;
  *reinterpret_cast<float4*>(d) = o;
}

// dx += sum_j keep_j / (1-p) * (dT_j A_j) (f32 in place, or bf16(dx + ...) to dxb): block = one 32-row tile, 8 waves
// taking the 32-column tiles w, w+8, ... Each wave computes the TRANSPOSED tile D[col][row] = sum_k A_j[k][col]
// dT_j[row][k] on v_mfma_f32_32x32x16_bf16 (A operand: the packed dx fragments of A_j, one contiguous KiB each; B
// operand: the wave's dT rows, f32 -> bf16, loaded once), so each lane owns one row and 4 consecutive columns per
// register group: dx is read and written with 16-B accesses and the lane's keep bits of a site are one word. The next
// column tile's loads are issued before the current tile's MFMAs.
template <int NS>
struct DxRegs {
  bf16x8 af[NS][2];
  float4 dxv[4];
  uint32_t kw[NS];
};

// Every global load is unconditional (rows past M read row M - 1 and are never stored; DROP is a template switch):
// a load inside a branch makes hipcc drain vmcnt(0) behind it, which serialised the dT row loads into 8 round trips.
template <int NS, bool DTB, bool DROP>  // DTB: dt rows are bf16; DROP: keep bits given
__global__ __launch_bounds__(512) void lora_dx_kernel(LoraBwdArgs a) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int row = blockIdx.x * 32 + r;
  const bool rok = row < a.M;
  const long rowc = rok ? row : a.M - 1;
  const int nct = a.Kin / 32;
  bf16x8 tb[NS][2];  // B operand: lane (row r, half h) holds dT_j[row][16 kb + 8 h + i]
#pragma unroll
  for (int j = 0; j < NS; ++j)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const long off = rowc * a.lddt + 32 * j + 16 * kb + 8 * h;
      if constexpr (DTB) {
        tb[j][kb] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(a.dt) + off);
      } else {
        const float* tp = a.dt + off;
        const float4 f0 = *reinterpret_cast<const float4*>(tp);
        const float4 f1 = *reinterpret_cast<const float4*>(tp + 4);
        tb[j][kb][0] = (bf16)f0.x; tb[j][kb][1] = (bf16)f0.y; tb[j][kb][2] = (bf16)f0.z; tb[j][kb][3] = (bf16)f0.w;
        tb[j][kb][4] = (bf16)f1.x; tb[j][kb][5] = (bf16)f1.y; tb[j][kb][6] = (bf16)f1.z; tb[j][kb][7] = (bf16)f1.w;
      }
    }
  if (a.dtb && w == 0 && rok && blockIdx.y == 0) {  // bf16 dT for slx_lora_grad: one wave of the row tile writes it
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        *reinterpret_cast<bf16x8*>(a.dtb + (long)row * a.lddtb + 32 * j + 16 * kb + 8 * h) = tb[j][kb];
  }
  auto load = [&](int ct, DxRegs<NS>& R) {
#pragma unroll
    for (int j = 0; j < NS; ++j) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        R.af[j][kb] = *reinterpret_cast<const bf16x8*>(a.A[j] + ((long)(2 * ct + kb) * 64 + lane) * 8);
      R.kw[j] = DROP ? a.bits[j][rowc * a.ldbits + ct] : 0u;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
      R.dxv[g] = *reinterpret_cast<const float4*>(a.dx + rowc * a.lddx + 32 * ct + 8 * g + 4 * h);
  };
  auto process = [&](int ct, const DxRegs<NS>& R) {
    f32x16 o[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
#pragma unroll
      for (int i = 0; i < 16; ++i) o[j][i] = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) o[j] = mfma32x32(R.af[j][kb], tb[j][kb], o[j]);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float v[4] = {R.dxv[g].x, R.dxv[g].y, R.dxv[g].z, R.dxv[g].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // register 4g+e: column 8g + 4h + e of the tile
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
          const float k = DROP ? (((R.kw[j] >> (8 * g + 4 * h + e)) & 1u) ? a.sc : 0.f) : 1.0f;
          sum += k * o[j][4 * g + e];
        }
        v[e] += sum;
      }
      if (rok) {
        const int col = 32 * ct + 8 * g + 4 * h;
        if (a.dxb) {
          bf16x4 b = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          *reinterpret_cast<bf16x4*>(a.dxb + (long)row * a.lddxb + col) = b;
        } else {
          *reinterpret_cast<float4*>(a.dx + (long)row * a.lddx + col) = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  };
  // the block's column tiles: wave w takes w + 8 y, then every 8 * gridDim.y-th (gridDim.y column groups per row tile)
  const int c0 = w + 8 * blockIdx.y, cs = 8 * gridDim.y;
  // a load for a tile past nct reads the wave's current tile again (L1/L2-hot) and is never processed: no branch
  // around a load
  DxRegs<NS> R0, R1;
  load(min(c0, nct - 1), R0);
  for (int ct = c0; ct < nct; ct += 2 * cs) {
    const bool more = ct + cs < nct;
    load(more ? ct + cs : ct, R1);
    process(ct, R0);
    if (!more) break;
    load(ct + 2 * cs < nct ? ct + 2 * cs : ct + cs, R0);
    process(ct + cs, R1);
  }
}

// ---- LoRA parameter gradients of a layer in one launch (slx_lora_grad) -------------------------------------------
// out_j (+)= alpha * T_j^T . X_j' for a list of jobs, X_j' = X (dB: X = dy, T = t) or bf16(X / (1-p)) & keep_j (dA: X = the
// site input, T = dT): the skinny [32 x N] = [32 x M] . [M x N] products whose standalone launches (split-K GEMMs for
// dB, lora_da_kernel for dA) stream their big operand at ~1-2 TB/s because every block's row range is only one or two
// 64-row sub-chunks deep, so each block waits one full memory latency per sub-chunk. Here all the products of a layer
// group are work items (job, 128-column block, row chunk) of one persistent launch sized to one item per block slot;
// each item walks its row chunk with two 64-row sub-chunks in flight (register sets R0 / R1) behind the one being
// multiplied, and ends with one set of f32 atomics (the [n][32] B-gradient layout through an LDS transpose, so the
// atomics stay coalesced). Operand staging, masks and MFMA forms are lora_da_kernel's.
constexpr int kLgMaxJobs = 12;
struct LgJob {
  const bf16* X; long ldx; int N;
  const bf16* T; long ldt;
  int ns;
  const uint32_t* bits[3]; long ldbits;
  float sc;      // 1 / (1 - p) (dropout scale of X, applied with the mask)
  float alpha;   // scale of the f32 product
  float* out[3]; int nr;
  int ncb, kch, item0;
  float* part[3];  // deterministic mode: per-row-chunk partials [nkc][32 N] of each site (same layout as out), summed
                   // in chunk order by det_reduce after the launch; null = f32 atomics into out
};
struct LgArgs { int M, njobs, nitems; LgJob j[kLgMaxJobs]; };

__device__ __forceinline__ LgJob lg_job(const LgArgs& a, int jb) {
  switch (jb) {  // static indices only: a dynamic index into the kernel-argument array would copy it to scratch
    case 0: return a.j[0];
    case 1: return a.j[1];
    case 2: return a.j[2];
    case 3: return a.j[3];
    case 4: return a.j[4];
    case 5: return a.j[5];
    case 6: return a.j[6];
    case 7: return a.j[7];
    case 8: return a.j[8];
    case 9: return a.j[9];
    case 10: return a.j[10];
    default: return a.j[11];
  }
}

template <int NS>
struct LgRegs {
  uint4 rx[4];    // X: row srow, 16-B chunks (tid & 3) * 4 + c4 of the 128 columns
  uint4 rt[NS];   // T: piece tid + 256 q of the [64][32 NS] tile (row p / (4 NS), chunk p % (4 NS))
  uint32_t rm[NS];
};

// One work item: rows [mb, me) x the 128 columns from c0 of job J (NS sites sharing X; DROP: keep-bit masks).
// NS and DROP are template parameters so the item loop is straight-line code in which the compiler counts the two
// sub-chunks in flight (vmcnt(N)) instead of draining both at each commit.
template <int NS, bool DROP>
__device__ __forceinline__ void lg_item(const LgJob J, int c0, int mb, int me, int kc, char* smem) {
  char* ts = smem + 6 * 8192;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int srow = tid >> 2;
  const int mycol = c0 + 32 * w + (lane & 31);
  f32x16 acc[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  // branch-free loads: rows past the chunk clamped to its last row (zeroed at commit), T columns past the sites
  // clamped to the last site's
  auto load = [&](int mm, LgRegs<NS>& R) {
    const int gm = min(mm + srow, me - 1);
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const int c = (tid & 3) * 4 + c4;
      R.rx[c4] = *reinterpret_cast<const uint4*>(J.X + (long)gm * J.ldx + c0 + 8 * c);
    }
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const int pc = tid + 256 * q, tr = min(mm + pc / (4 * NS), me - 1);
      R.rt[q] = *reinterpret_cast<const uint4*>(J.T + (long)tr * J.ldt + 8 * (pc % (4 * NS)));
    }
    if constexpr (DROP) {
#pragma unroll
      for (int j = 0; j < NS; ++j) R.rm[j] = J.bits[j][(long)gm * J.ldbits + (c0 >> 5) + (tid & 3)];
    }
  };
  auto commit = [&](const LgRegs<NS>& R, int mm) {
    const bool ok = mm + srow < me;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const int c = (tid & 3) * 4 + c4;
      uint4 v = ok ? R.rx[c4] : make_uint4(0u, 0u, 0u, 0u);
      uint32_t* u = reinterpret_cast<uint32_t*>(&v);
      if constexpr (DROP) {  // bf16(x / (1-p)), the rounding of peft's dropout output
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          bf16x2 o;
          o[0] = (bf16)(__uint_as_float(u[d] << 16) * J.sc);
          o[1] = (bf16)(__uint_as_float(u[d] & 0xFFFF0000u) * J.sc);
          u[d] = __builtin_bit_cast(uint32_t, o);
        }
      }
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        uint4 m = v;
        if constexpr (DROP) {
          uint32_t* mu = reinterpret_cast<uint32_t*>(&m);
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_sbfe((int)R.rm[j], 8 * c4 + 2 * d, 1);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_sbfe((int)R.rm[j], 8 * c4 + 2 * d + 1, 1);
            mu[d] &= (lo & 0xFFFFu) | (hi & 0xFFFF0000u);
          }
        }
        *reinterpret_cast<uint4*>(smem + (2 * j + (c >> 3)) * 8192 + la_sw(srow, c & 7)) = m;
      }
    }
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const int pc = tid + 256 * q, tr = pc / (4 * NS), ch = pc % (4 * NS);
      *reinterpret_cast<uint4*>(ts + (ch >> 3) * 8192 + la_sw(tr, ch & 7)) =
          mm + tr < me ? R.rt[q] : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto mma = [&]() {
    // the lane index laundered per call: its LDS addresses are recomputed (a few VALU per sub-chunk) instead of
    // hoisted out of the sub-chunk loop for every site and slice, which spilled at NS = 3
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int ms = 0; ms < 4; ++ms)
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const bf16x8 xm = la_tr(smem + (2 * j + (w >> 1)) * 8192, 16 * ms, 32 * (w & 1), ln);
        const bf16x8 ta = la_tr(ts + ((32 * j) >> 6) * 8192, 16 * ms, (32 * j) & 63, ln);
        acc[j] = mfma32x32(ta, xm, acc[j]);
      }
  };
  // D sub-chunks in flight behind the one being multiplied (depths 4 / 3 for single- / multi-site items measured the
  // same on the step as 2, profiles/round4_lora_grad_depth_ab.txt)
  constexpr int D = 2;
  const int nsub = (me - mb + 63) / 64;
  LgRegs<NS> R[D];
#pragma unroll
  for (int q = 0; q < D; ++q)
    if (q < nsub) load(mb + 64 * q, R[q]);
  for (int sb = 0; sb < nsub; sb += D) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      if (sb + q < nsub) {
        commit(R[q], mb + 64 * (sb + q));
        __syncthreads();
        if (sb + q + D < nsub) load(mb + 64 * (sb + q + D), R[q]);
        mma();
        __syncthreads();
      }
    }
  }
  const long pofs = (long)kc * 32 * J.N;  // this item's partial slot (deterministic mode)
  if (!J.nr) {
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int rr = (g & 3) + 8 * (g >> 2) + 4 * h;
        if (J.part[0]) J.part[j][pofs + (long)rr * J.N + mycol] = J.alpha * acc[j][g];
        else atomicAdd(J.out[j] + (long)rr * J.N + mycol, J.alpha * acc[j][g]);
      }
  } else {  // out[n][32]: transpose through LDS ([32][129] f32), then 32 consecutive r per 32 lanes
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < NS; ++j) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int rr = (g & 3) + 8 * (g >> 2) + 4 * h;
        red[rr * 129 + 32 * w + (lane & 31)] = acc[j][g];
      }
      __syncthreads();
      for (int e = tid; e < 32 * 128; e += 256) {
        const int col = e >> 5, r = e & 31;
        if (J.part[0]) J.part[j][pofs + (long)(c0 + col) * 32 + r] = J.alpha * red[r * 129 + col];
        else atomicAdd(J.out[j] + (long)(c0 + col) * 32 + r, J.alpha * red[r * 129 + col]);
      }
      __syncthreads();
    }
  }
}

// one block per work item (the host sizes the items to about one per block slot, so the grid is one round)
__global__ __launch_bounds__(256, 2) void lora_grad_kernel(LgArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[8 * 8192];  // X: 3 sites x 2 panels | T: 2 panels
  const int item = blockIdx.x;
  int jb = 0;
#pragma unroll
  for (int q = 1; q < kLgMaxJobs; ++q) jb += (q < a.njobs && item >= lg_job(a, q).item0) ? 1 : 0;
  const LgJob J = lg_job(a, jb);
  const int li = item - J.item0, cb = li % J.ncb, kc = li / J.ncb;
  const int c0 = cb * 128, mb = kc * J.kch, me = min(a.M, mb + J.kch);
  const bool drop = J.bits[0] != nullptr;
  switch (J.ns * 2 + (drop ? 1 : 0)) {
    case 2: lg_item<1, false>(J, c0, mb, me, kc, smem); break;
    case 3: lg_item<1, true>(J, c0, mb, me, kc, smem); break;
    case 4: lg_item<2, false>(J, c0, mb, me, kc, smem); break;
    case 5: lg_item<2, true>(J, c0, mb, me, kc, smem); break;
    case 6: lg_item<3, false>(J, c0, mb, me, kc, smem); break;
    default: lg_item<3, true>(J, c0, mb, me, kc, smem); break;
  }
}


// ---- the down site's LoRA dgrad fused with the SwiGLU backward (slx_lora_swiglu_bwd) ---------------------------------
// dgu = [d * u * silu'(g) | d * silu(g)] with d = resid + keep * (dT . A) / (1 - p): the Qwen2MLP backward from the
// gradient of the activation act = silu(g) * u (resid, the down projection's bf16 base dgrad) plus the down site's LoRA
// term (dT [M x 32] . A [32 x F], keep bits of the forward's dropout). The GEMM form of the same (a K = 64 DROPMASK_
// SWIGLU epilogue over the zero-padded A) walks 128 x 128 output tiles whose epilogue streams are the whole cost
// (~315 MB per layer); here a block owns 32 rows x 256 columns: it issues its 4 x 16 B of resid / gate / up per thread
// and the keep words first, runs the tiny K = 32 product on the MFMA (4 per wave, operands straight from global: dT
// rows and the A^T rows of the packed [F][32] copy), exchanges the [32 x 256] f32 tile through LDS and stores 16 B of
// gate and up gradient per chunk - row-contiguous 512-B streams in and out.
struct LswArgs {
  const bf16* dt; long lddt;
  const bf16* at; long ldat;  // A^T [F][32] bf16
  const bf16* resid; long ldr;
  const bf16* gu; long ldgu;
  const uint32_t* bits; long ldbits;
  float sc;  // 1 / (1 - p)
  bf16* dgu; long lddgu;
  int M, F;
};

// DROP: keep bits given (a compile-time switch: a keep-word load behind `a.bits ? ... :` was a branch around a load,
// after which hipcc drains vmcnt(0), serialising the block's four chunks of loads)
template <bool DROP>
__global__ __launch_bounds__(256) void lora_swiglu_bwd_kernel(LswArgs a) {
  __shared__ __attribute__((aligned(16))) float acc_s[32][256 + 4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // column block fastest in dispatch order: the blocks in flight together cover whole rows (DRAM page locality)
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 256;
  // epilogue operands first: chunk i of this thread = row (tid + 256 i) >> 5, 8 columns 8 ((tid + 256 i) & 31)
  uint4 rr[4], gg[4], uu[4];
  uint32_t kb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, row = c >> 5, n = n0 + 8 * (c & 31);
    const int m = min(m0 + row, a.M - 1);  // rows past M load row M-1 (never stored)
    rr[i] = *reinterpret_cast<const uint4*>(a.resid + (long)m * a.ldr + n);
    gg[i] = *reinterpret_cast<const uint4*>(a.gu + (long)m * a.ldgu + n);
    uu[i] = *reinterpret_cast<const uint4*>(a.gu + (long)m * a.ldgu + a.F + n);
    kb[i] = DROP ? (a.bits[(long)m * a.ldbits + (n >> 5)] >> (n & 31)) & 0xFFu : 0xFFu;
  }
  // [32 x 256] = dT [32 x 32] . A [32 x 256]: wave w takes column blocks 2w, 2w + 1
  const int mr = min(m0 + (lane & 31), a.M - 1);
  bf16x8 af[2], bfr[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
    af[kk] = *reinterpret_cast<const bf16x8*>(a.dt + (long)mr * a.lddt + 16 * kk + 8 * (lane >> 5));
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int n = n0 + 32 * (2 * w + q) + (lane & 31);
      bfr[q][kk] = *reinterpret_cast<const bf16x8*>(a.at + (long)n * a.ldat + 16 * kk + 8 * (lane >> 5));
    }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    f32x16 acc;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
    acc = mfma32x32(af[0], bfr[q][0], acc);
    acc = mfma32x32(af[1], bfr[q][1], acc);
#pragma unroll
    for (int j = 0; j < 16; ++j) acc_s[8 * (j >> 2) + 4 * (lane >> 5) + (j & 3)][32 * (2 * w + q) + (lane & 31)] = acc[j];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, row = c >> 5, cc = c & 31, n = n0 + 8 * cc;
    const int m = m0 + row;
    const float4 v0 = *reinterpret_cast<const float4*>(&acc_s[row][8 * cc]);
    const float4 v1 = *reinterpret_cast<const float4*>(&acc_s[row][8 * cc + 4]);
    const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const bf16x8 r8 = __builtin_bit_cast(bf16x8, rr[i]), g8 = __builtin_bit_cast(bf16x8, gg[i]),
                 u8 = __builtin_bit_cast(bf16x8, uu[i]);
    bf16x8 og, ou;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = ((kb[i] >> e) & 1u ? v[e] * a.sc : 0.f) + (float)r8[e];
      const float g = (float)g8[e], u = (float)u8[e];
      og[e] = (bf16)(d * u * silu_grad(g));
      ou[e] = (bf16)(d * silu(g));
    }
    if (m < a.M) {
      *reinterpret_cast<bf16x8*>(a.dgu + (long)m * a.lddgu + n) = og;
      *reinterpret_cast<bf16x8*>(a.dgu + (long)m * a.lddgu + a.F + n) = ou;
    }
  }
}

// ---- the same pass with the down site's dA and the gate / up sites' dB (slx_lora_swiglu_bwd_grads) ------------------
// slx_lora_grad's MLP-half launch streamed dgu (2F wide, 124 MB at the InternVL2-1B step) for dB_gate / dB_up and act
// (62 MB) for dA_down once more, after this kernel had both in registers. Here a block owns 128 columns of F and a
// group of 32-row chunks, two chunks' loads in flight (register sets R[0] / R[1]: resid / gate / up / keep, 2 x 16 B
// each per thread, and the three [32 x 32] LoRA operand tiles dT, tg, tu on the first 128 threads). Per chunk it forms
// the dgrad term (dT . A on the MFMA, 2 per wave, A^T fragments loaded once per block) and exchanges it through LDS;
// computes dgu exactly as lora_swiglu_bwd_kernel does and act / drop(act) exactly as the forward's
// swiglu_lora_down_kernel does; stores dgu and issues the loads of the chunk after next into the freed registers;
// stages dgu_gate, dgu_up, drop(act) and the operand tiles as [32][64] la_sw panels; and accumulates the three
// [32 x 128] products with lora_grad's transposed fragment reads (la_tr) on v_mfma_f32_32x32x16_bf16, 6 per wave.
// The block's three f32 partials go to ws [G][3][32 F] (the B gradients transposed through LDS to their [F][32]
// layout) and lsw_grads_reduce_kernel adds them in row-group order.
struct LswgArgs {
  LswArgs s;
  const bf16* tg; const bf16* tu; long ldtg;
  int kch;         // rows per block (a multiple of 32)
  float* part;     // [gridDim.y][3][32 F]
};

struct LswgRegs {
  uint4 rr[2], gg[2], uu[2], td, tgv, tuv;
  uint32_t kb[2];
  bf16x8 af[2];
};

// DROP: keep bits given (p > 0); a compile-time switch, so every load of the chunk loop is an unconditional global load
template <bool DROP>
__global__ __launch_bounds__(256, 2) void lora_swiglu_bwd_grads_kernel(LswgArgs g) {
  // region P (24 KiB): the [32][132] f32 dgrad-term exchange, then per chunk the panels og (0, 1), ou (2, 3),
  // drop(act) (4, 5) of 4 KiB each; region T (12 KiB): the dT, tg, tu panels (columns 0-31 used)
  constexpr int PB = 4096;
  __shared__ __attribute__((aligned(16))) char smem[9 * PB];  // >= the [32][129] f32 transpose of the partials
  float* acc_s = reinterpret_cast<float*>(smem);
  char* tp = smem + 6 * PB;
  const LswArgs& a = g.s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int n0 = blockIdx.x * 128;
  const int mb = blockIdx.y * g.kch, me = min(a.M, mb + g.kch);
  // A^T fragments of the dgrad term: wave w's column tile 32 w
  bf16x8 bfr[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
    bfr[kk] = *reinterpret_cast<const bf16x8*>(a.at + (long)(n0 + 32 * w + (lane & 31)) * a.ldat + 16 * kk + 8 * h);
  f32x16 accA, accG, accU;
#pragma unroll
  for (int j = 0; j < 16; ++j) accA[j] = accG[j] = accU[j] = 0.f;
  // piece c = tid + 256 i (i = 0, 1) is row c >> 4, columns n0 + 8 (c & 15); operand tiles (tid < 128): row tid >> 2,
  // 16-B chunk tid & 3; af: dT rows m0 + (lane & 31)
  auto load = [&](int m0, LswgRegs& R) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i, n = n0 + 8 * (c & 15);
      const int m = min(m0 + (c >> 4), a.M - 1);  // rows past M load row M-1 (zeroed in the panels, never stored)
      R.rr[i] = *reinterpret_cast<const uint4*>(a.resid + (long)m * a.ldr + n);
      R.gg[i] = *reinterpret_cast<const uint4*>(a.gu + (long)m * a.ldgu + n);
      R.uu[i] = *reinterpret_cast<const uint4*>(a.gu + (long)m * a.ldgu + a.F + n);
      R.kb[i] = DROP ? a.bits[(long)m * a.ldbits + (n >> 5)] : 0xFFFFFFFFu;  // shifted at use
    }
    {  // every thread loads (threads 128.. duplicate 0..127's pieces, L2 hits): no branch around a load
      const int tm = min(m0 + ((tid & 127) >> 2), a.M - 1), tc = 8 * (tid & 3);
      R.td = *reinterpret_cast<const uint4*>(a.dt + (long)tm * a.lddt + tc);
      R.tgv = *reinterpret_cast<const uint4*>(g.tg + (long)tm * g.ldtg + tc);
      R.tuv = *reinterpret_cast<const uint4*>(g.tu + (long)tm * g.ldtg + tc);
    }
    const int mr = min(m0 + (lane & 31), a.M - 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      R.af[kk] = *reinterpret_cast<const bf16x8*>(a.dt + (long)mr * a.lddt + 16 * kk + 8 * h);
  };
  auto process = [&](LswgRegs& R, int m0, bool more) {
    {  // dgrad term [32 x 128] = dT [32 x 32] . A [32 x 128]: wave w columns 32 w
      f32x16 acc;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = 0.f;
      acc = mfma32x32(R.af[0], bfr[0], acc);
      acc = mfma32x32(R.af[1], bfr[1], acc);
#pragma unroll
      for (int j = 0; j < 16; ++j) acc_s[(8 * (j >> 2) + 4 * h + (j & 3)) * 132 + 32 * w + (lane & 31)] = acc[j];
    }
    __syncthreads();
    float v[2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i, row = c >> 4, cc = c & 15;
      const float4 v0 = *reinterpret_cast<const float4*>(&acc_s[row * 132 + 8 * cc]);
      const float4 v1 = *reinterpret_cast<const float4*>(&acc_s[row * 132 + 8 * cc + 4]);
      v[i][0] = v0.x; v[i][1] = v0.y; v[i][2] = v0.z; v[i][3] = v0.w;
      v[i][4] = v1.x; v[i][5] = v1.y; v[i][6] = v1.z; v[i][7] = v1.w;
    }
    __syncthreads();  // region P is rewritten as panels below
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i, row = c >> 4, cc = c & 15, n = n0 + 8 * cc;
      const int m = m0 + row;
      const bool ok = m < me;
      const bf16x8 r8 = __builtin_bit_cast(bf16x8, R.rr[i]), g8 = __builtin_bit_cast(bf16x8, R.gg[i]),
                   u8 = __builtin_bit_cast(bf16x8, R.uu[i]);
      bf16x8 og, ou, dk;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool keep = (R.kb[i] >> ((8 * cc + e) & 31)) & 1u;
        const float d = (keep ? v[i][e] * a.sc : 0.f) + (float)r8[e];  // lora_swiglu_bwd_kernel's arithmetic
        const float gf = (float)g8[e], uf = (float)u8[e];
        og[e] = (bf16)(d * uf * silu_grad(gf));
        ou[e] = (bf16)(d * silu(gf));
        const bf16 act = (bf16)(silu(gf) * uf);  // swiglu_lora_down_kernel's (and slx_swiglu_fwd's) rounding
        dk[e] = keep ? (bf16)((float)act * a.sc) : (bf16)0.f;
      }
      if (ok) {
        *reinterpret_cast<bf16x8*>(a.dgu + (long)m * a.lddgu + n) = og;
        *reinterpret_cast<bf16x8*>(a.dgu + (long)m * a.lddgu + a.F + n) = ou;
      }
      const uint4 z = make_uint4(0u, 0u, 0u, 0u);
      const int po = (cc >> 3) * PB + la_sw(row, cc & 7);
      *reinterpret_cast<uint4*>(smem + po) = ok ? __builtin_bit_cast(uint4, og) : z;
      *reinterpret_cast<uint4*>(smem + 2 * PB + po) = ok ? __builtin_bit_cast(uint4, ou) : z;
      *reinterpret_cast<uint4*>(smem + 4 * PB + po) = ok ? __builtin_bit_cast(uint4, dk) : z;
    }
    if (tid < 128) {
      const int to = la_sw(tid >> 2, tid & 3);
      *reinterpret_cast<uint4*>(tp + to) = R.td;
      *reinterpret_cast<uint4*>(tp + PB + to) = R.tgv;
      *reinterpret_cast<uint4*>(tp + 2 * PB + to) = R.tuv;
    }
    // the chunk after next into the registers just consumed (past the block's rows: this chunk again, L2-hot; every
    // load of the loop is unconditional, so the compiler counts the loads in flight instead of draining them)
    __builtin_amdgcn_sched_barrier(0);
    load(more ? m0 + 64 : m0, R);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    {  // [32 x 32] per product and wave: columns 32 w of the block (panel w >> 1, panel columns 32 (w & 1))
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int pc = 32 * (w & 1), pn = (w >> 1) * PB;
#pragma unroll
      for (int ms = 0; ms < 2; ++ms) {
        accA = mfma32x32(la_tr(tp, 16 * ms, 0, ln), la_tr(smem + 4 * PB + pn, 16 * ms, pc, ln), accA);
        accG = mfma32x32(la_tr(tp + PB, 16 * ms, 0, ln), la_tr(smem + pn, 16 * ms, pc, ln), accG);
        accU = mfma32x32(la_tr(tp + 2 * PB, 16 * ms, 0, ln), la_tr(smem + 2 * PB + pn, 16 * ms, pc, ln), accU);
      }
    }
    __syncthreads();
  };
  LswgRegs R[2];
  load(mb, R[0]);
  __builtin_amdgcn_sched_barrier(0);  // R[0]'s loads all before R[1]'s: the in-loop waits then count R[1]'s as newer
  load(mb + 32 < me ? mb + 32 : mb, R[1]);
  __builtin_amdgcn_sched_barrier(0);
  for (int m0 = mb; m0 < me; m0 += 64) {  // a pair of chunks per trip (a chunk past me only adds zeros)
    process(R[0], m0, m0 + 64 < me);
    process(R[1], m0 + 32, m0 + 96 < me);
  }
  // partials: A in its [32][F] layout straight from the accumulators; G / U through an LDS transpose to [F][32]
  const long F32n = 32L * a.F;
  float* pb = g.part + (long)blockIdx.y * 3 * F32n;
  const int mycol = n0 + 32 * w + (lane & 31);
#pragma unroll
  for (int j = 0; j < 16; ++j) pb[(long)((j & 3) + 8 * (j >> 2) + 4 * h) * a.F + mycol] = accA[j];
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const f32x16& acc = q == 0 ? accG : accU;
#pragma unroll
    for (int j = 0; j < 16; ++j) red[((j & 3) + 8 * (j >> 2) + 4 * h) * 129 + 32 * w + (lane & 31)] = acc[j];
    __syncthreads();
    for (int e = tid; e < 32 * 128; e += 256) {
      const int col = e >> 5, r = e & 31;
      pb[(1 + q) * F32n + (long)(n0 + col) * 32 + r] = red[r * 129 + col];
    }
    __syncthreads();
  }
}

// out_q[k] += alpha_q * sum over the row groups y (in order) of part[y][q][k], q = 0 (dA_down), 1 (dB_gate), 2 (dB_up)
__global__ __launch_bounds__(256) void lsw_grads_reduce_kernel(const float* part, int ny, long n, float* o0, float* o1,
                                                               float* o2, float al0, float al12) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= 3 * n) return;
  const int q = (int)(e / n);
  const long k = e - q * n;
  float s = 0.f;
  for (int y = 0; y < ny; ++y) s += part[(long)y * 3 * n + e];
  float* o = q == 0 ? o0 : (q == 1 ? o1 : o2);
  o[k] += (q == 0 ? al0 : al12) * s;
}

// ---- the SwiGLU forward fused with the down site's LoRA down-projection (slx_swiglu_lora_down) ----------------------
// act = silu(g) * u (bf16, the Qwen2MLP activation the down projection reads) and t = drop(act) . A^T [M x 32] (peft's
// lora_A on down_proj, drop(act) = bf16(act / (1 - p)) & keep), in one pass over gu: a block owns 32 rows x 256
// columns, streams g / u as 16-B row chunks, stores act, stages drop(act) in LDS ([32][256] bf16, 16-B chunks XOR-
// swizzled by the row) and one wave runs its 32 x 32 x 256 slice of t on the MFMA (16 MFMAs, A rows straight from
// global, L2-resident) and stores the block's [32 x 32] f32 partial to the workspace; a second launch adds the F / 256 partials of every row in column-block order (deterministic) and writes t
// as bf16. Replaces slx_swiglu_fwd + slx_lora_down(down), which read act back from HBM with only M / 32 blocks.
struct SldArgs {
  const bf16* gu; long ldgu;
  bf16* act; long ldact;
  const bf16* A; long lda;        // lora_A [32][F] bf16
  const uint32_t* bits; long ldbits;
  float sc;
  bf16* t; long ldt;
  float* part;                    // [F / 256][M][32] f32 partials
  int M, F;
  uint32_t s1, thr; int gen;      // gen: the keep bits generated here (mask index m * F + n) and written to bits
};

template <bool DROP>  // as lora_swiglu_bwd_kernel's
__global__ __launch_bounds__(256) void swiglu_lora_down_kernel(SldArgs a) {
  __shared__ __attribute__((aligned(16))) char xs[32 * 512];  // drop(act) [32][256] bf16
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // column block fastest in dispatch order: the blocks in flight together cover whole rows (DRAM page locality)
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 256;
  uint4 gg[4], uu[4];
  uint32_t kb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, row = c >> 5, n = n0 + 8 * (c & 31);
    const int m = min(m0 + row, a.M - 1);
    gg[i] = *reinterpret_cast<const uint4*>(a.gu + (long)m * a.ldgu + n);
    uu[i] = *reinterpret_cast<const uint4*>(a.gu + (long)m * a.ldgu + a.F + n);
    if (!DROP || a.gen) kb[i] = 0xFFu;
    else kb[i] = (a.bits[(long)m * a.ldbits + (n >> 5)] >> (n & 31)) & 0xFFu;
  }
  if (DROP && a.gen) {  // the 8 keep bits of each piece hashed while its loads fly; byte (n / 8) % 4 of its word stored
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i, row = c >> 5, n = n0 + 8 * (c & 31);
      kb[i] = drop_keep8(a.s1, (unsigned long long)(m0 + row) * a.F + n, a.thr);
      if (m0 + row < a.M)
        reinterpret_cast<uint8_t*>(const_cast<uint32_t*>(a.bits))[((long)(m0 + row) * a.ldbits + (n >> 5)) * 4 + ((n >> 3) & 3)] =
            (uint8_t)kb[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, row = c >> 5, cc = c & 31, n = n0 + 8 * cc;
    const bf16x8 g8 = __builtin_bit_cast(bf16x8, gg[i]), u8 = __builtin_bit_cast(bf16x8, uu[i]);
    bf16x8 o, d;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = (bf16)(silu((float)g8[e]) * (float)u8[e]);  // slx_swiglu_fwd's rounding
      d[e] = (kb[i] >> e) & 1u ? (bf16)((float)o[e] * a.sc) : (bf16)0.f;
    }
    if (m0 + row < a.M) *reinterpret_cast<bf16x8*>(a.act + (long)(m0 + row) * a.ldact + n) = o;
    *reinterpret_cast<bf16x8*>(xs + row * 512 + ((cc ^ (row & 31)) << 4)) = d;
  }
  __syncthreads();
  if (w != 0) return;
  // wave 0: the block's [32 x 32] partial over its 256 columns, 16 MFMAs; A rows j = lane & 31 straight from global
  f32x16 acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(a.A + (long)(lane & 31) * a.lda + n0 + 16 * kk + 8 * (lane >> 5));
    const int row = lane & 31, cc = 2 * kk + (lane >> 5);
    const bf16x8 af = *reinterpret_cast<const bf16x8*>(xs + row * 512 + ((cc ^ (row & 31)) << 4));
    acc = mfma32x32(af, bfr, acc);
  }
  float* pb = a.part + ((long)blockIdx.x * a.M) * 32;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int row = 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3);
    if (m0 + row < a.M) pb[(long)(m0 + row) * 32 + (lane & 31)] = acc[j];
  }
}

// t[m][j] = bf16(sum over the column blocks y of part[y][m][j]), y in order: the kernel boundary makes every partial
// visible (an in-launch last-arriver hand-off needs an agent-scope release per block, i.e. an L2 write-back behind
// the block's act stores, which cost far more than this launch)
__global__ __launch_bounds__(256) void swiglu_lora_down_reduce_kernel(const float* part, int ny, long M, bf16* t,
                                                                      long ldt) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= M * 32) return;
  float v = 0.f;
  for (int y = 0; y < ny; ++y) v += part[(long)y * M * 32 + e];
  t[(e >> 5) * ldt + (e & 31)] = (bf16)v;
}

}  // namespace slx

using namespace slx;

extern "C" int slx_lora_down(const slx_lora_down_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d->nsites >= 1 && d->nsites <= 4 && d->r == 32, "slx_lora_down: 1..4 sites of rank 32");
  SLX_CHECK_ARG(d->Kin % 32 == 0 && d->ldx % 8 == 0, "slx_lora_down: Kin %% 32, ldx %% 8");
  SLX_CHECK_ARG(d->p >= 0.f && d->p < 1.f, "slx_lora_down: 0 <= p < 1");
  SLX_CHECK_ARG(d->bits[0] == nullptr || d->ldbits >= d->Kin / 32, "slx_lora_down: ldbits < Kin/32");
  if (d->M == 0) return 0;
  LoraDownArgs a;
  memset(&a, 0, sizeof(a));
  a.x = (const bf16*)d->x; a.ldx = d->ldx; a.M = (int)d->M; a.Kin = d->Kin; a.nsites = d->nsites;
  for (int i = 0; i < 4; ++i) {
    a.A[i] = (const bf16*)(i < d->nsites ? d->A[i] : d->A[0]);
    a.bits[i] = (i < d->nsites && d->p > 0.f) ? d->bits[i] : nullptr;
    SLX_CHECK_ARG(i >= d->nsites || d->p == 0.f || d->bits[i], "slx_lora_down: p > 0 needs the keep bits of every site");
  }
  a.ldbits = d->ldbits;
  a.t = (bf16*)d->t; a.ldt = d->ldt; a.p = d->p; a.ldmask = d->ldmask;
  a.gen = d->gen_bits && d->p > 0.f;
  if (a.gen) {
    SLX_CHECK_ARG(d->ldmask % 2 == 0, "slx_lora_down: gen_bits needs an even ldmask");
    a.thr = (uint32_t)(d->p * 65536.0f + 0.5f);  // slx_dropout_bits' threshold
    for (int i = 0; i < d->nsites; ++i) a.s1[i] = drop_seed_mix(d->seed[i]);
  }
  dim3 grid((unsigned)((d->M + 31) / 32));
  hipStream_t st = (hipStream_t)stream;
  switch (d->nsites) {
    case 1: hipLaunchKernelGGL(lora_down_kernel<1>, grid, dim3(512), 0, st, a); break;
    case 2: hipLaunchKernelGGL(lora_down_kernel<2>, grid, dim3(512), 0, st, a); break;
    case 3: hipLaunchKernelGGL(lora_down_kernel<3>, grid, dim3(512), 0, st, a); break;
    default: hipLaunchKernelGGL(lora_down_kernel<4>, grid, dim3(512), 0, st, a); break;
  }
  SLX_LAUNCH_CHECK("slx_lora_down");
  return 0;
}

extern "C" int slx_lora_pack_a(const void* A, int64_t lda, int Kin, int layout, void* Af, slx_stream_t stream) {
  SLX_CHECK_ARG(A && Af && Kin > 0 && Kin % 32 == 0 && lda >= Kin, "slx_lora_pack_a: A, Af, Kin %% 32, lda >= Kin");
  SLX_CHECK_ARG(layout == 0 || layout == 1, "slx_lora_pack_a: layout 0 (lora_down) or 1 (lora_bwd dx)");
  hipLaunchKernelGGL(lora_pack_a_kernel, dim3((unsigned)((32L * Kin + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)A, (long)lda, Kin, layout, (bf16*)Af);
  SLX_LAUNCH_CHECK("slx_lora_pack_a");
  return 0;
}

extern "C" int slx_dropout_bits(const slx_dropout_bits_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d && d->njobs >= 1 && d->njobs <= 8, "slx_dropout_bits: 1..8 jobs");
  SLX_CHECK_ARG(d->p > 0.f && d->p < 1.f, "slx_dropout_bits: 0 < p < 1");
  if (d->rows == 0) return 0;
  DropBitsArgs a;
  memset(&a, 0, sizeof(a));
  a.njobs = d->njobs; a.rows = d->rows;
  a.thr = (uint32_t)(d->p * 65536.0f + 0.5f);
  SLX_CHECK_ARG(d->rows <= 4L * 65535, "slx_dropout_bits: rows <= 262140");
  int off = 0;
  for (int j = 0; j < d->njobs; ++j) {
    const slx_dropout_bits_job& jb = d->job[j];
    SLX_CHECK_ARG(jb.bits && jb.cols % 32 == 0 && jb.cols > 0 && jb.ldbits >= jb.cols / 32 && jb.ldmask % 2 == 0,
                  "slx_dropout_bits: job %d needs bits, cols %% 32, ldbits >= cols/32, even ldmask", j);
    a.wpre[j] = off;
    a.s1[j] = drop_seed_mix(jb.seed);
    a.bits[j] = jb.bits; a.ldbits[j] = jb.ldbits; a.ldmask[j] = jb.ldmask;
    off += jb.cols / 32;
  }
  a.wpre[d->njobs] = off;
  hipLaunchKernelGGL(dropout_bits_kernel, dim3((unsigned)((off + 63) / 64), (unsigned)((d->rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, a);
  SLX_LAUNCH_CHECK("slx_dropout_bits");
  return 0;
}

template <int NS, bool DTB>
static void launch_bwd_t(const LoraBwdArgs& a, dim3 grid, hipStream_t st) {
  if (a.dA[0]) {
    hipLaunchKernelGGL((lora_da_kernel<NS, DTB>), grid, dim3(256), 0, st, a);
    if (a.dA_part) {
      const long per4 = (long)NS * 32 * a.Kin / 4, per_block = 256 / kDaRedLanes;
      hipLaunchKernelGGL(lora_da_reduce_kernel, dim3((unsigned)((per4 + per_block - 1) / per_block)), dim3(256), 0, st, a,
                         (int)grid.y);
    }
  }
  // column groups per 32-row tile (SLX_LORA_DX_GROUPS): 1. The 512-thread blocks hold 150-200 VGPRs, so one fits a CU;
  // two groups (400 blocks at Qwen2's M = 6384) ran as 1.56 rounds and measured 0.25 % slower on the step than one
  // group's 200 blocks of 3-4 pipelined tiles per wave (profiles/round5_lora_dx_groups_ab.txt)
  static const int dxg = [] { const char* e = getenv("SLX_LORA_DX_GROUPS"); return e ? atoi(e) : 1; }();
  const int nct = a.Kin / 32;
  int g = dxg < 1 ? 1 : dxg;
  while (g > 1 && 8 * g > nct) --g;
  const dim3 dgrid((unsigned)((a.M + 31) / 32), (unsigned)g);
  if (a.dx && a.bits[0]) hipLaunchKernelGGL((lora_dx_kernel<NS, DTB, true>), dgrid, dim3(512), 0, st, a);
  else if (a.dx) hipLaunchKernelGGL((lora_dx_kernel<NS, DTB, false>), dgrid, dim3(512), 0, st, a);
}
template <int NS>
static void launch_bwd(const LoraBwdArgs& a, dim3 grid, hipStream_t st) {
  if (a.dt_bf16) launch_bwd_t<NS, true>(a, grid, st);
  else launch_bwd_t<NS, false>(a, grid, st);
}

// row chunks of the dA pass (shared by the launch and the workspace size): fewer chunks mean fewer dA partials, more
// mean more blocks
static int lora_da_mchunk(long M, int Kin) {
  static const int tgt = [] { const char* e = getenv("SLX_LORA_DA_BLOCKS"); return e ? atoi(e) : 512; }();
  const int cb = Kin / 128;
  const int nch = (tgt + cb - 1) / cb;
  int mchunk = (int)((M + nch - 1) / nch);
  mchunk = ((mchunk + 63) / 64) * 64;
  return mchunk < 64 ? 64 : mchunk;
}

extern "C" int64_t slx_lora_bwd_ws_floats(int64_t M, int Kin, int nsites) {
  if (M <= 0 || Kin <= 0 || Kin % 128 != 0 || nsites < 1) return 0;
  const int mchunk = lora_da_mchunk(M, Kin);
  const long nch = (M + mchunk - 1) / mchunk;
  return nch * nsites * 32L * Kin;
}

static int lora_bwd_impl(const slx_lora_bwd_desc* d, float* ws, int64_t ws_floats, slx_stream_t stream);

extern "C" int slx_lora_bwd(const slx_lora_bwd_desc* d, slx_stream_t stream) {
  return lora_bwd_impl(d, nullptr, 0, stream);
}

extern "C" int slx_lora_bwd_ws(const slx_lora_bwd_desc* d, float* ws, int64_t ws_floats, slx_stream_t stream) {
  return lora_bwd_impl(d, ws, ws_floats, stream);
}

static int lora_bwd_impl(const slx_lora_bwd_desc* d, float* ws, int64_t ws_floats, slx_stream_t stream) {
  SLX_CHECK_ARG(d->nsites >= 1 && d->nsites <= 4 && d->r == 32, "slx_lora_bwd: 1..4 sites of rank 32");
  SLX_CHECK_ARG(d->Kin % 128 == 0 && d->ldx % 8 == 0 && d->lddt % 4 == 0, "slx_lora_bwd: Kin %% 128, ldx %% 8, lddt %% 4");
  SLX_CHECK_ARG(!d->dx || (d->lddx % 4 == 0 && (!d->dx_bf16 || d->lddx_bf16 % 4 == 0)),
                "slx_lora_bwd: lddx %% 4 (and lddx_bf16 %% 4): the dx term uses 16-B accesses");
  SLX_CHECK_ARG(d->p >= 0.f && d->p < 1.f, "slx_lora_bwd: 0 <= p < 1");
  SLX_CHECK_ARG(d->p == 0.f || (d->bits[0] && d->ldbits >= d->Kin / 32), "slx_lora_bwd: p > 0 needs the keep bits");
  SLX_CHECK_ARG(!d->dx_bf16 || d->dx, "slx_lora_bwd: dx_bf16 needs dx (the f32 base gradient it is added to)");
  SLX_CHECK_ARG(d->dA[0] || d->dx, "slx_lora_bwd: nothing to do (neither dA nor dx)");
  for (int i = 1; i < d->nsites; ++i)
    SLX_CHECK_ARG((d->dA[i] != nullptr) == (d->dA[0] != nullptr), "slx_lora_bwd: dA for all sites or none");
  if (d->M == 0) return 0;
  LoraBwdArgs a;
  memset(&a, 0, sizeof(a));
  a.x = (const bf16*)d->x; a.ldx = d->ldx; a.M = (int)d->M; a.Kin = d->Kin; a.nsites = d->nsites;
  a.dt = d->dt; a.lddt = d->lddt; a.dt_bf16 = d->dt_bf16;
  SLX_CHECK_ARG(!d->dt_bf16 || d->lddt % 8 == 0, "slx_lora_bwd: bf16 dt needs lddt %% 8 (16-B row loads)");
  for (int i = 0; i < 4; ++i) {
    a.A[i] = (const bf16*)(i < d->nsites ? d->A[i] : d->A[0]);
    a.bits[i] = (d->p > 0.f && i < d->nsites) ? d->bits[i] : nullptr;
    a.dA[i] = i < d->nsites ? d->dA[i] : d->dA[0];
  }
  a.ldbits = d->ldbits;
  a.dx = d->dx; a.lddx = d->lddx;
  a.dxb = (bf16*)d->dx_bf16; a.lddxb = d->lddx_bf16;
  a.dtb = (bf16*)d->dt_bf16_out; a.lddtb = d->ld_dt_bf16_out;
  SLX_CHECK_ARG(!a.dtb || (d->dx && a.lddtb % 8 == 0 && ((uintptr_t)a.dtb & 15) == 0),
                "slx_lora_bwd: dt_bf16_out needs the dx term (its kernel converts dT), 16-B aligned rows");
  a.sc = 1.0f / (1.0f - d->p);
  const int cb = d->Kin / 128;
  a.mchunk = lora_da_mchunk(d->M, d->Kin);
  dim3 grid((unsigned)cb, (unsigned)((d->M + a.mchunk - 1) / a.mchunk));
  SLX_CHECK_ARG(!ws || !d->dA[0] || ws_floats >= slx_lora_bwd_ws_floats(d->M, d->Kin, d->nsites),
                "slx_lora_bwd_ws: workspace holds %lld floats, slx_lora_bwd_ws_floats asks for %lld", (long long)ws_floats,
                (long long)slx_lora_bwd_ws_floats(d->M, d->Kin, d->nsites));
  if (!ws && d->dA[0] && det_mode().on &&  // deterministic mode: the slab path, in the mode's workspace
      det_mode().ws_floats >= slx_lora_bwd_ws_floats(d->M, d->Kin, d->nsites)) {
    ws = det_mode().ws;
    ws_floats = det_mode().ws_floats;
  }
  SLX_CHECK_ARG(!d->dA[0] || ws || !det_mode().on, "slx_lora_bwd: deterministic workspace too small for the dA partials");
  a.dA_part = (ws && d->dA[0]) ? ws : nullptr;
  SLX_CHECK_ARG(!a.dA_part || (long)grid.y <= (long)kDaRedLanes * kDaRedPer,
                "slx_lora_bwd_ws: %u row chunks, at most %d (SLX_LORA_DA_BLOCKS too high for M)", grid.y,
                kDaRedLanes * kDaRedPer);
  hipStream_t st = (hipStream_t)stream;
  switch (d->nsites) {
    case 1: launch_bwd<1>(a, grid, st); break;
    case 2: launch_bwd<2>(a, grid, st); break;
    case 3: launch_bwd<3>(a, grid, st); break;
    default: launch_bwd<4>(a, grid, st); break;
  }
  SLX_LAUNCH_CHECK("slx_lora_bwd");
  return 0;
}

extern "C" int slx_lora_grad(const slx_lora_grad_job* jobs, int njobs, int64_t M, slx_stream_t stream) {
  SLX_CHECK_ARG(jobs && njobs >= 1 && njobs <= kLgMaxJobs, "slx_lora_grad: 1..%d jobs", kLgMaxJobs);
  SLX_CHECK_ARG(M >= 0 && M < (1LL << 31), "slx_lora_grad: M out of range");
  if (M == 0) return 0;
  LgArgs a;
  memset(&a, 0, sizeof(a));
  a.M = (int)M; a.njobs = njobs;
  long ncb_sum = 0;
  for (int i = 0; i < njobs; ++i) {
    const slx_lora_grad_job& d = jobs[i];
    SLX_CHECK_ARG(d.x && d.t && d.nsites >= 1 && d.nsites <= 3 && d.n > 0 && d.n % 128 == 0 && d.ldx % 8 == 0 &&
                  ((uintptr_t)d.x & 15) == 0, "slx_lora_grad: job %d needs x (16-B aligned, ldx %% 8), n %% 128, 1..3 sites", i);
    SLX_CHECK_ARG(d.t_bf16 == 1 && d.ldt % 8 == 0 && ((uintptr_t)d.t & 15) == 0,
                  "slx_lora_grad: job %d: t bf16 (t_bf16 = 1), 16-B aligned, ldt %% 8", i);
    SLX_CHECK_ARG(d.p >= 0.f && d.p < 1.f && (d.p == 0.f || (d.bits[0] && d.ldbits >= d.n / 32)),
                  "slx_lora_grad: job %d: 0 <= p < 1, p > 0 needs keep bits", i);
    LgJob& J = a.j[i];
    J.X = (const bf16*)d.x; J.ldx = d.ldx; J.N = d.n;
    J.T = (const bf16*)d.t; J.ldt = d.ldt;
    J.ns = d.nsites;
    for (int j = 0; j < 3; ++j) {
      SLX_CHECK_ARG(j >= d.nsites || d.out[j], "slx_lora_grad: job %d site %d has no output", i, j);
      SLX_CHECK_ARG(j >= d.nsites || d.p == 0.f || d.bits[j], "slx_lora_grad: job %d site %d has no keep bits", i, j);
      J.out[j] = j < d.nsites ? d.out[j] : nullptr;
      J.bits[j] = (d.p > 0.f && j < d.nsites) ? d.bits[j] : nullptr;
    }
    J.ldbits = d.ldbits;
    J.sc = 1.0f / (1.0f - d.p);
    J.alpha = d.alpha;
    J.nr = d.out_nr;
    J.ncb = d.n / 128;
    ncb_sum += J.ncb;
  }
  // row chunks: about one item per block slot (2 per CU), each chunk a whole number of 64-row sub-chunks
  static const int slots = [] { const char* e = getenv("SLX_LORA_GRAD_ITEMS"); return e ? atoi(e) : 512; }();
  const long nsub = (M + 63) / 64;
  long nkc = (slots + ncb_sum - 1) / ncb_sum;
  nkc = nkc < 1 ? 1 : (nkc > nsub ? nsub : nkc);
  const int kch = (int)(((nsub + nkc - 1) / nkc) * 64);
  nkc = (M + kch - 1) / kch;
  int items = 0;
  for (int i = 0; i < njobs; ++i) {
    a.j[i].kch = kch;
    a.j[i].item0 = items;
    items += a.j[i].ncb * (int)nkc;
  }
  a.nitems = items;
  const DetMode& dm = det_mode();
  if (dm.on) {  // partial slots [nkc][32 N] per (job, site) in the deterministic workspace
    long off = 0;
    for (int i = 0; i < njobs; ++i)
      for (int j = 0; j < a.j[i].ns; ++j) {
        a.j[i].part[j] = dm.ws + off;
        off += nkc * 32L * a.j[i].N;
      }
    SLX_CHECK_ARG(off <= dm.ws_floats, "slx_lora_grad: deterministic workspace holds %ld floats, the partials need %ld",
                  dm.ws_floats, off);
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(lora_grad_kernel, dim3(items), dim3(256), 0, st, a);
  SLX_LAUNCH_CHECK("slx_lora_grad");
  if (dm.on)
    for (int i = 0; i < njobs; ++i)
      for (int j = 0; j < a.j[i].ns; ++j)
        if (det_reduce(a.j[i].part[j], (int)nkc, 32L * a.j[i].N, 32L * a.j[i].N, a.j[i].out[j], 1, st)) return -1000;
  return 0;
}

extern "C" int slx_lora_swiglu_bwd(const slx_lora_swiglu_bwd_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d && d->dt && d->at && d->resid && d->gu && d->dgu, "slx_lora_swiglu_bwd: null operand");
  SLX_CHECK_ARG(d->F > 0 && d->F % 256 == 0 && d->M >= 0, "slx_lora_swiglu_bwd: F %% 256 == 0 (got %d)", d->F);
  SLX_CHECK_ARG(d->lddt % 8 == 0 && d->ldat % 8 == 0 && d->ldat >= 32 && d->ldr % 8 == 0 && d->ldgu % 8 == 0 &&
                d->lddgu % 8 == 0 && ((((uintptr_t)d->dt | (uintptr_t)d->at | (uintptr_t)d->resid | (uintptr_t)d->gu |
                                        (uintptr_t)d->dgu) & 15) == 0),
                "slx_lora_swiglu_bwd: 16-B aligned rows (leading dims %% 8)");
  SLX_CHECK_ARG(d->p >= 0.f && d->p < 1.f && (d->p == 0.f || (d->bits && d->ldbits >= d->F / 32)),
                "slx_lora_swiglu_bwd: 0 <= p < 1, p > 0 needs the keep bits");
  if (d->M == 0) return 0;
  LswArgs a;
  a.dt = (const bf16*)d->dt; a.lddt = d->lddt; a.at = (const bf16*)d->at; a.ldat = d->ldat;
  a.resid = (const bf16*)d->resid; a.ldr = d->ldr; a.gu = (const bf16*)d->gu; a.ldgu = d->ldgu;
  a.bits = d->p > 0.f ? d->bits : nullptr; a.ldbits = d->ldbits;
  a.sc = 1.0f / (1.0f - d->p);
  a.dgu = (bf16*)d->dgu; a.lddgu = d->lddgu;
  a.M = (int)d->M; a.F = d->F;
  const dim3 grid((unsigned)(d->F / 256), (unsigned)((d->M + 31) / 32));
  if (a.bits) hipLaunchKernelGGL(lora_swiglu_bwd_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(lora_swiglu_bwd_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, a);
  SLX_LAUNCH_CHECK("slx_lora_swiglu_bwd");
  return 0;
}

// rows per block of slx_lora_swiglu_bwd_grads: about two blocks per CU over the F / 128 column blocks
static int lswg_kch(int64_t M, int F) {
  const long nch = (M + 63) / 64, ncb = F / 128;
  long groups = (512 + ncb - 1) / ncb;
  groups = groups < 1 ? 1 : (groups > nch ? nch : groups);
  return (int)(((nch + groups - 1) / groups) * 64);
}

extern "C" int64_t slx_lora_swiglu_bwd_grads_ws_floats(int64_t M, int F) {
  if (M <= 0 || F <= 0 || F % 128 != 0) return 0;
  const int kch = lswg_kch(M, F);
  return (int64_t)((M + kch - 1) / kch) * 3 * 32 * F;
}

extern "C" int slx_lora_swiglu_bwd_grads(const slx_lora_swiglu_bwd_grads_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d && d->sw.dt && d->sw.at && d->sw.resid && d->sw.gu && d->sw.dgu && d->tg && d->tu && d->dA_down &&
                d->dB_gate && d->dB_up && d->ws, "slx_lora_swiglu_bwd_grads: null operand");
  const slx_lora_swiglu_bwd_desc& s = d->sw;
  SLX_CHECK_ARG(s.F > 0 && s.F % 128 == 0 && s.M >= 0 && s.M < (1LL << 31), "slx_lora_swiglu_bwd_grads: F %% 128 (got %d)",
                s.F);
  SLX_CHECK_ARG(s.lddt % 8 == 0 && s.ldat % 8 == 0 && s.ldat >= 32 && s.ldr % 8 == 0 && s.ldgu % 8 == 0 &&
                s.lddgu % 8 == 0 && d->ldtg % 8 == 0 &&
                ((((uintptr_t)s.dt | (uintptr_t)s.at | (uintptr_t)s.resid | (uintptr_t)s.gu | (uintptr_t)s.dgu |
                   (uintptr_t)d->tg | (uintptr_t)d->tu) & 15) == 0),
                "slx_lora_swiglu_bwd_grads: 16-B aligned rows (leading dims %% 8)");
  SLX_CHECK_ARG(s.p >= 0.f && s.p < 1.f && (s.p == 0.f || (s.bits && s.ldbits >= s.F / 32)),
                "slx_lora_swiglu_bwd_grads: 0 <= p < 1, p > 0 needs the keep bits");
  SLX_CHECK_ARG(d->ws_floats >= slx_lora_swiglu_bwd_grads_ws_floats(s.M, s.F),
                "slx_lora_swiglu_bwd_grads: workspace holds %lld floats, needs %lld", (long long)d->ws_floats,
                (long long)slx_lora_swiglu_bwd_grads_ws_floats(s.M, s.F));
  if (s.M == 0) return 0;
  LswgArgs g;
  LswArgs& a = g.s;
  a.dt = (const bf16*)s.dt; a.lddt = s.lddt; a.at = (const bf16*)s.at; a.ldat = s.ldat;
  a.resid = (const bf16*)s.resid; a.ldr = s.ldr; a.gu = (const bf16*)s.gu; a.ldgu = s.ldgu;
  a.bits = s.p > 0.f ? s.bits : nullptr; a.ldbits = s.ldbits;
  a.sc = 1.0f / (1.0f - s.p);
  a.dgu = (bf16*)s.dgu; a.lddgu = s.lddgu;
  a.M = (int)s.M; a.F = s.F;
  g.tg = (const bf16*)d->tg; g.tu = (const bf16*)d->tu; g.ldtg = d->ldtg;
  g.kch = lswg_kch(s.M, s.F);
  g.part = d->ws;
  const int groups = (int)((s.M + g.kch - 1) / g.kch);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(s.F / 128), (unsigned)groups);
  if (a.bits) hipLaunchKernelGGL(lora_swiglu_bwd_grads_kernel<true>, grid, dim3(256), 0, st, g);
  else hipLaunchKernelGGL(lora_swiglu_bwd_grads_kernel<false>, grid, dim3(256), 0, st, g);
  const long n = 32L * s.F;
  hipLaunchKernelGGL(lsw_grads_reduce_kernel, dim3((unsigned)((3 * n + 255) / 256)), dim3(256), 0, st,
                     (const float*)d->ws, groups, n, d->dA_down, d->dB_gate, d->dB_up, 1.0f, d->alpha_b);
  SLX_LAUNCH_CHECK("slx_lora_swiglu_bwd_grads");
  return 0;
}

extern "C" int64_t slx_swiglu_lora_down_ws_floats(int64_t M, int F) {
  return (M <= 0 || F <= 0 || F % 256 != 0) ? 0 : (int64_t)(F / 256) * M * 32;
}

extern "C" int slx_swiglu_lora_down(const slx_swiglu_lora_down_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d && d->gu && d->act && d->A && d->t && d->ws, "slx_swiglu_lora_down: null operand");
  SLX_CHECK_ARG(d->F > 0 && d->F % 256 == 0 && d->M >= 0 && d->M < (1LL << 31), "slx_swiglu_lora_down: F %% 256 (got %d)",
                d->F);
  SLX_CHECK_ARG(d->ldgu % 8 == 0 && d->ldact % 8 == 0 && d->lda % 8 == 0 && d->lda >= d->F &&
                ((((uintptr_t)d->gu | (uintptr_t)d->act | (uintptr_t)d->A) & 15) == 0),
                "slx_swiglu_lora_down: 16-B aligned rows (leading dims %% 8)");
  SLX_CHECK_ARG(d->p >= 0.f && d->p < 1.f && (d->p == 0.f || (d->bits && d->ldbits >= d->F / 32)),
                "slx_swiglu_lora_down: 0 <= p < 1, p > 0 needs the keep bits");
  SLX_CHECK_ARG(d->ws_floats >= slx_swiglu_lora_down_ws_floats(d->M, d->F),
                "slx_swiglu_lora_down: workspace holds %lld floats, needs %lld", (long long)d->ws_floats,
                (long long)slx_swiglu_lora_down_ws_floats(d->M, d->F));
  if (d->M == 0) return 0;
  SldArgs a;
  a.gu = (const bf16*)d->gu; a.ldgu = d->ldgu; a.act = (bf16*)d->act; a.ldact = d->ldact;
  a.A = (const bf16*)d->A; a.lda = d->lda;
  a.bits = d->p > 0.f ? d->bits : nullptr; a.ldbits = d->ldbits;
  a.sc = 1.0f / (1.0f - d->p);
  a.t = (bf16*)d->t; a.ldt = d->ldt;
  a.part = d->ws;
  a.M = (int)d->M; a.F = d->F;
  a.gen = d->gen_bits && d->p > 0.f;
  a.s1 = drop_seed_mix(d->seed);
  a.thr = (uint32_t)(d->p * 65536.0f + 0.5f);  // slx_dropout_bits' threshold
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(d->F / 256), (unsigned)((d->M + 31) / 32));
  if (a.bits) hipLaunchKernelGGL(swiglu_lora_down_kernel<true>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(swiglu_lora_down_kernel<false>, grid, dim3(256), 0, st, a);
  hipLaunchKernelGGL(swiglu_lora_down_reduce_kernel, dim3((unsigned)((d->M * 32 + 255) / 256)), dim3(256), 0, st,
                     (const float*)d->ws, d->F / 256, (long)d->M, (bf16*)d->t, (long)d->ldt);
  SLX_LAUNCH_CHECK("slx_swiglu_lora_down");
  return 0;
}
