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
// Backward: two launches, no atomics. First a dQ pass shaped like the forward (128 queries per workgroup, K/V tiles
// through LDS, dS^T in registers, dQ^T += K^T dS^T) that also computes delta = rowsum(dO*O) per query in its prologue
// and stores it; then a dK/dV pass (one workgroup = 4 waves = 128 keys of one (b, kv-head), sweeping the GQA group's
// q-heads x 64-query chunks, S and dP recomputed with the key on the lane so their accumulators feed dV^T/dK^T
// directly). Summing dQ over key blocks with f32 atomics instead (one kernel) was bound by the ~1.3 TB/s atomic rate.
#include <cstdlib>

#include "common.h"
#include "../../include/slx.h"

// Tuning knobs (A/B builds through tools/attn_ab.py pass -D overrides): blocks per CU of each kernel.
#ifndef ATTN_FWD_OCC
#define ATTN_FWD_OCC 2
#endif
#ifndef ATTN_DQ_OCC
#define ATTN_DQ_OCC 2
#endif
#ifndef ATTN_KV_SB
#define ATTN_KV_SB 0
#endif

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
  float* dq_acc;               // [B*S, Hq*64] f32, written by the dQ pass (finalized to bf16 + RoPE^T)
  float* dk_acc; float* dv_acc;  // [nsplit][B*S, Hkv*64] f32 when GQA/RoPE (finalized), else null: direct bf16
  bf16* dk; bf16* dv; long lddk, lddv;
  float* dbq; float* dbk; float* dbv;  // optional bias-gradient column sums of dq / dk / dv (f32, accumulated)
  int hsplit, nsplit;            // dK/dV pass: q-heads of a GQA group per workgroup, workgroups per group
  bf16* dq; long lddq;           // dQ pass output: bf16, RoPE^T applied with rcos/rsin (pos = query index) if given
  const float* rcos; const float* rsin;
  int tail_first;                // non-causal: each XCD's partial last row blocks dispatched first (SLX_ATTN_TAIL_FIRST)
  int tailv;                     // non-causal DMA forms: a short last key / query tile (<= kTailMax rows) on the VALU
  // non-causal: the rows past the last whole 128-row block (S % 128 <= kTailQ, InternViT's 1025th token) folded into
  // that block's workgroup instead of a workgroup of their own (the forward / dQ passes: queries; dK/dV: keys)
  int qtail, nqb;                // query blocks launched (S / 128 with a folded tail, else ceil(S / 128))
  int ktail, nkb;                // key blocks launched (dK/dV pass)
};

constexpr float LOG2E = 1.4426950408889634f;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
constexpr float LAZY = 8.0f;  // forward lazy-rescale threshold (log2 units)
constexpr float MASKED = -INFINITY;

// XCD-aware block order: the hardware deals consecutive block ids round-robin over the 8 XCDs (each
// with its own L2). Map the physical id to a logical one so every XCD gets a contiguous logical range,
// and order logical ids (b, kv-head, q-head in group, 128-row block) fastest-last: all blocks that read
// one (b, kv-head)'s K/V (or Q/dO in backward) then share one L2 instead of fetching it eight times.
// Causal launches (Qwen2) instead deal the blocks heaviest-first in dispatch order, with the row block as the slowest
// logical dimension (order 1: highest query block first, for the forward / dQ passes; order 2: lowest key block first,
// for the dK/dV pass): a query block's work grows with its index, and the last blocks dispatched should be the light
// ones, not a mix that leaves a few heavy blocks running alone at the tail. Every XCD gets the same mix (round-robin
// dealing); the whole K/V of a 798-token batch (3.3 MB) fits one XCD's L2 anyway.
struct BlockCoord { int blk, h, b; };
__device__ __forceinline__ BlockCoord attn_block(int nblk, int Hq, int Hkv, int B, int order = 0, int tail_first = 0) {
  const int nwg = nblk * Hq * B;
  int bid = blockIdx.x;
  const int G = Hq / Hkv;
  BlockCoord c;
  if (order != 0) {
    const int per = Hq * B;
    const int r = bid / per;
    c.blk = order == 1 ? nblk - 1 - r : r;
    int t = bid - r * per;
    const int hg = t % G;
    t /= G;
    const int hk = t % Hkv;
    c.b = t / Hkv;
    c.h = hk * G + hg;
    return c;
  }
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  if (tail_first && r == 0 && q % nblk == 0 && nblk > 1) {
    // within the XCD's range (whole (b, h) groups): its groups' last, partial row blocks first, then the rest
    const int base = (bid / q) * q, j = bid - base, npair = q / nblk;
    const int pair = j < npair ? j : (j - npair) / (nblk - 1);
    const int blk = j < npair ? nblk - 1 : (j - npair) % (nblk - 1);
    bid = base + pair * nblk + blk;
  }
  c.blk = bid % nblk;
  int t = bid / nblk;
  const int hg = t % G;
  t /= G;
  const int hk = t % Hkv;
  c.b = t / Hkv;
  c.h = hk * G + hg;
  return c;
}

// max over the two 32-lane halves (lane l and l^32) without an LDS round trip
__device__ __forceinline__ float half_swap_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// One 64-key tile of the forward for one wave (32 queries, query on the lane): S^T = K Q^T, online
// softmax in the log2 domain with the scale folded into one FMA per score (max taken on raw scores,
// c > 0), P^T from the accumulator straight into O^T += V^T P^T. MASK only for boundary tiles.
// Measured on the InternViT shape (tools/attn_ab.py): the structure itself - MFMAs fed from LDS, one barrier per
// 64-key tile - runs at ~860 TF with the softmax removed; the softmax costs ~30 %, of which the lean form below
// (row sum on the MFMA, lazy rescale) recovers ~2 %.
template <bool MASK>
__device__ __forceinline__ void fwd_tile(const char* Kl, const char* Vl, const bf16x8 (&qf)[4], f32x16& o0, f32x16& o1,
                                         f32x16& lacc, float& m, float c, int key0, int kvlen, int myq, bool causal,
                                         int lane) {
  const int hl = lane >> 5;
  f32x16 s[2];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) s[kb] = mfma32(row_frag(Kl, kb * 32, kk, lane), qf[kk], s[kb]);
  }
  if constexpr (MASK) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const bool ok = (key < kvlen) & (!causal | (key <= myq));
        s[kb][r] = ok ? s[kb][r] : MASKED;
      }
  }
  // VALU-lean softmax: the row sum comes out of the PV MFMAs (ones x P^T into lacc, so l sums exactly the bf16 P
  // that O accumulates), and O/l are rescaled only when some lane's max grows by more than LAZY (log2 units):
  // p = exp2(s c - m) <= 2^LAZY otherwise.
  float mx = s[0][0];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
  mx = half_swap_max(mx) * c;
  if (__builtin_amdgcn_ballot_w64(mx > m + LAZY)) {
    const float mnew = fmaxf(m, mx);
    const float alpha = __builtin_amdgcn_exp2f(m - mnew);
    m = mnew;
#pragma unroll
    for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; lacc[r] *= alpha; }
  }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kb][r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kb][r], c, -m));
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf16x8 pb = acc_frag(s[kb], st);
      o0 = mfma32(tr_frag(Vl, kb * 32 + 16 * st, 0, lane), pb, o0);
      o1 = mfma32(tr_frag(Vl, kb * 32 + 16 * st, 32, lane), pb, o1);
      lacc = mfma32(ones, pb, lacc);
    }
}

// ---- backward, dK/dV pass: one workgroup = 4 waves = 128 keys of one (b, kv-head); sweeps every q-head of
// the group x 64-query chunks (Q, dO, lse, delta staged through LDS). S and dP are computed with the key on
// the lane, so their accumulators are the B operands of dV^T += dO^T P and dK^T += Q^T dS. dK/dV of the
// whole GQA group accumulate in registers: no atomics, no cross-workgroup partials.
template <bool MASK>
__device__ __forceinline__ void bwd_kv_chunk(const char* Ql, const char* Dl, const float* lse_l, const float* del_l,
                                             const bf16x8 (&kf)[4], const bf16x8 (&vf)[4], f32x16& dk0, f32x16& dk1,
                                             f32x16& dv0, f32x16& dv1, float c, int qc, int S, int mykey, int kvlen,
                                             bool causal, int lane) {
  const int hl = lane >> 5;
#pragma unroll
  for (int qa = 0; qa < 2; ++qa) {
    f32x16 sp, dp;
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // dP^T starts from -delta of each register's query (row constants in LDS, negated)
      const f32x4 D4 = *reinterpret_cast<const f32x4*>(del_l + qa * 32 + 8 * g + 4 * hl);
#pragma unroll
      for (int e = 0; e < 4; ++e) { sp[4 * g + e] = 0.f; dp[4 * g + e] = D4[e]; }
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      sp = mfma32(row_frag(Ql, qa * 32, kk, lane), kf[kk], sp);
      dp = mfma32(row_frag(Dl, qa * 32, kk, lane), vf[kk], dp);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ql = qa * 32 + 8 * g + 4 * hl;  // local query of register 4g
      const f32x4 L4 = *reinterpret_cast<const f32x4*>(lse_l + ql);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * g + e;
        float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sp[r], c, -L4[e]));
        if constexpr (MASK) {
          const int q = qc + ql + e;
          const bool ok = (q < S) & (mykey < kvlen) & (!causal | (mykey <= q));
          p = ok ? p : 0.f;
        }
        sp[r] = p;
        dp[r] = p * dp[r];
      }
    }
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf16x8 pb = acc_frag(sp, st);
      const bf16x8 sb = acc_frag(dp, st);
      dv0 = mfma32(tr_frag(Dl, qa * 32 + 16 * st, 0, lane), pb, dv0);
      dv1 = mfma32(tr_frag(Dl, qa * 32 + 16 * st, 32, lane), pb, dv1);
      dk0 = mfma32(tr_frag(Ql, qa * 32 + 16 * st, 0, lane), sb, dk0);
      dk1 = mfma32(tr_frag(Ql, qa * 32 + 16 * st, 32, lane), sb, dk1);
    }
#if ATTN_KV_SB
    __builtin_amdgcn_sched_barrier(0);  // A/B: keep the two 32-query halves' live ranges apart
#endif
  }
}

// dst[0..63] += column sums over the block's 128 rows (4 waves x 32 lanes) of a [row x 64] gradient tile, for the
// q/k/v bias gradients (InternViT qkv.b): lane (row l & 31, half hl) holds dims 8g + 4hl + e in v0[4g + e] and
// 32 + 8g + 4hl + e in v1[4g + e] (rows that do not exist pass zeros). Each wave transposes its 32 rows through a
// wave-private [32][64] f32 LDS tile (float4 groups XOR-swizzled by row & 15), lane = dim sums its column, and the 4
// wave partials meet in `red`: one f32 atomic per dim and block. All 256 threads must call it; `lds` >= 32 KiB.
__device__ __forceinline__ void block_colsum64(char* lds, float* red, const float (&v0)[16], const float (&v1)[16],
                                               float* dst, int lane, int w) {
  __syncthreads();  // the tile area is free (main loop done, or the previous call's reads finished)
  float* t = reinterpret_cast<float*>(lds) + w * 2048;
  const int q = lane & 31, hl = lane >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int c4 = 2 * g + hl;
    *reinterpret_cast<float4*>(t + q * 64 + ((c4 ^ (q & 15)) << 2)) =
        make_float4(v0[4 * g], v0[4 * g + 1], v0[4 * g + 2], v0[4 * g + 3]);
    *reinterpret_cast<float4*>(t + q * 64 + (((8 + c4) ^ (q & 15)) << 2)) =
        make_float4(v1[4 * g], v1[4 * g + 1], v1[4 * g + 2], v1[4 * g + 3]);
  }
  __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private tile written (LDS is in order per wave)
  float sum = 0.f;
  const int c4 = lane >> 2, e = lane & 3;
#pragma unroll
  for (int r = 0; r < 32; ++r) sum += t[r * 64 + ((c4 ^ (r & 15)) << 2) + e];
  red[w * 64 + lane] = sum;
  __syncthreads();
  if (w == 0) atomicAdd(dst + lane, red[lane] + red[64 + lane] + red[128 + lane] + red[192 + lane]);
}

// ---- backward, dQ pass (the forward's structure): one workgroup = 4 waves = 128 queries of one (b, h);
// K/V tiles of 64 keys double-buffered through LDS; per tile S^T = K Q^T and dP^T = V dO^T with the query on
// the lane, dS^T = P^T (dP^T - delta) in registers, dQ^T += K^T dS^T (K read transposed); it stores -delta for the dK/dV
// pass (the initial accumulator of its dP chains, loaded as is by the LDS-DMA form). Plain stores, no
// atomics: recomputing S and dP here costs less than summing dQ over key blocks with f32 atomics
// (~1.3 TB/s chip-wide), which bounded the single-kernel backward.
template <bool MASK>
__device__ __forceinline__ void bwd_dq_tile(const char* Kl, const char* Vl, const bf16x8 (&qf)[4], const bf16x8 (&df)[4],
                                            f32x16& dq0, f32x16& dq1, float c, float lse, const f32x16& negd, int key0,
                                            int kvlen, int myq, bool causal, int lane) {
  const int hl = lane >> 5;
  f32x16 s[2], dp[2];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
    s[kb] = mfma32(row_frag(Kl, kb * 32, 0, lane), qf[0], s[kb]);
    dp[kb] = mfma32(row_frag(Vl, kb * 32, 0, lane), df[0], negd);  // dP^T - delta: the chain starts from -delta
#pragma unroll
    for (int kk = 1; kk < 4; ++kk) {
      s[kb] = mfma32(row_frag(Kl, kb * 32, kk, lane), qf[kk], s[kb]);
      dp[kb] = mfma32(row_frag(Vl, kb * 32, kk, lane), df[kk], dp[kb]);
    }
  }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kb][r], c, -lse));
      if constexpr (MASK) {
        const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const bool ok = (key < kvlen) & (!causal | (key <= myq));
        p = ok ? p : 0.f;
      }
      dp[kb][r] = p * dp[kb][r];
    }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf16x8 sb = acc_frag(dp[kb], st);
      dq0 = mfma32(tr_frag(Kl, kb * 32 + 16 * st, 0, lane), sb, dq0);
      dq1 = mfma32(tr_frag(Kl, kb * 32 + 16 * st, 32, lane), sb, dq1);
    }
}
// The RoPE table entries of a lane's 16 dQ dims (d = 8 g + 4 hl + e, as float4 per g), issued together: read per
// element inside `if (a.rcos)`, each load was drained (vmcnt(0)) before the next, 16 round trips per dQ store
__device__ __forceinline__ void rope_lane_tables(const float* rcos, const float* rsin, long qi, int hl, float4 (&cs)[4],
                                                 float4 (&sn)[4]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    cs[g] = *reinterpret_cast<const float4*>(rcos + qi * 32 + 8 * g + 4 * hl);
    sn[g] = *reinterpret_cast<const float4*>(rsin + qi * 32 + 8 * g + 4 * hl);
  }
}

// ---- the kernels: tiles staged by LDS-DMA (round 4) ----------------------------------------------------------------
// Tiles arrive by LDS-DMA (buffer_load_dwordx4 ... lds, the v3 GEMM's staging): a ring of NSLOT slots, each tile
// issued NSLOT - 1 tiles ahead right after the barrier that frees its slot, a counted vmcnt before that barrier (every
// wave issues the same number of pieces per tile; tiles past the end are all-sentinel pieces that land zeros in a slot
// nobody reads), no staging registers, no ds_write. (The round-1..3 register-staged forms - global loads one tile
// ahead, ds_write_b128 into a 2-slot ring - and the round-4 8-wave ping-pong forms, 1.5x slower on the backward, were
// retired in round 6; the compute bodies fwd_tile, bwd_dq_tile and bwd_kv_chunk are theirs.)
constexpr unsigned kAttnSent = 0x7FFFFFF0u;  // past every descriptor: the DMA lands zeros

__device__ __forceinline__ int sw_xor(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }  // sw_off's swizzle

// descriptor over rows [0, nrows) of a token-major bf16 slice (row stride ld elements, 64 columns)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slice_rsrc(const void* base, long ld, int nrows, int esize) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(((long)(nrows > 0 ? nrows - 1 : 0) * ld + 64) * esize), 0x00020000);
}

// One LDS-DMA piece (buffer_load_dword[x4] ... lds; M0 = the wave-uniform LDS destination) issued by inline asm.
// hipcc's wait-count pass cannot tell which LDS bytes a builtin LDS DMA writes, so it drained vmcnt(0) before the next
// ds_read of any address: right after each loop trip issued the next tile, before the current tile's fragment reads,
// so no DMA ever overlapped the MFMAs (and deeper rings could not help). Issued here, the pieces are ordered only by
// the ring's own protocol (counted wait_vmcnt before the barrier that publishes a slot). Every LDS DMA of this file
// goes through this helper, so hipcc keeps no value of its own in M0 (checked in the .s: M0 is written only here).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
template <int BYTES>
__device__ __forceinline__ void lds_dma(__amdgpu_buffer_rsrc_t rs, const char* lds, unsigned off) {
  static_assert(BYTES == 16 || BYTES == 4, "dwordx4 or dword pieces");
  const unsigned m = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)lds);
  if constexpr (BYTES == 16)
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m), "v"(off), "s"(rs)
                 : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds" ::"s"(m), "v"(off), "s"(rs)
                 : "memory", "m0");
}
#pragma clang diagnostic pop

// vmcnt(0) through the intrinsic hipcc's wait-count pass understands (lgkmcnt / expcnt left at their maxima), placed
// before a ring's first pieces: the loads issued before it (Q / dO fragments, lse) are then known complete at the tile
// loop's header. Without it the pass re-waits for them inside the loop, and those counted waits (vmcnt(3) .. (0))
// also wait for the asm-issued pieces in flight, which the hardware counter includes.
__device__ __forceinline__ void drain_known_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Wave w's two of the eight 1-KiB pieces of a 64-row x 64-column bf16 tile (rows row0 .. row0 + 63 of the slice)
// into the sw_off image at lds: lane l of piece p carries row 8p + (l >> 3) into physical chunk l & 7, i.e. logical
// (source) chunk (l & 7) ^ sw_xor(row) - the swizzle is applied on the source side. lane_off[i] = the lane's byte
// offset within the tile for piece 2w + i (dma_lane_offsets); rows >= nrows land zeros.
__device__ __forceinline__ void dma_lane_offsets(long ld, int w, int lane, int (&lane_off)[2], int (&lane_row)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * w + 8 * i + (lane >> 3);
    lane_row[i] = r;
    lane_off[i] = (int)(r * ld + 8 * ((lane & 7) ^ sw_xor(r))) * 2;
  }
}
__device__ __forceinline__ void dma_tile64(__amdgpu_buffer_rsrc_t rs, char* lds, long ld, int row0, int nrows, int w,
                                           const int (&lane_off)[2], const int (&lane_row)[2]) {
  const int tile_off = (int)(row0 * ld * 2);  // < 2 GiB: slices are one sample's rows
  const int lim = nrows - row0;               // rows of this tile that exist
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const unsigned off = lane_row[i] < lim ? (unsigned)(tile_off + lane_off[i]) : kAttnSent;
    lds_dma<16>(rs, lds + (2 * w + i) * 1024, off);
  }
}

// 64 consecutive f32 (elements i0 .. i0 + 63 of a row vector, valid below n) to lds[0..255] with one 4-B DMA
__device__ __forceinline__ void dma_row64_f32(__amdgpu_buffer_rsrc_t rs, char* lds, int i0, int n, int lane) {
  const int i = i0 + lane;
  const unsigned off = i < n ? (unsigned)(i * 4) : kAttnSent;
  lds_dma<4>(rs, lds, off);
}

// ---- short tails on the VALU (non-causal; InternViT: T = 1025 = 16 * 64 + 1) ----------------------------------
// A 64-row tile holding one valid key (forward / dQ) or query (dK/dV) costs the MFMAs and the masked softmax of a
// whole tile: 1/17 of each pass. Up to kTailMax such rows are instead folded in after the tile loop, one row at a time
// on the VALU: the same bf16 operands, f32 products, and P / dS rounded to bf16 exactly where the MFMA forms round
// them (only the f32 summation order differs). Operand rows come straight from global memory (every lane of a half
// reads the same 16-B pieces: broadcast loads).
constexpr int kTailMax = 4;

// Tail rows are copied to LDS when the workgroup starts (their global latency then hides under the tile loop, whose
// first barrier publishes them): rows[2 * j] = a[j], rows[2 * j + 1] = b[j] for j < n (64 bf16 each)
__device__ __forceinline__ void tail_stage(bf16* rows, const bf16* a0, long lda, const bf16* b0, long ldb, int n) {
  const int t = threadIdx.x;
  if (t < 16 * n) {
    const int j = t >> 4, which = (t >> 3) & 1, piece = t & 7;
    const bf16* src = which ? b0 + (long)j * ldb : a0 + (long)j * lda;
    *reinterpret_cast<uint4*>(rows + (2 * j + which) * 64 + 8 * piece) = *reinterpret_cast<const uint4*>(src + 8 * piece);
  }
}

// sum over the 64 dims of row . (the lane's fragments): lane (i, half hl) holds dims 16kk + 8hl + j of its own row
__device__ __forceinline__ float tail_dot(const bf16* row, const bf16x8 (&f)[4], int hl) {
  float sum = 0.f;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(row + 16 * kk + 8 * hl);
#pragma unroll
    for (int j = 0; j < 8; ++j) sum = __builtin_fmaf((float)f[kk][j], (float)x[j], sum);
  }
  return sum + __shfl_xor(sum, 32, 64);
}

// acc0[r] += w * row[dim(r)], acc1[r] += w * row[32 + dim(r)] for the accumulator layout dim(r) = 8(r >> 2) + 4hl + (r & 3)
__device__ __forceinline__ void tail_axpy(const bf16* row, float w, f32x16& acc0, f32x16& acc1, int hl) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const bf16x4 lo = *reinterpret_cast<const bf16x4*>(row + 8 * g + 4 * hl);
    const bf16x4 hi = *reinterpret_cast<const bf16x4*>(row + 32 + 8 * g + 4 * hl);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc0[4 * g + e] = __builtin_fmaf(w, (float)lo[e], acc0[4 * g + e]);
      acc1[4 * g + e] = __builtin_fmaf(w, (float)hi[e], acc1[4 * g + e]);
    }
  }
}

// ---- the row tail folded into the last whole block (round 6) ------------------------------------------------------
// InternViT's T = 1025 = 8 * 128 + 1: with ceil(T / 128) blocks, 256 of the 2304 workgroups of each pass carry ONE
// query (forward / dQ) or ONE key (dK/dV) through the whole sweep, half a round of slots on the 512-slot chip
// (isolated: forward 121.7 us at T = 1025 against 90.1 at T = 1024, backward 325.7 against 274.0; profiles/
// round6_attn_tail.txt). Here the last whole block's workgroup takes those rows (<= kTailQ) along: per 64-row tile
// the 4 waves split the tile's 64 rows 16 each, a lane = (row 16w + l / 4, dim quarter l & 3) forms its quarter of
// the tail row's dot products (two 16-B LDS reads against the tail row staged in LDS, a quad sum), and the weighted
// column sums over the wave's 16 rows run with lane = dim (16 readlanes + 16 LDS reads). The forward keeps one
// online-softmax state (m, l, o) per wave, merged across the 4 waves at the end; the dQ / dK-dV sums are plain sums
// over the waves. Same bf16 operands, f32 products, p / dS rounded to bf16 where the MFMA forms round them.
constexpr int kTailQ = 2;

__device__ __forceinline__ float wave_sum64(float x) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);
  return x;
}
__device__ __forceinline__ float rdlane(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
// x + x of the lane (l ^ 1), then (l ^ 2): DPP quad permutations, no LDS round trip (a __shfl_xor is a ds_bpermute)
__device__ __forceinline__ float quad_sum(float x) {
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true));  // quad_perm [1, 0, 3, 2]
  return x + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, true));  // [2, 3, 0, 1]
}
// dims [16 qd, 16 qd + 16) of row `row` of an sw_off tile . the same dims of a 64-dim bf16 row in LDS, summed over the
// lane's quad (lanes 4i .. 4i + 3 hold the four quarters of row i): every lane of the quad gets the full dot product
__device__ __forceinline__ float quarter_dot(const char* tile, int row, int qd, const bf16* v) {
  const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(tile + sw_off(row, 2 * qd));
  const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(tile + sw_off(row, 2 * qd + 1));
  const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(v + 16 * qd);
  const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(v + 16 * qd + 8);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s = __builtin_fmaf((float)a0[j], (float)b0[j], s);
#pragma unroll
  for (int j = 0; j < 8; ++j) s = __builtin_fmaf((float)a1[j], (float)b1[j], s);
  return quad_sum(s);
}
// acc + sum over kk < 16 of wv(lane 4 kk) * tile[r0 + kk][lane]  (lane = dim)
__device__ __forceinline__ float col_axpy16(const char* tile, int r0, float wv, int lane, float acc) {
#pragma unroll
  for (int kk = 0; kk < 16; ++kk)
    acc = __builtin_fmaf(rdlane(wv, 4 * kk), (float)*reinterpret_cast<const bf16*>(tile + sw_elem(r0 + kk, lane)), acc);
  return acc;
}

// forward: the tail query rows (tq: q_j at rows 2j of a pair-staged buffer) against one K/V tile, this wave's 16 keys.
// The wave's running max tm moves only when a score exceeds it by LAZY (ballot; a wave reduction then), as in fwd_tile,
// so the common tile needs no cross-lane reduction: each key's lanes hold p, lane-private partial sums tl (one lane per
// key counts) are reduced once at the end, and O accumulates with lane = dim.
__device__ __forceinline__ void fwd_qtail_tile(const char* Kl, const char* Vl, const bf16* tq, int nq, int key0, int klim,
                                               float c, int w, int lane, float (&tm)[kTailQ], float (&tl)[kTailQ],
                                               float (&to)[kTailQ]) {
  const int kr = 16 * w + (lane >> 2), qd = lane & 3;
  const bool kok = key0 + kr < klim;
#pragma unroll
  for (int j = 0; j < kTailQ; ++j) {
    if (j < nq) {
      const float s = kok ? quarter_dot(Kl, kr, qd, tq + 2 * j * 64) * c : -INFINITY;
      if (__builtin_amdgcn_ballot_w64(s > tm[j] + LAZY)) {
        float mx = s;
#pragma unroll
        for (int o = 4; o < 64; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        const float mnew = fmaxf(tm[j], mx);
        const float alpha = __builtin_amdgcn_exp2f(tm[j] - mnew);
        tl[j] *= alpha;
        to[j] *= alpha;
        tm[j] = mnew;
      }
      const float p = kok ? (float)(bf16)__builtin_amdgcn_exp2f(s - tm[j]) : 0.f;
      tl[j] += qd == 0 ? p : 0.f;
      to[j] = col_axpy16(Vl, 16 * w, p, lane, to[j]);
    }
  }
}

// dQ pass: the tail queries (tq pairs: q_j, dO_j; ts[2j] = lse_j, ts[2j + 1] = delta_j) against one K/V tile
__device__ __forceinline__ void dq_qtail_tile(const char* Kl, const char* Vl, const bf16* tq, const float* ts, int nq,
                                              int key0, int klim, float c, int w, int lane, float (&tdq)[kTailQ]) {
  const int kr = 16 * w + (lane >> 2), qd = lane & 3;
  const bool kok = key0 + kr < klim;
#pragma unroll
  for (int j = 0; j < kTailQ; ++j) {
    if (j < nq) {
      const float sv = quarter_dot(Kl, kr, qd, tq + 2 * j * 64);
      const float dpv = quarter_dot(Vl, kr, qd, tq + (2 * j + 1) * 64);
      const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -ts[2 * j]));
      const float ds = kok ? (float)(bf16)(pv * (dpv - ts[2 * j + 1])) : 0.f;
      tdq[j] = col_axpy16(Kl, 16 * w, ds, lane, tdq[j]);
    }
  }
}

// dK/dV pass: the tail keys (tk pairs: k_j, v_j) against one (q-head, 64-query chunk) stage, this wave's 16 queries
__device__ __forceinline__ void kv_ktail_stage(const char* Ql, const char* Dl, const float* lse_l, const float* nd_l,
                                               const bf16* tk, int nk, int qc, int S, float c, int w, int lane,
                                               float (&tdk)[kTailQ], float (&tdv)[kTailQ]) {
  const int qr = 16 * w + (lane >> 2), qd = lane & 3;
  const bool qok = qc + qr < S;
#pragma unroll
  for (int j = 0; j < kTailQ; ++j) {
    if (j < nk) {
      const float sv = quarter_dot(Ql, qr, qd, tk + 2 * j * 64);
      const float dpv = quarter_dot(Dl, qr, qd, tk + (2 * j + 1) * 64);
      const float pv = qok ? __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -lse_l[qr])) : 0.f;
      const float pb = (float)(bf16)pv, sb = (float)(bf16)(pv * (dpv + nd_l[qr]));  // nd_l: -delta
      tdv[j] = col_axpy16(Dl, 16 * w, pb, lane, tdv[j]);
      tdk[j] = col_axpy16(Ql, 16 * w, sb, lane, tdk[j]);
    }
  }
}

#ifndef ATTN_NSLOT
#ifndef ATTN_NSLOT
#define ATTN_NSLOT 2  // one tile ahead: fastest of 2 / 3 / 4 slots on both shapes (profiles/round4_attn_dma_ab.txt)
#endif
#endif

// forward: one workgroup = 4 waves = 128 queries of one (b, h); the K/V tiles of the (b, kv-head) streamed through an
// NSLOT ring (16 KiB per slot), fwd_tile per 64-key tile
__global__ __launch_bounds__(256, ATTN_FWD_OCC) void attn_fwd_dma_kernel(AttnArgs a) {
  constexpr int NS = ATTN_NSLOT;
  __shared__ __attribute__((aligned(1024))) char smem[NS * 16384];
  const BlockCoord bc = attn_block(a.nqb, a.Hq, a.Hkv, a.B, a.causal ? 1 : 0, a.tail_first);
  const int qb = bc.blk, h = bc.h, b = bc.b;
  const int hk = h / (a.Hq / a.Hkv);
  const int S = a.S;
  const int kvlen = a.seqlens ? min(a.seqlens[b], S) : S;
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);  // the DMA pieces' wave index (M0 must be uniform)
  const int q0 = qb * 128 + w * 32;
  const int myq = q0 + (lane & 31);
  const bool active = q0 < S;
  const float c = a.scale * LOG2E;
  const bf16* kbase = a.k + (long)b * S * a.ldk + hk * 64;
  const bf16* vbase = a.v + (long)b * S * a.ldv + hk * 64;
  const __amdgpu_buffer_rsrc_t rk = slice_rsrc(kbase, a.ldk, S, 2), rv = slice_rsrc(vbase, a.ldv, S, 2);
  // the folded query tail (workgroup-uniform): rows a.nqb * 128 .. + nq - 1 ride with the last whole block
  const int nq = (a.qtail && qb == a.nqb - 1) ? a.qtail : 0;
  __shared__ __attribute__((aligned(16))) bf16 tqrows[2 * kTailQ * 64];
  {
    const bf16* tqa = a.q + ((long)b * S + a.nqb * 128) * a.ldq + h * 64;
    tail_stage(tqrows, tqa, a.ldq, tqa, a.ldq, nq);
  }
  float tm[kTailQ], tl[kTailQ], to[kTailQ];
#pragma unroll
  for (int j = 0; j < kTailQ; ++j) { tm[j] = -1e30f; tl[j] = 0.f; to[j] = 0.f; }

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
  const int ntail = (!a.causal && a.tailv && (kend & 63) <= kTailMax) ? (kend & 63) : 0;  // keys on the VALU
  const int nt = (kend - ntail + 63) / 64;
  __shared__ __attribute__((aligned(16))) bf16 trows[2 * kTailMax * 64];
  tail_stage(trows, kbase + (long)(kend - ntail) * a.ldk, a.ldk, vbase + (long)(kend - ntail) * a.ldv, a.ldv, ntail);
  if (nt == 0) __syncthreads();
  int ko[2], kr_[2], vo[2], vr_[2];
  dma_lane_offsets(a.ldk, wu, lane, ko, kr_);
  dma_lane_offsets(a.ldv, wu, lane, vo, vr_);
  auto issue = [&](int t) {  // 4 pieces per wave per tile; t >= nt: sentinel pieces only
    char* slot = smem + (t % NS) * 16384;
    const int r0 = t < nt ? t * 64 : S;
    dma_tile64(rk, slot, a.ldk, r0, S, wu, ko, kr_);
    dma_tile64(rv, slot + 8192, a.ldv, r0, S, wu, vo, vr_);
  };


  f32x16 o0, o1, lacc;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; lacc[r] = 0.f; }
  float m = -1e30f;
  drain_known_vm();
#pragma unroll
  for (int j = 0; j < NS - 1; ++j) issue(j);
  for (int t = 0; t < nt; ++t) {
    wait_vmcnt<4 * (NS - 2)>();  // this wave's pieces of tile t landed (tiles t+1 .. t+NS-2 may still fly)
    __syncthreads();             // every wave's pieces landed; every wave is done with tile t-1 (its slot is free)
    issue(t + NS - 1);
    const char* Kl = smem + (t % NS) * 16384;
    const char* Vl = Kl + 8192;
    if (active && !(a.causal && t * 64 > q0 + 31)) {  // causal: tiles wholly above this wave's diagonal skipped
      const int kfull = a.causal ? min(kvlen, q0 + 1) : kvlen;
      if ((t + 1) * 64 <= kfull) fwd_tile<false>(Kl, Vl, qf, o0, o1, lacc, m, c, t * 64, kvlen, myq, false, lane);
      else fwd_tile<true>(Kl, Vl, qf, o0, o1, lacc, m, c, t * 64, kvlen, myq, a.causal, lane);
    }
    if (nq) fwd_qtail_tile(Kl, Vl, tqrows, nq, t * 64, kend - ntail, c, w, lane, tm, tl, to);
  }
  wait_vmcnt<0>();  // the trailing sentinel pieces have landed before the workgroup's LDS is released
  if (active) {
    for (int j = 0; j < ntail; ++j) {  // the short key tail: s, the online max, bf16 p, O += p v, l += p
      const float sc = tail_dot(trows + 2 * j * 64, qf, hl) * c;
      if (__builtin_amdgcn_ballot_w64(sc > m + LAZY)) {
        const float mnew = fmaxf(m, sc);
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);
        m = mnew;
#pragma unroll
        for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; lacc[r] *= alpha; }
      }
      const float pb = (float)(bf16)__builtin_amdgcn_exp2f(sc - m);
      lacc[0] += pb;
      tail_axpy(trows + (2 * j + 1) * 64, pb, o0, o1, hl);
    }
  }
  if (nq) {  // the folded tail queries: the short key tail (wave 0, lane = dim), then the 4 waves' states merged
    __shared__ float tqred[kTailQ][4][66];
#pragma unroll
    for (int j = 0; j < kTailQ; ++j) tl[j] = wave_sum64(tl[j]);  // the lane-private partial sums of fwd_qtail_tile
    if (w == 0) {
#pragma unroll
      for (int j = 0; j < kTailQ; ++j) {
        if (j >= nq) continue;
        const float qv = (float)tqrows[2 * j * 64 + lane];
        for (int jj = 0; jj < ntail; ++jj) {
          const float sc = wave_sum64(qv * (float)trows[2 * jj * 64 + lane]) * c;
          const float mnew = fmaxf(tm[j], sc);
          const float alpha = __builtin_amdgcn_exp2f(tm[j] - mnew);
          const float pb = (float)(bf16)__builtin_amdgcn_exp2f(sc - mnew);
          tl[j] = tl[j] * alpha + pb;
          to[j] = __builtin_fmaf(pb, (float)trows[(2 * jj + 1) * 64 + lane], to[j] * alpha);
          tm[j] = mnew;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kTailQ; ++j) {
      if (j < nq) {
        tqred[j][w][lane] = to[j];
        if (lane == 0) { tqred[j][w][64] = tm[j]; tqred[j][w][65] = tl[j]; }
      }
    }
    __syncthreads();
    if (w == 0) {
      for (int j = 0; j < nq; ++j) {
        float M = tqred[j][0][64];
#pragma unroll
        for (int ww = 1; ww < 4; ++ww) M = fmaxf(M, tqred[j][ww][64]);
        float L = 0.f, O = 0.f;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) {
          const float f = __builtin_amdgcn_exp2f(tqred[j][ww][64] - M);
          L = __builtin_fmaf(tqred[j][ww][65], f, L);
          O = __builtin_fmaf(tqred[j][ww][lane], f, O);
        }
        const long row = a.nqb * 128 + j;
        a.o[((long)b * S + row) * a.ldo + h * 64 + lane] = (bf16)(O / L);
        if (lane == 0 && a.lse) a.lse[((long)b * a.Hq + h) * S + row] = M + __log2f(L);
      }
    }
  }
  if (!active || myq >= S) return;
  const float lt = lacc[0];
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

// dQ pass (the forward's shape): 128 queries of one (b, h) per workgroup, the K/V tiles through the NSLOT ring
__global__ __launch_bounds__(256, ATTN_DQ_OCC) void attn_bwd_dq_dma_kernel(AttnArgs a) {
  constexpr int NS = ATTN_NSLOT;
  __shared__ __attribute__((aligned(1024))) char smem[NS * 16384];
  const BlockCoord bc = attn_block(a.nqb, a.Hq, a.Hkv, a.B, a.causal ? 1 : 0, a.tail_first);
  const int qb = bc.blk, h = bc.h, b = bc.b;
  const int hk = h / (a.Hq / a.Hkv);
  const int S = a.S;
  const int kvlen = a.seqlens ? min(a.seqlens[b], S) : S;
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);  // the DMA pieces' wave index (M0 must be uniform)
  const int q0 = qb * 128 + w * 32;
  const int myq = q0 + (lane & 31);
  const bool active = q0 < S;
  const float c = a.scale * LOG2E;
  const bf16* kbase = a.k + (long)b * S * a.ldk + hk * 64;
  const bf16* vbase = a.v + (long)b * S * a.ldv + hk * 64;
  const __amdgpu_buffer_rsrc_t rk = slice_rsrc(kbase, a.ldk, S, 2), rv = slice_rsrc(vbase, a.ldv, S, 2);
  // the folded query tail (workgroup-uniform): q / dO rows staged in LDS, lse and delta per row in tqst (delta from
  // dO . O by wave 0, stored negated for the dK/dV pass like every other row's)
  const int nq = (a.qtail && qb == a.nqb - 1) ? a.qtail : 0;
  __shared__ __attribute__((aligned(16))) bf16 tqrows[2 * kTailQ * 64];
  __shared__ float tqst[2 * kTailQ];
  {
    const long r0 = (long)b * S + a.nqb * 128;
    tail_stage(tqrows, a.q + r0 * a.ldq + h * 64, a.ldq, a.dout + r0 * a.lddo + h * 64, a.lddo, nq);
    if (w == 0) {
      for (int j = 0; j < nq; ++j) {
        const float dv = (float)a.dout[(r0 + j) * a.lddo + h * 64 + lane], ov = (float)a.o[(r0 + j) * a.ldo + h * 64 + lane];
        const float dl = wave_sum64(dv * ov);
        const long li = ((long)b * a.Hq + h) * S + a.nqb * 128 + j;
        if (lane == 0) {
          tqst[2 * j] = a.lse[li];
          tqst[2 * j + 1] = dl;
          const_cast<float*>(a.delta)[li] = -dl;
        }
      }
    }
  }
  float tdq[kTailQ];
#pragma unroll
  for (int j = 0; j < kTailQ; ++j) tdq[j] = 0.f;

  bf16x8 qf[4], df[4];
  float lse = 0.f, dlt = 0.f;
  {
    const int qr = min(myq, S - 1);
    const bf16* qrow = a.q + ((long)b * S + qr) * a.ldq + h * 64;
    const bf16* drow = a.dout + ((long)b * S + qr) * a.lddo + h * 64;
    const bf16* orow = a.o + ((long)b * S + qr) * a.ldo + h * 64;
    bf16x8 of[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      qf[kk] = *reinterpret_cast<const bf16x8*>(qrow + 16 * kk + 8 * hl);
      df[kk] = *reinterpret_cast<const bf16x8*>(drow + 16 * kk + 8 * hl);
      of[kk] = *reinterpret_cast<const bf16x8*>(orow + 16 * kk + 8 * hl);
    }
    const long li = ((long)b * a.Hq + h) * S + qr;
    lse = a.lse[li];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt = __builtin_fmaf((float)df[kk][j], (float)of[kk][j], dlt);
    dlt += __shfl_xor(dlt, 32, 64);
    if (hl == 0 && active && myq < S) const_cast<float*>(a.delta)[li] = -dlt;
  }
  f32x16 negd;
#pragma unroll
  for (int r = 0; r < 16; ++r) negd[r] = -dlt;
  int kend = kvlen;
  if (a.causal) kend = min(kend, qb * 128 + 128);
  const int ntail = (!a.causal && a.tailv && (kend & 63) <= kTailMax) ? (kend & 63) : 0;  // keys on the VALU
  const int nt = (kend - ntail + 63) / 64;
  __shared__ __attribute__((aligned(16))) bf16 trows[2 * kTailMax * 64];
  tail_stage(trows, kbase + (long)(kend - ntail) * a.ldk, a.ldk, vbase + (long)(kend - ntail) * a.ldv, a.ldv, ntail);
  if (nt == 0) __syncthreads();
  int ko[2], kr_[2], vo[2], vr_[2];
  dma_lane_offsets(a.ldk, wu, lane, ko, kr_);
  dma_lane_offsets(a.ldv, wu, lane, vo, vr_);
  auto issue = [&](int t) {  // 4 pieces per wave per tile; t >= nt: sentinel pieces only
    char* slot = smem + (t % NS) * 16384;
    const int r0 = t < nt ? t * 64 : S;
    dma_tile64(rk, slot, a.ldk, r0, S, wu, ko, kr_);
    dma_tile64(rv, slot + 8192, a.ldv, r0, S, wu, vo, vr_);
  };

  f32x16 dq0, dq1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { dq0[r] = 0.f; dq1[r] = 0.f; }
  drain_known_vm();
#pragma unroll
  for (int j = 0; j < NS - 1; ++j) issue(j);
  for (int t = 0; t < nt; ++t) {
    wait_vmcnt<4 * (NS - 2)>();
    __syncthreads();
    issue(t + NS - 1);
    const char* Kl = smem + (t % NS) * 16384;
    const char* Vl = Kl + 8192;
    if (active && !(a.causal && t * 64 > q0 + 31)) {
      const int kfull = a.causal ? min(kvlen, q0 + 1) : kvlen;
      if ((t + 1) * 64 <= kfull) bwd_dq_tile<false>(Kl, Vl, qf, df, dq0, dq1, c, lse, negd, t * 64, kvlen, myq, false, lane);
      else bwd_dq_tile<true>(Kl, Vl, qf, df, dq0, dq1, c, lse, negd, t * 64, kvlen, myq, a.causal, lane);
    }
    if (nq) dq_qtail_tile(Kl, Vl, tqrows, tqst, nq, t * 64, kend - ntail, c, w, lane, tdq);
  }
  wait_vmcnt<0>();
  if (active) {
    for (int j = 0; j < ntail; ++j) {  // the short key tail: dS = p (dP - delta) in bf16, dQ += dS k
      const bf16* krow = trows + 2 * j * 64;
      const float sv = tail_dot(krow, qf, hl);
      const float dpv = tail_dot(trows + (2 * j + 1) * 64, df, hl);
      const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -lse));
      tail_axpy(krow, (float)(bf16)(pv * (dpv - dlt)), dq0, dq1, hl);
    }
  }
  if (nq) {  // the folded tail queries: the short key tail (wave 0, lane = dim), the 4 waves' sums, the dQ rows
    __shared__ float tqred[kTailQ][4][64];
    if (w == 0) {
#pragma unroll
      for (int j = 0; j < kTailQ; ++j) {
        if (j >= nq) continue;
        const float qv = (float)tqrows[2 * j * 64 + lane], dov = (float)tqrows[(2 * j + 1) * 64 + lane];
        for (int jj = 0; jj < ntail; ++jj) {
          const float kv = (float)trows[2 * jj * 64 + lane];
          const float sv = wave_sum64(qv * kv);
          const float dpv = wave_sum64(dov * (float)trows[(2 * jj + 1) * 64 + lane]);
          const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -tqst[2 * j]));
          tdq[j] = __builtin_fmaf((float)(bf16)(pv * (dpv - tqst[2 * j + 1])), kv, tdq[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kTailQ; ++j)
      if (j < nq) tqred[j][w][lane] = tdq[j];
    __syncthreads();
    if (w == 0) {
      for (int j = 0; j < nq; ++j) {
        const float x = ((tqred[j][0][lane] + tqred[j][1][lane]) + (tqred[j][2][lane] + tqred[j][3][lane])) * a.scale;
        const bf16 xb = (bf16)x;
        a.dq[((long)b * S + a.nqb * 128 + j) * a.lddq + h * 64 + lane] = xb;
        if (a.dbq) atomicAdd(a.dbq + h * 64 + lane, (float)xb);
      }
    }
  }
  __syncthreads();  // the ring is free for the bias column sums' LDS tiles
  const bool qvalid = active && myq < S;
  float c0[16], c1[16];
  const long qi = qvalid ? myq : 0;
  bf16* qrow = a.dq + ((long)b * S + qi) * a.lddq + h * 64;
  float4 rtc[4], rts[4];
  if (a.rcos) rope_lane_tables(a.rcos, a.rsin, qi, hl, rtc, rts);
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hl;
    bf16x4 v0, v1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x0 = dq0[4 * g + e] * a.scale, x1 = dq1[4 * g + e] * a.scale;
      if (a.rcos) {
        const float cs = reinterpret_cast<const float*>(&rtc[g])[e], sn = reinterpret_cast<const float*>(&rts[g])[e];
        const float y0 = x0 * cs + x1 * sn, y1 = x1 * cs - x0 * sn;
        x0 = y0;
        x1 = y1;
      }
      v0[e] = (bf16)x0;
      v1[e] = (bf16)x1;
      c0[4 * g + e] = qvalid ? (float)v0[e] : 0.f;
      c1[4 * g + e] = qvalid ? (float)v1[e] : 0.f;
    }
    if (qvalid) {
      *reinterpret_cast<bf16x4*>(qrow + d) = v0;
      *reinterpret_cast<bf16x4*>(qrow + 32 + d) = v1;
    }
  }
  if (a.dbq) {
    __shared__ float red[256];
    block_colsum64(smem, red, c0, c1, a.dbq + h * 64, lane, w);
  }
}

// dK/dV pass: 128 keys of one (b, kv-head) per workgroup, sweeping the group's q-heads; each (q-head, 64-query chunk) stage - Q tile, dO tile, lse[64], -delta[64] -
// through the NSLOT ring (16.5 KiB per slot). Per wave and stage 5 DMA instructions: Q and dO pieces (2 + 2) and one
// 4-B row piece (wave 0: lse, wave 1: -delta, waves 2-3: a sentinel piece into the slot's scratch row).
constexpr int KV_SLOT = 16384 + 4 * 256;
#ifndef ATTN_KV_OCC
#define ATTN_KV_OCC 2
#endif
__global__ __launch_bounds__(256, ATTN_KV_OCC) void attn_bwd_kv_dma_kernel(AttnArgs a) {
  constexpr int NS = ATTN_NSLOT;
  __shared__ __attribute__((aligned(1024))) char smem[NS * KV_SLOT];
  const BlockCoord bc = attn_block(a.nkb, a.Hkv * a.nsplit, a.Hkv * a.nsplit, a.B, a.causal ? 2 : 0, a.tail_first);
  const int kblk = bc.blk, hk = bc.h / a.nsplit, sp = bc.h % a.nsplit, b = bc.b;
  const int G = a.Hq / a.Hkv;
  const int hg0 = sp * a.hsplit;
  const int ng = min(G, hg0 + a.hsplit) - hg0;
  const int S = a.S;
  const int kvlen = a.seqlens ? min(a.seqlens[b], S) : S;
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);  // the DMA pieces' wave index (M0 must be uniform)
  const int k0 = kblk * 128;
  const int kw0 = k0 + 32 * w;
  const int mykey = kw0 + (lane & 31);
  const float c = a.scale * LOG2E;

  bf16x8 kf[4], vf[4];
  {
    const int kr = min(mykey, S - 1);
    const bf16* kp = a.k + ((long)b * S + kr) * a.ldk + hk * 64;
    const bf16* vp = a.v + ((long)b * S + kr) * a.ldv + hk * 64;
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
  // queries on the VALU (one q-head per workgroup: InternViT)
  const int qtail = (!a.causal && a.tailv && ng == 1 && (S & 63) <= kTailMax) ? (S & 63) : 0;
  const int nch = qstart < S ? (S - qtail - qstart + 63) / 64 : 0;
  __shared__ __attribute__((aligned(16))) bf16 trows[2 * kTailMax * 64];
  {
    const int h = hk * G + hg0;
    tail_stage(trows, a.q + ((long)b * S + S - qtail) * a.ldq + h * 64, a.ldq,
               a.dout + ((long)b * S + S - qtail) * a.lddo + h * 64, a.lddo, qtail);
    if (nch == 0) __syncthreads();
  }
  const int nit = nch * ng;
  // the folded key tail (workgroup-uniform): keys a.nkb * 128 .. + nk - 1 ride with the last whole key block (k / v
  // rows staged in LDS; a key past kvlen contributes nothing)
  const int nk = (a.ktail && kblk == a.nkb - 1 && a.nkb * 128 < kvlen) ? min(a.ktail, kvlen - a.nkb * 128) : 0;
  __shared__ __attribute__((aligned(16))) bf16 tkrows[2 * kTailQ * 64];
  {
    const long r0 = (long)b * S + a.nkb * 128;
    tail_stage(tkrows, a.k + r0 * a.ldk + hk * 64, a.ldk, a.v + r0 * a.ldv + hk * 64, a.ldv, nk);
  }
  float tdk[kTailQ], tdv[kTailQ];
#pragma unroll
  for (int j = 0; j < kTailQ; ++j) { tdk[j] = 0.f; tdv[j] = 0.f; }
  int qo[2], qr_[2], doo[2], dr_[2];
  dma_lane_offsets(a.ldq, wu, lane, qo, qr_);
  dma_lane_offsets(a.lddo, wu, lane, doo, dr_);
  // (q-head, chunk) of the next stage to issue, advanced by one per issue: issue() is called for it = 0, 1, 2, ...
  // in order, so no per-iteration integer division by nch (a ~40-instruction scalar sequence each)
  int ih = 0, ic = 0;
  // the q-head's buffer descriptors (Q, dO, lse | delta rows), rebuilt only when the issued head changes
  int rh = -1;
  __amdgpu_buffer_rsrc_t rsq = slice_rsrc(a.q, a.ldq, S, 2), rsd = rsq, rsl = rsq;
  auto issue = [&](int it) {
    char* slot = smem + (it % NS) * KV_SLOT;
    const bool real = it < nit;
    const int h = hk * G + hg0 + (real ? ih : 0), qc = real ? qstart + ic * 64 : S;
    if (++ic == nch) { ic = 0; ++ih; }
    if (h != rh) {
      rh = h;
      rsq = slice_rsrc(a.q + (long)b * S * a.ldq + h * 64, a.ldq, S, 2);
      rsd = slice_rsrc(a.dout + (long)b * S * a.lddo + h * 64, a.lddo, S, 2);
      const long base = ((long)b * a.Hq + h) * S;
      rsl = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wu == 0 ? a.lse + base : a.delta + base), (short)0,
                                              S * 4, 0x00020000);
    }
    dma_tile64(rsq, slot, a.ldq, qc, S, wu, qo, qr_);
    dma_tile64(rsd, slot + 8192, a.lddo, qc, S, wu, doo, dr_);
    dma_row64_f32(rsl, slot + 16384 + 256 * wu, qc, wu < 2 ? S : 0, lane);
  };


  drain_known_vm();
#pragma unroll
  for (int j = 0; j < NS - 1; ++j) issue(j);
  int cc = 0;  // chunk index of stage `it` (it % nch, advanced incrementally)
  for (int it = 0; it < nit; ++it) {
    wait_vmcnt<5 * (NS - 2)>();
    __syncthreads();
    const int qc = qstart + cc * 64;
    if (++cc == nch) cc = 0;
    const char* slot = smem + (it % NS) * KV_SLOT;
    const char* Ql = slot;
    const char* Dl = slot + 8192;
    const float* lse_l = reinterpret_cast<const float*>(slot + 16384);
    const bool full = (qc + 64 <= S) && (kw0 + 32 <= kvlen) && (!a.causal || kw0 + 31 <= qc);
    if (kw0 >= kvlen || (a.causal && kw0 > qc + 63)) {  // padding keys, or every key of the wave above the chunk
    } else if (full) bwd_kv_chunk<false>(Ql, Dl, lse_l, lse_l + 64, kf, vf, dk0, dk1, dv0, dv1, c, qc, S, mykey, kvlen, false, lane);
    else bwd_kv_chunk<true>(Ql, Dl, lse_l, lse_l + 64, kf, vf, dk0, dk1, dv0, dv1, c, qc, S, mykey, kvlen, a.causal, lane);
    if (nk) kv_ktail_stage(Ql, Dl, lse_l, lse_l + 64, tkrows, nk, qc, S, c, w, lane, tdk, tdv);
    issue(it + NS - 1);  // into slot (it - 1) % NS: every wave finished stage it - 1 before this iteration's barrier
  }
  wait_vmcnt<0>();
  if (qtail && kw0 < kvlen) {  // the short query tail: dV += p dO, dK += dS q (bf16 p, dS)
    const int h = hk * G + hg0;
    for (int j = 0; j < qtail; ++j) {
      const long li = ((long)b * a.Hq + h) * S + S - qtail + j;
      const bf16* qrow = trows + 2 * j * 64;
      const bf16* drow = trows + (2 * j + 1) * 64;
      const float sv = tail_dot(qrow, kf, hl);
      const float dpv = tail_dot(drow, vf, hl);
      float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -a.lse[li]));
      pv = mykey < kvlen ? pv : 0.f;
      tail_axpy(drow, (float)(bf16)pv, dv0, dv1, hl);
      tail_axpy(qrow, (float)(bf16)(pv * (dpv + a.delta[li])), dk0, dk1, hl);  // a.delta holds -delta
    }
  }
  if (nk) {  // the folded tail keys: the short query tail (wave 0, lane = dim), the 4 waves' sums, the dK / dV rows
    __shared__ float tkred[2][kTailQ][4][64];
    if (w == 0) {
      const int h = hk * G + hg0;
#pragma unroll
      for (int j = 0; j < kTailQ; ++j) {
        if (j >= nk) continue;
        const float kv = (float)tkrows[2 * j * 64 + lane], vv = (float)tkrows[(2 * j + 1) * 64 + lane];
        for (int jq = 0; jq < qtail; ++jq) {
          const long li = ((long)b * a.Hq + h) * S + S - qtail + jq;
          const float qv = (float)trows[2 * jq * 64 + lane], dov = (float)trows[(2 * jq + 1) * 64 + lane];
          const float sv = wave_sum64(qv * kv), dpv = wave_sum64(dov * vv);
          const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c, -a.lse[li]));
          tdv[j] = __builtin_fmaf((float)(bf16)pv, dov, tdv[j]);
          tdk[j] = __builtin_fmaf((float)(bf16)(pv * (dpv + a.delta[li])), qv, tdk[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kTailQ; ++j) {
      if (j < nk) { tkred[0][j][w][lane] = tdk[j]; tkred[1][j][w][lane] = tdv[j]; }
    }
    __syncthreads();
    if (w == 0) {
      for (int j = 0; j < nk; ++j) {
        const bf16 kx = (bf16)(((tkred[0][j][0][lane] + tkred[0][j][1][lane]) + (tkred[0][j][2][lane] + tkred[0][j][3][lane]))
                               * a.scale);
        const bf16 vx = (bf16)((tkred[1][j][0][lane] + tkred[1][j][1][lane]) + (tkred[1][j][2][lane] + tkred[1][j][3][lane]));
        const long row = (long)b * S + a.nkb * 128 + j;
        a.dk[row * a.lddk + hk * 64 + lane] = kx;
        a.dv[row * a.lddv + hk * 64 + lane] = vx;
        if (a.dbk) {
          atomicAdd(a.dbk + hk * 64 + lane, (float)kx);
          atomicAdd(a.dbv + hk * 64 + lane, (float)vx);
        }
      }
    }
  }
  __syncthreads();  // ring free for the bias column sums' LDS tiles

  const bool kvalid = mykey < S;
  float ck0[16], ck1[16], cv0[16], cv1[16];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hl;
    if (!kvalid) {
#pragma unroll
      for (int e = 0; e < 4; ++e) ck0[4 * g + e] = ck1[4 * g + e] = cv0[4 * g + e] = cv1[4 * g + e] = 0.f;
    } else if (a.dk_acc) {
      const long off = (long)sp * a.B * S * (a.Hkv * 64) + ((long)b * S + mykey) * (a.Hkv * 64) + hk * 64;
      float* kp = a.dk_acc + off;
      float* vp = a.dv_acc + off;
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
        ck0[4 * g + e] = (float)k0v[e];
        ck1[4 * g + e] = (float)k1v[e];
        cv0[4 * g + e] = (float)v0v[e];
        cv1[4 * g + e] = (float)v1v[e];
      }
      *reinterpret_cast<bf16x4*>(kp + d) = k0v;
      *reinterpret_cast<bf16x4*>(kp + 32 + d) = k1v;
      *reinterpret_cast<bf16x4*>(vp + d) = v0v;
      *reinterpret_cast<bf16x4*>(vp + 32 + d) = v1v;
    }
  }
  if (a.dbk) {
    __shared__ float red[256];
    block_colsum64(smem, red, ck0, ck1, a.dbk + hk * 64, lane, w);
    block_colsum64(smem, red, cv0, cv1, a.dbv + hk * 64, lane, w);
  }
}

__device__ __forceinline__ void rope_pair(float& x0, float& x1, float cs, float sn, bool inverse) {
  const float a = x0, b = x1;
  if (!inverse) { x0 = a * cs - b * sn; x1 = b * cs + a * sn; }
  else { x0 = a * cs + b * sn; x1 = b * cs - a * sn; }
}

struct RopeArgs {
  bf16* x; long ldx; int ntok, S, nheads; const float* cos; const float* sin; int inverse;
  const float* src_f32; long ldsrc;  // optional f32 source (finalize: dq/dk accumulators)
  int nsplit; long split_stride;     // f32 source: sum of nsplit partials split_stride floats apart
};

// One thread per (token, head, i<32 pair-group of 4): 8 pairs per thread -> 256 threads per row. The table entries and
// the f32 partials are read as float4 groups, all issued before use (a table read per element inside `if (r.cos)` was
// drained before the next: 16 round trips); same sums in the same order
__device__ __forceinline__ void set8(float (&v)[8], const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void add8(float (&v)[8], const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
}
__device__ __forceinline__ void rope_rows(const RopeArgs& r) {
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
  float cs[8], sn[8];
  if (r.cos) {
    const float* c = r.cos + (long)pos * 32 + i0;
    const float* q = r.sin + (long)pos * 32 + i0;
    const float4 c0 = *reinterpret_cast<const float4*>(c), c1 = *reinterpret_cast<const float4*>(c + 4);
    const float4 s0 = *reinterpret_cast<const float4*>(q), s1 = *reinterpret_cast<const float4*>(q + 4);
    cs[0] = c0.x; cs[1] = c0.y; cs[2] = c0.z; cs[3] = c0.w; cs[4] = c1.x; cs[5] = c1.y; cs[6] = c1.z; cs[7] = c1.w;
    sn[0] = s0.x; sn[1] = s0.y; sn[2] = s0.z; sn[3] = s0.w; sn[4] = s1.x; sn[5] = s1.y; sn[6] = s1.z; sn[7] = s1.w;
  }
  float v0[8], v1[8];
  if (r.src_f32) {
    const float* s = r.src_f32 + tok * r.ldsrc + hh * 64;
    set8(v0, s + i0);
    set8(v1, s + 32 + i0);
    for (int p = 1; p < r.nsplit; ++p) {
      add8(v0, s + p * r.split_stride + i0);
      add8(v1, s + p * r.split_stride + 32 + i0);
    }
  } else {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(x + i0);
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(x + 32 + i0);
#pragma unroll
    for (int j = 0; j < 8; ++j) { v0[j] = (float)a[j]; v1[j] = (float)b[j]; }
  }
  bf16x8 oa, ob;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (r.cos) rope_pair(v0[j], v1[j], cs[j], sn[j], r.inverse != 0);
    oa[j] = (bf16)v0[j];
    ob[j] = (bf16)v1[j];
  }
  *reinterpret_cast<bf16x8*>(x + i0) = oa;
  *reinterpret_cast<bf16x8*>(x + 32 + i0) = ob;
}
__global__ void rope_kernel(RopeArgs r) { rope_rows(r); }
// the dK and dV finalizes of one backward as one launch (blockIdx.y selects the tensor)
__global__ void rope2_kernel(RopeArgs r0, RopeArgs r1) { rope_rows(blockIdx.y ? r1 : r0); }

// GQA finalize: dst[t, hk, :] = sum_{j<G} src[t, hk*G + j, :] (f32 per-q-head partials, row stride
// Hq*64) -> optional RoPE^T -> bf16. One thread per (token, kv head, quarter of the pairs).
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


// ---- decode attention, one workgroup per kv head (agent decode, caches of <= 1024 rows) ---------------------------
// The new token's G query heads over cache rows [0, pos] of one kv head, without a key split (so no partials, no
// cross-workgroup merge): 16 waves; wave w owns 32-key blocks w and w + 16. S = K Q^T on the MFMA with K fragments
// loaded straight from the cache rows (natural order) and the rotated q heads as the B operand (head on the lane,
// padded to 32 with zero rows); softmax max / sum per head through one LDS exchange each; O^T += V^T P^T with V staged
// in swizzled LDS and P^T taken from the score accumulator (the training forward's operand forms); the 16 wave
// partials of O^T summed through LDS. Cache row layout [q (Hq*64) | k (Hkv*64) | v (Hkv*64)], rows < pos hold rotated
// k; this kernel rotates q and row pos's k (writing that k back for later steps).
struct DecMfmaArgs {
  bf16* cache; long ld; int Hq, Hkv;
  const float* cos; const float* sin;
  bf16* out;
  const int* st;  // slx_dec_state: [0] pos, [2] done
  float scale;
};

constexpr int kDecKeys = 1024;

__device__ __forceinline__ void dec_attn_mfma_body(const DecMfmaArgs& a, int g, char* smem) {
  char* Vl = smem;                          // [kDecKeys][64] bf16, swizzled (128 KB); reused for the O^T partials
  char* Ql = smem + kDecKeys * 128;         // [32][64] bf16 rotated q heads (rows >= G zero), swizzled
  float* kpos = reinterpret_cast<float*>(Ql + 32 * 128);  // [64] rotated k of row pos (bf16 values)
  float* red = kpos + 64;                   // [16 waves][32 heads]
  float* Mh = red + 16 * 32;                // [32]
  float* Lh = Mh + 32;                      // [32]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hl = lane >> 5;
  const int pos = a.st[0], L = pos + 1;
  const int G = a.Hq / a.Hkv;
  const int qn = a.Hq * 64, kn = a.Hkv * 64;
  const int nb = (L + 31) >> 5;  // 32-key blocks
  const bf16* kcol = a.cache + qn + g * 64;
  const bf16* vcol = a.cache + qn + kn + g * 64;
  // ---- every global read up front: K fragments of this wave's blocks, V rows (16-B chunks), q / k rows of pos
  bf16x8 kf[2][4];
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
    const int blk = w + 16 * bb;
    const int key = min(blk * 32 + (lane & 31), L - 1);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      kf[bb][kk] = blk < nb ? *reinterpret_cast<const bf16x8*>(kcol + (long)key * a.ld + 16 * kk + 8 * hl) : bf16x8{};
  }
  uint4 vr[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = tid + 1024 * i, row = c >> 3;
    vr[i] = row < L ? *reinterpret_cast<const uint4*>(vcol + (long)row * a.ld + 8 * (c & 7)) : make_uint4(0u, 0u, 0u, 0u);
  }
  bf16* prow = a.cache + (long)pos * a.ld;
  const float* cs = a.cos + (long)pos * 32;
  const float* sn = a.sin + (long)pos * 32;
  if (tid < 32 * 32) {  // rotate_half RoPE of the G q heads into Ql (rows >= G: zeros)
    const int h = tid >> 5, j = tid & 31;
    float r0 = 0.f, r1 = 0.f;
    if (h < G) {
      const bf16* q = prow + (g * G + h) * 64;
      const float q0 = (float)q[j], q1 = (float)q[j + 32];
      r0 = q0 * cs[j] - q1 * sn[j];
      r1 = q1 * cs[j] + q0 * sn[j];
    }
    *reinterpret_cast<bf16*>(Ql + sw_elem(h, j)) = (bf16)r0;
    *reinterpret_cast<bf16*>(Ql + sw_elem(h, j + 32)) = (bf16)r1;
  }
  if (w == 15 && lane < 32) {  // k of this token: rotated, written back once
    const int j = lane;
    bf16* k = prow + qn + g * 64;
    const float k0 = (float)k[j], k1 = (float)k[j + 32];
    const bf16 r0 = (bf16)(k0 * cs[j] - k1 * sn[j]), r1 = (bf16)(k1 * cs[j] + k0 * sn[j]);
    k[j] = r0;
    k[j + 32] = r1;
    kpos[j] = (float)r0;
    kpos[j + 32] = (float)r1;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = tid + 1024 * i, row = c >> 3;
    if (row < nb * 32) *reinterpret_cast<uint4*>(Vl + sw_off(row, c & 7)) = vr[i];
  }
  __syncthreads();
  // the lanes holding row pos take the rotated k
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
    if (w + 16 * bb == (pos >> 5) && (lane & 31) == (pos & 31)) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int j = 0; j < 8; ++j) kf[bb][kk][j] = (bf16)kpos[16 * kk + 8 * hl + j];
    }
  }
  // ---- scores S[key][head] = K q^T, head on the lane (l & 31), 16 keys per lane and block
  bf16x8 qf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) qf[kk] = row_frag(Ql, 0, kk, lane);
  const float c = a.scale * LOG2E;
  f32x16 s[2];
  float mx = -INFINITY;
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[bb][r] = 0.f;
    if (w + 16 * bb < nb) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) s[bb] = mfma32(kf[bb][kk], qf[kk], s[bb]);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = (w + 16 * bb) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        s[bb][r] = key < L ? s[bb][r] * c : -INFINITY;
        mx = fmaxf(mx, s[bb][r]);
      }
    }
  }
  mx = half_swap_max(mx);
  if (lane < 32) red[w * 32 + lane] = mx;
  __syncthreads();
  if (tid < 32) {
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) m = fmaxf(m, red[i * 32 + tid]);
    Mh[tid] = m;
  }
  __syncthreads();
  const float M = Mh[lane & 31];
  float ls = 0.f;
  f32x16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
    if (w + 16 * bb < nb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[bb][r] = __builtin_amdgcn_exp2f(s[bb][r] - M);
        ls += (float)(bf16)s[bb][r];  // the bf16 P the MFMA sums
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 pb = acc_frag(s[bb], st);
        o0 = mfma32(tr_frag(Vl, (w + 16 * bb) * 32 + 16 * st, 0, lane), pb, o0);
        o1 = mfma32(tr_frag(Vl, (w + 16 * bb) * 32 + 16 * st, 32, lane), pb, o1);
      }
    }
  }
  {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(ls), __float_as_uint(ls), false, false);
    ls = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  __syncthreads();  // every wave is done with Vl: reuse it for the O^T partials [16][G][64]
  float* op = reinterpret_cast<float*>(Vl);
  if (lane < 32) red[w * 32 + lane] = ls;
  const int h = lane & 31;
  if (h < G) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = 8 * (r >> 2) + 4 * hl + (r & 3);
      op[(w * G + h) * 64 + d] = o0[r];
      op[(w * G + h) * 64 + 32 + d] = o1[r];
    }
  }
  __syncthreads();
  if (tid < 32) {
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) l += red[i * 32 + tid];
    Lh[tid] = l;
  }
  __syncthreads();
  if (tid < G * 64) {
    const int hh = tid >> 6, d = tid & 63;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += op[(i * G + hh) * 64 + d];
    const bf16 o = (bf16)(acc / Lh[hh]);
    a.out[(g * G + hh) * 64 + d] = o;
  }
}

__global__ __launch_bounds__(1024) void dec_attn_mfma_kernel(DecMfmaArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (a.st[2]) return;
  dec_attn_mfma_body(a, blockIdx.x, smem);
}

// ---- decode attention split over keys, merged by the O GEMV (slx_dec_attn_o_split) ----------------------------------
// Grid (Hkv, ns), 4 waves: workgroup (g, sp) takes the 32-key blocks [sp*bpw, (sp+1)*bpw) of kv head g (bpw =
// ceil(nb/ns) <= 8; wave w owns blocks w and w + 4) with the operand forms of dec_attn_mfma_body, and stores its
// partial softmax state per query head, unnormalised: m (max of the log2-domain scores), l (sum of the bf16 P) and
// o[64] = sum P v, at ws + (g*ns + sp) * G*66 (m[G], l[G], o[G][64]). No counter and no merge in this launch: the O
// GEMV that follows reads every split's partial (the kernel boundary makes them visible) and merges them while its
// weight rows are in flight, so the attention costs one short launch on Hkv*ns CUs instead of one CU per kv head
// loading the whole cache.
__global__ __launch_bounds__(256) void dec_attn_mfma_split_kernel(DecMfmaArgs a, float* ws) {
  __shared__ __attribute__((aligned(16))) char Vl[256 * 128];  // this split's V rows, swizzled; then O^T partials
  __shared__ __attribute__((aligned(16))) char Ql[32 * 128];
  __shared__ float kpos[64];
  __shared__ float red[4 * 32];
  __shared__ float Mh[32], Lh[32];
  if (a.st[2]) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hl = lane >> 5;
  const int g = blockIdx.x, sp = blockIdx.y, ns = gridDim.y;
  const int pos = a.st[0], L = pos + 1;
  const int G = a.Hq / a.Hkv;
  const int qn = a.Hq * 64, kn = a.Hkv * 64;
  const int nb = (L + 31) >> 5;
  const int bpw = (nb + ns - 1) / ns;
  const int b0 = sp * bpw, b1 = min(nb, b0 + bpw);
  float* part = ws + ((long)g * ns + sp) * (G * 66);
  if (b0 >= b1) {  // empty split: neutral partial (m = -inf, l = 0, o = 0)
    for (int i = tid; i < G * 66; i += 256) part[i] = i < G ? -INFINITY : 0.f;
    return;
  }
  const int r0 = b0 * 32, nrow = min(L, b1 * 32) - r0;  // this split's cache rows [r0, r0 + nrow)
  const bf16* kcol = a.cache + qn + g * 64;
  const bf16* vcol = a.cache + qn + kn + g * 64;
  bf16x8 kf[2][4];
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
    const int blk = b0 + w + 4 * bb;
    const int key = min(blk * 32 + (lane & 31), L - 1);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      kf[bb][kk] = blk < b1 ? *reinterpret_cast<const bf16x8*>(kcol + (long)key * a.ld + 16 * kk + 8 * hl) : bf16x8{};
  }
  uint4 vr[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = tid + 256 * i, row = c >> 3;
    vr[i] = row < nrow ? *reinterpret_cast<const uint4*>(vcol + (long)(r0 + row) * a.ld + 8 * (c & 7))
                       : make_uint4(0u, 0u, 0u, 0u);
  }
  bf16* prow = a.cache + (long)pos * a.ld;
  const float* cs = a.cos + (long)pos * 32;
  const float* sn = a.sin + (long)pos * 32;
  for (int e = tid; e < 32 * 32; e += 256) {  // rotate_half RoPE of the G q heads into Ql (rows >= G: zeros)
    const int h = e >> 5, j = e & 31;
    float q0r = 0.f, q1r = 0.f;
    if (h < G) {
      const bf16* q = prow + (g * G + h) * 64;
      const float q0 = (float)q[j], q1 = (float)q[j + 32];
      q0r = q0 * cs[j] - q1 * sn[j];
      q1r = q1 * cs[j] + q0 * sn[j];
    }
    *reinterpret_cast<bf16*>(Ql + sw_elem(h, j)) = (bf16)q0r;
    *reinterpret_cast<bf16*>(Ql + sw_elem(h, j + 32)) = (bf16)q1r;
  }
  const bool has_pos = (pos >> 5) < b1;  // the last split with keys holds row pos
  if (has_pos && w == 0 && lane < 32) {  // k of this token: rotated, written back once
    const int j = lane;
    bf16* k = prow + qn + g * 64;
    const float k0 = (float)k[j], k1 = (float)k[j + 32];
    const bf16 kr0 = (bf16)(k0 * cs[j] - k1 * sn[j]), kr1 = (bf16)(k1 * cs[j] + k0 * sn[j]);
    k[j] = kr0;
    k[j + 32] = kr1;
    kpos[j] = (float)kr0;
    kpos[j + 32] = (float)kr1;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = tid + 256 * i, row = c >> 3;
    if (row < (b1 - b0) * 32) *reinterpret_cast<uint4*>(Vl + sw_off(row, c & 7)) = vr[i];
  }
  __syncthreads();
  if (has_pos) {
#pragma unroll
    for (int bb = 0; bb < 2; ++bb)
      if (b0 + w + 4 * bb == (pos >> 5) && (lane & 31) == (pos & 31)) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int j = 0; j < 8; ++j) kf[bb][kk][j] = (bf16)kpos[16 * kk + 8 * hl + j];
      }
  }
  bf16x8 qf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) qf[kk] = row_frag(Ql, 0, kk, lane);
  const float c = a.scale * LOG2E;
  f32x16 s[2];
  float mx = -INFINITY;
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[bb][r] = 0.f;
    const int blk = b0 + w + 4 * bb;
    if (blk < b1) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) s[bb] = mfma32(kf[bb][kk], qf[kk], s[bb]);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = blk * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        s[bb][r] = key < L ? s[bb][r] * c : -INFINITY;
        mx = fmaxf(mx, s[bb][r]);
      }
    }
  }
  mx = half_swap_max(mx);
  if (lane < 32) red[w * 32 + lane] = mx;
  __syncthreads();
  if (tid < 32) {
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) m = fmaxf(m, red[i * 32 + tid]);
    Mh[tid] = m;
  }
  __syncthreads();
  const float M = Mh[lane & 31];
  float ls = 0.f;
  f32x16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
    const int blk = b0 + w + 4 * bb;
    if (blk < b1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[bb][r] = __builtin_amdgcn_exp2f(s[bb][r] - M);
        ls += (float)(bf16)s[bb][r];  // the bf16 P the MFMA sums
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 pb = acc_frag(s[bb], st);
        const int lrow = (blk - b0) * 32 + 16 * st;
        o0 = mfma32(tr_frag(Vl, lrow, 0, lane), pb, o0);
        o1 = mfma32(tr_frag(Vl, lrow, 32, lane), pb, o1);
      }
    }
  }
  {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(ls), __float_as_uint(ls), false, false);
    ls = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  __syncthreads();  // every wave is done with Vl: reuse it for the O^T partials [4][G][64]
  float* op = reinterpret_cast<float*>(Vl);
  if (lane < 32) red[w * 32 + lane] = ls;
  const int h = lane & 31;
  if (h < G) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = 8 * (r >> 2) + 4 * hl + (r & 3);
      op[(w * G + h) * 64 + d] = o0[r];
      op[(w * G + h) * 64 + 32 + d] = o1[r];
    }
  }
  __syncthreads();
  if (tid < G) {
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) l += red[i * 32 + tid];
    part[tid] = Mh[tid];
    part[G + tid] = l;
  }
  for (int e = tid; e < G * 64; e += 256) {
    const int hh = e >> 6, d = e & 63;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc += op[(i * G + hh) * 64 + d];
    part[2 * G + e] = acc;
  }
}

int dec_attn_split_launch(void* cache, long ld, int Hq, int Hkv, const float* cos_tab, const float* sin_tab,
                          float* ws, int ns, const void* st, hipStream_t s) {
  DecMfmaArgs a{(bf16*)cache, ld, Hq, Hkv, cos_tab, sin_tab, nullptr, (const int*)st, 0.125f};
  hipLaunchKernelGGL(dec_attn_mfma_split_kernel, dim3(Hkv, ns), dim3(256), 0, s, a, ws);
  SLX_LAUNCH_CHECK("slx_dec_attn_o_split(attention)");
  return 0;
}

int dec_attn_mfma_launch(void* cache, long ld, int Hq, int Hkv, const float* cos_tab, const float* sin_tab, void* out,
                         const void* st, hipStream_t s) {
  constexpr int LDS = kDecKeys * 128 + 32 * 128 + (64 + 16 * 32 + 32 + 32) * 4;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)dec_attn_mfma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  DecMfmaArgs a{(bf16*)cache, ld, Hq, Hkv, cos_tab, sin_tab, (bf16*)out, (const int*)st, 0.125f};
  hipLaunchKernelGGL(dec_attn_mfma_kernel, dim3(Hkv), dim3(1024), LDS, s, a);
  SLX_LAUNCH_CHECK("slx_dec_attn(mfma)");
  return 0;
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
  // default on: +0.1-0.2 % on the VLA step (profiles/round2_s3_tail_swiglu_ab.txt)
  static const int tf = [] { const char* e = getenv("SLX_ATTN_TAIL_FIRST"); return e ? atoi(e) : 1; }();
  a.tail_first = (!d->causal && d->S % 128 != 0) ? tf : 0;
  static const int tv = [] { const char* e = getenv("SLX_ATTN_TAILV"); return e ? atoi(e) : 1; }();
  a.tailv = tv;
  a.nqb = a.nkb = (d->S + 127) / 128;
  return 0;
}

// the row tail (S % 128 <= kTailQ) folded into the last whole block: non-causal, at least one whole block
// (SLX_ATTN_QTAIL=0 launches the tail rows' own workgroups as before, A/B)
static int row_tail(const AttnArgs& a) {
  static const int on = [] { const char* e = getenv("SLX_ATTN_QTAIL"); return e ? atoi(e) : 1; }();
  const int r = a.S % 128;
  return (on && !a.causal && a.tailv && a.S >= 128 && r > 0 && r <= kTailQ) ? r : 0;
}

extern "C" int slx_attn_fwd(const slx_attn_desc* d, slx_stream_t stream) {
  AttnArgs a;
  int rc = fill_common(a, d);
  if (rc) return rc;
  if (a.B == 0 || a.S == 0) return 0;
  a.qtail = row_tail(a);
  a.nqb = a.qtail ? a.S / 128 : (a.S + 127) / 128;
  dim3 grid(a.nqb * a.Hq * a.B);
  hipLaunchKernelGGL(attn_fwd_dma_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
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
  a.dq_acc = g->dq_acc;
  a.dq = (bf16*)g->dq; a.lddq = g->lddq; a.rcos = g->rope_cos; a.rsin = g->rope_sin;
  SLX_CHECK_ARG(a.dq && a.lddq % 4 == 0, "slx_attn_bwd: dq (bf16, lddq %% 4 == 0) is required");
  const bool gqa = d->Hq != d->Hkv;
  const bool f32kv = gqa || g->rope_cos;  // dK needs RoPE^T or the layout differs: finalize from f32
  SLX_CHECK_ARG(a.lse && a.delta && a.dq_acc, "slx_attn_bwd: lse, delta_ws and dq_acc are required");
  SLX_CHECK_ARG(!f32kv || (g->dk_acc && g->dv_acc), "slx_attn_bwd: GQA/RoPE needs dk_acc/dv_acc workspaces");
  a.dk_acc = f32kv ? g->dk_acc : nullptr;
  a.dv_acc = f32kv ? g->dv_acc : nullptr;
  a.dk = (bf16*)g->dk; a.dv = (bf16*)g->dv; a.lddk = g->lddk; a.lddv = g->lddv;
  a.dbq = g->dbias_q; a.dbk = g->dbias_k; a.dbv = g->dbias_v;
  SLX_CHECK_ARG((a.dbk == nullptr) == (a.dbv == nullptr), "slx_attn_bwd: dbias_k and dbias_v go together");
  SLX_CHECK_ARG(!a.dbk || !f32kv, "slx_attn_bwd: dk/dv bias sums need the bf16 dK/dV path (no GQA, no RoPE)");
  const long ntok = (long)a.B * a.S;
  // the folded row tails: queries in the dQ pass (its dQ store has no RoPE^T for them), keys in the dK/dV pass (bf16
  // dK / dV written directly: no GQA, no RoPE)
  a.qtail = a.rcos ? 0 : row_tail(a);
  a.nqb = a.qtail ? a.S / 128 : (a.S + 127) / 128;
  a.ktail = f32kv ? 0 : row_tail(a);
  a.nkb = a.ktail ? a.S / 128 : (a.S + 127) / 128;
  // dQ pass first: it computes delta = rowsum(dO * O) per query in its prologue and stores it for the dK/dV pass
  hipLaunchKernelGGL(attn_bwd_dq_dma_kernel, dim3(a.nqb * a.Hq * a.B), dim3(256), 0, st, a);
  SLX_LAUNCH_CHECK("slx_attn_bwd(dq)");
  {  // split a GQA group's q-heads over workgroups: one q-head per workgroup (Qwen2: 7 x 112 = 784 workgroups; with the
     // heaviest-first order +0.25 % on the step over the 4-way split that just fills the chip,
     // profiles/round2_s3_kv_gu_ab.txt); SLX_ATTN_KV_NS overrides (A/B)
    const int G = a.Hq / a.Hkv;
    static const int ns_env = [] { const char* e = getenv("SLX_ATTN_KV_NS"); return e ? atoi(e) : 0; }();
    int ns = ns_env > 0 ? ns_env : G;
    ns = ns < 1 ? 1 : (ns > G ? G : ns);
    if (!f32kv) ns = 1;
    a.hsplit = (G + ns - 1) / ns;
    a.nsplit = (G + a.hsplit - 1) / a.hsplit;
  }
  hipLaunchKernelGGL(attn_bwd_kv_dma_kernel, dim3(a.nkb * a.Hkv * a.nsplit * a.B), dim3(256), 0, st, a);
  SLX_LAUNCH_CHECK("slx_attn_bwd(dk/dv)");
  // finalize: f32 -> bf16, summing head-split partials and applying the RoPE transpose where asked
  auto rope_args = [&](const float* src, int heads, bf16* dst, long ld, bool rope, int nsplit) {
    RopeArgs r;
    memset(&r, 0, sizeof(r));
    r.ntok = ntok; r.S = a.S; r.inverse = 1;
    r.cos = rope ? g->rope_cos : nullptr;
    r.sin = rope ? g->rope_sin : nullptr;
    r.x = dst; r.ldx = ld; r.nheads = heads; r.src_f32 = src; r.ldsrc = (long)heads * 64;
    r.nsplit = nsplit; r.split_stride = ntok * heads * 64;
    return r;
  };
  if (f32kv && a.nsplit > 1) {  // GQA: dK (RoPE^T) and dV finalized by one launch
    const RopeArgs rk = rope_args(a.dk_acc, a.Hkv, (bf16*)g->dk, g->lddk, true, a.nsplit);
    const RopeArgs rv = rope_args(a.dv_acc, a.Hkv, (bf16*)g->dv, g->lddv, false, a.nsplit);
    const long total = ntok * a.Hkv * 4;
    hipLaunchKernelGGL(rope2_kernel, dim3((total + 255) / 256, 2), dim3(256), 0, st, rk, rv);
    SLX_LAUNCH_CHECK("slx_attn_bwd(finalize dk+dv)");
    return 0;
  }
  auto conv = [&](const float* src, int heads, bf16* dst, long ld, bool rope, int nsplit) -> int {
    if ((rope && g->rope_cos) || nsplit > 1) {
      const RopeArgs r = rope_args(src, heads, dst, ld, rope, nsplit);
      const long total = ntok * heads * 4;
      hipLaunchKernelGGL(rope_kernel, dim3((total + 255) / 256), dim3(256), 0, st, r);
    } else {
      const long total = ntok * heads * 8;
      hipLaunchKernelGGL(f32_to_bf16_rows_kernel, dim3((total + 255) / 256), dim3(256), 0, st, src, (long)heads * 64, dst, ld, ntok, heads * 64);
    }
    SLX_LAUNCH_CHECK("slx_attn_bwd(finalize)");
    return 0;
  };
  if (f32kv) {
    if ((rc = conv(a.dk_acc, a.Hkv, (bf16*)g->dk, g->lddk, true, a.nsplit))) return rc;
    if ((rc = conv(a.dv_acc, a.Hkv, (bf16*)g->dv, g->lddv, false, a.nsplit))) return rc;
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
