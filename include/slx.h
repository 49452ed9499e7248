/*
 * slx.h — C-ABI of libslx_hip.so, the MI355X (gfx950) kernels behind the SimLingo VLA hot path.
 *
 * Conventions (SURVEY.md §8b "Ownership"/"Error convention"):
 *   - Plain pointers + sizes + element strides; no framework types. bf16 tensors are uint16 bit
 *     patterns, f32 tensors are float. Caller allocates every buffer; kernels never allocate.
 *   - Every call takes the HIP stream it is enqueued on (slx_stream_t == hipStream_t).
 *   - Every call returns 0 on success, a negative code on failure (-22 = bad argument,
 *     <= -1000 = HIP launch error); slx_last_error() returns a thread-local message.
 *   - Calls are asynchronous and reentrant per stream; the library holds no global mutable state.
 *
 * Each entry point names the reference interface it replaces (file:line under the reference
 * repository TimS-ml/simlingo, or the third-party kernel it stands for).
 */
#ifndef SLX_H_
#define SLX_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef void* slx_stream_t;

/* ---- library ------------------------------------------------------------------------------ */
const char* slx_last_error(void);
int slx_abi_version(void);
int slx_device_sync(void);
/* Deterministic-reduction mode (reproducible gradients; off by default). on = 1: every cross-block f32 reduction of
 * the step (LoRA parameter gradients, column sums, norm parameter gradients, the gradient sum of squares, GEMM split-K)
 * stores per-block partials in ws and sums them in a fixed order instead of f32 atomics, and GEMM split-K runs only in
 * its in-launch slab form; two runs on the same inputs then give bitwise-equal gradients. ws (>= 2^20 floats; 16 Mi
 * floats cover the InternVL2-1B step) is used by one call at a time and must outlive the mode. Process-wide switch,
 * for one stream at a time (a test / reproducibility mode, not thread-safe against concurrent launches).          */
int slx_set_deterministic(int on, float* ws, int64_t ws_floats);
int slx_get_deterministic(void);

/* ---- GEMM ---------------------------------------------------------------------------------
 * C[M,N] = alpha * sum_k A(m,k) B(k,n)   (+ epilogue), bf16 operands, f32 accumulation (MFMA).
 * Replaces cuBLAS behind every nn.Linear of InternViT / mlp1 / Qwen2+LoRA / LM head
 * (simlingo_training/models/encoder/internvl2_model.py:114 -> remote InternVisionModel;
 *  simlingo_training/models/driving.py:217 -> Qwen2ForCausalLM; llm.py:106-119 LoRA).       */
enum {
  SLX_GEMM_NT = 0, /* A [M][K] (lda), B [N][K] (ldb): Y = X W^T          (forward Linear)  */
  SLX_GEMM_NN = 1, /* A [M][K],       B [K][N]:       dX = dY W            (data grad)     */
  SLX_GEMM_TN = 2, /* A [K][M],       B [K][N]:       dW = dY^T X          (weight grad)   */
  SLX_GEMM_TT = 3  /* A [K][M],       B [N][K]                                              */
};
enum {
  SLX_EPI_STORE = 0,      /* C (+)= alpha*acc + bias[n]                                       */
  SLX_EPI_GELU = 1,       /* aux_out = h = alpha*acc + bias; C = gelu_erf(h)   (bf16)          */
  SLX_EPI_RESID_LS = 2,   /* y = alpha*acc + bias; aux_out = y (bf16, optional);
                             C(f32) = resid + ls[n]*y   (InternViT layer-scale residual)      */
  SLX_EPI_GELU_BWD = 3,   /* C = alpha*acc * gelu_erf'(aux[m,n])                              */
  SLX_EPI_SWIGLU_BWD = 4, /* aux=[g|u] (ld ldaux, width 2N): C[m,n]=d*u*silu'(g), C[m,N+n]=d*silu(g) */
  SLX_EPI_DROPMASK = 5,   /* C (+)= alpha*acc * keep(seed, m*ldmask+n)/(1-p)   (LoRA dropout bwd) */
  SLX_EPI_DROPMASK_SWIGLU = 6, /* d = resid + keep*alpha*acc; C[:, :N] = d*u*silu'(g), C[:, N:] = d*silu(g),
                                  aux = [g | u] (Qwen2MLP down_proj LoRA dgrad fused into the SwiGLU backward) */
  SLX_EPI_QGELU = 7,      /* aux_out = h = alpha*acc + bias; C = h*sigmoid(1.702h)  (CLIP quick_gelu, bf16) */
  SLX_EPI_QGELU_BWD = 8   /* C = alpha*acc * quick_gelu'(aux[m,n])                                         */
};
typedef struct slx_gemm_desc {
  int layout, epilogue, out_f32;
  int M, N, K, batch;
  const void* A; int64_t lda; int64_t sA;
  const void* B; int64_t ldb; int64_t sB;
  void* C; int64_t ldc; int64_t sC;
  float alpha;
  const float* bias;   /* [N] f32 or NULL */
  const float* ls;     /* [N] f32 (RESID_LS) */
  const void* aux; int64_t ldaux;       /* bf16 epilogue input */
  void* aux_out; int64_t ldaux_out;     /* bf16 epilogue output */
  const float* resid; int64_t ldr;      /* f32 residual (RESID_LS) */
  int accumulate;
  uint64_t seed; float drop_p; int64_t ldmask;
  int ksplit_max;   /* 0 = automatic split-K for under-filled f32 STORE GEMMs, < 0 = never, > 0 = cap */
  int variant;      /* 0 = automatic main-loop choice (tuning/testing hook; see gemm.hip)         */
  int drop_operand; /* 0 none; 1/2: LoRA dropout applied to A/B while loading, mask index =
                       storage_row*ldmask + storage_col, hash of slx_dropout (seed, drop_p)      */
  float* colsum;    /* optional [N] f32: += column sums of the epilogue's f32 output (the bias gradient
                       of the layer whose output gradient this GEMM produces, e.g. fc1.b from the
                       GELU_BWD dgrad); STORE (no split-K) / GELU_BWD / QGELU_BWD, N % 8 == 0        */
  float* colsum_ws; /* required with colsum: [ceil(M/64), N] f32 partials (one row per 64-row subtile,
                       plain stores, then one small reduce launch: no same-address atomics)          */
  const uint32_t* maskbits; int64_t ldbits; /* DROPMASK epilogues: keep bits [M][ldbits] written by
                       slx_lora_down (bit n&31 of word n>>5); NULL = regenerate from (seed, drop_p, ldmask)  */
  float* rem_ws; int64_t rem_ws_floats; /* optional scratch for the M % 256 remainder rows (<= 64 of them):
                       split-K f32 partials [splits][rem][N] summed by the v3 launch itself (A K-contiguous)
                       or by one epilogue pass; its LAST 4096 words are arrival counters that must be zero
                       before first use (every call leaves them zero; one workspace per stream). Without it
                       (or if it is too small) the remainder runs as a latency-bound 16..64-row tile      */
  int resid_bf16;   /* DROPMASK_SWIGLU: resid holds bf16 rows (the bf16 base gradient of a bf16 Linear backward)  */
  float* split_ws; int64_t split_ws_floats; /* optional scratch for split-K f32 STORE GEMMs on the 256x256 kernel
                       (weight gradients, slx_gemm_bf16_pair): [tiles][ksplit][65536] f32 partial slabs summed inside
                       the launch by each tile's last-arriving split (deterministic split order) instead of f32
                       atomics into C; its LAST 16384 words are arrival counters that must be zero before first use
                       (every call leaves them zero; one workspace per stream). NULL = atomics                     */
  const float* rope_cos; const float* rope_sin; /* optional, STORE bf16 only: RoPE on the output columns < rope_ncols
                       (64-wide heads, dims d / d + 32 rotated as a pair; position = row % rope_S, tables [rope_S][32]
                       f32 as slx_rope takes them), applied to alpha*acc + bias before the bf16 rounding: the Qwen2
                       q|k projection (modeling_qwen2 apply_rotary_pos_emb) fused into its GEMM                       */
  int rope_S; int rope_ncols;
  int aux_grad;     /* GELU / QGELU: aux_out receives the activation's derivative at the pre-activation,
                       bf16(gelu'(h)), instead of h; GELU_BWD / QGELU_BWD: aux holds that derivative and is multiplied
                       in directly (the backward epilogue then evaluates no transcendental)                           */
} slx_gemm_desc;
int slx_gemm_bf16(const slx_gemm_desc* d, slx_stream_t stream);

/* Plain GEMM through hipBLASLt (round 6): D[M][N] = alpha * A[M][K] . B[N][K]^T + beta * C[M][N], row-major, A / B
   bf16, C / D both f32 (out_f32) or both bf16, f32 accumulation. The step's plain GEMMs where the vendor library's
   tiles beat slx_gemm_bf16 (measured per shape): the Qwen2 gate/up data gradient ([dx | dt] = dgu . W_cat, no
   epilogue) and the Qwen2 o / down projections with their residual (C = the f32 residual stream, beta = 1: Qwen2's
   `hidden_states = residual + mlp(...)`, modeling_qwen2 decoder layer, reached through llm.py:88-119). Replaces the
   same torch.nn.Linear calls as slx_gemm_bf16. The plan (descriptors + the heuristic's algorithm) is cached per
   shape; workspace: caller-owned, ws_bytes (0 allowed). Not bitwise reproducible against slx_gemm_bf16 (another
   summation order); callers in deterministic-reduction mode keep slx_gemm_bf16. */
typedef struct slx_gemm_lt_desc {
  int64_t M, N, K;
  const void* A; int64_t lda;   /* bf16 [M][K] */
  const void* B; int64_t ldb;   /* bf16 [N][K] */
  const void* C; int64_t ldc;   /* [M][N], read when beta != 0 (may equal D) */
  void* D; int64_t ldd;         /* [M][N] */
  float alpha, beta;
  int out_f32;                  /* C and D f32 (1) or bf16 (0) */
  void* ws; int64_t ws_bytes;
} slx_gemm_lt_desc;
int slx_gemm_lt(const slx_gemm_lt_desc* d, slx_stream_t stream);
/* Two independent accumulating f32 STORE GEMMs (same layout and K, no bias / colsum / batch) in one launch:
 * the InternViT weight-gradient pairs (fc2.w + fc1.w, proj.w + qkv.w; the torch autograd wgrad GEMMs of
 * internvl2 InternMLP / InternAttention, K = tokens) share one round of 256 split-K blocks.
 * d1->ksplit_max caps the split count (0 = automatic).                                                     */
int slx_gemm_bf16_pair(const slx_gemm_desc* d1, const slx_gemm_desc* d2, slx_stream_t stream);

/* ---- Attention (head_dim 64) ----------------------------------------------------------------
 * Replaces flash-attn 2.7.0.post2 (README.md:67-68) inside the InternVL2-1B remote code:
 * InternViT non-causal MHA (internvl2_model.py:114 -> extract_feature) and Qwen2 causal GQA with
 * key padding (driving.py:217-223, attention_mask = inputs_mask, valid-first layout).
 * q/k/v/o: token-major rows [B*S, ld], head h at columns h*64..h*64+63.
 * Deviation: the key-padding mask is a per-sequence valid-key COUNT (seqlens), i.e. keys [0, seqlens[b]) valid.
 * That is the only layout AdaptorList.forward produces (adaptors.py: inputs are packed valid-first, padding
 * after); an arbitrary [B, S] mask (holes, left padding of keys) is not expressible here, and the Python seam
 * (vlm.py _valid_lengths) raises NotImplementedError for one instead of silently mis-masking.        */
typedef struct slx_attn_desc {
  int B, S, Hq, Hkv, head_dim, causal;
  const void* q; int64_t ldq;
  const void* k; int64_t ldk;
  const void* v; int64_t ldv;
  void* o; int64_t ldo;
  float* lse;           /* [B, Hq, S] f32, log2 domain (written by fwd, read by bwd)        */
  const int* seqlens;   /* [B] valid keys per sequence (key-padding mask) or NULL           */
  float scale;          /* softmax scale (1/sqrt(64))                                       */
} slx_attn_desc;
typedef struct slx_attn_bwd_desc {
  const void* dout; int64_t lddo;
  void* dq; int64_t lddq;
  void* dk; int64_t lddk;
  void* dv; int64_t lddv;
  float* delta_ws;              /* [B, Hq, S]                                            */
  float* dq_acc;                /* [B*S, Hq*64] f32 workspace (fully overwritten)        */
  float* dk_acc; float* dv_acc; /* [B*S, Hq*64] f32 workspaces, required for GQA or RoPE */
  const float* rope_cos; const float* rope_sin; /* [S, 32] tables: apply RoPE^T to dq/dk */
  float* dbias_q; float* dbias_k; float* dbias_v; /* optional [Hq*64] / [Hkv*64] f32: += column sums of dq / dk / dv
                                   over all B*S rows (the q/k/v bias gradients of InternViT's qkv Linear,
                                   qkv_bias=True); dk/dv sums need Hq == Hkv and no RoPE                      */
} slx_attn_bwd_desc;
int slx_attn_fwd(const slx_attn_desc* d, slx_stream_t stream);
int slx_attn_bwd(const slx_attn_desc* d, const slx_attn_bwd_desc* g, slx_stream_t stream);
/* Qwen2 rotary embedding, rotate_half convention, theta baked into the [S,32] cos/sin tables
 * (HF Qwen2RotaryEmbedding, rope_theta 1e6; position_ids=None -> arange, driving.py:207).    */
int slx_rope(void* x, int64_t ldx, int64_t ntok, int S, int nheads, const float* cos_tab,
             const float* sin_tab, int inverse, slx_stream_t stream);

/* ---- LayerNorm / RMSNorm ---------------------------------------------------------------------
 * InternViT norm1/norm2 (eps 1e-6), mlp1 LayerNorm(4096, eps 1e-5) with the pixel_shuffle(0.5)
 * gather fused in (pixel_shuffle_grid = 32, tokens_per_image = 1025), Qwen2RMSNorm (eps 1e-6).
 * x: f32 rows, y: bf16 rows. D % 4 == 0, D <= 4096.                                           */
typedef struct slx_norm_desc {
  int rms;
  const float* x; int64_t ldx;
  const float* gamma; const float* beta;
  void* y; int64_t ldy;
  float* mean; float* rstd;   /* [rows] saved statistics */
  int64_t rows; int D; float eps;
  int pixel_shuffle_grid; int tokens_per_image;
  int y_f32;                  /* 1: y rows are f32 (ldy in floats) instead of bf16               */
  void* dx_bf16; int64_t lddx_bf16; /* bwd, optional: bf16 copy of the (accumulated) dx rows, written
                                       in the same pass (the next dgrad GEMM's operand; no cast kernel) */
  /* bwd, optional (D <= 1024, no pixel shuffle, dx_accumulate): the slx_ls_branch_bwd of the residual branch that
   * precedes this norm in the backward, applied to the updated dx rows in the same pass: ls_g = bf16(dx * ls),
   * ls_dls += sum dx * ls_y, ls_dbias += sum dx * ls (InternViT x = x_in + ls * branch(...), ls != NULL)     */
  const float* ls; const void* ls_y; int64_t ld_ls_y; void* ls_g; int64_t ld_ls_g; float* ls_dls; float* ls_dbias;
  int dy_bf16;                /* bwd: 1 = the dy argument of slx_norm_bwd points to bf16 rows (lddy in elements):
                                 the bf16 gradient a bf16 Linear's backward hands LayerNorm under autocast      */
} slx_norm_desc;
int slx_norm_fwd(const slx_norm_desc* d, slx_stream_t stream);
int slx_norm_bwd(const slx_norm_desc* d, const float* dy, int64_t lddy, float* dx, int64_t lddx,
                 int dx_accumulate, float* dgamma, float* dbeta, int param_accumulate,
                 float* partial_ws, slx_stream_t stream);
int slx_norm_partial_ws_floats(int D);

/* ---- glue kernels ----------------------------------------------------------------------------- */
/* InternViT patch embedding Conv2d(3,1024,k14,s14) as im2col (K padded to kpad) + GEMM.      */
int slx_im2col_patch(const float* pix, int N, int H, int W, int P, int kpad, void* out, slx_stream_t s);
/* x0 = [cls; patches] + pos_embed   (InternVisionEmbeddings; no interpolation at 448)        */
int slx_vit_embed_fwd(const float* patch, const float* cls, const float* pos, float* out, int N, int T, int D, slx_stream_t s);
int slx_vit_embed_bwd(const float* dx, int N, int T, int D, float* dpos, float* dcls, void* dpatch, slx_stream_t s);
/* Qwen2MLP act: silu(gate) * up, gu = [gate | up] (fused gate/up GEMM output)                  */
int slx_swiglu_fwd(const void* gu, int64_t ldgu, void* out, int64_t ldo, int64_t M, int F, slx_stream_t s);
/* bias gradients: out[c] (+)= sum_r x[r,c]; mode 0 bf16 x, 1 f32 x                              */
int slx_colsum(int mode, const void* x, int64_t ldx, int64_t M, int N, float* out, int accumulate, float* ws, slx_stream_t s);
int slx_colsum_ws_floats(int N);
/* InternViT layer-scale branch backward: g = dres*ls (bf16), dls = sum dres*y, dbias = sum g.
 * ls may be NULL (ls = 1: CLIP's plain residual), y and dls NULL together (no layer scale).     */
int slx_ls_branch_bwd(const float* dres, int64_t ldr, const float* ls, const void* y, int64_t ldy, void* g, int64_t ldg,
                      int64_t M, int N, float* dls, float* dbias, int accumulate, float* ws, slx_stream_t s);
/* LLM input assembly (AdaptorList.forward adaptors.py:301-331 + replace_placeholder_tokens
 * internvl2_model.py:44-142 restated as one gather): code = kind<<28 | index,
 * kind 0 token (embed_tokens, ids clamped to V-1), 1 image row, 2 wp_encoder row, 3 query.    */
int slx_assemble_tokens(const int* code, int64_t n, int D, const void* embed, int V, const void* img, const float* wp,
                        const float* query, float* out, slx_stream_t s);
int slx_gather_rows(const float* src, int64_t lds, const int* idx, int64_t n, int D, void* dst, int64_t ldd, int dst_bf16, slx_stream_t s);
int slx_gather_rows_bf16(const void* src, int64_t lds, const int* idx, int64_t n, int D, void* dst, int64_t ldd, slx_stream_t s);
int slx_gather_sum(const float* src, int64_t lds, const int* pos, int B, int nq, int D, float* out, int accumulate, slx_stream_t s);
/* peft LoRA dropout (lora_dropout, llm.py:113) with a counter-hash mask regenerated in backward */
int slx_dropout(const void* src, int64_t lds, void* dst, int64_t ldd, int64_t M, int N, uint64_t seed, float p, int64_t ldmask, slx_stream_t s);
/* LoRA dropout keep masks (peft lora_dropout, llm.py:113) as bits: for each job, bits[row][w] bit c =
 * keep(seed, row*ldmask + 32w + c) (common.h drop_keep: one hash per index pair, 16-bit uniforms, p -> round(p*65536)),
 * rows x cols (cols % 32 == 0, ldmask even). One launch for up to 8 jobs (a layer's 7 sites); every LoRA consumer
 * (slx_lora_down, slx_lora_bwd, the GEMM DROPMASK epilogues) reads these bits.                   */
typedef struct { uint64_t seed; uint32_t* bits; int64_t ldbits; int64_t ldmask; int cols; } slx_dropout_bits_job;
typedef struct {
  int njobs; float p; int64_t rows;
  slx_dropout_bits_job job[8];
} slx_dropout_bits_desc;
int slx_dropout_bits(const slx_dropout_bits_desc* d, slx_stream_t stream);
/* LoRA down-projection of the sites sharing one input (peft LoraLayer.forward lora_A(dropout(x)),
 * llm.py:106-119 / peft lora/layer.py): t[:, 32j:32j+32] = drop_j(x) A_j^T, bf16 out; r must be 32, Kin % 32 == 0.
 * p > 0: the keep mask of site j is read from bits[j] ([M][ldbits] uint32, slx_dropout_bits); seed is unused.
 * A_j is passed in the packed fragment order slx_lora_pack_a writes (refreshed once per optimizer step).  */
typedef struct {
  const void* x; int64_t ldx;         /* bf16 [M, Kin] */
  int64_t M; int Kin; int r; int nsites;
  const void* A[4];                   /* bf16 packed A_j (slx_lora_pack_a), 32 * Kin elements per site */
  uint64_t seed[4];
  void* t; int64_t ldt;               /* bf16 [M, >= 32*nsites] */
  float p; int64_t ldmask;
  const uint32_t* bits[4]; int64_t ldbits;  /* keep bits per site (p > 0), ldbits >= Kin/32 words per row */
  int gen_bits;  /* p > 0: 0 = read the keep bits (slx_dropout_bits wrote them); 1 = GENERATE them from seed[j] /
                  * ldmask while x is read (drop_keep, the same hash as slx_dropout_bits) and write them to bits[j] for
                  * the backward (round 6: no separate keep-bit launch)                                           */
} slx_lora_down_desc;
int slx_lora_down(const slx_lora_down_desc* d, slx_stream_t stream);
/* A [32, Kin] bf16 (row stride lda, the peft lora_A.weight layout) -> Af, a packed fragment order (Kin % 32 == 0):
 * layout 0, read by slx_lora_down:        Af[((2*(k/32) + (k/16)%2) * 64 + r + 32*((k/8)%2)) * 8 + k%8] = A[r][k];
 * layout 1, read by slx_lora_bwd (dx):    Af[((2*(k/32) + r/16) * 64 + k%32 + 32*((r/8)%2)) * 8 + r%8]  = A[r][k]. */
int slx_lora_pack_a(const void* A, int64_t lda, int Kin, int layout, void* Af, slx_stream_t stream);
/* LoRA backward of the sites sharing one input (peft lora_A backward + the dropout's input gradient):
 *   dA_j[32, Kin] += dT_j^T drop_j(x)                     (f32 atomics)
 *   dx[M, Kin]    += sum_j keep_j/(1-p) * (dT_j A_j)      (if dx; or bf16(dx + ...) written to dx_bf16 instead)
 * dT_j = columns 32j..32j+31 of dt (f32 [M, >= 32*nsites]: the extra columns of the fused [dy | s dy B] dgrad GEMM).
 * keep_j from bits[j] (slx_dropout_bits); p == 0: no mask. Kin % 128 == 0.                        */
typedef struct {
  const void* x; int64_t ldx;         /* bf16 [M, Kin] (undropped forward input) */
  int64_t M; int Kin; int r; int nsites;
  const float* dt; int64_t lddt;      /* f32 [M, >= 32*nsites] (bf16 with dt_bf16) */
  const void* A[4];                   /* bf16 packed A_j, slx_lora_pack_a layout 1 (read by the dx term only) */
  const uint32_t* bits[4]; int64_t ldbits;
  float* dA[4];                       /* f32 [32, Kin] per site, accumulated; all NULL: dx only (the dA pass can
                                         then run on another stream: nothing downstream in the backward reads it) */
  float* dx; int64_t lddx;            /* f32 [M, Kin] or NULL (no input gradient) */
  void* dx_bf16; int64_t lddx_bf16;   /* optional bf16 [M, Kin] output instead of updating dx in place */
  float p;
  int dt_bf16;                        /* 1: dt points to bf16 rows (lddt % 8 == 0), e.g. the bf16 dgrad GEMM output */
  void* dt_bf16_out; int64_t ld_dt_bf16_out;  /* optional bf16 [M, 32*nsites]: the dx term also writes dT as bf16 here
                                                 (the operand slx_lora_grad takes) */
} slx_lora_bwd_desc;
int slx_lora_bwd(const slx_lora_bwd_desc* d, slx_stream_t stream);
/* The same with dA summed without atomics: each (column block, row chunk) block stores its f32 partial into ws and a
 * second launch adds the row chunks' partials into dA_j in a fixed order (deterministic). ws_floats must be at least
 * slx_lora_bwd_ws_floats(M, Kin, nsites) (a smaller ws is an argument error). */
int64_t slx_lora_bwd_ws_floats(int64_t M, int Kin, int nsites);
int slx_lora_bwd_ws(const slx_lora_bwd_desc* d, float* ws, int64_t ws_floats, slx_stream_t stream);
/* The LoRA parameter gradients of one layer group in ONE launch: per job, out_j += alpha * t_j^T . x_j' over the M rows,
 * where x_j' = x (B gradients: x = the site's output gradient dy [M][n], t = its forward down-projection t_j, alpha = s,
 * out_nr = 1: out is the [n][32] B gradient) or x_j' = bf16(x / (1-p)) & keep_j (A gradients: x = the site input,
 * t = dT_j, alpha = 1, out_nr = 0: out is the [32][n] A gradient; up to 3 sites share one x). Replaces the dB
 * split-K GEMMs and the dA part of slx_lora_bwd (peft lora_B / lora_A weight gradients, llm.py:106-119).
 * n % 128 == 0, ldx % 8, x 16-B aligned; t bf16 [M][32*nsites], 16-B aligned, ldt % 8 (t_bf16 must be 1: a dT
 * that lives in f32 comes as bf16 from slx_lora_bwd's dt_bf16_out); at most 12 jobs.                              */
typedef struct slx_lora_grad_job {
  const void* x; int64_t ldx; int n;
  const void* t; int64_t ldt; int t_bf16;
  int nsites;
  const uint32_t* bits[3]; int64_t ldbits; float p;
  float alpha;
  float* out[3]; int out_nr;
} slx_lora_grad_job;
int slx_lora_grad(const slx_lora_grad_job* jobs, int njobs, int64_t M, slx_stream_t s);
/* The down site's LoRA dgrad fused with the SwiGLU backward (Qwen2MLP, llm.py:106-119 peft lora on down_proj):
 * dgu[m, f] = d * u * silu'(g), dgu[m, F + f] = d * silu(g) with d = resid[m, f] + keep[m, f] (dT . A)[m, f] / (1 - p),
 * g = gu[m, f], u = gu[m, F + f]. dT bf16 [M][>= 32] (the fused dgrad GEMM's LoRA columns), at = A^T bf16 [F][32]
 * (lora_A.weight transposed), resid bf16 [M][F] (the base dgrad dact), gu bf16 [M][2F] (the gate|up GEMM output), bits
 * the forward's keep bits [M][>= F/32] (p > 0). F % 256 == 0, 16-B aligned rows.                                  */
typedef struct slx_lora_swiglu_bwd_desc {
  const void* dt; int64_t lddt;
  const void* at; int64_t ldat;
  const void* resid; int64_t ldr;
  const void* gu; int64_t ldgu;
  const uint32_t* bits; int64_t ldbits;
  float p;
  void* dgu; int64_t lddgu;
  int64_t M; int F;
} slx_lora_swiglu_bwd_desc;
int slx_lora_swiglu_bwd(const slx_lora_swiglu_bwd_desc* d, slx_stream_t stream);
/* slx_lora_swiglu_bwd plus three LoRA parameter gradients from the same pass (the peft lora_A / lora_B weight grads of
 * Qwen2MLP's down and gate/up sites, llm.py:106-119), so neither the 2F-wide dgu nor act is read again:
 *   dA_down [32][F] += dT^T . drop(act),  act = bf16(silu(g) * u) (the forward's activation, recomputed bit-exactly),
 *                      drop(act) = bf16(act / (1 - p)) & keep (the down site's keep bits, as in the dgrad term);
 *   dB_gate [F][32] += alpha_b * dgu[:, :F]^T . tg,  dB_up [F][32] += alpha_b * dgu[:, F:]^T . tu  (bf16 dgu as stored);
 * tg / tu bf16 [M][32]: the gate / up sites' forward t = drop(x) . A^T. Row-group partials go to ws (size from
 * slx_lora_swiglu_bwd_grads_ws_floats) and are summed in row-group order by a second launch (deterministic in every
 * mode); F % 128 == 0. dgu is bitwise what slx_lora_swiglu_bwd writes.                                           */
typedef struct slx_lora_swiglu_bwd_grads_desc {
  slx_lora_swiglu_bwd_desc sw;
  const void* tg; const void* tu; int64_t ldtg;
  float* dA_down; float* dB_gate; float* dB_up;
  float alpha_b;
  float* ws; int64_t ws_floats;
} slx_lora_swiglu_bwd_grads_desc;
int64_t slx_lora_swiglu_bwd_grads_ws_floats(int64_t M, int F);
int slx_lora_swiglu_bwd_grads(const slx_lora_swiglu_bwd_grads_desc* d, slx_stream_t stream);
/* The SwiGLU forward fused with the down site's LoRA down-projection (Qwen2MLP act_fn(gate) * up, then peft lora_A
 * on down_proj with its dropout; llm.py:106-119): act = bf16(silu(g) * u) from gu bf16 [M][2F] (the gate|up GEMM
 * output), written to act [M][F], and t = drop(act) . A^T written as bf16 to t [M][32], drop(x) = bf16(x / (1 - p)) &
 * keep (the forward's keep bits [M][>= F/32], p > 0). A = lora_A bf16 [32][F]. ws: f32 scratch of
 * slx_swiglu_lora_down_ws_floats(M, F) floats (per-column-block partials of t, summed in order by a second launch).
 * F % 256 == 0.                                                                                                      */
typedef struct slx_swiglu_lora_down_desc {
  const void* gu; int64_t ldgu;
  void* act; int64_t ldact;
  const void* A; int64_t lda;
  const uint32_t* bits; int64_t ldbits;
  float p;
  void* t; int64_t ldt;
  float* ws; int64_t ws_floats;
  int64_t M; int F;
  uint64_t seed; int gen_bits;  /* p > 0 and gen_bits: the keep bits are generated here (seed, ldmask = F) and
                                 * written to bits, as slx_lora_down's gen_bits                              */
} slx_swiglu_lora_down_desc;
int slx_swiglu_lora_down(const slx_swiglu_lora_down_desc* d, slx_stream_t stream);
int64_t slx_swiglu_lora_down_ws_floats(int64_t M, int F);

/* small strided f32 GEMM (driving heads adaptors.py:113-132, WaypointInputAdaptor :80)        */
enum { SLX_ACT_NONE = 0, SLX_ACT_RELU = 1, SLX_ACT_SILU = 2 };
typedef struct slx_sgemm_desc {
  int M, N, K, act, accumulate;
  const float* A; int64_t sam, sak;
  const float* B; int64_t sbk, sbn;
  float* C; int64_t scm, scn;
  const float* bias;
  float* pre; int64_t ldpre;   /* optional pre-activation output [M][ldpre] */
  float alpha;
} slx_sgemm_desc;
int slx_sgemm(const slx_sgemm_desc* d, slx_stream_t s);
int slx_act_bwd(const float* dact, const float* pre, float* dpre, int64_t n, int act, slx_stream_t s);

/* ---- losses ---------------------------------------------------------------------------------
 * LanguageAdaptor.compute_loss (adaptors.py:259-274) on the gathered loss rows only,
 * DrivingAdaptor.compute_loss (adaptors.py:183-221: cumsum + smooth_l1(beta 1).sum(-1)),
 * summarise_losses (models/utils.py:7-41).                                                      */
int slx_ce_fwd(const float* logits, int64_t ld, const int* labels, int64_t R, int V, float* loss, float* lse, slx_stream_t s);
int slx_ce_bwd(const float* logits, int64_t ld, const int* labels, const float* lse, int64_t R, int V, const float* gscale,
               void* dlogits, int64_t ldd, slx_stream_t s);
/* Fused LM head + CE over the R gathered loss rows (the training step; replaces lm_head + slx_ce_fwd / slx_ce_bwd and
 * their f32 [R, V] logits): feat [R][D] bf16 (ld ldf), W = lm_head [>=V][D] bf16 (ld ldw), labels [R] (-1 ignored).
 * fwd: the LM-head GEMM's epilogue reduces each row's logits to (max, sum exp) per 64-column sub-tile and the label
 * logit into ws (slx_lmhead_ce_ws_floats(R, V) floats); a combine pass writes loss[R] and lse[R].
 * bwd: the GEMM recomputed with the softmax-gradient epilogue: dlogits [R][ldd] bf16 = (softmax - onehot) * gscale[0],
 * zero past V (ldd >= V rounded up to 128), the operand of the dlogits x lm_head dgrad.                         */
int slx_lmhead_ce_ws_floats(int64_t R, int V);
int slx_lmhead_ce_fwd(const void* feat, int64_t ldf, const void* W, int64_t ldw, const int* labels, int64_t R, int V,
                      int D, float* loss, float* lse, float* ws, int64_t ws_floats, slx_stream_t s);
int slx_lmhead_ce_bwd(const void* feat, int64_t ldf, const void* W, int64_t ldw, const int* labels, const float* lse,
                      int64_t R, int V, int D, const float* gscale, void* dlogits, int64_t ldd, slx_stream_t s);
/* kind 0: smooth_l1(beta=1).sum(-1) per point (simlingo_training adaptors.py:205-213);
 * kind 1: mse.sum(-1) per point (simlingo_base_training adaptors.py:226)                       */
int slx_wp_loss_fwd(const float* out, const float* label, int B, int n, int dims, int kind, float* pred, float* loss,
                    slx_stream_t s);
int slx_wp_loss_bwd(const float* pred, const float* label, int B, int n, int dims, int kind, const float* gscale,
                    float* dout, slx_stream_t s);
int slx_loss_finalize(const float* lang, int nl, const float* route, int nr, const float* speed, int ns, float* out, slx_stream_t s);
/* gs[0..2] = (dl[0] + dl[1+i]) / n_i : per-item gradient scales from the upstream grads of
 * [total, lang, route, speed] (dl may be NULL -> d total = 1).                                 */
int slx_loss_gscale(const float* dl, int nl, int nr, int ns, float* gs, slx_stream_t s);
int slx_scatter_rows(const float* src, int64_t lds, const int* idx, int64_t n, int D, float* dst, int64_t ldd, int accumulate, slx_stream_t s);
int slx_gather_rows_b2f(const void* src, int64_t lds, const int* idx, int64_t n, int D, float* dst, int64_t ldd, slx_stream_t s);
/* SwiGLU backward from f32 d(act) (used when LoRA adds to d(act) before the activation backward) */
int slx_swiglu_bwd(const float* dact, int64_t ldd, const void* gu, int64_t ldgu, void* dgu, int64_t lddgu, int64_t M, int F, slx_stream_t s);
int slx_cast_rows(const float* src, int64_t lds, void* dst, int64_t ldd, int64_t M, int N, slx_stream_t s);

/* ---- optimizer (torch.optim.AdamW semantics, driving.py:718-724; clip_grad_norm 0.3, train.py:206) */
int slx_sumsq(const float* g, int64_t n, float* out, int zero_first, slx_stream_t s);
/* grad_scale multiplies the gradient (1/world after a SUM all-reduce); clipping uses the scaled norm */
int slx_adamw(float* p, const float* g, float* m, float* v, void* p_bf16, int64_t n, float lr, float beta1, float beta2,
              float eps, float weight_decay, int step, const float* sumsq, float max_norm, float grad_scale, slx_stream_t s);
/* The same clip + AdamW, and the sum of squares, reading the gradients as bf16: the summed data-parallel gradient on
 * the bf16 all-reduce wire (simlingo_amd/ddp.py wire="bf16"), scaled by grad_scale (1/world) and widened to f32 inside
 * the kernel, so no cast-back pass runs between the last all-reduce and the optimizer (train.py:160-168).          */
int slx_adamw_bf16g(float* p, const void* g_bf16, float* m, float* v, void* p_bf16, int64_t n, float lr, float beta1,
                    float beta2, float eps, float weight_decay, int step, const float* sumsq, float max_norm,
                    float grad_scale, slx_stream_t s);
int slx_sumsq_bf16(const void* g_bf16, int64_t n, float* out, int zero_first, slx_stream_t s);
/* The same sum of squares as per-block partials in `ws` (>= SLX_SUMSQ_PARTS floats) summed in block order: bitwise
 * reproducible, so data-parallel replicas that hold identical summed gradients compute the identical clip factor and
 * stay bitwise identical (torch's clip_grad_norm_ reduces in a fixed order too, train.py:206). The engines use these. */
#define SLX_SUMSQ_PARTS 2048
int slx_sumsq_ws(const float* g, int64_t n, float* out, int zero_first, float* ws, int64_t ws_floats, slx_stream_t s);
int slx_sumsq_bf16_ws(const void* g_bf16, int64_t n, float* out, int zero_first, float* ws, int64_t ws_floats,
                      slx_stream_t s);
int slx_cast_f32_bf16(const float* src, void* dst, int64_t n, slx_stream_t s);

/* ---- SimLingo-Base (LLaVA-NeXT CLIP encoder + tiny Llama, BASELINE configs[1]) ----------------- */
/* NormZeroOne (simlingo_base_training/models/driving.py:89-103): out = x * scale + shift        */
int slx_affine(const float* x, int64_t n, float scale, float shift, float* out, slx_stream_t s);
/* out = a + b + c (projection bias + temporal_encoding + camera_encoding, llavanext.py:98-110)  */
int slx_vec_sum3(const float* a, const float* b, const float* c, int64_t n, float* out, slx_stream_t s);
/* LingoLlavaNextModel.forward_image spatial merge (llavanext_model.py:128-157): per image the
 * npatch_h x npatch_w patches of g x g projector rows -> unpad_image rows [r0, r0+hu) x cols
 * [c0, c0+wu) -> avg_pool2d(pool) -> + image_newline column: slx_llava_merge_tokens() rows of C.
 * src/out bf16; bwd: dsrc (bf16, every source row; 0 where unpadded away) from dout (f32).      */
int slx_llava_merge_tokens(int hu, int wu, int pool);
int slx_llava_merge_fwd(const void* src, int C, int64_t n_img, int npatch_h, int npatch_w, int g, int r0, int hu, int c0,
                        int wu, int pool, const float* newline, void* out, slx_stream_t s);
int slx_llava_merge_bwd(const float* dout, int C, int64_t n_img, int npatch_h, int npatch_w, int g, int r0, int hu, int c0,
                        int wu, int pool, void* dsrc, slx_stream_t s);
/* table: n device-resident entries {src f32*, lds, dst*, ldd, rows, cols, float-bits scale, mode}:
 * dst = src * scale, mode 0 bf16, 1 f32 (the fp32 parity mode), 2 bf16 in slx_lora_pack_a's fragment order
 * (rows == 32), 3 bf16 in layout 1 of slx_lora_pack_a, 4 bf16 transposed (dst[c * ldd + r]).
 * Packs LoRA B (scaled by lora_alpha/r) into the fused
 * [W | s*B] operands and LoRA A into the packed copies slx_lora_down / slx_lora_bwd read, once per optimizer step. */
int slx_pack_scaled(const int64_t* table, int n, slx_stream_t s);
/* The same packing over a flat grid of equal chunks (round 6): block b packs chunk block_map[b] >> 16 (SLX_PACK_CHUNK
   elements) of entry block_map[b] & 0xFFFF (n <= 65536); block_map: nblocks device int32 built by the caller. One
   block per 2048 elements instead of 32 blocks per entry whatever its size. */
#define SLX_PACK_CHUNK 2048
int slx_pack_scaled_flat(const int64_t* table, int n, const int* block_map, int nblocks, slx_stream_t s);
/* table: n device-resident entries {src bf16*, lds, dst bf16*, ldd, rows, cols}: dst[c][r] = src[r][c].
 * max_tiles >= the largest ceil(rows/64)*ceil(cols/64) of the entries. Refreshes the [in][out] copies of the
 * weights whose data-gradient GEMM then runs in the NT layout (no reference counterpart: a layout choice of
 * this implementation for torch.nn.Linear's backward, dX = dY W). */
int slx_transpose_bf16(const int64_t* table, int n, int64_t max_tiles, slx_stream_t s);

/* ---- KV-cached greedy decode (agent call, BASELINE configs[4]) -------------------------------------
 * Replaces the no-cache loop of LLM.greedy_sample (simlingo_training/models/language_model/llm.py:
 * 178-250, called from DrivingModel.forward driving.py:131-176): the prefix runs once through the
 * batched kernels above; every further token is slx_dec_begin + per layer {QKV GEMV (RMSNorm fused,
 * row `pos` of the layer's q|k|v cache), slx_dec_attn (RoPE fused), O GEMV (+residual), gate/up GEMV
 * (RMSNorm + SwiGLU fused), down GEMV (+residual)} + LM-head GEMV with the argmax folded in.
 * Per-step scalars live in device memory (hipGraph-capturable); after EOS every kernel early-exits.*/
typedef struct slx_dec_state {
  int pos;      /* position of the token being processed (prefill leaves S0 - 1)               */
  int n_gen;    /* tokens recorded so far                                                       */
  int done;     /* 1 after EOS / max_new tokens were recorded                                   */
  int max_new;  /* max_new_tokens (llm.py:181)                                                  */
  int eos;      /* eos_token_id (driving.py:136-141)                                            */
  int pad[3];
} slx_dec_state;
enum { SLX_DEC_STORE_ROW = 0, SLX_DEC_RESID = 1, SLX_DEC_SWIGLU = 2, SLX_DEC_ARGMAX = 3 };
typedef struct slx_dec_gemv_desc {
  int mode;
  const void* W; int64_t ldw; int N; int K;   /* W bf16 [N][K] (SWIGLU: gate rows [0,N), up [N,2N)) */
  const float* X; const float* gamma; float eps; /* input = RMSNorm(X f32 [K]) * gamma, or ...      */
  const void* xb;                               /* ... a bf16 vector [K]                            */
  const float* bias;
  void* out; int64_t out_ld;                    /* STORE_ROW: bf16 row state->pos; SWIGLU: bf16 [N] */
  float* resid;                                 /* RESID: resid[n] += y                            */
  unsigned long long* keys;                     /* ARGMAX: slx_dec_key_shards() u64 keys (zeroed)  */
  const slx_dec_state* state;                   /* NULL -> pos 0, never done                        */
} slx_dec_gemv_desc;
int slx_dec_key_shards(void);
/* record the token of the previous step (argmax keys -> tokens[n_gen]), X = embed[token] f32     */
int slx_dec_begin(slx_dec_state* st, unsigned long long* keys, const void* embed, int D, float* X, int* tokens,
                  slx_stream_t s);
int slx_dec_gemv(const slx_dec_gemv_desc* d, slx_stream_t s);
/* one query row (cache row state->pos) over cache rows [0, pos]; q/k rotated with cos/sin row pos;
 * split over keys (slx_dec_attn_nsplit(lmax) workgroups per kv head, partials in ws), merged in the
 * same launch by the last-arriving workgroup of each kv head (arrival counters at the end of ws: ws
 * must be zeroed once before first use; every call leaves the counters at 0 again);
 * out bf16 [Hq*64]; lmax = cache rows allocated (the split count is fixed by it: graph-safe)      */
int slx_dec_attn_nsplit(int lmax);
/* tools only: record phase timestamps (wall_clock64 ticks) of the next slx_dec_attn launches into buf
 * (>= 64 + Hkv * nsplit int64); NULL turns tracing off                                                  */
void slx_dec_attn_set_trace(long long* buf);
/* tests / tools only: 1 = use the split form even for caches of <= 1024 rows (which otherwise run one MFMA
 * workgroup per kv head, no split)                                                                        */
void slx_dec_attn_force_split(int on);
/* the attention split over keys WITHOUT an in-launch merge (SLX_DEC_SPLIT_NS workgroups per kv head, default 8, each
 * at most 8 key blocks of 32: lmax <= 256 * ns; partials in ws, sized by slx_dec_attn_ws_floats), then the O GEMV +
 * residual X[n] += W_o[n, :] . out, whose prologue merges the partials (two launches, no counters). out (optional, bf16
 * [Hq*64]) receives the merged attention output. Replaces slx_dec_attn + the O GEMV (the o_proj call of
 * Qwen2Attention inside llm.py:178-250's greedy loop).                                                          */
int slx_dec_attn_o_split(void* cache, int64_t ld, int Hq, int Hkv, const float* cos_tab, const float* sin_tab,
                         int lmax, float* ws, void* out, const slx_dec_state* st, const void* Wo, int64_t ldwo, int N,
                         int K, float* X, slx_stream_t s);
/* 1 if slx_dec_attn_o_split supports a cache of lmax rows under this process's SLX_DEC_SPLIT_NS, else 0 (the caller
 * then runs slx_dec_attn + the O GEMV)                                                                           */
int slx_dec_attn_o_split_ok(int lmax);
int slx_dec_attn_ws_floats(int Hq, int Hkv, int lmax);
int slx_dec_attn(void* cache, int64_t ld, int Hq, int Hkv, const float* cos_tab, const float* sin_tab, int lmax,
                 float* ws, void* out, const slx_dec_state* st, slx_stream_t s);

/* ---- collate image path: uint8 frames -> InternVL2 pixel tiles (csrc/frames.hip) --------
 * Replaces preprocess_image_batch (simlingo_training/utils/internvl2_utils.py:179-203) per batch: the bottom crop
 * (dataloader/dataset_base.py:464-467) is a row count, dynamic_preprocess (internvl2_utils.py:231-266) picks the
 * grid on the host, and one kernel does Pillow's BICUBIC Image.resize (Resample.c ImagingResample, bit-exact
 * uint8), the 448-tile crop, ToTensor and Normalize (build_transform, internvl2_utils.py:206-214).
 * slx_resample_ksize / slx_resample_coeffs are host functions (no GPU): Pillow's precompute_coeffs +
 * normalize_coeffs_8bpc for one axis, in_size -> out_size, box = whole axis; bounds[2*o] = first source
 * index, bounds[2*o+1] = tap count, kk[o*kmax + j] = 22-bit fixed-point weight. Returns ksize (or < 0). */
int slx_resample_ksize(int in_size, int out_size);
int slx_resample_coeffs(int in_size, int out_size, int kmax, int32_t* bounds, int32_t* kk);
typedef struct {
  const uint8_t* src;               /* frames, element strides: frame sb, row sy, pixel sx, channel sc (RGB)  */
  int64_t sb, sy, sx, sc;
  int B, H, W;                      /* H = rows kept by the bottom crop (rows 0..H-1 are read)                */
  int tw, th, tile;                 /* resized size (multiples of tile) and tile edge (448)                    */
  const int32_t* hbounds;           /* device: slx_resample_coeffs(W, tw) tables (unused when need_h == 0)      */
  const int32_t* hcoeffs;
  int hksize;
  const int32_t* vbounds;           /* device: slx_resample_coeffs(H, th) tables (unused when need_v == 0)      */
  const int32_t* vcoeffs;
  int vksize;
  int need_h, need_v;               /* Pillow skips a pass (and its rounding) when that axis keeps its size     */
  int rows_per_block, cols_per_block; /* output rows x columns per block                                     */
  int lds_rows, lds_cols;           /* max source rows / columns any block reads (LDS window <= 64 KiB)        */
  float mean[3], std[3];            /* Normalize constants as f32 (IMAGENET_MEAN / IMAGENET_STD)               */
  float* out;                       /* [B][tiles][3][tile][tile] f32, tile t = row-major over the tile grid     */
} slx_frame_desc;
int slx_frames_to_tiles(const slx_frame_desc* d, slx_stream_t stream);

/* ---- fp32 parity mode (SURVEY.md §7 hard part 2; csrc/precise.hip) ---------------------------
 * f32 twins of the bf16-only forward entry points, used by VLAEngine / BaseEngine(precise=True) to run the
 * engines' own launch sequence with f32 activations and weights, so the forward can be held to the north-star
 * tolerance (waypoint L2 <= 1e-4 m, LM CE <= 1e-4) against the reference fixtures. Same arguments and meaning
 * as the bf16 entry point named; every void* operand is f32. Not tuned.                              */
int slx_gemm_f32(const slx_gemm_desc* d, slx_stream_t stream);        /* slx_gemm_bf16, epilogues STORE /
                                                       GELU / QGELU / RESID_LS / GELU_BWD / QGELU_BWD (no colsum) */
int slx_attn_fwd_f32(const slx_attn_desc* d, slx_stream_t stream);    /* slx_attn_fwd                     */
int slx_rope_f32(void* x, int64_t ldx, int64_t ntok, int S, int nheads, const float* cos_tab,
                 const float* sin_tab, int inverse, slx_stream_t stream);                 /* slx_rope */
int slx_swiglu_fwd_f32(const void* gu, int64_t ldgu, void* out, int64_t ldo, int64_t M, int F, slx_stream_t s);
int slx_im2col_patch_f32(const float* pix, int N, int H, int W, int P, int kpad, void* out, slx_stream_t s);
int slx_assemble_tokens_f32(const int* code, int64_t n, int D, const void* embed, int V, const void* img,
                            const float* wp, const float* query, float* out, slx_stream_t s);
int slx_llava_merge_fwd_f32(const void* src, int C, int64_t n_img, int npatch_h, int npatch_w, int g, int r0,
                            int hu, int c0, int wu, int pool, const float* newline, void* out, slx_stream_t s);
/* backward twins (the trained path at the north-star tolerance, VLAEngine(precise=True).backward) */
int slx_attn_bwd_f32(const slx_attn_desc* d, const slx_attn_bwd_desc* g,
                     slx_stream_t stream);                        /* slx_attn_bwd without RoPE / dbias: dq, dk, dv of the
                                                                     rotated q / k (callers apply slx_rope_f32 inverse
                                                                     and slx_colsum); delta_ws [B, Hq, S] required */
int slx_swiglu_bwd_f32(const float* dact, int64_t ldd, const void* gu, int64_t ldgu, void* dgu, int64_t lddgu,
                       int64_t M, int F, slx_stream_t s);        /* slx_swiglu_bwd                       */
int slx_mul_f32(int mode, const float* x, int64_t ldx, const float* y, int64_t ldy, float* out, int64_t ldo,
                int64_t M, int N, slx_stream_t s);               /* out = x*y (mode 0) or x*y[col] (1): the
                                                                     layer-scale branch products of slx_ls_branch_bwd */
int slx_ce_bwd_f32(const float* logits, int64_t ld, const int* labels, const float* lse, int64_t R, int V,
                   const float* gscale, float* dlogits, int64_t ldd, slx_stream_t s);     /* slx_ce_bwd  */
int slx_vit_embed_bwd_f32(const float* dx, int N, int T, int D, float* dpos, float* dcls, float* dpatch,
                          slx_stream_t s);                       /* slx_vit_embed_bwd                    */

/* ---- on-box calibration (the bf16 MFMA ceiling measured on the box, reported beside the spec) ------ */
/* grid workgroups of 4 waves, each wave iters x 4 back-to-back v_mfma_f32_32x32x16_bf16 on random register operands;
 * FLOPs = grid * 4 * iters * 4 * 32768; out >= grid * 256 floats (the reduced accumulators, so the loop is live)   */
int slx_mfma_peak(int grid, int iters, float* out, slx_stream_t s);

#ifdef __cplusplus
}
#endif
#endif /* SLX_H_ */
