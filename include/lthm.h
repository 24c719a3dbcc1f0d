/*
 * lthm.h — C ABI of the MI355X (gfx950) LTHM training hot path.
 *
 * Every entry point takes plain device pointers, element counts and a
 * hipStream_t passed as `void*`; nothing in here depends on torch.  All buffers
 * are caller-allocated (the Python host layer uses the torch caching
 * allocator); the library owns no device memory.  Return value: 0 on success,
 * otherwise a hipError_t code (1 = hipErrorInvalidValue for bad arguments).
 * Launches are stream-ordered and never synchronise the host.
 *
 * dtype codes: LTHM_F32 = 0, LTHM_BF16 = 1.
 *
 * Each function cites the reference interface it replaces
 * (paths relative to the reference repository ranjanbalappa-nykaa/recommendations).
 */
#ifndef LTHM_H_
#define LTHM_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LTHM_ABI_VERSION 43 /* bumped on any signature / struct layout change */

#define LTHM_F32 0
#define LTHM_BF16 1
#define LTHM_FP8_E4M3 2 /* OCP e4m3fn (gfx950), GEMM operands only */

/* KShift finalisation modes */
#define LTHM_KSHIFT_SCALE 0      /* x / sqrt(K)               commons/layers.py:170 */
#define LTHM_KSHIFT_NORMALIZE 1  /* F.normalize(x, 2, -1)     commons/layers.py:168 */
#define LTHM_KSHIFT_NONE 2       /* plain sum (FlatEmbedding, K = 1)               */

/* ------------------------------------------------------------------------- */
/* version / capability                                                      */
/* ------------------------------------------------------------------------- */
/* returns LTHM_ABI_VERSION of the built library */
int lthm_abi_version(void);
/* number of gfx950 devices visible (0 on a host without a GPU); never fails */
int lthm_device_count(void);

/* ------------------------------------------------------------------------- */
/* Embedding gather / pool — commons/layers.py                               */
/* ------------------------------------------------------------------------- */

/* KShiftEmbedding.get_row_idx for every (id, c), c = 0..K-1.
 * rows[i*K + c] = row of ids[i] for rotation c.  Replaces commons/layers.py:174-185. */
int lthm_kshift_rows(const int64_t* ids, int64_t n, int64_t P, int32_t K,
                     int64_t* rows, void* stream);

/* KShiftEmbedding.forward (commons/layers.py:152-172) fused: K row indices,
 * in-order fp32 sum of the K table rows, then x / sqrt(K) or F.normalize.
 * W: [P, D] (w_dtype), out: [n, D] (out_dtype), norms: optional [n] f32
 * (pre-normalisation L2 norm, needed by the normalize backward).
 * Row offset `row_base` is added to every row (table-batched storage). */
int lthm_kshift_fwd(const int64_t* ids, int64_t n, const void* W, int32_t w_dtype,
                    int64_t P, int64_t row_base, int32_t D, int32_t K, int32_t mode,
                    void* out, int32_t out_dtype, float* norms, void* stream);

/* Same as lthm_kshift_fwd for F features stored in one table-batched weight:
 * ids [n, F]; feature f uses rows [f*P, (f+1)*P) of W [F*P, D]; out [n, F, D]. */
int lthm_kshift_fwd_multi(const int64_t* ids, int64_t n, int32_t F, const void* W,
                          int32_t w_dtype, int64_t P, int32_t D, int32_t K, int32_t mode,
                          void* out, int32_t out_dtype, float* norms, void* stream);
/* lthm_kshift_fwd_multi writing item (b, f)'s row at out + b * out_ld + f * D (elements): the F x D
 * rows of a sample inside a wider row, e.g. the ranker's MLP input [dense | F tables], built without a
 * concatenation pass (round 6, ABI 42).  out_ld > F * D needs K = 1. */
int lthm_kshift_fwd_multi_ld(const int64_t* ids, int64_t n, int32_t F, const void* W, int32_t w_dtype, int64_t P,
                             int32_t D, int32_t K, int32_t mode, void* out, int32_t out_dtype, int64_t out_ld,
                             float* norms, void* stream);

/* Item-embedding artifact forward (embedding_module_gen.py:32-41 ModelWrapper, consumed
 * at encoder.py:25-29 via torch.jit.load): out[i] = KShift_K(ids[i]; W [P, D], mode)
 * * sigmoid(w2 . QuickGELU(W1 m + b1) + b2) with m = KShift_Km(ids[i]; Wm [Pm, Dm]) / sqrt(Km)
 * (the mask model: KShiftEmbedding(normalize_output=False) -> commons MLP with one
 * hidden layer, W1 [H1, Dm], b1 [H1], w2 [H1], b2 [1]; all f32).  Dm % 4 == 0, Dm <= 16,
 * H1 <= 256, Wm 16-B aligned; W f32 or bf16, out f32 or bf16 [n, D].  Forward only. */
int lthm_item_artifact_fwd(const int64_t* ids, int64_t n, const void* W, int32_t w_dtype, int64_t P, int32_t D,
                           int32_t K, int32_t mode, const float* Wm, int64_t Pm, int32_t Dm, int32_t Km,
                           const float* W1, const float* b1, int32_t H1, const float* w2, const float* b2, void* out,
                           int32_t out_dtype, void* stream);

/* Pool K rows of a gathered buffer W [R, D] given explicit row indices
 * rows [n, K] (< R): same in-order f32 sum and finalisation as lthm_kshift_fwd.
 * The row-sharded item table (C3) pools the rows its all_to_all exchange
 * returned with it, bit-identical to the unsharded gather. */
int lthm_gather_pool(const int64_t* rows, int64_t n, int32_t K, const void* W, int32_t w_dtype, int64_t R, int32_t D,
                     int32_t mode, void* out, int32_t out_dtype, float* norms, void* stream);
/* Backward of lthm_kshift_fwd(_multi) into a dense f32 gradient dW [F*P, D]
 * (accumulated, caller zeroes).  LDS-staged dedup: each workgroup sorts its
 * (row, id) pairs in LDS, reduces duplicate rows wave-segment-wise, and emits
 * one f32 add per unique row.  dY: [n, F, D] (dy_dtype); out/norms are the
 * forward's output and norms (only read for LTHM_KSHIFT_NORMALIZE).
 * F = 1 for the single-table form. */
int lthm_kshift_bwd_dense(const int64_t* ids, int64_t n, int32_t F, const void* dY,
                          int32_t dy_dtype, const void* out, int32_t out_dtype,
                          const float* norms, int64_t P, int32_t D, int32_t K,
                          int32_t mode, float* dW, void* stream);

/* Same, plus the touched-row list for the sparse row-wise optimizers: the first
 * add to a row sets flags[row] (int32 [F*P], caller keeps it zeroed; lthm_sparse_adamw /
 * lthm_sparse_adagrad re-zero the entries of the rows they update, or none with flags = NULL) and appends
 * the row to list (int64 [>= n*F*K]) at atomic index *count (int64, zeroed). */
int lthm_kshift_bwd_sparse(const int64_t* ids, int64_t n, int32_t F, const void* dY,
                           int32_t dy_dtype, const void* out, int32_t out_dtype,
                           const float* norms, int64_t P, int32_t D, int32_t K, int32_t mode,
                           float* dW, int32_t* flags, int64_t* list, int64_t* count, void* stream);
/* The K = 1, plain-output case of lthm_kshift_bwd_sparse (FlatEmbedding / table-batched flat
 * lookups, the C4 ranker: commons/layers.py:56-61's nn.Embedding backward) with the rows of
 * first touch STORED: the item that sets the row's bit writes its row of dW (no prior contents
 * needed: rows are stored, not accumulated), every other item of a touched row is added
 * afterwards with f32 atomics.  flags here is a BITMAP: bit (row & 31) of 32-bit word row >> 5,
 * [>= ceil(F * P / 32)] words, kept zeroed by the caller (the row-wise optimizer clears it whole
 * after its step).  dup_ws: int64 [>= n * F + 1] workspace.  Same dW / list / count result as
 * lthm_kshift_bwd_sparse with K = 1, mode LTHM_KSHIFT_SCALE, up to the f32 summation order of
 * duplicated rows. */
int lthm_kshift_bwd_sparse_first(const int64_t* ids, int64_t n, int32_t F, const void* dY, int32_t dy_dtype,
                                 int64_t P, int32_t D, float* dW, int32_t* flags, int64_t* list, int64_t* count,
                                 int64_t* dup_ws, int64_t dup_cap, void* stream);
/* lthm_kshift_bwd_sparse_first reading item (b, f)'s gradient row at dY + b * dy_ld + f * D
 * (the gradient of the strided lthm_kshift_fwd_multi_ld output, in place in the wider row). */
int lthm_kshift_bwd_sparse_first_ld(const int64_t* ids, int64_t n, int32_t F, const void* dY, int32_t dy_dtype,
                                    int64_t dy_ld, int64_t P, int32_t D, float* dW, int32_t* flags, int64_t* list,
                                    int64_t* count, int64_t* dup_ws, int64_t dup_cap, void* stream);

/* Fused dedup + row-wise Adagrad of a KShift table: lthm_kshift_bwd_sparse followed by
 * lthm_sparse_adagrad_ex in one call, with no gradient row stored.  For the item-embedding
 * generator, whose tables step right after their backward with torch.optim.Adagrad and nothing
 * in between (embedding_module_gen.py:137,151-153 and :97-99,113-115): the pairs (row, item) of
 * every (item, shift) are radix-sorted by row (stable, so a row's pairs stay in item order), each
 * row's gradient -- sum over its pairs of the item's pooled-sum gradient (dy / sqrt(K), dy, or the
 * F.normalize backward, as lthm_kshift_bwd_sparse) -- is summed in that order and the row updated
 * once, unfused f32:  s = s + g * g;  W = W - (clr * g) / (sqrt(s) + eps).  A row with more than
 * 256 pairs is summed in chunks of 256 pairs, the chunk sums in 16 contiguous groups, the group
 * sums in order (oracle/ref.py kshift_adagrad_ref restates the order).  Deterministic.
 * clr = lr / (1 + (step - 1) * lr_decay) (torch.optim.Adagrad; no weight decay).  ids / dY / out /
 * norms as lthm_kshift_bwd_sparse ([n, F] ids, item i of table i % F); W, state_sum [F * P, D] f32.
 * Requires F * P <= 2^32, n * F * K < 2^31, D <= 256, K <= 64; workspace 256-B aligned, >=
 * lthm_kshift_adagrad_ws_bytes(n * F, K, D) bytes (-1: invalid sizes). */
int64_t lthm_kshift_adagrad_ws_bytes(int64_t n_items, int32_t K, int32_t D);
int lthm_kshift_adagrad_fused(const int64_t* ids, int64_t n, int32_t F, const void* dY, int32_t dy_dtype,
                              const void* out, int32_t out_dtype, const float* norms, int64_t P, int32_t D, int32_t K,
                              int32_t mode, float* W, float* state_sum, float clr, float eps, void* workspace,
                              int64_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------- */
/* GEMM: every nn.Linear on the path (commons/transformers/layers.py:240-241,   */
/* :274-276; commons/layers.py:65-81; models/lthm/sequence/ Linears)          */
/* ------------------------------------------------------------------------- */
#define LTHM_ACT_NONE 0
#define LTHM_ACT_GELU 1        /* nn.GELU(approximate='tanh')  transformers/layers.py:275 */
#define LTHM_ACT_QGELU 2       /* QuickGELU x*sigmoid(1.702x)   commons/layers.py:9-11    */
#define LTHM_ACT_GELU_GRAD 3   /* multiply by GELU'(aux)   (backward epilogue)            */
#define LTHM_ACT_QGELU_GRAD 4  /* multiply by QuickGELU'(aux)                             */
#define LTHM_ACT_GELU_D 5      /* GELU, but aux_out receives GELU'(x) (bf16), not x      */
#define LTHM_ACT_MUL_AUX 6     /* multiply by aux (a derivative saved by LTHM_ACT_GELU_D) */

/* C[b] = epi(alpha * A[b] . B[b]), bf16 operands, fp32 accumulation (MFMA).
 *   a_kcontig: A is [M][K] (row stride lda) else A is [K][M] (row stride lda)
 *   b_kcontig: B is [N][K] (row stride ldb) else B is [K][N] (row stride ldb)
 * epilogue, in order: + bias[N]; act (GELU/QGELU store the pre-activation to
 * aux_out, *_GRAD multiply by act'(aux)); + res1; + res2; cast to out_dtype.
 * splits > 1: split-K over `workspace` (splits*batch*M*N f32), then combine. */
typedef struct lthm_gemm_desc {
  const void* A;
  const void* B;
  void* C;
  int64_t M;
  int64_t N;
  int64_t K;
  int64_t lda;
  int64_t ldb;
  int64_t ldc;
  int64_t sA;
  int64_t sB;
  int64_t sC;
  int32_t batch;
  int32_t a_kcontig;
  int32_t b_kcontig;
  int32_t out_dtype;
  float alpha;
  int32_t act;
  const float* bias;
  const void* aux;
  void* aux_out;
  int64_t ldaux;
  const void* res1;
  const void* res2;
  int64_t ldr1;
  int64_t ldr2;
  int32_t res1_dtype;
  int32_t res2_dtype;
  int32_t splits;
  int32_t pad0;
  float* workspace;
  size_t workspace_bytes;
  int32_t ab_dtype;
  int32_t pad1;
  const float* a_scale;
  const float* b_scale;
  int32_t* amax_out; /* optional: atomic max of |C| (as f32 bits) over the stored values */
} lthm_gemm_desc;

/* ab_dtype LTHM_BF16 (0 is read as bf16 too) or LTHM_FP8_E4M3: A [M, K] and B [N, K]
 * both K-contiguous e4m3 bytes (lda / ldb in bytes), per-tensor device scales
 * a_scale / b_scale (C = epi(alpha * a_scale * b_scale * A.B)); batch 1, no split-K,
 * K % 128 == 0 -- the fp8 encoder GEMMs of the C5 config, on
 * v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales. */
int lthm_gemm(const lthm_gemm_desc* desc, void* stream);

/* Per-tensor fp8 quantisation: scale = amax(|x|) / 448 (1 if x == 0),
 * q = e4m3(clamp(x / scale, -448, 448)) round-to-nearest-even.  x: n f32 / bf16
 * (n % 8 == 0, 16-B aligned); q: n bytes; scale: device f32; work: 4-byte scratch. */
int lthm_quantize_fp8(const void* x, int32_t dtype, int64_t n, uint8_t* q, float* scale, int32_t* work,
                      void* stream);
/* The same quantisation with amax(|x|) already reduced by the producer (the f32 bits of
 * the maximum in *amax: lthm_layernorm_fwd_amax, lthm_gemm's amax_out, lthm_amax), so
 * x is read once: the C5 encoder's fused quantisation. */
int lthm_quantize_fp8_amax(const void* x, int32_t dtype, int64_t n, const int32_t* amax, uint8_t* q, float* scale,
                           void* stream);
/* *amax = max(*amax, amax(|x|)) as f32 bits (x: n f32 / bf16, n % 8 == 0, 16-B aligned);
 * the caller zeroes *amax before the first producer. */
int lthm_amax(const void* x, int32_t dtype, int64_t n, int32_t* amax, void* stream);

/* ------------------------------------------------------------------------- */
/* Fused encoder MLP: _MLP.forward, commons/transformers/layers.py:279-284      */
/* (c_fc -> GELU(tanh) -> c_proj, dropout 0) with the [M, HID] hidden kept on   */
/* chip.  x: ln_2 output bf16 [M, D]; W1 = c_fc.weight bf16 [HID, D];           */
/* W2T = c_proj.weight^T bf16 [HID, D]; biases f32 (NULL for bias=False).        */
/* Supported shapes: lthm_mlp_supported(D, HID) (D 128 or 256, HID % 32 == 0).  */
/* ------------------------------------------------------------------------- */
int lthm_mlp_supported(int32_t D, int32_t HID);
/* out f32 [M, D] = res1 [+ res2] + c_proj(GELU(c_fc(x))); res1 / res2 f32 [M, D] or NULL
 * (replaces TransformerBlock's x + mlp(ln_2 x), commons/transformers/layers.py:371). */
int lthm_mlp_fwd(const void* x, int64_t M, int32_t D, int32_t HID, const void* W1, const float* b1,
                 const void* W2T, const float* b2, const float* res1, const float* res2, float* out,
                 void* stream);
/* lthm_mlp_fwd with ln_2 fused into the prologue: the input rows are LayerNorm(x) (x f32 [M, D],
 * ln_w / ln_b f32 [D], eps 1e-5, ln_b NULL for bias=False); h_out (bf16 [M, D]), mean and rstd
 * (f32 [M]) receive the LayerNorm output and statistics for the backward (each may be NULL).
 * Replaces the block's x + mlp(ln_2(x)) (commons/transformers/layers.py:371, :142-149). */
int lthm_mlp_fwd_ln(const float* x, const float* ln_w, const float* ln_b, int64_t M, int32_t D, int32_t HID,
                    const void* W1, const float* b1, const void* W2T, const float* b2, const float* res1,
                    const float* res2, float* out, void* h_out, float* mean, float* rstd, void* stream);
/* The training backward with the hidden RECOMPUTED (never stored by the forward):
 * pre = x W1^T + b1; G = GELU(pre); dP = (dY W2) * GELU'(pre); dX = dP W1.  dY bf16 [M, D]
 * (gradient of the MLP output), dX [M, D] in dx_dtype (LTHM_F32 / LTHM_BF16), G and dP bf16
 * [M, HID]: the operands of dW2 = dY^T G and dW1 = dP^T x (db1 = colsum dP), which the
 * weight-gradient GEMM computes.  Replaces the c_proj / c_fc dgrad pair of
 * commons/transformers/layers.py:279-284's backward. */
int lthm_mlp_bwd(const void* x, const void* dY, int64_t M, int32_t D, int32_t HID, const void* W1, const float* b1,
                 const void* W2T, void* dX, int32_t dx_dtype, void* G, void* dP, void* stream);
/* The same recompute without dX (G and dP only; two waves per SIMD): dX = dP W1 then runs on the
 * GEMM.  HID <= 4096. */
int lthm_mlp_bwd_hidden(const void* x, const void* dY, int64_t M, int32_t D, int32_t HID, const void* W1,
                        const float* b1, const void* W2T, void* G, void* dP, void* stream);
/* The training backward with NO [M, HID] operand in HBM (round 5): two recompute kernels.
 * lthm_mlp_bwd_dx: dX = ((dY W2) * GELU'(x W1^T + b1)) W1 alone (dX in dx_dtype). */
int lthm_mlp_bwd_dx(const void* x, const void* dY, int64_t M, int32_t D, int32_t HID, const void* W1,
                    const float* b1, const void* W2T, void* dX, int32_t dx_dtype, void* stream);
/* lthm_mlp_wgrad: dW1 = dP^T x (f32 [HID, D], c_fc.weight's gradient), dW2 = dY^T G (f32 [D, HID],
 * c_proj.weight's), db1 = colsum dP (f32 [HID], or NULL) with G / dP recomputed per token tile
 * inside the kernel; partial sums per token slice go to the workspace (>= lthm_mlp_wgrad_ws_bytes)
 * and are folded in slice order (deterministic).  HID % 128 == 0.  Replaces the c_fc / c_proj
 * weight-gradient products of commons/transformers/layers.py:279-284's backward. */
int64_t lthm_mlp_wgrad_ws_bytes(int64_t M, int32_t D, int32_t HID);
int lthm_mlp_wgrad(const void* x, const void* dY, int64_t M, int32_t D, int32_t HID, const void* W1,
                   const float* b1, const void* W2T, float* dW1, float* dW2, float* db1, void* workspace,
                   int64_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------- */
/* LayerNorm (commons/transformers/layers.py:142-149, eps 1e-5)               */
/* ------------------------------------------------------------------------- */
/* x f32 [M, D] -> y (y_dtype) [M, D], mean/rstd f32 [M]. b may be NULL (bias=False). */
int lthm_layernorm_fwd(const float* x, int64_t M, int32_t D, const float* w, const float* b,
                       void* y, int32_t y_dtype, float* mean, float* rstd, void* stream);
/* lthm_layernorm_fwd that also folds amax(|y|) (of the stored, rounded y) into *amax
 * (f32 bits, atomic max; the caller zeroes it): the fp8 quantisation's reduction. */
int lthm_layernorm_fwd_amax(const float* x, int64_t M, int32_t D, const float* w, const float* b, void* y,
                            int32_t y_dtype, float* mean, float* rstd, int32_t* amax, void* stream);
/* number of row blocks the backward uses (partials is [2, blocks, D] f32) */
int lthm_layernorm_bwd_blocks(int64_t M);
/* dx = LN'(dy) + res1 + res2 (f32; res may be NULL), optional bf16 copy of dx;
 * partials[0] = per-block dweight sums, partials[1] = per-block dbias sums. */
int lthm_layernorm_bwd(const void* dy, int32_t dy_dtype, const float* x, int64_t M, int32_t D,
                       const float* w, const float* mean, const float* rstd, const float* res1,
                       const float* res2, float* dx, void* dx_bf16, float* partials, void* stream);
/* flags bit 0 (D % 4 == 0): dx (f32) = LN'(dy) + 2 res1 + res2 while dx_bf16 = LN'(dy) + res1 + res2:
 * the double-residual block's ln_2 backward hands ln_1's backward its two residual gradients
 * as one f32 tensor (query_tower.py:135, x + block(x)) */
int lthm_layernorm_bwd_ex(const void* dy, int32_t dy_dtype, const float* x, int64_t M, int32_t D,
                          const float* w, const float* mean, const float* rstd, const float* res1,
                          const float* res2, float* dx, void* dx_bf16, float* partials, int32_t flags, void* stream);
/* The input-gradient GEMM that feeds a LayerNorm backward, fused with it (round 5): dh = dy W
 * (dy [M, K] bf16, wt = W^T [256, K] bf16, K % 64 == 0: the block's c_fc / c_attn dgrad,
 * commons/transformers/layers.py:271-284 and :247-265) and then lthm_layernorm_bwd_ex over
 * dh in f32 (layers.py:142-149): dx = LN'(dh) + res1 + res2 (+ res1 again with flags bit 0),
 * its bf16 copy (dx_bf16 may be null), and per-tile weight / bias gradient partials
 * (partials: f32 [2, lthm_dgrad_layernorm_bwd_tiles(M), 256], rows summed by the caller).
 * D must be 256 (one column tile holds whole rows); 16-B aligned operands. */
int lthm_dgrad_layernorm_bwd_tiles(int64_t M);
/* The block's c_proj forward and ln_2 in one kernel (round 5): x1 = res1 + x W^T + bias
 * (x [M, K] bf16, W [256, K] bf16 = nn.Linear weight, K % 64 == 0; transformers/layers.py:
 * 264 + the residual of :371) written in f32, then lthm_layernorm_fwd of x1 (layers.py:142-149,
 * eps 1e-5): h bf16 [M, 256], mean / rstd [M].  bias / res1 / ln_b may be null. */
int lthm_linear_layernorm_fwd(const void* x, const void* w, const float* bias, const float* res1, int64_t M,
                              int32_t D, int64_t K, const float* ln_w, const float* ln_b, float* x1,
                              void* h, float* mean, float* rstd, void* stream);
int lthm_dgrad_layernorm_bwd(const void* dy, const void* wt, int64_t M, int32_t D, int64_t K,
                             const float* x, const float* w, const float* mean, const float* rstd,
                             const float* res1, const float* res2, float* dx, void* dx_bf16,
                             float* partials, int32_t flags, void* stream);

/* ------------------------------------------------------------------------- */
/* Attention with relative position bias + causal mask                       */
/* (commons/transformers/layers.py:13-61, :202-265)                          */
/* ------------------------------------------------------------------------- */
typedef struct lthm_attn_desc {
  const void* q;
  const void* k;
  const void* v;
  int64_t q_tok_stride;
  int64_t k_tok_stride;
  int64_t v_tok_stride;
  int64_t q_head_stride;
  int64_t k_head_stride;
  int64_t v_head_stride;
  int64_t q_batch_stride;
  int64_t k_batch_stride;
  int64_t v_batch_stride;
  void* out;
  int64_t o_tok_stride;
  int64_t o_head_stride;
  int64_t o_batch_stride;
  const float* table;
  int64_t table_rows;
  float* lse;
  int32_t B;
  int32_t T;
  int32_t H;
  int32_t E;
  int32_t causal;
  int32_t pad0;
  const void* dout;
  void* dq;
  void* dk;
  void* dv;
  float* dtable_part;
  float* delta;
  const float* mask;          /* optional additive mask, f32 [., ., T, T] (NULL: none) */
  int64_t mask_batch_stride;  /* 0 broadcasts one mask over the batch */
  int64_t mask_head_stride;   /* 0 broadcasts over the heads */
  int64_t mask_row_stride;    /* >= T */
  /* packed rows (shared pad prefix, lthm_pad_prefix_*; T > 256, E = 64, no mask): when row_map
   * is set the batch strides are unused and row t of sequence b is row row_map[b * T + t] of
   * q / k / v (and of out / dout / dq through live_map, -1 = not this sequence's row: its dout
   * reads as zero, its out / dq are not written, and query tiles with no live row are skipped).
   * dK / dV of a key in the chain (row < chain_rows) go to dk_chain / dv_chain row
   * b * chain_rows + t (token stride chain_ts, head stride = k / v head stride), the others to
   * dk / dv at their packed row. */
  const int32_t* row_map;
  const int32_t* live_map;
  void* dk_chain;
  void* dv_chain;
  int64_t chain_ts;
  int32_t chain_rows;
  int32_t pad1;
} lthm_attn_desc;

/* bf16 q/k/v/out, f32 table [table_rows, H] (row q-k+T), lse f32 [B, H, T].
 * T <= 256: one workgroup per (batch, head) holds K and V whole in LDS.
 * 256 < T <= 4096 (E = 32/64/128): 64-row workgroups stream K/V windows.
 * mask != NULL: S[b, h, q, k] += mask[b * mask_batch_stride + h * mask_head_stride
 * + q * mask_row_stride + k] (the reference's general additive attn_mask, SDPA :57-58,
 * TransformerBlock.inner_forward :404-408, on top of the causal flag); served by the
 * whole-head VALU kernels, so T <= 256 and K, V, Q, dO of one head fit in LDS. */
int lthm_attn_fwd(const lthm_attn_desc* desc, void* stream);
/* dq/dk/dv bf16 (same strides as q/k/v); dtable_part f32 [parts, 2T+1, H] with
 * parts = lthm_attn_bwd_parts(B, T) (reduce over the first dim; = B for T <= 256);
 * delta: f32 [B, H, T] workspace, required when T > 256. */
int lthm_attn_bwd(const lthm_attn_desc* desc, void* stream);
int64_t lthm_attn_bwd_parts(int32_t B, int32_t T);
/* 1 when lthm_attn_fwd / lthm_attn_bwd take PACKED rows (row_map set) at this T and E with no
 * mask: the long-T' 32x32x16 kernels serve it (T > 256, E = 64, both LDS images fit, not
 * switched off by the A/B environment switches); 0: the caller unpacks to full sequences. */
int lthm_attn_packed_ok(int32_t T, int32_t E);

/* ------------------------------------------------------------------------- */
/* LTHM towers (models/lthm/sequence/ encoder, product and query towers)     */
/* ------------------------------------------------------------------------- */
#define LTHM_MAX_CVE 8

/* history flip, right padding -> left padding (encoder.py:52-54, 60-61) */
int lthm_flip_tokens(const int64_t* in, int64_t* out, int64_t B, int32_t T, void* stream);

/* ProductTower.forward (product_tower.py:43-62) with its 6 CosineVectorEmbedding
 * modules (commons/transformers/layers.py:443-471) fused per token. */
typedef struct lthm_ptower_desc {
  const int64_t* ids;
  const void* x;
  int32_t x_dtype;
  int32_t Din;
  int64_t n;
  int32_t Dout;
  int32_t n_mod;
  const float* w_map;
  const float* b_map;
  const float* proj;
  const float* grids;
  const void* tables;
  const void* hist;
  int32_t tab_dtype;
  int32_t proj_total;
  int32_t grid_total;
  int32_t cve_rows;
  int32_t norm_bins;
  float norm_threshold;
  int32_t cve_only;       /* 1: plain CosineVectorEmbedding(s): sum of bags only, one normalisation */
  int32_t emb_dtype;      /* dtype of emb_out: LTHM_F32 or LTHM_BF16 */
  int32_t mod_nproj[8];
  int32_t mod_nbins[8];
  int32_t mod_row_off[8];
  int32_t mod_proj_off[8];
  int32_t mod_grid_off[8];
  void* emb_out;
  uint16_t* rows_out;
  void* xn_out;
  uint8_t* mask_out;
} lthm_ptower_desc;

int lthm_product_tower_fwd(const lthm_ptower_desc* desc, void* stream);

/* Row gather (scatter = 0: dst row i = src row idx[i], a zero row where idx[i] < 0) or scatter
 * (scatter = 1: dst row idx[i] = src row i, skipped where idx[i] < 0) of `count` rows of
 * row_bytes (a multiple of 16; 16-B aligned pointers and leading dims).  The product tower's
 * token compaction (models/lthm/sequence/product_tower.py:43-62: a pad token's embedding is
 * masked to zero, so the tower runs on the non-pad tokens only). */
int lthm_rows_move(const void* src, int64_t src_ld_bytes, const int32_t* idx, int64_t count, void* dst,
                   int64_t dst_ld_bytes, int64_t row_bytes, int32_t scatter, void* stream);

/* Shared pad prefix (query_tower.py:99-137 over left-padded histories, encoder.py:52): with causal
 * attention, no dropout and the same position-0 token for every sequence, a pad position's state
 * depends only on its position, so the encoder runs the pad chain (positions 0 .. P) once and
 * each sequence's positions past its pads ("packed" rows: the chain first, then the sequences'
 * valid positions in order).
 *   stats:  npad[b] = leading set bytes of mask row b; stats = {1 if every row is a prefix mask,
 *           sum of T - npad, P = max npad, the first b with npad = P (the chain's owner)}.
 *   maps:   full row f = b Tp + p (Tp = T + 1) -> packed row pof[f] (the chain row p for p <= npad[b]);
 *           pof_x[f] the same but -1 at the pad rows of every sequence except the owner;
 *           fop[r] = the full row of packed row r (chain rows: the owner's).  voff[b] = exclusive
 *           prefix sum of T - npad.
 *   sum:    dst[p] (p <= P, packed chain rows) = sum over b with npad[b] >= p of src[b Tp + p]
 *           (W elements of rows src_ld / dst_ld elements apart, bf16 or f32, W, src_ld, dst_ld
 *           multiples of 8; fixed order); ws of lthm_pad_prefix_ws_bytes bytes. */
int lthm_pad_prefix_stats(const uint8_t* mask, int64_t mask_stride, int32_t B, int32_t T, int32_t* npad,
                          int32_t* stats, void* stream);
int lthm_pad_prefix_maps(const int32_t* npad, const int64_t* voff, int32_t B, int32_t Tp, int32_t P, int32_t owner,
                         int32_t* pof, int32_t* pof_x, int32_t* fop, void* stream);
int64_t lthm_pad_prefix_ws_bytes(int32_t B, int32_t P, int32_t W);
int lthm_pad_prefix_sum(const void* src, int64_t src_ld, int32_t dtype, int32_t W, const int32_t* npad, int32_t B,
                        int32_t Tp, int32_t P, void* dst, int64_t dst_ld, void* ws, int64_t ws_bytes, void* stream);

/* dW[rows[t, i]] += dY[t, :] for all tokens t, slots i < nidx <= 64 (0xffff = skip).
 * LDS-privatised EmbeddingBag / Embedding backward for tables of R < 65535 rows.
 * `workspace` (device, may be NULL) holds per-token-chunk partial sums; with
 * >= 2 * R * D * 4 bytes the tokens are split into chunks that are folded into
 * dW in a fixed order (no global atomics).  dW is accumulated into. */
int lthm_small_table_bwd(const uint16_t* rows, int32_t nidx, const void* dY, int32_t dy_dtype, int64_t ldy,
                         int64_t n, int32_t R, int32_t D, float* dW, void* workspace, int64_t workspace_bytes,
                         void* stream);
/* Same, with the slots grouped into nseg (<= 64) segments: segment s covers slots
 * [seg_slot0[s], +seg_nslot[s]) (nslot <= 64) whose rows all lie in
 * [seg_row0[s], +seg_nrow[s]); segment row ranges are disjoint.  A segment's
 * [nrow, 64] f32 slice is held in LDS, so nrow <= 640 (<= 256 keeps two blocks
 * per CU).  The seg_* arrays are HOST arrays. */
int lthm_segmented_table_bwd(const uint16_t* rows, int32_t nidx, int32_t nseg, const int32_t* seg_slot0,
                             const int32_t* seg_nslot, const int32_t* seg_row0, const int32_t* seg_nrow,
                             const void* dY, int32_t dy_dtype, int64_t ldy, int64_t n, int32_t D, float* dW,
                             void* workspace, int64_t workspace_bytes, void* stream);
/* CosineVectorEmbedding / EmbeddingBag gradient for CVE-structured tables on
 * MFMA: module j covers slots [mod_slot0[j], +mod_nslot[j]) and slot s owns rows
 * [mod_row0[j] + (s - mod_slot0[j]) * mod_rps[j], +mod_rps[j]) (module row ranges
 * disjoint, nmod <= 16, <= 64 tiles of 128 rows).  dY bf16 [n, D] with D in
 * {16, 32, 64, 128, 256} (f32 dY is split into bf16 hi + lo); dW f32 accumulated;
 * workspace as lthm_small_table_bwd.
 * (commons/transformers/layers.py:462-471 backward; product_tower.py:43-62).
 * The mod_* arrays are HOST arrays. */
int lthm_cve_table_bwd(const uint16_t* rows, int32_t nidx, int32_t nmod, const int32_t* mod_slot0,
                       const int32_t* mod_nslot, const int32_t* mod_row0, const int32_t* mod_rps,
                       const void* dY, int32_t dy_dtype, int64_t ldy, int64_t n, int32_t D, float* dW,
                       void* workspace, int64_t workspace_bytes, void* stream);
/* Same one-hot MFMA gradient for a small table of R rows whose nidx <= 8 slots
 * may each reference any row (0xffff = skip): dW[rows[t, i]] += dY[t, :]
 * (nn.Embedding / EmbeddingBag-sum backward: the query tower's action, time,
 * position and pad tables, outcome conditioning).  dY f32 (hi + lo bf16 split)
 * or bf16 [n, D], D in {16, 32, 64, 128, 256}; R <= 8192. */
int lthm_table_bwd_mfma(const uint16_t* rows, int32_t nidx, int32_t R, const void* dY, int32_t dy_dtype,
                        int64_t ldy, int64_t n, int32_t D, float* dW, void* workspace, int64_t workspace_bytes,
                        void* stream);
/* QuantileMapper (commons/transformers/layers.py:477-487) on x [B, F]:
 * out = bucketize(x[:, f], q_f) / (nq + 1) - 0.5; quantiles [shared ? 1 : F, nq]. */
int lthm_quantile_map(const float* x, int64_t B, int32_t F, const float* quantiles, int32_t nq, int32_t shared,
                      float* out, void* stream);

/* Vector-feature layers (commons/transformers/layers.py), f32, all device pointers.
 * rowproj_fwd: z[r, j] = s_r sum_k x[r, k] W[j, k] with W[j, k] at w[j*ldj + k*ldk], x [rows, dim].
 *   mode 0 SimhashVectorIndexer (:426-437): out int64 [rows] = sum_j (z[r, j] > 0) << j, P <= 64;
 *   mode 1 CosineLinear (:517-525) forward with w = normalize(W) [P, dim]:
 *          out f32 [rows, P] = z / max(|x_r|, 1e-12). */
int lthm_rowproj_fwd(const float* x, int64_t rows, int32_t dim, const float* w, int64_t ldj, int64_t ldk, int32_t P,
                     int32_t mode, void* out, void* stream);
/* F.normalize(x, dim=-1) over f32 rows */
int lthm_l2norm_rows(const float* x, int64_t rows, int32_t dim, float* y, void* stream);
/* its backward dx = (g - y (y . g)) / |x| (g / eps when |x| <= eps); exactly one of
 * g [rows, dim] or dz [rows, P] (then g = dz @ w_hat, w_hat [P, dim]: CosineLinear's x
 * side) is given; rinv [rows] (may be NULL) receives 1 / max(|x|, eps). */
int lthm_l2norm_rows_bwd(const float* x, int64_t rows, int32_t dim, const float* g, const float* dz,
                         const float* w_hat, int32_t P, float* dx, float* rinv, void* stream);
/* CosineLinear weight side: dw_hat[j, k] += sum_r dz[r, j] x[r, k] rinv[r] (accumulates). */
int lthm_cosine_wgrad(const float* dz, const float* x, const float* rinv, int64_t rows, int32_t P, int32_t dim,
                      float* dw_hat, void* stream);
/* Gaussian bins of LearnableCosineVectorEmbedding / ProbabilityVectorEmbedding
 * (:558-569, :588-595): z [n] f32 with n = rows * P, element i at projection p = i % P,
 * mean [P, nb] (nb <= 64): out[i, b] = normalize_b(topk_b(exp(-0.5 (z_i - mean[p, b])^2 / sigma2)));
 * top_k 0 = no top-k.  out_dtype LTHM_F32 or LTHM_BF16.  bwd: dz [n] (may be NULL) and
 * dmean [P, nb] (accumulated) from gout [n, nb] (g_dtype F32 / BF16). */
int lthm_gauss_bins_fwd(const float* z, int64_t n, int32_t P, const float* mean, int32_t nb, float sigma2,
                        int32_t top_k, void* out, int32_t out_dtype, void* stream);
int lthm_gauss_bins_bwd(const float* z, int64_t n, int32_t P, const float* mean, int32_t nb, float sigma2,
                        int32_t top_k, const void* gout, int32_t g_dtype, float* dz, float* dmean, void* stream);

/* MoELinear (commons/transformers/layers.py:101-136), the parts around its GEMMs.
 * gate: probs[m, :] = softmax(g) with g = scale * logits[m, :] and, when top_k > 0,
 * g[e] -> -inf where g[e] is below the top_k-th largest (:123-127); E <= 64.
 * gate_bwd: dlogits = scale * p (dp - sum_j p_j dp_j).
 * scale: GH[m, e P + p] = probs[m, e] * H[m, e P + p]   (bf16 in / out).
 * hidden_bwd: dg[m, e] = sum_p dGH H;  dpre = probs[m, e] dGH gelu_tanh'(pre)  (bf16 out). */
int lthm_moe_gate_fwd(const float* logits, int64_t M, int32_t E, float scale, int32_t top_k, float* probs,
                      void* stream);
int lthm_moe_gate_bwd(const float* probs, const float* dprobs, int64_t M, int32_t E, float scale, float* dlogits,
                      void* stream);
int lthm_moe_scale(const void* H, const float* probs, int64_t M, int32_t E, int32_t P, void* GH, void* stream);
int lthm_moe_hidden_bwd(const float* dGH, const void* H, const void* pre, const float* probs, int64_t M, int32_t E,
                        int32_t P, void* dpre, float* dg, void* stream);

/* Binary cross-entropy with logits, mean reduction
 * (F.binary_cross_entropy_with_logits; the ranker's click loss and
 * embedding_module_gen.py:112-116's mask-model loss).
 * fwd: *loss_sum += inv_n * sum_i [max(z,0) - z y + log1p(exp(-|z|))]  (caller zeroes it)
 * bwd: dz_i = (sigmoid(z_i) - y_i) * (*gscale) * inv_n                      */
int lthm_bce_logits_fwd(const float* z, const float* y, int64_t n, float inv_n, float* loss_sum, void* stream);
int lthm_bce_logits_bwd(const float* z, const float* y, int64_t n, const float* gscale, float inv_n, float* dz,
                        void* stream);

/* nn.MSELoss (embedding_module_gen.py:139-150): loss_sum += inv_n * sum (y - x)^2 (zero it
 * first); bwd dy = 2 (y - x) * (*gscale) * inv_n.  y F32 or BF16 (dy the same), x f32. */
int lthm_mse_fwd(const void* y, int32_t y_dtype, const float* x, int64_t n, float inv_n, float* loss_sum, void* stream);
int lthm_mse_bwd(const void* y, int32_t y_dtype, const float* x, int64_t n, const float* gscale, float inv_n, void* dy,
                 void* stream);

/* QueryTower input assembly (query_tower.py:89-111): action + time embeddings,
 * pad substitution, zero/CLS token, reversed position embedding. */
typedef struct lthm_tokens_desc {
  const void* P;
  int32_t p_dtype;
  int32_t d;
  const int64_t* labels;
  const int64_t* ts;
  const uint8_t* mask;
  int64_t B;
  int32_t T_full;
  int32_t trim;
  const float* act;
  const float* hod;
  const float* how;
  const float* dow;
  const float* wpe;
  const float* pad;
  const float* ctx;
  int32_t off_act;
  int32_t off_hod;
  int32_t off_how;
  int32_t off_dow;
  int32_t off_wpe;
  int32_t off_pad;
  int64_t div_hod;
  int64_t mod_hod;
  int64_t div_how;
  int64_t mod_how;
  int64_t div_dow;
  int64_t mod_dow;
  float* x0;
  uint16_t* rows_out;
} lthm_tokens_desc;

int lthm_tokens_fwd(const lthm_tokens_desc* desc, void* stream);
/* dP (bf16 [B, T, d]) = unmasked dx0[:, 1:], dctx (f32 [B, d], may be NULL) = dx0[:, 0] */
int lthm_tokens_bwd(const lthm_tokens_desc* desc, const float* dx0, void* dP, float* dctx, void* stream);
/* out = bf16(x + table[outcome mod n_outcomes]) (query_tower.py:118-122); rows_out [B*(T+1)] */
int lthm_outcome_fwd(const float* x, const int64_t* labels, int64_t B, int32_t T_full, int32_t trim,
                     int64_t future, const float* table, int32_t n_outcomes, int32_t D, void* out,
                     uint16_t* rows, void* stream);

/* Row-sharded KShift lookup routing (C3 item table; commons/layers.py:152-185 row math,
 * SURVEY §8e): global row r on rank r % world at local index r / world.
 * lthm_shard_route: the K rows of n_items ids, deduplicated per workgroup of 2,048 (row, shift)
 * pairs (LDS bitonic sort), laid out owner-major in send_rows [capacity n_items * K];
 * send_counts [world] and owner_base [world + 1] (owner_base[world] = the request total) stay on
 * the device; inv [n_items * K] holds, for every pair, the position of its row's value in the
 * buffer the exchange returns (owner-major, the send order).  Replaces torch.unique / argsort /
 * bincount of the reference-style exchange; workspace: lthm_shard_route_ws_bytes bytes.
 * 1 <= world <= 256 (the per-owner counts live in LDS); larger worlds are refused. */
int64_t lthm_shard_route_ws_bytes(int64_t n_pairs, int32_t world);
int lthm_shard_route(const int64_t* ids, int64_t n_items, int32_t K, int64_t P, int32_t world, int64_t* send_rows,
                     int64_t* send_counts, int64_t* owner_base, int64_t* inv, void* workspace, int64_t ws_bytes,
                     void* stream);
/* out[i] = shard[rows[i] / world] (row_bytes a multiple of 16) for i < min(*count, cap) (count NULL: cap);
 * the owner side of the exchange (and the whole lookup at world 1) */
int lthm_shard_gather(const void* shard, int64_t n_local, int32_t row_bytes, const int64_t* rows,
                      const int64_t* count, int64_t cap, int32_t world, void* out, void* stream);

/* ------------------------------------------------------------------------- */
/* In-batch contrastive loss (models/lthm/sequence/wrapper.py:114-245)        */
/* ------------------------------------------------------------------------- */
/* F.normalize of rows: out bf16 [rows, D], norms f32 [rows] (wrapper.py:118-119).
 * row_mask (may be NULL): rows r with row_mask[(r / mask_group) * mask_stride + r % mask_group]
 * set get a zero output row (the loss zeroes the `in` rows of pad positions, which
 * every logit of them excludes; their norm is still written). */
int lthm_rownorm(const void* x, int32_t x_dtype, int64_t rows, int32_t D, void* out_bf16, float* norms,
                 const uint8_t* row_mask, int64_t mask_group, int64_t mask_stride, void* stream);
/* backward of lthm_rownorm: dx = (g - y (y.g)) / |x|; writes dx_bf16 and/or dx_f32 */
int lthm_rownorm_bwd(const void* x, int32_t x_dtype, const float* norms, const float* g, int64_t rows,
                     int32_t D, void* dx_bf16, float* dx_f32, void* stream);

typedef struct lthm_contrastive_desc {
  const void* out_n;      /* bf16 [B, T+1, n_heads, De] normalised next_token_emb */
  const void* in_n;       /* bf16 [B, T, De] normalised current_token_emb */
  const uint8_t* mask;    /* [B, mask_stride] pad mask (already offset by the trim) */
  int64_t mask_stride;
  int64_t B;
  int32_t T;
  int32_t n_heads;
  int32_t head;
  int32_t De;
  int32_t mb_size;        /* train_mini_batch_size (32) */
  int32_t n_mb;
  int32_t n_max;          /* >= mb_size * T, a multiple of 64, n_max * T < 2^32 (no other limit: val_step
                             runs the whole batch as one mini-batch, wrapper.py:75-80) */
  float tau;              /* softmax_temperature */
  const int32_t* offsets; /* [n_mb, n_heads] lookahead offset per mini-batch and head */
  float* lse;             /* [n_mb, n_max] per-row buffers (this head) */
  float* pos;
  int32_t* cnt;
  int32_t* rank;
  float* diag;            /* forward: positive logit (-inf: pad row / r >= n);
                             backward: scratch for the per-row exp2 shift */
  float* w;               /* row weights, written by the forward, read by the backward */
  const float* gscale;    /* device scalar: upstream gradient of the loss (backward) */
  float* d_out;           /* f32 [B, T+1, n_heads, De]: every row of this head is written (no pre-zeroing) */
  float* d_in;            /* f32 [B, T, De] (accumulated over heads) */
  const float* logq;      /* NULL, or f32 [B, logq_stride]: additive logit correction -beta * logQ(id)
                             of every input token (wrapper.py:131-135, 204-208; zero on the positive) */
  int64_t logq_stride;
  float* logq_col;        /* with logq: [n_mb, n_max] scratch written by the forward, read by the backward */
  const void* y_raw;      /* backward, optional: [B, T+1, n_heads, De] next_token_emb before F.normalize (dtype y_dtype;
                             bf16 only without t_raw) */
  const float* y_norm;    /* with y_raw: f32 [B, T+1, n_heads] its row norms (lthm_rownorm) */
  void* dy;               /* with y_raw: [B, T+1, n_heads, De] (dtype y_dtype) written INSTEAD of d_out: the gradient through
                             F.normalize (wrapper.py:118-119), every row of this head written */
  int32_t heads_run;      /* forward: heads head .. head + heads_run - 1 in one set of launches (0 or 1: one) */
  int64_t head_stride;    /* with heads_run > 1: elements between consecutive heads' lse / pos / cnt / rank /
                             diag / w / logq_col buffers; stats rows advance by n_mb * nstat */
  int32_t y_dtype;        /* LTHM_F32 / LTHM_BF16: dtype of y_raw and dy */
  const void* t_raw;      /* backward, with y_raw / dy: [B, T, De] current_token_emb before F.normalize (dtype t_dtype);
                             then every head runs in ONE call (head 0, heads_run = n_heads) and dIn is summed over
                             the heads on chip: dt is written once, through F.normalize, instead of d_in */
  int32_t t_dtype;
  const float* t_norm;    /* with t_raw: f32 [B, T] its row norms (lthm_rownorm) */
  void* dt;               /* with t_raw: [B, T, De] (dtype t_dtype): d current_token_emb, every row written */
  void* stats_ws;         /* forward: device workspace of lthm_contrastive_ws_bytes(n_mb, n_max, heads_run)
                             bytes (rank histograms + per-block partial sums) */
  int64_t stats_ws_bytes;
  int32_t rows_done;      /* backward: the forward already wrote dy (it was given y_raw / y_norm / dy at the fixed
                             shift: the fused forward + ROWS pass) for a unit upstream gradient; the backward
                             then runs the COLS side only and scales dy by *gscale */
  void* main_ev0;         /* optional hipEvent_t pair recorded on the stream around the call's main pass alone
                             (forward: cl_fr32_k / cl_fwd_k; backward: the cl_bwd32_k columns / rows passes),
                             for live per-kernel timing (bench.py); NULL: not recorded */
  void* main_ev1;
  void* vc_ws;            /* optional, training at the fixed shift (the fused forward + ROWS pass and its rows_done
                             backward): device workspace of lthm_contrastive_vc_ws_bytes bytes, the SAME buffer for the
                             forward and its backward.  The S passes then run over the valid (non-pad) indices of each
                             (mini-batch, head) only -- every logit of a pad row or column is excluded anyway
                             (wrapper.py:175-190).  Requires head 0, heads_run = n_heads, head_stride = n_mb * n_max,
                             mb_size <= 4096.  NULL: the full n x n passes */
  int64_t vc_ws_bytes;
} lthm_contrastive_desc;

/* bytes of lthm_contrastive_desc.vc_ws (-1: invalid sizes) */
int64_t lthm_contrastive_vc_ws_bytes(int64_t B, int32_t T, int32_t n_heads, int32_t mb_size, int32_t n_mb,
                                     int32_t n_max);
/* bytes of lthm_contrastive_desc.stats_ws for one forward launch (-1: invalid sizes) */
int64_t lthm_contrastive_ws_bytes(int32_t n_mb, int32_t n_max, int32_t heads);

/* Forward for one head (or heads_run consecutive heads) over all mini-batches.  stats [n_mb, nstat] f32 per head
 * (nstat >= 8 + nk): {mean CE over the used tokens, used rows (effective batch), mean negatives, min negatives,
 *  mean rank, median rank, offset, used tokens, hit@ks[0..nk)}; a used row whose CE is NaN leaves the mean and
 *  the used tokens (wrapper.py:210-214); loss_scale multiplies the row weights (1 / n_mb).
 * Training at the fixed shift (2 / tau <= 80, no logq) with y_raw / y_norm / dy given (heads 0 .. n_heads - 1,
 * mb_size <= 4096 sequences): one pass per row block computes the forward AND the row side of the backward,
 * writing dy for a unit upstream gradient; the backward is then called with rows_done = 1. */
int lthm_contrastive_fwd(const lthm_contrastive_desc* desc, float* stats, int32_t nstat, const int32_t* ks,
                         int32_t nk, float loss_scale, void* stream);
int lthm_contrastive_bwd(const lthm_contrastive_desc* desc, void* stream);

/* ------------------------------------------------------------------------- */
/* Optimizers and gradient transforms                                        */
/* ------------------------------------------------------------------------- */
/* torch.optim.AdamW step on a flat fp32 tensor (wrapper.py:263-275); optional bf16
 * shadow of the updated parameter; grad_scale multiplies g (clipping). */
int lthm_adamw(float* p, float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
               float eps, float weight_decay, int64_t step, float grad_scale, void* bf16_shadow,
               int32_t zero_grad, void* stream);
/* Multi-tensor form of lthm_adamw (optional bf16 shadows pb, no grad zeroing): `count` tensors given by
 * host arrays of device pointers p/g/m/v and element counts n, all with the same
 * hyper-parameters and step; one launch per 48 tensors (torch.optim.AdamW foreach). */
int lthm_adamw_multi(int32_t count, float** p, float** g, float** m, float** v,
                     const int64_t* n, float lr, float beta1, float beta2, float eps, float weight_decay,
                     int64_t step, float grad_scale, void* stream);
/* torch.optim.Adagrad step (embedding_module_gen.py:97,137) */
int lthm_adagrad(float* p, float* g, float* state_sum, int64_t n, float lr, float lr_decay, float eps,
                 float weight_decay, int64_t step, int32_t zero_grad, void* stream);
/* row-wise (lazy) AdamW / Adagrad over the touched rows of a [R, D] table; each
 * consumed gradient row is re-zeroed and its flag cleared.  max_rows bounds *count. */
int lthm_sparse_adamw(const int64_t* rows, const int64_t* count, int64_t max_rows, int32_t D, float* p,
                      float* g, float* m, float* v, int32_t* flags, float lr, float beta1, float beta2,
                      float eps, float weight_decay, int64_t step, void* bf16_shadow, void* stream);
int lthm_sparse_adagrad(const int64_t* rows, const int64_t* count, int64_t max_rows, int32_t D, float* p,
                        float* g, float* state_sum, int32_t* flags, float lr, float lr_decay, float eps,
                        int64_t step, void* bf16_shadow, void* stream);
/* lthm_sparse_adamw / lthm_sparse_adagrad with keep_grad = 1: the consumed gradient rows are NOT
 * re-zeroed -- for tables whose next backward overwrites a row at its first touch
 * (lthm_kshift_bwd_sparse_first with a touched-row bitmap the caller clears after the step), so the
 * zero store is dead traffic; keep_grad = 0 is the plain entry point.  Round 6 (ABI 41). */
int lthm_sparse_adamw_ex(const int64_t* rows, const int64_t* count, int64_t max_rows, int32_t D, float* p,
                         float* g, float* m, float* v, int32_t* flags, float lr, float beta1, float beta2,
                         float eps, float weight_decay, int64_t step, void* bf16_shadow, int32_t keep_grad,
                         void* stream);
int lthm_sparse_adagrad_ex(const int64_t* rows, const int64_t* count, int64_t max_rows, int32_t D, float* p,
                           float* g, float* state_sum, int32_t* flags, float lr, float lr_decay, float eps,
                           int64_t step, void* bf16_shadow, int32_t keep_grad, void* stream);
/* *out_accum += sum(x^2) */
int lthm_sumsq(const void* x, int32_t dtype, int64_t n, float* out_accum, void* stream);
/* max_norm <= 0: y = x / (sqrt(*sumsq) + add_eps)   (cap_gradients, commons/functional.py:23)
 * max_norm  > 0: y = x * min(1, max_norm / (sqrt(*sumsq) + 1e-6))   (clip_grad_norm_) */
int lthm_scale_by_norm(const void* x, void* y, int32_t dtype, int64_t n, const float* sumsq, float add_eps,
                       float max_norm, void* stream);

/* ------------------------------------------------------------------------- */
/* streaming helpers                                                         */
/* ------------------------------------------------------------------------- */
int lthm_cast(const void* in, int32_t in_dtype, void* out, int32_t out_dtype, int64_t n, void* stream);
/* out[t][i] = bf16(in[t][i]) for count tensors of n[t] f32 elements (host arrays of
 * device pointers): the bf16 GEMM operands of a model's fp32 weights, cast in one
 * launch per 48 tensors at the start of each forward (no cross-step copies to go stale) */
int lthm_cast_multi_bf16(int32_t count, float** in, void** out, const int64_t* n, void* stream);
/* out[c] (+)= sum_r in[r*ld + c], c < cols (f32 out) */
int lthm_colsum(const void* in, int32_t dtype, int64_t rows, int64_t cols, int64_t ld, float* out,
                int32_t accumulate, void* stream);
int lthm_fill_f32(float* p, float value, int64_t n, void* stream);
/* nn.Dropout(p) (commons/transformers/layers.py:253-256, 264, 283; query_tower.py:133).
 * Element i is kept iff (splitmix64(seed + i * 0x9E3779B97F4A7C15) >> 40) / 2^24 >= p,
 * kept values are scaled by 1 / (1 - p); the backward calls the same entry point with
 * the forward's seed.  0 <= p < 1.
 * lthm_dropout:      y = [res1] + [res2] + dropout(x)   (res1 / res2: f32 or NULL)
 * lthm_dropout_rows: x [rows, groups * cols] in place, row r of group g scaled by the
 *                    decision for index g * rows + r (token dropout of q / k / v)
 * lthm_dropout_mask: out[i] = keep decision (uint8), for tests and inspection */
int lthm_dropout(const void* x, int32_t x_dtype, void* y, int32_t y_dtype, int64_t n, float p, uint64_t seed,
                 const float* res1, const float* res2, void* stream);
int lthm_dropout_rows(void* x, int32_t dtype, int64_t rows, int32_t cols, int32_t groups, float p, uint64_t seed,
                      void* stream);
int lthm_dropout_mask(uint8_t* out, int64_t n, float p, uint64_t seed, void* stream);
/* Streaming logQ for the LTHM loss (commons/layers.py:189-237 CascadedStreamingLogQ-
 * CorrectionModule, as wrapper.py:126-136 drives it per mini-batch of mb_size sequences):
 * for mini-batch k in order, train_step on its non-pad ids at batch index batch_idx0 + k,
 * then out[b, t] = -beta * min_m(-log b_m[(id + hash_offsets[m]) mod num_buckets]) for
 * all its ids.  b_tables / a_tables: f32 [n_modules, num_buckets] (the modules' b / a
 * buffers stacked), updated in place, bit-identical to the reference's sequence of
 * train_steps.  ids [B, ids_stride], mask [B, mask_stride] (1 = pad; NULL = no pads), out
 * f32 [B, T] or NULL (update only: the β = 0 case, where the reference trains the
 * estimates but the correction vanishes).  update = 0 skips the train_step (the module's
 * plain forward; beta = -1 then returns min_m -log b).  With update, workspace holds
 * lthm_logq_ws_bytes(B, T, mb_size, n_modules) bytes (a per-call bucket table; every
 * mini-batch's updates run in parallel over buckets).  n_modules * num_buckets < 2^32 - 1. */
int64_t lthm_logq_ws_bytes(int64_t B, int32_t T, int32_t mb_size, int32_t n_modules);
int lthm_logq_stream(const int64_t* ids, int64_t ids_stride, const uint8_t* mask, int64_t mask_stride, int64_t B,
                     int32_t T, int32_t mb_size, float* b_tables, float* a_tables, const int64_t* hash_offsets,
                     int32_t n_modules, int64_t num_buckets, float alpha, int64_t batch_idx0, float beta,
                     int32_t update, float* out, void* workspace, int64_t ws_bytes, void* stream);
/* History-trim statistics of mask [B, T] (uint8, 1 = pad) for query_tower.py:73-86:
 * work[0] = first column holding a non-pad entry (T if none), work[1] = number of
 * all-pad columns; work is a device int32 buffer of T + 2 entries (work[2..] scratch). */
int lthm_trim_stats(const uint8_t* mask, int64_t B, int32_t T, int32_t* work, void* stream);
/* y = act(x) (dy == NULL) or y = dy * act'(x); act = LTHM_ACT_GELU / LTHM_ACT_QGELU */
int lthm_activation(const void* x, const void* dy, void* y, int32_t dtype, int64_t n, int32_t act, void* stream);

/* ------------------------------------------------------------------------- */
/* Id ingest — commons/feature_utils.py (host CPU unless noted)              */
/* ------------------------------------------------------------------------- */
/* xxHash32 / xxHash64 of a byte string (python-xxhash intdigest()) */
uint32_t lthm_xxh32(const void* data, int64_t len, uint32_t seed);
uint64_t lthm_xxh64(const void* data, int64_t len, uint64_t seed);
/* hash_string_to_long (feature_utils.py:40-46) over n packed UTF-8 strings
 * bytes[offsets[i] .. offsets[i+1]): out[i] = xxh64(s_i, seed) - 2^63.  With
 * to_lower, ASCII letters are lowered here; strings holding non-ASCII bytes are
 * flagged in needs_unicode_lower[i] (may be NULL) and left for the caller
 * (Python str.lower()).  Returns the number flagged, or -1 on bad arguments. */
int64_t lthm_hash_strings(const uint8_t* bytes, const int64_t* offsets, int64_t n, uint64_t seed, int32_t to_lower,
                          int64_t* out, uint8_t* needs_unicode_lower);
/* hash_string_to_long(str(v), seed) for int64 values v (decimal str(), no lowering) */
int lthm_hash_int64_str(const int64_t* vals, int64_t n, uint64_t seed, int64_t* out);
/* the same on the GPU: device pointers, stream-ordered */
int lthm_hash_int64_str_dev(const int64_t* vals, int64_t n, uint64_t seed, int64_t* out, void* stream);
/* handle_categorical_history_feature / pad_array (feature_utils.py:21-25, 149-183):
 * row r = items[row_offsets[r] .. row_offsets[r+1]) (already hashed), optionally
 * dropping entries equal to history_id[r], capped to `length`, right-padded with
 * `pad` -> out [n_rows, length]. */
int lthm_history_pad(const int64_t* items, const int64_t* row_offsets, int64_t n_rows, const int64_t* history_id,
                     int32_t remove_history_id, int32_t length, int64_t pad, int64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* LTHM_H_ */
