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

#define LTHM_F32 0
#define LTHM_BF16 1

/* KShift finalisation modes */
#define LTHM_KSHIFT_SCALE 0      /* x / sqrt(K)               commons/layers.py:170 */
#define LTHM_KSHIFT_NORMALIZE 1  /* F.normalize(x, 2, -1)     commons/layers.py:168 */
#define LTHM_KSHIFT_NONE 2       /* plain sum (FlatEmbedding, K = 1)               */

/* ------------------------------------------------------------------------- */
/* version / capability                                                      */
/* ------------------------------------------------------------------------- */
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

/* ------------------------------------------------------------------------- */
/* GEMM: every nn.Linear on the path (commons/transformers/layers.py:240-241,   */
/* :274-276; commons/layers.py:65-81; models/lthm/sequence/ Linears)          */
/* ------------------------------------------------------------------------- */
#define LTHM_ACT_NONE 0
#define LTHM_ACT_GELU 1        /* nn.GELU(approximate='tanh')  transformers/layers.py:275 */
#define LTHM_ACT_QGELU 2       /* QuickGELU x*sigmoid(1.702x)   commons/layers.py:9-11    */
#define LTHM_ACT_GELU_GRAD 3   /* multiply by GELU'(aux)   (backward epilogue)            */
#define LTHM_ACT_QGELU_GRAD 4  /* multiply by QuickGELU'(aux)                             */

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
} lthm_gemm_desc;

int lthm_gemm(const lthm_gemm_desc* desc, void* stream);

/* ------------------------------------------------------------------------- */
/* LayerNorm (commons/transformers/layers.py:142-149, eps 1e-5)               */
/* ------------------------------------------------------------------------- */
/* x f32 [M, D] -> y (y_dtype) [M, D], mean/rstd f32 [M]. b may be NULL (bias=False). */
int lthm_layernorm_fwd(const float* x, int64_t M, int32_t D, const float* w, const float* b,
                       void* y, int32_t y_dtype, float* mean, float* rstd, void* stream);
/* number of row blocks the backward uses (partials is [2, blocks, D] f32) */
int lthm_layernorm_bwd_blocks(int64_t M);
/* dx = LN'(dy) + res1 + res2 (f32; res may be NULL), optional bf16 copy of dx;
 * partials[0] = per-block dweight sums, partials[1] = per-block dbias sums. */
int lthm_layernorm_bwd(const void* dy, int32_t dy_dtype, const float* x, int64_t M, int32_t D,
                       const float* w, const float* mean, const float* rstd, const float* res1,
                       const float* res2, float* dx, void* dx_bf16, float* partials, void* stream);

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
} lthm_attn_desc;

/* bf16 q/k/v/out, f32 table [table_rows, H] (row q-k+T), lse f32 [B, H, T]. T <= 256. */
int lthm_attn_fwd(const lthm_attn_desc* desc, void* stream);
/* dq/dk/dv bf16 (same strides as q/k/v); dtable_part f32 [B, 2T+1, H] (reduce over B). */
int lthm_attn_bwd(const lthm_attn_desc* desc, void* stream);

/* ------------------------------------------------------------------------- */
/* streaming helpers                                                         */
/* ------------------------------------------------------------------------- */
int lthm_cast(const void* in, int32_t in_dtype, void* out, int32_t out_dtype, int64_t n, void* stream);
/* out[c] (+)= sum_r in[r*ld + c], c < cols (f32 out) */
int lthm_colsum(const void* in, int32_t dtype, int64_t rows, int64_t cols, int64_t ld, float* out,
                int32_t accumulate, void* stream);
int lthm_fill_f32(float* p, float value, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LTHM_H_ */
