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

#ifdef __cplusplus
}
#endif
#endif /* LTHM_H_ */
