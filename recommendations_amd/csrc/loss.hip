// Fused in-batch contrastive loss of the LTHM wrapper
// (models/lthm/sequence/wrapper.py:114-245), forward + backward, for gfx950.
//
// Per mini-batch of <= 32 sequences and per lookahead head i with offset o
// (drawn per mini-batch, wrapper.py:147-153):
//   rows r = (b, t), t < L = T - o:   out_r = normalize(next_token_emb[b, t, i])
//   cols c = (b', t'):                in_c  = normalize(current_token_emb[b', t' + o])
//   logits = out . in^T / tau, -inf where same sequence & r != c, or col/row pad;
//   rows kept iff not pad and >= 1 finite negative; CE(logits, r) averaged.
// The [n, n] logits (n <= 32 T) are never written: transposed 64 x 32 tiles
// S^T = img . regrows^T are produced by bf16 MFMA (K = 128) from LDS-staged
// column tiles and reduced on the fly to per-row (sum-exp, finite count, rank
// of the positive).  The backward recomputes each tile from the saved LSE; dS
// is already in the A-operand lanes of the second MFMA, so the row kernel
// accumulates dOut and the column kernel (roles swapped) dIn in registers —
// no atomics, no LDS round trip, no T^2 buffer.
// The argsort / topk metrics (wrapper.py:228-238) become the in-kernel rank
// count #{c != r : logit[r, c] > logit[r, r]}.
#include "common.hpp"

#include <algorithm>
#include <cstdlib>

namespace lthm {

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

// two f32 -> packed bf16 pair, round-to-nearest-even (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){lo, hi}, bf16x2v));
}

constexpr int DE = 128;  // product_emb_dim (model/lthm.yaml:22)

// 256-B rows of 16 x 16-B chunks, chunk ch of row r at slot ch ^ swz(r), swz a
// permutation of row & 15 chosen (by exhaustive search) so that both read
// patterns are bank-conflict-free under gfx950's lane groups
// (MI355X_MICROARCH.md, LDS table):
//  * row fragments, ds_read_b128: lane l reads row l & 15, chunk c + (l >> 4);
//    groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32) need 16 distinct slots;
//  * transposed fragments, ds_read_b64_tr_b16: lanes 0-31 read rows 0-7 (32-63:
//    rows 8-15) x one 32-B chunk pair, so swz >> 1 must differ within each 8 rows.
// swz = 0 2 4 6 8 10 12 14 | 9 11 13 15 1 3 5 7
__device__ __forceinline__ int swz(int row) {
  const int h = (row >> 3) & 1;
  return ((((row & 7) << 1) + (h << 3)) & 15) | h;
}
__device__ __forceinline__ int ks_off256(int row, int ch) { return row * 256 + ((ch ^ swz(row)) << 4); }
// The 32x32x16 tile engine's image (cdna_hip_programming.md T10, image (b)): chunk ch of
// row r at slot ch ^ swz32(r), conflict-free for the ds_read_b128 row fragments of the
// 32x32x16 A operand and for the ds_read_b64_tr_b16 transposed B fragments (each aligned
// quad of rows takes four distinct aligned blocks of four slots).
__device__ __forceinline__ int swz32(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int ko32(int row, int ch) { return row * 256 + ((ch ^ swz32(row)) << 4); }

// ---------------------------------------------------------------- row normalisation
// out[r] = bf16(x[r] / max(|x[r]|, 1e-12)), norms[r] = |x[r]|   (F.normalize, wrapper.py:118-119)
template <typename TX>
__global__ __launch_bounds__(256) void rownorm_k(const TX* __restrict__ x, int64_t rows, int D, bf16_t* __restrict__ out,
                                                 float* __restrict__ norms, const uint8_t* __restrict__ mask,
                                                 int64_t mgroup, int64_t mstride) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    float v[4];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      v[i] = (c < D) ? Elem<TX>::ld(x + r * D + c) : 0.f;
      ss += v[i] * v[i];
    }
    const float nrm = sqrtf(wave_sum(ss));
    const float den = fmaxf(nrm, 1e-12f);
    const bool zero = mask && mask[(r / mgroup) * mstride + r % mgroup];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      if (c < D) out[r * D + c] = zero ? (bf16_t)0 : f2bf(v[i] / den);
    }
    if (lane == 0) norms[r] = nrm;
  }
}

// dx[r] = (g - y (y . g)) / max(|x|, eps)  with y = x / |x|  (eps branch: g / eps)
template <typename TX>
__global__ __launch_bounds__(256) void rownorm_bwd_k(const TX* __restrict__ x, const float* __restrict__ norms,
                                                     const float* __restrict__ g, int64_t rows, int D,
                                                     bf16_t* __restrict__ dx_bf, float* __restrict__ dx_f) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    const float nrm = norms[r];
    float y[4], gv[4];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      y[i] = (c < D) ? Elem<TX>::ld(x + r * D + c) / fmaxf(nrm, 1e-12f) : 0.f;
      gv[i] = (c < D) ? g[r * D + c] : 0.f;
      dot += y[i] * gv[i];
    }
    dot = wave_sum(dot);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        const float o = (nrm > 1e-12f) ? (gv[i] - y[i] * dot) / nrm : gv[i] / 1e-12f;
        if (dx_bf) dx_bf[r * D + c] = f2bf(o);
        if (dx_f) dx_f[r * D + c] = o;
      }
    }
  }
}

// Vectorised forms (D % 8 == 0, D <= 256): 16 lanes per row, 8 contiguous
// elements (16 B of bf16 / 32 B of f32) per lane and pass, NC passes.
template <typename TX>
__device__ __forceinline__ void ld8(const TX* p, float* v) {
  if constexpr (sizeof(TX) == 2) {
    load_vec<TX, 16>(p, v);
  } else {
    load_vec<TX, 16>(p, v);
    load_vec<TX, 16>(p + 4, v + 4);
  }
}
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// rows whose mask byte mask[(r / mgroup) * mstride + r % mgroup] is set get a zero
// output row (their norm is still written, for the backward)
template <typename TX, int NC>
__global__ __launch_bounds__(256) void rownorm_v8_k(const TX* __restrict__ x, int64_t rows, int D,
                                                    bf16_t* __restrict__ out, float* __restrict__ norms,
                                                    const uint8_t* __restrict__ mask, int64_t mgroup,
                                                    int64_t mstride) {
  const int sub = threadIdx.x & 15;
  for (int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4; r < rows; r += (int64_t)gridDim.x * 16) {
    float v[NC][8];
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int e = (sub + 16 * c) * 8;
      if (e < D) ld8(x + r * D + e, v[c]);
      else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = 0.f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    }
    const float nrm = sqrtf(group16_sum(ss));
    const float den = fmaxf(nrm, 1e-12f);
    const bool zero = mask && mask[(r / mgroup) * mstride + r % mgroup];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int e = (sub + 16 * c) * 8;
      if (e < D) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = zero ? 0.f : v[c][i] / den;
        store_vec<bf16_t, 8>(out + r * D + e, o);
      }
    }
    if (sub == 0) norms[r] = nrm;
  }
}

template <typename TX, int NC>
__global__ __launch_bounds__(256) void rownorm_bwd_v8_k(const TX* __restrict__ x, const float* __restrict__ norms,
                                                        const float* __restrict__ g, int64_t rows, int D,
                                                        bf16_t* __restrict__ dx_bf, float* __restrict__ dx_f) {
  const int sub = threadIdx.x & 15;
  for (int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4; r < rows; r += (int64_t)gridDim.x * 16) {
    const float nrm = norms[r];
    const float den = fmaxf(nrm, 1e-12f);
    float y[NC][8], gv[NC][8];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int e = (sub + 16 * c) * 8;
      if (e < D) {
        ld8(x + r * D + e, y[c]);
        ld8(g + r * D + e, gv[c]);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) y[c][i] = gv[c][i] = 0.f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        y[c][i] /= den;
        dot += y[c][i] * gv[c][i];
      }
    }
    dot = group16_sum(dot);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int e = (sub + 16 * c) * 8;
      if (e < D) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (nrm > 1e-12f) ? (gv[c][i] - y[c][i] * dot) / nrm : gv[c][i] / 1e-12f;
        if (dx_bf) store_vec<bf16_t, 8>(dx_bf + r * D + e, o);
        if (dx_f) {
          store_vec<float, 4>(dx_f + r * D + e, o);
          store_vec<float, 4>(dx_f + r * D + e + 4, o + 4);
        }
      }
    }
  }
}

// ---------------------------------------------------------------- arguments and geometry
struct ClArgs {
  const bf16_t* out_n;  // [B, Tp, NH, DE]
  const bf16_t* in_n;   // [B, T, DE]
  const uint8_t* mask;  // [B, mask_stride] (already offset by trim)
  int64_t mask_stride;
  int64_t B;
  int T, NH, head, mbs, n_mb, n_max;
  const int* offsets;   // [n_mb, NH]
  float tau;
  float* lse; float* pos; int* cnt; int* rank;  // [n_mb, n_max]  (this head)
  float* diag;                                     // [n_mb, n_max]
  const float* w;                                  // [n_mb, n_max] row weights (bwd)
  const float* gscale;                             // device scalar dL (bwd)
  float* d_out;                                    // f32 [B, Tp, NH, DE]
  float* d_in;                                     // f32 [B, T, DE] (accumulated)
  float* colb;  // forward only: per-column exp2 bias (-1/tau log2 e, -inf for pad / beyond n),
                // kept in the row-weight buffer until cl_stats_k overwrites it
  // logQ correction (wrapper.py:131-135, 204-208): lq [B, lq_stride] is the additive
  // logit correction -beta * logQ(id) of every input token (natural log units), or
  // null; lqcol [n_mb, n_max] its per-column copy (0 for pad / beyond n), written by
  // cl_diag_k and read by both passes.  With lq the kernels take the online-max
  // (non-FIXED) path, whose per-element masking applies it to every c != r.
  const float* lq;
  int64_t lq_stride;
  float* lqcol;
  // ROWS epilogue through F.normalize: dy = (g - y (y . g)) / |x| with y = x / |x|
  const bf16_t* y_raw;  // [B, Tp, NH, DE] or null
  const float* y_norm;  // [B, Tp, NH]
  bf16_t* dy;           // [B, Tp, NH, DE], written instead of d_out
  int64_t head_stride;  // several heads per launch: per-head buffer stride (head = head0 + z)
  int y_dtype;          // dtype of y_raw / dy (LTHM_F32 / LTHM_BF16)
  int heads_run;        // heads head0 .. head0 + heads_run - 1
  // COLS epilogue through F.normalize: dt = (g - t^ (t^ . g)) / |t| of current_token_emb
  const void* t_raw;    // [B, T, DE], dtype t_dtype
  int t_dtype;
  const float* t_norm;  // [B, T]
  void* dt;             // [B, T, DE], dtype t_dtype, every row written
  int xcd_order;        // fused forward: XCD-remapped block order (A/B switch LTHM_CL_FR_XCD)
  // valid-row compaction (training at the fixed shift, lthm_contrastive_desc.vc_ws): the valid
  // indices of each (mini-batch, head) in order; per head, advanced by head_args
  int* vm;        // [NH][n_mb] valid count m
  int* vcs;       // [NH][n_mb][mbs + 1] compact start of each sequence (vcs[Bm] = m)
  int* vridx;     // [NH][n_mb][n_max] index r of compact row i
  float* vsh;     // [NH][n_mb][n_max] backward: exp2 shift of compact row i
  float* vw;      // [NH][n_mb][n_max] backward: row weight of compact row i
  int* vcmap;     // [NH][n_mb][mbs T] physical `in` row b T + t of the mini-batch -> compact column, or -1
  bf16_t* vR;     // [NH][n_mb][n_max][DE] compact `out` rows
  bf16_t* vC;     // [NH][n_mb][n_max][DE] compact `in` rows (column images)
  int* vpidx;     // [n_mb][mbs T] the mini-batch's valid physical `in` rows b T + t, in order
  int* vnp;       // [n_mb] their count
  float* vnorm_out;  // compact forward without a normalised `out` (out_n null): y_norm, written by the gather
};

// the per-head view of a multi-head forward launch: head head0 + z, buffers advanced by z strides
__device__ __forceinline__ ClArgs head_args(const ClArgs& a0, int z) {
  ClArgs a = a0;
  if (z) {
    const int64_t o = (int64_t)z * a0.head_stride;
    a.head += z;
    a.lse += o; a.pos += o; a.cnt += o; a.rank += o; a.diag += o;
    a.w += o;
    if (a.colb) a.colb += o;
    if (a.lqcol) a.lqcol += o;
    if (a.vm) {
      const int64_t hv = (int64_t)z * a0.n_mb * a0.n_max;
      a.vm += (int64_t)z * a0.n_mb;
      a.vcs += (int64_t)z * a0.n_mb * (a0.mbs + 1);
      a.vridx += hv; a.vsh += hv; a.vw += hv;
      a.vcmap += (int64_t)z * a0.n_mb * a0.mbs * a0.T;
      a.vR += hv * DE; a.vC += hv * DE;
    }
  }
  return a;
}

struct Geo {
  int L, off, Bm, n;
  int64_t b0;
  uint64_t Lm;  // ceil(2^32 / L): seq(c) = c / L by one 32 x 64 multiply (exact for c < 2^32 / L)
};
// sequence index c / L of a row / column c < n (exact while n L < 2^32, cl_check)
__device__ __forceinline__ int seq_of(const Geo& g, int c) {
  return (int)(((uint64_t)(uint32_t)c * g.Lm) >> 32);
}

__device__ __forceinline__ Geo geo(const ClArgs& a, int mb) {
  Geo g;
  g.off = a.offsets[mb * a.NH + a.head];
  g.L = a.T - g.off;
  g.b0 = (int64_t)mb * a.mbs;
  g.Bm = (int)min((int64_t)a.mbs, a.B - g.b0);
  g.n = g.L > 0 ? g.Bm * g.L : 0;
  g.Lm = g.L > 0 ? ((1ull << 32) + (uint64_t)g.L - 1) / (uint64_t)g.L : 0;
  return g;
}
__device__ __forceinline__ const bf16_t* out_row(const ClArgs& a, const Geo& g, int r) {
  const int b = r / g.L, t = r - (r / g.L) * g.L;
  return a.out_n + (((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head) * DE;
}
__device__ __forceinline__ const bf16_t* in_row(const ClArgs& a, const Geo& g, int c) {
  const int b = c / g.L, t = c - (c / g.L) * g.L;
  return a.in_n + ((g.b0 + b) * a.T + t + g.off) * DE;
}
__device__ __forceinline__ bool pad_of(const ClArgs& a, const Geo& g, int c) {
  const int b = c / g.L, t = c - (c / g.L) * g.L;
  return a.mask[(g.b0 + b) * a.mask_stride + t + g.off] != 0;
}

__device__ __forceinline__ bf16x8v row_frag(const unsigned char* img, int row, int chunk) {
  return __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(img + ks_off256(row, chunk)));
}

// load this wave's 16 register rows as 4 k32 A fragments
template <typename RowFn>
__device__ __forceinline__ void reg_frags(bf16x8v (&f)[4], int lane, int cnt, int rbase, RowFn rowp) {
  const int r = rbase + (lane & 15);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r < cnt) v = *reinterpret_cast<const u32x4*>(rowp(r) + (s * 4 + (lane >> 4)) * 8);
    f[s] = __builtin_bit_cast(bf16x8v, v);
  }
}

// diag[r] = out_r . in_r / tau (fp32 dot of the bf16 operands), per (mb, row);
// -inf for pad rows and for the rows n <= r < n_max (the forward reads the
// diag of its columns as their pad flag)
__global__ __launch_bounds__(256) void cl_diag_k(ClArgs a0) {
  const ClArgs a = head_args(a0, blockIdx.z);
  const int mb = blockIdx.y;
  const Geo g = geo(a, mb);
  const int lane = threadIdx.x & 63, sub = lane & 15;
  // 16 lanes per row (one 16-B chunk of each operand per lane), 4 rows per wave
  for (int r = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + (lane >> 4); r - (lane >> 4) < a.n_max;
       r += gridDim.x * 16) {
    float s = -INFINITY;
    const bool live = r < g.n && !pad_of(a, g, min(r, g.n - 1));
    float acc = 0.f;
    if (live) {
      const u32x4 ov = *reinterpret_cast<const u32x4*>(out_row(a, g, r) + sub * 8);
      const u32x4 iv = *reinterpret_cast<const u32x4*>(in_row(a, g, r) + sub * 8);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc = fmaf(__uint_as_float(ov[k] << 16), __uint_as_float(iv[k] << 16), acc);
        acc = fmaf(__uint_as_float(ov[k] & 0xffff0000u), __uint_as_float(iv[k] & 0xffff0000u), acc);
      }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) acc += __shfl_xor(acc, o, 64);
    if (live) s = acc / a.tau;
    if (sub == 0 && r < a.n_max) {
      a.diag[(int64_t)mb * a.n_max + r] = s;
      if (a.colb) a.colb[(int64_t)mb * a.n_max + r] = s == -INFINITY ? -INFINITY : -(1.f / a.tau) * 1.4426950408889634f;
      if (a.lq) {
        float q = 0.f;
        if (s != -INFINITY) {
          const int b = r / g.L, t = r - (r / g.L) * g.L;
          q = a.lq[(g.b0 + b) * a.lq_stride + t + g.off];
        }
        a.lqcol[(int64_t)mb * a.n_max + r] = q;
      }
    }
  }
}

// backward prologue: shift[r] = log2 w_r - lse_r log2 e (-inf where w_r = 0 or r >= n),
// the exp2 shift that folds the row weight into dS = w (e^(S/tau - lse) - [r == c])
__global__ __launch_bounds__(256) void cl_shift_k(ClArgs a0) {
  const ClArgs a = head_args(a0, blockIdx.z);
  float* shift = a.colb;  // = diag of this head (the backward's scratch for the shift)
  const int mb = blockIdx.y;
  const Geo g = geo(a, mb);
  const int64_t base = (int64_t)mb * a.n_max;
  for (int r = blockIdx.x * 256 + threadIdx.x; r < a.n_max; r += gridDim.x * 256) {
    const float wv = r < g.n ? a.w[base + r] : 0.f;
    shift[base + r] = wv != 0.f ? __log2f(wv) - a.lse[base + r] * 1.4426950408889634f : -INFINITY;
  }
  // d_out / dy rows of this head that the ROWS kernel never writes (t >= L of each of the
  // mini-batch's sequences) are zeroed here, so they need no whole-tensor fill
  const int tl0 = max(g.L, 0), ntail = a.T + 1 - tl0;
  const int per_seq = ntail * (DE / 4);
  const int64_t cnt = (int64_t)g.Bm * per_seq;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / per_seq), rem = (int)(i - (int64_t)b * per_seq);
    const int t = tl0 + rem / (DE / 4), c4 = rem % (DE / 4);
    const int64_t o = (((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head) * DE + c4 * 4;
    if (a.dy && a.y_dtype == LTHM_BF16) *reinterpret_cast<uint2*>(a.dy + o) = uint2{0u, 0u};
    else if (a.dy) *reinterpret_cast<float4*>((float*)a.dy + o) = float4{0.f, 0.f, 0.f, 0.f};
    else if (a.d_out) *reinterpret_cast<float4*>(a.d_out + o) = float4{0.f, 0.f, 0.f, 0.f};
  }
}

// ---------------------------------------------------------------- stats
// Three launches, any n (the rank histogram and the per-row flags live in HBM, no
// per-block limit on the rows of a mini-batch):
//  cl_rowstats_k  (CL_SROWS rows per block): per row, used = not pad and >= 1 finite
//                 negative (wrapper.py:193-201); a used row whose CE is NaN is dropped from
//                 the mean and from used_tokens (wrapper.py:210-214) but stays in the
//                 effective batch, the negatives and the ranks, as there; block partial sums
//                 {CE, negatives, ranks, used, min negatives, used tokens} in fixed order
//                 (f64), the used-token flag into w, one integer atomic per used row into the
//                 rank histogram (order-free, deterministic);
//  cl_stats_k     (one block per (mini-batch, head)): the partials in fixed order, hits@k as
//                 prefix counts of the histogram, the median rank from its order statistics;
//  cl_wscale_k    row weights w_r = token_r * loss_scale / U_tokens.
// stats[mb][*] = {mean CE over the used tokens, used (effective batch), mean negatives, min
//                 negatives, mean rank, median rank, offset, used tokens, hits@k...}
constexpr int CL_SROWS = 2048;
constexpr int CL_NPART = 6;  // f64 partials per (head, mb, block)
constexpr int CL_NSTAT = 8;  // stats before hits@k

__device__ __forceinline__ double block_dsum(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const double t = red[0];
  __syncthreads();
  return t;
}

// workspace: [heads][n_mb][n_max] int32 histogram, then [heads][n_mb][nblk][CL_NPART] f64
__global__ __launch_bounds__(256) void cl_rowstats_k(ClArgs a0, int* __restrict__ hist, double* __restrict__ part) {
  const ClArgs a = head_args(a0, blockIdx.z);
  const int mb = blockIdx.y, nblk = gridDim.x;
  const int64_t hm = (int64_t)blockIdx.z * a0.n_mb + mb;
  hist += hm * a0.n_max;
  part += (hm * nblk + blockIdx.x) * CL_NPART;
  const Geo g = geo(a, mb);
  const int tid = threadIdx.x;
  const int64_t base = (int64_t)mb * a.n_max;
  float ls = 0.f, neg = 0.f, rks = 0.f;  // <= 8 rows per thread: integer sums stay exact
  int used = 0, tok = 0, mneg = 0x7fffffff;
  for (int i = 0; i < CL_SROWS / 256; ++i) {
    const int r = blockIdx.x * CL_SROWS + tid + 256 * i;
    if (r >= a.n_max) break;
    bool u = false, t = false;
    if (r < g.n) {
      const int nn = a.cnt[base + r] - 1;
      u = !pad_of(a, g, r) && nn > 0;
      if (u) {
        const int rk = a.rank[base + r];
        const float ce = a.lse[base + r] - a.pos[base + r];
        t = !__builtin_isnan(ce);  // wrapper.py:210-211: NaN CE rows leave the mean and used_tokens
        if (t) {
          ls += ce;
          tok += 1;
        }
        neg += (float)nn;
        rks += (float)rk;
        used += 1;
        mneg = min(mneg, nn);
        atomicAdd(hist + rk, 1);
      }
    }
    a.colb[base + r] = t ? 1.f : 0.f;  // used-token flag into w (colb = w in the forward); cl_wscale_k scales it
  }
  __shared__ double red[256];
  __shared__ int imn[256];
  const double Ls = block_dsum(ls, red), Ns = block_dsum(neg, red), Rs = block_dsum(rks, red);
  const double U = block_dsum(used, red), Ut = block_dsum(tok, red);
  imn[tid] = mneg;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) imn[tid] = min(imn[tid], imn[tid + s]);
    __syncthreads();
  }
  if (tid == 0) {
    part[0] = Ls; part[1] = Ns; part[2] = Rs; part[3] = U; part[4] = (double)imn[0]; part[5] = Ut;
  }
}

__global__ __launch_bounds__(256) void cl_stats_k(ClArgs a0, const int* __restrict__ hist,
                                                  const double* __restrict__ part, int nblk, float* __restrict__ stats,
                                                  int nstat, const int* __restrict__ ks, int nk) {
  const ClArgs a = head_args(a0, blockIdx.z);
  const int mb = blockIdx.x;
  const int64_t hm = (int64_t)blockIdx.z * a0.n_mb + mb;
  hist += hm * a0.n_max;
  part += hm * nblk * CL_NPART;
  float* st = stats + hm * nstat;
  const Geo g = geo(a, mb);
  const int tid = threadIdx.x;
  __shared__ double red[256];
  __shared__ int ired[256];
  __shared__ int sel[2];
  double v[4] = {0.0, 0.0, 0.0, 0.0}, vt = 0.0;
  double mn = 2147483647.0;
  for (int b = tid; b < nblk; b += 256) {  // fixed order: thread tid folds blocks tid, tid + 256, ...
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] += part[b * CL_NPART + k];
    mn = fmin(mn, part[b * CL_NPART + 4]);
    vt += part[b * CL_NPART + 5];
  }
  const double Ls = block_dsum(v[0], red), Ns = block_dsum(v[1], red), Rs = block_dsum(v[2], red);
  const int U = (int)block_dsum(v[3], red);
  const int Ut = (int)block_dsum(vt, red);  // used tokens: the used rows with a finite CE
  ired[tid] = (int)mn;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) ired[tid] = min(ired[tid], ired[tid + s]);
    __syncthreads();
  }
  const int Mn = ired[0];
  __syncthreads();
  // hits@k (wrapper.py:235-238): rank < min(k, min negatives), a prefix count of the histogram
  for (int q = 0; q < nk; ++q) {
    const int kq = min(ks[q], Mn);
    int h = 0;
    for (int i = tid; i < kq && i < a.n_max; i += 256) h += hist[i];
    const int H = (int)block_dsum(h, red);
    if (tid == 0) st[CL_NSTAT + q] = U > 0 ? (float)((double)H / U) : 0.f;
  }
  // median of the used ranks (torch.quantile(0.5): linear interpolation between the order
  // statistics p_lo and p_hi): each thread owns a contiguous run of bins, an exclusive scan of
  // the run totals, then the owner of each order statistic reports its bin
  const int p_lo = U > 0 ? (U - 1) / 2 : 0;
  const int p_hi = U > 0 ? min(p_lo + 1, U - 1) : 0;
  const int nb = g.n > 0 ? g.n : 1;  // ranks < n
  const int per = (nb + 255) / 256;
  const int i0 = min(tid * per, nb), i1 = min(i0 + per, nb);
  int csum = 0;
  for (int i = i0; i < i1; ++i) csum += hist[i];
  ired[tid] = csum;
  if (tid < 2) sel[tid] = 0;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // inclusive Hillis-Steele scan
    const int t = tid >= o ? ired[tid - o] : 0;
    __syncthreads();
    ired[tid] += t;
    __syncthreads();
  }
  int run = ired[tid] - csum;
  if (U > 0 && p_hi >= run && p_lo < run + csum) {
    for (int i = i0; i < i1; ++i) {
      const int c = hist[i];
      if (c > 0) {
        if (p_lo >= run && p_lo < run + c) sel[0] = i;
        if (p_hi >= run && p_hi < run + c) sel[1] = i;
      }
      run += c;
    }
  }
  __syncthreads();
  if (tid == 0) {
    st[0] = Ut > 0 ? (float)(Ls / Ut) : 0.f;  // wrapper.py:212-217: mean over the finite rows, 0 if none
    st[1] = (float)U;
    st[2] = U > 0 ? (float)(Ns / U) : 0.f;
    st[3] = (float)(U > 0 ? Mn : 0);
    st[4] = U > 0 ? (float)(Rs / U) : 0.f;
    float med = 0.f;
    if (U > 0) {
      const float p = 0.5f * (float)(U - 1);
      med = (float)sel[0] + (p - (float)p_lo) * (float)(sel[1] - sel[0]);
    }
    st[5] = med;
    st[6] = (float)g.off;
    st[7] = (float)Ut;
  }
}

__global__ __launch_bounds__(256) void cl_wscale_k(ClArgs a0, const float* __restrict__ stats, int nstat,
                                                   float loss_scale) {
  const ClArgs a = head_args(a0, blockIdx.z);
  const int mb = blockIdx.y;
  const float U = stats[((int64_t)blockIdx.z * a0.n_mb + mb) * nstat + 7];  // used tokens
  const float wr = U > 0.f ? loss_scale / U : 0.f;
  float* w = a.colb + (int64_t)mb * a.n_max;  // = the row weights w in the forward
  for (int r = blockIdx.x * 256 + threadIdx.x; r < a.n_max; r += gridDim.x * 256) w[r] = w[r] != 0.f ? wr : 0.f;
}

// ---------------------------------------------------------------- tile engine
// 128 register rows per block (each wave: 32 rows = two 16-row MFMA tiles),
// 64-row column tiles streamed into a 3-deep LDS ring by LDS-DMA
// (global_load_lds_dwordx4): tile t + 2 is issued right after the barrier that
// opens tile t, so two tiles of loads are in flight behind the math; a counted
// `s_waitcnt vmcnt` plus a raw `s_barrier` retire tile t (no vmcnt(0) drain).
// The DMA's LDS destination is lane-linear, so the ks_off256 swizzle is applied
// to the source chunk.  Rows beyond n are read from a zero row; the wrapper
// zeroes the normalised `in` rows of pad positions, so pad columns of the
// forward / dOut images are zero rows too.
//
// Rows are L2-normalised, so every logit lies in [-1/tau, 1/tau] (up to bf16
// rounding): with 2/tau <= 80 the softmax shift is the constant 1/tau (no
// running max, exp never under- or overflows); smaller tau falls back to a
// per-tile online max.
//
// Clean tiles.  With the fixed shift, a column tile that holds no column of
// the sequences of the block's rows (no same-sequence exclusion, no diagonal)
// needs no per-element masking: pad columns are zero image rows with a -inf
// exponent shift (forward: their logit 0 is removed from the rank by count),
// so an element costs one fma + one v_exp (+ one compare for the rank).  Only
// the <= 3-4 tiles that meet the block's own sequences take the masked path.
// Exponentials are exp2 with log2(e) folded into the scale and the row weights
// folded into the shift (w e^t = 2^(t log2 e + log2 w)).
constexpr int CL_ROWS = 128;
constexpr int CL_NBUF = 3;
constexpr float LOG2E = 1.4426950408889634f;

// M1: whether the second per-column vector is used (the fixed-shift forward has none,
// which brings its LDS under 160 KiB / 3 for three blocks, i.e. three waves per SIMD)
template <bool M1 = true, int NB = CL_NBUF>
struct ClTile {
  unsigned char img[NB][64 * 256];
  float m0[NB][4][64];             // per-wave copies of a per-column vector (fwd: diag; bwd COLS: shift)
  float m1[NB][4][M1 ? 64 : 1];    // bwd COLS: row weights of the image rows; fwd: logQ of the columns
};

__device__ __attribute__((aligned(16))) unsigned char cl_zero_row[256];
__device__ float cl_ninf = -INFINITY;  // per-column values for the columns past n_max of a tile
__device__ float cl_zero_f = 0.f;


// Image-row staging.  Wave w stages rows 16w .. 16w + 15 of every tile with four
// DMAs of 4 rows x 256 B; lane l lands at row 16w + 4k + l/16, slot l%16 and so
// loads chunk slot ^ swz(row), which puts chunk ch at ks_off256(row, ch).  The
// source row of column c = (b, t) (sequence b of the mini-batch, position t) sits
// at base + b * sb + t * st elements; the cursor advances (b, t) by 64 columns a
// tile without a division.
template <bool SW32 = false, int NK = 4>
struct RowCursor {
  const bf16_t* base;
  int sb, st, L, q64, r64;
  int b[NK], t[NK], choff[NK];
  int c;  // column of this lane's k = 0 row in the next tile to stage
  __device__ __forceinline__ void init(const bf16_t* base_, int sb_, int st_, int L_, int w, int lane) {
    base = base_; sb = sb_; st = st_; L = L_;
    q64 = 64 / L; r64 = 64 - q64 * L;
    c = 4 * NK * w + (lane >> 4);
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int row = c + 4 * k;
      b[k] = row / L;
      t[k] = row - b[k] * L;
      choff[k] = ((lane & 15) ^ (SW32 ? swz32(row) : swz(row))) * 8;
    }
  }
  // stage the next tile into img (the tile's 64-row image), then advance by 64 columns
  __device__ __forceinline__ void stage(unsigned char* img, int n, int w, int lane) {
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const void* src = (c + 4 * k < n) ? (const void*)(base + ((int64_t)b[k] * sb + t[k] * st + choff[k]))
                                        : (const void*)(cl_zero_row + 16 * (lane & 15));
      glds16(src, img + (4 * NK * w + 4 * k) * 256);
      t[k] += r64;
      b[k] += q64;
      if (t[k] >= L) { t[k] -= L; b[k] += 1; }
    }
    c += 64;
  }
};

// transposed-k fragment: B[k][n = nb + (lane&15)] with k = 0..3 -> image rows
// kb + 4(lane>>4) + k and k = 4..7 -> rows kb + 16 + 4(lane>>4) + k-4, i.e. the k
// order in which a transposed S^T tile's C registers already sit per lane.
// Since swz(row) depends only on row & 15, the byte offset splits into a per-lane
// part for each 16-column block nd (trp_offsets, loop invariant) plus kb * 256 and
// 16 * 256 for the upper 4 k, which become ds_read immediates.
__device__ __forceinline__ void trp_offsets(int (&off)[8], int lane) {
  const int gq = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int row = 4 * gq + q;
#pragma unroll
  for (int nd = 0; nd < 8; ++nd) off[nd] = row * 256 + (((2 * nd + (p >> 1)) ^ swz(row)) << 4) + 8 * (p & 1);
}
typedef __attribute__((address_space(3))) unsigned char lds_u8;
// per-tile base of column block nd, laundered through an empty asm so the compiler
// cannot re-associate it with the kb / k offsets (which then fold into ds_read
// immediates instead of costing two VALU adds per read)
__device__ __forceinline__ lds_u8* trp_base(const unsigned char* img, int off) {
  lds_u8* p = (lds_u8*)img + off;
  asm volatile("" : "+v"(p));
  return p;
}
__device__ __forceinline__ bf16x8v trp_frag(lds_u8* base, int kb) {
  lds_u8* a0 = base + kb * 256;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0 + 16 * 256));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8v, v);
}

// S^T tile: acc[mi][yb][j] = img[yb*16 + 4(lane>>4) + j] . X[xbase + 16 mi + (lane&15)]
// (the register rows' A fragments double as the B operand)
__device__ __forceinline__ void st_tile(f32x4 (&acc)[2][4], const bf16x8v (&qf)[2][4], const unsigned char* img,
                                        int lane) {
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int yb = 0; yb < 4; ++yb) acc[mi][yb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int yb = 0; yb < 4; ++yb) {
      const bf16x8v af = row_frag(img, yb * 16 + (lane & 15), s * 4 + (lane >> 4));
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
        acc[mi][yb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, qf[mi][s], acc[mi][yb], 0, 0, 0);
    }
}

// this lane's 16 per-column values v[yb*16 + rg + j] of a 64-entry LDS row
__device__ __forceinline__ void col_vals(float (&o)[4][4], const float* v, int rg) {
#pragma unroll
  for (int yb = 0; yb < 4; ++yb) {
    const float4 q = *reinterpret_cast<const float4*>(v + yb * 16 + rg);
    o[yb][0] = q.x; o[yb][1] = q.y; o[yb][2] = q.z; o[yb][3] = q.w;
  }
}

// the column range [lo, hi) of the sequences that the block's rows [x0, x0 + 128) touch
__device__ __forceinline__ void own_cols(const Geo& g, int x0, int& lo, int& hi) {
  const int xe = min(x0 + CL_ROWS, g.n) - 1;
  lo = (x0 / g.L) * g.L;
  hi = (xe / g.L + 1) * g.L;
}

__device__ __forceinline__ float next_up(float t) {
  if (t != t || t == INFINITY) return t;
  if (t == 0.f) return __int_as_float(1);
  const int b = __float_as_int(t);
  return __int_as_float(t > 0.f ? b + 1 : b - 1);
}
// the largest float t with fl(t * it) <= dg, so that (a > t) == (fl(a * it) > dg)
// for every float a (a -> fl(a * it) is monotone for it > 0)
__device__ __forceinline__ float rank_threshold(float dg, float it, float tau) {
  float t = dg * tau;
  for (int k = 0; k < 16 && t * it > dg; ++k) t = -next_up(-t);
  for (int k = 0; k < 16 && next_up(t) * it <= dg; ++k) t = next_up(t);
  return t;
}

// NB: LDS ring depth (3: two tiles of loads in flight behind the math; 2: one), OCC:
// blocks per CU the registers and LDS are sized for
template <bool FIXED, int NB, int OCC>
__global__ __launch_bounds__(256, OCC) void cl_fwd_k(ClArgs a0) {
  __shared__ __attribute__((aligned(16))) ClTile<!FIXED, NB> sh;
  // (row block, mini-batch, head) from one XCD-remapped linear id: each XCD walks a
  // contiguous run of (head, mini-batch) pairs
  const int per_head = gridDim.x * gridDim.y;
  const int lin = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), per_head * gridDim.z);
  const int z = lin / per_head, bid = lin - z * per_head;
  const ClArgs a = head_args(a0, z);
  const int mb = bid / gridDim.x;
  const Geo g = geo(a, mb);
  const int r0 = (bid - mb * gridDim.x) * CL_ROWS;
  if (r0 >= g.n) return;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, rg = 4 * (lane >> 4);
  const int64_t base = (int64_t)mb * a.n_max;
  bf16x8v qf[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
    reg_frags(qf[mi], lane, g.n, r0 + 32 * w + 16 * mi, [&](int r) { return out_row(a, g, r); });
  const float it = 1.f / a.tau, c1 = it * LOG2E, cs = -it * LOG2E;
  int spec_lo, spec_hi;
  own_cols(g, r0, spec_lo, spec_hi);
  // this lane's rows: r = r0 + 32 w + 16 mi + col  (one per mi)
  float m[2], l[2], pv[2], dg[2], thr[2];
  int cn[2], rk[2], rsq[2], rr[2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int r = r0 + 32 * w + 16 * mi + col;
    rr[mi] = r;
    m[mi] = FIXED ? it : -INFINITY;
    l[mi] = 0.f; pv[mi] = -INFINITY; cn[mi] = 0; rk[mi] = 0;
    dg[mi] = (r < g.n) ? a.diag[base + r] : 0.f;
    thr[mi] = rank_threshold(dg[mi], it, a.tau);
    rsq[mi] = (r < g.n) ? seq_of(g, r) : -2;
  }
  const int ntile = (g.n + 63) / 64;
  // 5 DMAs per wave and tile: 4 image pieces + the diag (pad flag) of the tile's columns
  RowCursor<> cur_in;
  cur_in.init(a.in_n + ((g.b0 * a.T) + g.off) * DE, a.T * DE, DE, g.L, w, lane);
  auto stage = [&](int t) {
    const int buf = t % NB;
    cur_in.stage(sh.img[buf], g.n, w, lane);
    glds4(t * 64 + lane < a.n_max ? a.colb + base + t * 64 + lane : &cl_ninf, sh.m0[buf][w]);
    if (!FIXED) glds4(a.lq && t * 64 + lane < a.n_max ? a.lqcol + base + t * 64 + lane : &cl_zero_f, sh.m1[buf][w]);
  };
  retire_loads();
  stage(0);
  if (NB > 2 && ntile > 1) stage(1);
  for (int tI = 0; tI < ntile; ++tI) {
    const int cur = tI % NB, c0 = tI * 64;
    if (NB > 2 && tI + 1 < ntile) wait_vm<FIXED ? 5 : 6>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (tI + NB - 1 < ntile) stage(tI + NB - 1);
    f32x4 acc[2][4];
    st_tile(acc, qf, sh.img[cur], lane);
    const float* cdg = sh.m0[cur][w];  // column exp2 bias: cs, or -inf for a pad column / beyond n
    const float* clq = sh.m1[cur][w];  // !FIXED: logQ correction of the columns (0 without logQ)
    const bool special = !FIXED || (c0 < spec_hi && c0 + 64 > spec_lo);
    if (!special) {
      float cb[4][4];
      col_vals(cb, cdg, rg);
      const int np = __popcll(__ballot(cdg[lane] == -INFINITY));
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        int k = 0;
#pragma unroll
        for (int yb = 0; yb < 4; ++yb)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            l[mi] += __builtin_amdgcn_exp2f(__builtin_fmaf(acc[mi][yb][j], c1, cb[yb][j]));
            k += acc[mi][yb][j] > thr[mi] ? 1 : 0;
          }
        // the zero pad / beyond-n rows give logit 0: count them once per row (lane group 0)
        if (rg == 0) {
          cn[mi] += 64 - np;
          k -= (0.f > thr[mi]) ? np : 0;
        }
        rk[mi] += k;
      }
    } else {
      int csq[4][4];
      bool cok[4][4];
#pragma unroll
      for (int yb = 0; yb < 4; ++yb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cl = yb * 16 + rg + j;
          cok[yb][j] = cdg[cl] != -INFINITY;
          csq[yb][j] = seq_of(g, c0 + cl);
        }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const int r = rr[mi];
        if constexpr (!FIXED) {
          float bm = -INFINITY;
#pragma unroll
          for (int yb = 0; yb < 4; ++yb)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int c = c0 + yb * 16 + rg + j;
              const float vq = acc[mi][yb][j] * it + (c == r ? 0.f : clq[yb * 16 + rg + j]);
              if (cok[yb][j] && (csq[yb][j] != rsq[mi] || c == r)) bm = fmaxf(bm, vq);
            }
          bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
          bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
          const float mn = fmaxf(m[mi], bm);
          if (mn != -INFINITY) {
            l[mi] *= (m[mi] == -INFINITY) ? 0.f : __expf(m[mi] - mn);
            m[mi] = mn;
          }
        }
#pragma unroll
        for (int yb = 0; yb < 4; ++yb)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int c = c0 + yb * 16 + rg + j;
            const float v = acc[mi][yb][j] * it;
            if (c == r) pv[mi] = v;
            if (cok[yb][j] && (csq[yb][j] != rsq[mi] || c == r)) {
              // the CE sees the logQ-corrected logit, the rank the plain one (wrapper.py:204-233)
              l[mi] += __expf((FIXED || c == r ? v : v + clq[yb * 16 + rg + j]) - m[mi]);
              cn[mi] += 1;
              rk[mi] += (c != r && v > dg[mi]) ? 1 : 0;
            }
          }
      }
    }
  }
  // combine the 4 lane groups that share each row
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    float mm = m[mi], ll = l[mi], pp = pv[mi];
    int cc = cn[mi], kk = rk[mi];
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      if constexpr (FIXED) {
        ll += __shfl_xor(ll, o, 64);
      } else {
        const float m2 = __shfl_xor(mm, o, 64), l2 = __shfl_xor(ll, o, 64);
        const float mn = fmaxf(mm, m2);
        ll = (mm == -INFINITY ? 0.f : ll * __expf(mm - mn)) + (m2 == -INFINITY ? 0.f : l2 * __expf(m2 - mn));
        mm = mn;
      }
      pp = fmaxf(pp, __shfl_xor(pp, o, 64));
      cc += __shfl_xor(cc, o, 64);
      kk += __shfl_xor(kk, o, 64);
    }
    const int r = rr[mi];
    if (rg == 0 && r < g.n) {
      const int64_t o = base + r;
      a.lse[o] = (cc > 0) ? mm + __logf(ll) : -INFINITY;
      a.pos[o] = pp;
      a.cnt[o] = cc;
      a.rank[o] = kk;
    }
  }
}

// ROWS = true : register rows are `out` rows r, image rows are `in` cols c  -> dOut
// ROWS = false: register rows are `in` cols c, image rows are `out` rows r  -> dIn
// The S^T tile leaves dS in the A-operand lanes of dS . img (k order matched by
// trp_frag), so no LDS round trip is needed between the two MFMAs.
// dS[r][c] = w_r (exp(S[r][c] / tau - lse_r) - [r == c]) on kept (r, c), computed
// as 2^(S c1 + shift_r) - w_r [r == c] (shift from cl_shift_k, in a.diag).
// ROWS: pad columns are zero image rows, so their dS never reaches dOut (with a
// running shift the exponent is capped at log2 w_r, where every kept dS lies,
// so it stays finite).
template <bool ROWS, bool FIXED>
__global__ __launch_bounds__(256, 2) void cl_bwd_k(ClArgs a) {
  __shared__ __attribute__((aligned(16))) ClTile<> sh;
  const int bid = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
  const int mb = bid / gridDim.x;
  const Geo g = geo(a, mb);
  const int x0 = (bid - mb * gridDim.x) * CL_ROWS;
  if (x0 >= g.n) return;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, rg = 4 * (lane >> 4);
  const int64_t base = (int64_t)mb * a.n_max;
  const float* shift = a.diag;
  const float it = 1.f / a.tau, c1 = it * LOG2E;
  int spec_lo, spec_hi;
  own_cols(g, x0, spec_lo, spec_hi);
  bf16x8v qf[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    if (ROWS) reg_frags(qf[mi], lane, g.n, x0 + 32 * w + 16 * mi, [&](int r) { return out_row(a, g, r); });
    else reg_frags(qf[mi], lane, g.n, x0 + 32 * w + 16 * mi, [&](int c) { return in_row(a, g, c); });
  }
  // this lane's register row per mi (x = x0 + 32 w + 16 mi + col)
  float xsh[2], xw[2], xcap[2], xq[2];
  bool xpad[2];
  int xsq[2], xx[2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int x = x0 + 32 * w + 16 * mi + col;
    const bool in = x < g.n;
    xx[mi] = x;
    xw[mi] = (ROWS && in) ? a.w[base + x] : 0.f;
    xsh[mi] = (ROWS && in) ? shift[base + x] : -INFINITY;
    xcap[mi] = xw[mi] != 0.f ? __log2f(xw[mi]) : -INFINITY;
    xpad[mi] = in ? (ROWS ? false : pad_of(a, g, x)) : true;
    xsq[mi] = in ? seq_of(g, x) : -2;
    // COLS: the logQ correction of this register row's column (log2 units)
    xq[mi] = (!FIXED && !ROWS && a.lq && in) ? a.lqcol[base + x] * LOG2E : 0.f;
  }
  f32x4 dacc[2][8];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int i = 0; i < 8; ++i) dacc[mi][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  int toff[8];
  trp_offsets(toff, lane);
  const int ntile = (g.n + 63) / 64;
  // ROWS: 4 image DMAs per wave and tile; COLS: + shift and weight of the image rows
  RowCursor<> cur_img;
  if (ROWS) cur_img.init(a.in_n + ((g.b0 * a.T) + g.off) * DE, a.T * DE, DE, g.L, w, lane);
  else cur_img.init(a.out_n + (g.b0 * (a.T + 1) * a.NH + a.head) * DE, (a.T + 1) * a.NH * DE, a.NH * DE, g.L, w,
                    lane);
  auto stage = [&](int t) {
    const int buf = t % CL_NBUF, y0 = t * 64;
    cur_img.stage(sh.img[buf], g.n, w, lane);
    if (!ROWS) {
      const bool inr = y0 + lane < a.n_max;  // past n_max: shift -inf, weight 0
      glds4(inr ? shift + base + y0 + lane : &cl_ninf, sh.m0[buf][w]);
      glds4(inr ? a.w + base + y0 + lane : &cl_zero_f, sh.m1[buf][w]);
    } else if (!FIXED) {  // ROWS: the logQ correction of the image rows (columns)
      glds4(a.lq && y0 + lane < a.n_max ? a.lqcol + base + y0 + lane : &cl_zero_f, sh.m0[buf][w]);
    }
  };
  retire_loads();
  stage(0);
  if (ntile > 1) stage(1);
  for (int tI = 0; tI < ntile; ++tI) {
    const int cur = tI % CL_NBUF, y0 = tI * 64;
    if (tI + 1 < ntile) {
      if (ROWS) wait_vm<FIXED ? 4 : 5>();
      else wait_vm<6>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (tI + 2 < ntile) stage(tI + 2);
    const unsigned char* img = sh.img[cur];
    f32x4 acc[2][4];
    st_tile(acc, qf, img, lane);
    const bool special = !FIXED || (y0 < spec_hi && y0 + 64 > spec_lo);
    // dS in place: acc[mi][yb][j] <- dS[x][y],  y = y0 + yb*16 + rg + j
    if (!special) {
      if (ROWS) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int yb = 0; yb < 4; ++yb)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[mi][yb][j] = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[mi][yb][j], c1, xsh[mi]));
      } else {
        float ysh[4][4];
        col_vals(ysh, sh.m0[cur][w], rg);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int yb = 0; yb < 4; ++yb)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[mi][yb][j] = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[mi][yb][j], c1, ysh[yb][j]));
      }
    } else {
#pragma unroll
      for (int yb = 0; yb < 4; ++yb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int yl = yb * 16 + rg + j, y = y0 + yl;
          const int ysq = y < g.n ? seq_of(g, y) : -1;
          const float ysh = ROWS ? 0.f : sh.m0[cur][w][yl], yw = ROWS ? 0.f : sh.m1[cur][w][yl];
          const float yq = (ROWS && !FIXED) ? sh.m0[cur][w][yl] * LOG2E : 0.f;
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) {
            const int x = xx[mi];
            float ds = 0.f;
            const bool keep = (ysq != xsq[mi] || x == y);
            if (ROWS) {
              if (keep && xw[mi] != 0.f) {
                float t = __builtin_fmaf(acc[mi][yb][j], c1, xsh[mi] + (x == y ? 0.f : yq));
                if (!FIXED) t = fminf(t, xcap[mi]);
                ds = __builtin_amdgcn_exp2f(t) - (x == y ? xw[mi] : 0.f);
              }
            } else {
              if (!xpad[mi] && keep && yw != 0.f)
                ds = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[mi][yb][j], c1, ysh + (x == y ? 0.f : xq[mi]))) -
                     (x == y ? yw : 0.f);
            }
            acc[mi][yb][j] = ds;
          }
        }
    }
    // dacc[32 x 128] += dS[32 x 64] . img[64 x 128]   (k = y, in trp_frag order)
    lds_u8* tb[8];
#pragma unroll
    for (int nd = 0; nd < 8; ++nd) tb[nd] = trp_base(img, toff[nd]);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8v af[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const f32x4& p = acc[mi][2 * ks];
        const f32x4& q = acc[mi][2 * ks + 1];
        const u32x4 h = {pk_bf16(p[0], p[1]), pk_bf16(p[2], p[3]), pk_bf16(q[0], q[1]), pk_bf16(q[2], q[3])};
        af[mi] = __builtin_bit_cast(bf16x8v, h);
      }
#pragma unroll
      for (int nd = 0; nd < 8; ++nd) {
        const bf16x8v bfr = trp_frag(tb[nd], ks * 32);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          dacc[mi][nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr, dacc[mi][nd], 0, 0, 0);
      }
    }
  }
  // write: dacc[mi][nd][j] = d[x = x0 + 32 w + 16 mi + rg + j][e = nd*16 + col]
  // (COLS: pad `in` rows get no gradient; their dacc is not written)
  const float gs = (a.gscale ? *a.gscale : 1.f) * it;
  if (ROWS && a.dy) {
    // through F.normalize (the separate lthm_rownorm_bwd pass and the f32 d_out round trip
    // disappear): the 16 lanes of a lane group hold one row's 128 columns (col + 16 nd)
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int x = x0 + 32 * w + 16 * mi + rg + j;
        const int xc = min(x, g.n - 1);  // every lane takes part in the row reduction
        const int b = xc / g.L, t = xc - (xc / g.L) * g.L;
        const int64_t ro = ((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head;
        const float nrm = a.y_norm[ro], den = fmaxf(nrm, 1e-12f);
        float yv[8], dot = 0.f;
#pragma unroll
        for (int nd = 0; nd < 8; ++nd) {
          yv[nd] = bf2f(a.y_raw[ro * DE + nd * 16 + col]) / den;
          dot += yv[nd] * (gs * dacc[mi][nd][j]);
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) dot += __shfl_xor(dot, o, 64);
        if (x < g.n) {
#pragma unroll
          for (int nd = 0; nd < 8; ++nd) {
            const float gv = gs * dacc[mi][nd][j];
            a.dy[ro * DE + nd * 16 + col] = f2bf(nrm > 1e-12f ? (gv - yv[nd] * dot) / nrm : gv / 1e-12f);
          }
        }
      }
    return;
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = x0 + 32 * w + 16 * mi + rg + j;
      if (x >= g.n) continue;
      const int b = x / g.L, t = x - (x / g.L) * g.L;
      if (!ROWS && pad_of(a, g, x)) continue;
      float* dst = ROWS ? a.d_out + (((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head) * DE
                        : a.d_in + ((g.b0 + b) * a.T + t + g.off) * DE;
#pragma unroll
      for (int nd = 0; nd < 8; ++nd) {
        const float v = gs * dacc[mi][nd][j];
        if (ROWS) dst[nd * 16 + col] = v;
        else dst[nd * 16 + col] += v;
      }
    }
}


// ---------------------------------------------------------------- backward on 32x32x16 MFMA
// The same tile math as cl_bwd_k with v_mfma_f32_32x32x16_bf16: an MFMA holds the SIMD's
// vector issue for 8 of its 32 cycles instead of 8 of 16 (MI355X_MICROARCH.md, constants),
// so the per-element exp2 / fma / bf16 packing of dS fits beside the matrix work.
//  * S^T tile (64 image rows x 32 register rows per wave): acc[ib][v] = img[32 ib + 8(v>>2) +
//    4 hh + (v&3)] . X[x], hh = lane >> 5; the lane's register row x = x0 + 32 w + (lane & 31)
//    is the MFMA column, so every per-row quantity is a per-lane scalar.
//  * dS in place, then dS^T . img as the A operand with no lane movement (registers
//    8s..8s+7 of block ib are k-step 2 ib + s; cdna_hip_programming.md §3): the B operand is
//    read transposed from the same image (ds_read_b64_tr_b16), rows in that k order.
//  * the accumulator is restaged through LDS for the epilogue, where the gradient goes
//    through F.normalize (wrapper.py:118-119) and is written once in the operand's dtype.
// ROWS: grid (row blocks, n_mb, heads): register rows = out rows of one head; image = `in`.
// COLS: grid (physical-row blocks, n_mb): register rows = physical `in` rows (b, t) (the same
//   operand for every head); the image walks the out rows of every head in turn, so dIn is
//   summed over the heads in registers (no f32 d_in read-modify-write per head).
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(bf16x8v a, bf16x8v b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

constexpr int CL_EPS = 132;  // epilogue restage row stride (floats): conflict-free b32 writes / b128 reads

constexpr int CL_NB32 = 4;  // image ring depth of the 32x32x16 backward: three tiles of DMA in flight
template <int NW>
struct ClTile32 {
  union {
    struct {
      unsigned char img[CL_NB32][64 * 256];
      float m0[CL_NB32][NW][64];  // per-wave copies of a per-image-row vector (COLS: shift; ROWS !FIXED: logQ)
      float m1[CL_NB32][NW][64];  // COLS: row weights of the image rows
    } r;
    float ep[NW][32][CL_EPS];     // epilogue: each wave's 32 x 128 f32 accumulator, row-major
  };
};

// per-lane byte offsets of the 8 row fragments (k-step s) of an image row block and of the
// 8 transposed fragments (column block nd, lower / upper 4 k) of a 16-row k-step
__device__ __forceinline__ void frag32_offsets(int (&roff)[8], int (&toff)[4][2], int lane) {
  const int hh = lane >> 5, r32 = lane & 31, sw = swz32(r32);
#pragma unroll
  for (int s = 0; s < 8; ++s) roff[s] = r32 * 256 + (((2 * s + hh) ^ sw) << 4);
  const int g16 = lane >> 4, colhalf = g16 & 1, li = lane & 15, q = li >> 2, pp = li & 3;
#pragma unroll
  for (int nd = 0; nd < 4; ++nd)
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) {
      const int row = 4 * hh + 8 * hi + q;
      toff[nd][hi] = row * 256 + (((4 * nd + 2 * colhalf + (pp >> 1)) ^ swz32(row)) << 4) + 8 * (pp & 1);
    }
}

__device__ __forceinline__ bf16x8v tr_frag32(const unsigned char* img, int off_lo, int off_hi) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)((lds_u8*)img + off_lo));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)((lds_u8*)img + off_hi));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8v, v);
}

// the register row's per-lane state for one head
struct XRow {
  int x;        // row / column index in the head's logit matrix (-1: none)
  int sq;       // sequence of x (-2: none)
  bool live;    // contributes (COLS: a valid, non-pad column of this head; ROWS: x < n)
  float sh;     // ROWS: exp2 shift of row x (log2 w - lse log2 e)
  float w;      // ROWS: row weight
  float cap;    // ROWS, running shift: log2 w
  float q;      // COLS, logQ: the correction of column x (log2 units)
};

// dacc[nd] += dS^T . img over every image tile of one head (ROWS: image = `in` columns of the
// head; COLS: image = out rows of the head).  The special range [spec_lo, spec_hi) holds the
// image rows of the register rows' own sequences (diagonal, same-sequence exclusion).
template <bool ROWS, bool FIXED, int NW>
__device__ __forceinline__ void cl_bwd32_head(ClTile32<NW>& sh, f32x16 (&dacc)[4], const bf16x8v (&qf)[8],
                                              const int (&roff)[8], const int (&toff)[4][2], const ClArgs& a,
                                              const Geo& g, int64_t base, const XRow& xr, bool wmask, int spec_lo,
                                              int spec_hi, RowCursor<true, 16 / NW>& cur, int w, int lane) {
  const int hh = lane >> 5;
  const float it = 1.f / a.tau, c1 = it * LOG2E;
  const float* shift = a.diag;
  const int ntile = (g.n + 63) / 64;
  const int xlo = xr.sq >= 0 ? xr.sq * g.L : -(1 << 30);  // first image row of the register row's sequence
  auto stage = [&](int t) {
    const int buf = t % CL_NB32, y0 = t * 64;
    cur.stage(sh.r.img[buf], g.n, w, lane);
    if (!ROWS) {
      const bool inr = y0 + lane < a.n_max;  // past n_max: shift -inf, weight 0
      glds4(inr ? shift + base + y0 + lane : &cl_ninf, sh.r.m0[buf][w]);
      glds4(inr ? a.w + base + y0 + lane : &cl_zero_f, sh.r.m1[buf][w]);
    } else if (!FIXED) {
      glds4(a.lq && y0 + lane < a.n_max ? a.lqcol + base + y0 + lane : &cl_zero_f, sh.r.m0[buf][w]);
    }
  };
  constexpr int NK = 16 / NW;
  constexpr int PT = ROWS ? (FIXED ? NK : NK + 1) : NK + 2;  // DMAs per wave and tile
  retire_loads();
  stage(0);
  if (ntile > 1) stage(1);
  if (ntile > 2) stage(2);
  for (int tI = 0; tI < ntile; ++tI) {
    const int cb = tI % CL_NB32, y0 = tI * 64;
    if (tI + 2 < ntile) wait_vm<2 * PT>();
    else if (tI + 1 < ntile) wait_vm<PT>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (tI + 3 < ntile) stage(tI + 3);
    const unsigned char* img = sh.r.img[cb];
    f32x16 acc[2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[ib][v] = 0.f;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const bf16x8v af = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(img + ib * 8192 + roff[s]));
        acc[ib] = mfma32(af, qf[s], acc[ib]);
      }
    }
    const bool special = !FIXED || (y0 < spec_hi && y0 + 64 > spec_lo);
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      if (!special) {
        if (ROWS) {
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[ib][v] = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[ib][v], c1, xr.sh));
        } else {
#pragma unroll
          for (int qd = 0; qd < 4; ++qd) {
            const float4 ys = *reinterpret_cast<const float4*>(&sh.r.m0[cb][w][32 * ib + 8 * qd + 4 * hh]);
            const float yv[4] = {ys.x, ys.y, ys.z, ys.w};
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[ib][4 * qd + j] = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[ib][4 * qd + j], c1, yv[j]));
          }
        }
      } else {
        // y0 laundered: without it loop strength reduction keeps a 64-bit running product of
        // seq_of for each of the 32 elements across the tile loop (64 VGPRs, spills)
        int ys0 = y0;
        asm volatile("" : "+s"(ys0));
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int yl = 32 * ib + 8 * (v >> 2) + 4 * hh + (v & 3), y = ys0 + yl;
#if defined(CL_SP2)
          // branch-free: the register row's own sequence is [xlo, xlo + L); beyond-n image rows
          // are zero (ROWS) or carry weight 0 (COLS)
          const bool same = (unsigned)(y - xlo) < (unsigned)g.L;
          const bool keep = xr.live && (!same || xr.x == y);
          const bool dg = xr.x == y;
          float ds;
          if (ROWS) {
            const float yq = FIXED ? 0.f : sh.r.m0[cb][w][yl] * LOG2E;
            float t = __builtin_fmaf(acc[ib][v], c1, xr.sh + (dg ? 0.f : yq));
            if (!FIXED) t = fminf(t, xr.cap);
            const float e = __builtin_amdgcn_exp2f(t) - (dg ? xr.w : 0.f);
            ds = (keep && xr.w != 0.f) ? e : 0.f;
          } else {
            const float ysh = sh.r.m0[cb][w][yl], yw = sh.r.m1[cb][w][yl];
            const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[ib][v], c1, ysh + (dg ? 0.f : xr.q))) -
                            (dg ? yw : 0.f);
            ds = (keep && yw != 0.f) ? e : 0.f;
          }
          acc[ib][v] = ds;
#else
          const int ysq = y < g.n ? seq_of(g, y) : -1;
          const bool keep = xr.live && (ysq != xr.sq || xr.x == y);
          float ds = 0.f;
          if (ROWS) {
            const float yq = FIXED ? 0.f : sh.r.m0[cb][w][yl] * LOG2E;
            if (keep && xr.w != 0.f) {
              float t = __builtin_fmaf(acc[ib][v], c1, xr.sh + (xr.x == y ? 0.f : yq));
              if (!FIXED) t = fminf(t, xr.cap);
              ds = __builtin_amdgcn_exp2f(t) - (xr.x == y ? xr.w : 0.f);
            }
          } else {
            const float ysh = sh.r.m0[cb][w][yl], yw = sh.r.m1[cb][w][yl];
            if (keep && yw != 0.f)
              ds = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[ib][v], c1, ysh + (xr.x == y ? 0.f : xr.q))) -
                   (xr.x == y ? yw : 0.f);
          }
          acc[ib][v] = ds;
#endif
        }
      }
      // dacc[32 x 128] += dS[32 x 32] . img[32 x 128] of this image block: k-step ks = 2 ib + hf
      // holds image rows 16 ks + 8 (j>>2) + 4 hh + (j&3) in element j (registers 8 hf .. 8 hf + 7)
  #pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int ks = 2 * ib + hf, o = 8 * hf;
        const f32x16& pv = acc[ib];
        u32x4 hpk = {pk_bf16(pv[o], pv[o + 1]), pk_bf16(pv[o + 2], pv[o + 3]), pk_bf16(pv[o + 4], pv[o + 5]),
                     pk_bf16(pv[o + 6], pv[o + 7])};
        if (wmask && !xr.live) hpk = u32x4{0u, 0u, 0u, 0u};  // COLS: a column this head does not have
        const bf16x8v af = __builtin_bit_cast(bf16x8v, hpk);
#pragma unroll
        for (int nd = 0; nd < 4; ++nd) {
          const bf16x8v bfr = tr_frag32(img, toff[nd][0] + ks * 4096, toff[nd][1] + ks * 4096);
          dacc[nd] = mfma32(af, bfr, dacc[nd]);
        }
      }
      }
  }
}

// gradient through F.normalize, written in the operand's dtype: dx = (g - y (y . g)) / |x|,
// y = x / max(|x|, eps) (the eps branch: g / eps).  16 lanes per row, 8 columns per lane.
__device__ __forceinline__ void normalize_bwd_store(const float (&gv)[8], const void* xraw, int xdt, float nrm,
                                                    void* dst, int64_t elem, bool write) {
  const float den = fmaxf(nrm, 1e-12f);
  float yv[8], dot = 0.f;
  if (xdt == LTHM_BF16) load_vec<bf16_t, 16>((const bf16_t*)xraw + elem, yv);
  else {
    load_vec<float, 16>((const float*)xraw + elem, yv);
    load_vec<float, 16>((const float*)xraw + elem + 4, yv + 4);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    yv[i] /= den;
    dot += yv[i] * gv[i];
  }
  dot = group16_sum(dot);
  if (!write) return;
  float o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = nrm > 1e-12f ? (gv[i] - yv[i] * dot) / nrm : gv[i] / 1e-12f;
  if (xdt == LTHM_BF16) store_vec<bf16_t, 8>((bf16_t*)dst + elem, o);
  else {
    store_vec<float, 4>((float*)dst + elem, o);
    store_vec<float, 4>((float*)dst + elem + 4, o + 4);
  }
}

// NW waves per workgroup (32 NW register rows): 4 (two workgroups per CU) or 8 (one workgroup
// per CU: each image tile is staged once for 256 register rows, half the DMA issue per wave)
template <bool ROWS, bool FIXED, int NW>
__global__ __launch_bounds__(64 * NW, 2) void cl_bwd32_k(ClArgs a0) {
  constexpr int XR = 32 * NW;  // register rows per workgroup
  __shared__ __attribute__((aligned(16))) ClTile32<NW> sh;
  const int nz = ROWS ? gridDim.z : 1;
  const int per = gridDim.x * gridDim.y;
  const int lin = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * (ROWS ? blockIdx.z : 0)), per * nz);
  const int z = lin / per, bid = lin - z * per;
  const int mb = bid / gridDim.x, xb = bid - mb * gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int64_t base = (int64_t)mb * a0.n_max;
  const int64_t b0 = (int64_t)mb * a0.mbs;
  const int Bm = (int)min((int64_t)a0.mbs, a0.B - b0);
  int roff[8], toff[4][2];
  frag32_offsets(roff, toff, lane);
  f32x16 dacc[4];
#pragma unroll
  for (int nd = 0; nd < 4; ++nd)
#pragma unroll
    for (int v = 0; v < 16; ++v) dacc[nd][v] = 0.f;
  bf16x8v qf[8];
  const float gs = (a0.gscale ? *a0.gscale : 1.f) / a0.tau;
  if (ROWS) {
    const ClArgs a = head_args(a0, z);
    const Geo g = geo(a, mb);
    const int x0 = xb * XR;
    if (x0 >= g.n) return;
    XRow xr;
    xr.x = x0 + 32 * w + r32;
    xr.live = xr.x < g.n;
    {
      const bf16_t* rp = xr.live ? out_row(a, g, xr.x) : nullptr;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        u32x4 v = {0u, 0u, 0u, 0u};
        if (xr.live) v = *reinterpret_cast<const u32x4*>(rp + 16 * s + 8 * (lane >> 5));
        qf[s] = __builtin_bit_cast(bf16x8v, v);
      }
    }
    xr.w = xr.live ? a.w[base + xr.x] : 0.f;
    xr.sh = xr.live ? a.diag[base + xr.x] : -INFINITY;
    xr.cap = xr.w != 0.f ? __log2f(xr.w) : -INFINITY;
    xr.sq = xr.live ? seq_of(g, xr.x) : -2;
    xr.q = 0.f;
    const int spec_lo = (x0 / g.L) * g.L, spec_hi = ((min(x0 + XR, g.n) - 1) / g.L + 1) * g.L;
    RowCursor<true, 16 / NW> cur;
    cur.init(a.in_n + ((g.b0 * a.T) + g.off) * DE, a.T * DE, DE, g.L, w, lane);
    cl_bwd32_head<true, FIXED, NW>(sh, dacc, qf, roff, toff, a, g, base, xr, false, spec_lo, spec_hi, cur, w, lane);
    // epilogue: restage, then 16 lanes per row through F.normalize into dy
    __syncthreads();
#pragma unroll
    for (int nd = 0; nd < 4; ++nd)
#pragma unroll
      for (int v = 0; v < 16; ++v) sh.ep[w][8 * (v >> 2) + 4 * (lane >> 5) + (v & 3)][32 * nd + r32] = dacc[nd][v];
    const int sub = lane & 15;
#pragma unroll 1
    for (int ps = 0; ps < 8; ++ps) {
      const int rl = 4 * ps + (lane >> 4), x = x0 + 32 * w + rl;
      const int xc = min(x, g.n - 1);  // every lane takes part in the row reduction
      const int b = xc / g.L, t = xc - b * g.L;
      const int64_t ro = ((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head;
      float gv[8];
      const float4 u0 = *reinterpret_cast<const float4*>(&sh.ep[w][rl][8 * sub]);
      const float4 u1 = *reinterpret_cast<const float4*>(&sh.ep[w][rl][8 * sub + 4]);
      gv[0] = gs * u0.x; gv[1] = gs * u0.y; gv[2] = gs * u0.z; gv[3] = gs * u0.w;
      gv[4] = gs * u1.x; gv[5] = gs * u1.y; gv[6] = gs * u1.z; gv[7] = gs * u1.w;
      normalize_bwd_store(gv, a.y_raw, a.y_dtype, a.y_norm[ro], a.dy, ro * DE + 8 * sub, x < g.n);
    }
    return;
  }
  // COLS: physical `in` rows p = b T + t of the mini-batch
  const int T = a0.T;
  const int nphys = Bm * T;
  const int p0 = xb * XR;
  if (p0 >= nphys) return;
  const int p = p0 + 32 * w + r32;
  const bool pin = p < nphys;
  const int pb = pin ? p / T : 0, pt = pin ? p - pb * T : 0;
  const bool ppad = !pin || a0.mask[(b0 + pb) * a0.mask_stride + pt] != 0;
  {
    const bf16_t* rp = a0.in_n + ((b0 + pb) * T + pt) * DE;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (pin) v = *reinterpret_cast<const u32x4*>(rp + 16 * s + 8 * (lane >> 5));
      qf[s] = __builtin_bit_cast(bf16x8v, v);
    }
  }
  const int b_lo = p0 / T, b_hi = (min(p0 + XR, nphys) - 1) / T;
  const int nrun = a0.heads_run;
#pragma unroll 1
  for (int hz = 0; hz < nrun; ++hz) {
    const ClArgs a = head_args(a0, hz);
    const Geo g = geo(a, mb);
    if (g.n == 0) continue;
    XRow xr;
    xr.live = !ppad && pt >= g.off;
    xr.x = xr.live ? pb * g.L + pt - g.off : -1;
    xr.sq = xr.live ? pb : -2;
    xr.sh = 0.f; xr.w = 0.f; xr.cap = 0.f;
    xr.q = (!FIXED && a.lq && xr.live) ? a.lqcol[base + xr.x] * LOG2E : 0.f;
    const bool wmask = __ballot(!xr.live) != 0ull;
    RowCursor<true, 16 / NW> cur;
    cur.init(a.out_n + (g.b0 * (a.T + 1) * a.NH + a.head) * DE, (a.T + 1) * a.NH * DE, a.NH * DE, g.L, w, lane);
    __syncthreads();  // the previous head's last tiles are read before this head's prologue restages the ring
    cl_bwd32_head<false, FIXED, NW>(sh, dacc, qf, roff, toff, a, g, base, xr, wmask, b_lo * g.L, (b_hi + 1) * g.L, cur,
                                w, lane);
  }
  __syncthreads();
#pragma unroll
  for (int nd = 0; nd < 4; ++nd)
#pragma unroll
    for (int v = 0; v < 16; ++v) sh.ep[w][8 * (v >> 2) + 4 * (lane >> 5) + (v & 3)][32 * nd + r32] = dacc[nd][v];
  const int sub = lane & 15;
#pragma unroll 1
  for (int ps = 0; ps < 8; ++ps) {
    const int rl = 4 * ps + (lane >> 4), q = p0 + 32 * w + rl;
    const int qc = min(q, nphys - 1);
    const int b = qc / T, t = qc - b * T;
    const int64_t ro = (b0 + b) * T + t;
    const bool pad = a0.mask[(b0 + b) * a0.mask_stride + t] != 0;
    float gv[8];
    const float4 u0 = *reinterpret_cast<const float4*>(&sh.ep[w][rl][8 * sub]);
    const float4 u1 = *reinterpret_cast<const float4*>(&sh.ep[w][rl][8 * sub + 4]);
    const float gz = pad ? 0.f : gs;  // pad rows of `in`: every logit against them is excluded
    gv[0] = gz * u0.x; gv[1] = gz * u0.y; gv[2] = gz * u0.z; gv[3] = gz * u0.w;
    gv[4] = gz * u1.x; gv[5] = gz * u1.y; gv[6] = gz * u1.z; gv[7] = gz * u1.w;
    normalize_bwd_store(gv, a0.t_raw, a0.t_dtype, a0.t_norm[ro], a0.dt, ro * DE + 8 * sub, q < nphys);
  }
}

// ---------------------------------------------------------------- fused forward + ROWS
// Training at the fixed shift: P[x][y] = p / Z_x with p = 2^(S c1 - log2 e / tau) needs no lse
// before the pass over the columns, so ONE pass gives the forward's Z_x (lse), counts and
// ranks AND U_x = sum_y p[x][y] in_y; at the end dOut_x = w_x (U_x / Z_x - in_x) goes
// through F.normalize into dy (unit upstream gradient: the backward scales dy by it).  The
// row weights w_x are known before the pass (cl_used_k: they depend on the pad mask only),
// so the row side of the backward costs no S recompute: forward + backward execute
// 8 n^2 De per head, the algorithmic count.

// row weights w_r = used_r * loss_scale / U of every head and mini-batch from the pad mask:
// row r is used when it is not a pad and some valid column lies outside its sequence (the
// forward's "at least one finite negative", wrapper.py:193-201); U = used rows of the
// mini-batch.  Also zeroes the dy rows the fused kernel never writes (t >= L).  Grid
// (n_mb, heads), one block each; V[b] valid tokens per sequence in LDS (Bm <= CL_UMAXB).
constexpr int CL_UMAXB = 4096;
__global__ __launch_bounds__(256) void cl_used_k(ClArgs a0, float* __restrict__ w0, float loss_scale) {
  const ClArgs a = head_args(a0, blockIdx.y);
  float* wout = w0 + (int64_t)blockIdx.y * a0.head_stride;
  const int mb = blockIdx.x;
  const Geo g = geo(a, mb);
  const int tid = threadIdx.x;
  const int64_t base = (int64_t)mb * a.n_max;
  __shared__ int V[CL_UMAXB];
  __shared__ double red[256];
  int nv = 0;
  for (int b = tid; b < g.Bm; b += 256) {
    int v = 0;
    for (int t = 0; t < g.L; ++t) v += pad_of(a, g, b * g.L + t) ? 0 : 1;
    V[b] = v;
    nv += v;
  }
  const int N = (int)block_dsum((double)nv, red);  // block_dsum syncs: V is complete
  int u = 0;
  for (int b = tid; b < g.Bm; b += 256) u += (N - V[b] > 0) ? V[b] : 0;
  const int U = (int)block_dsum((double)u, red);
  const float wr = U > 0 ? loss_scale / (float)U : 0.f;
  for (int r = tid; r < a.n_max; r += 256) {
    float wv = 0.f;
    if (r < g.n) {
      const int b = seq_of(g, r);
      wv = (!pad_of(a, g, r) && N - V[b] > 0) ? wr : 0.f;
    }
    wout[base + r] = wv;
  }
  const int tl0 = max(g.L, 0), ntail = a.T + 1 - tl0;
  const int per_seq = ntail * (DE / 4);
  const int64_t cnt = (int64_t)g.Bm * per_seq;
  for (int64_t i = tid; i < cnt; i += 256) {
    const int b = (int)(i / per_seq), rem = (int)(i - (int64_t)b * per_seq);
    const int t = tl0 + rem / (DE / 4), c4 = rem % (DE / 4);
    const int64_t o = (((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head) * DE + c4 * 4;
    if (a.y_dtype == LTHM_BF16) *reinterpret_cast<uint2*>(a.dy + o) = uint2{0u, 0u};
    else *reinterpret_cast<float4*>((float*)a.dy + o) = float4{0.f, 0.f, 0.f, 0.f};
  }
}

// dy *= *gscale (the fused forward wrote dy for a unit upstream gradient); nothing to do at 1
template <typename TY>
__global__ __launch_bounds__(256) void cl_dyscale_k(TY* __restrict__ dy, int64_t n, const float* __restrict__ gscale) {
  const float gs = *gscale;
  if (gs == 1.f) return;
  for (int64_t i = (blockIdx.x * (int64_t)256 + threadIdx.x) * 8; i < n; i += (int64_t)gridDim.x * 256 * 8) {
    float v[8];
    if (i + 8 <= n) {
      if constexpr (sizeof(TY) == 2) {
        load_vec<TY, 16>(dy + i, v);
      } else {
        load_vec<TY, 16>(dy + i, v);
        load_vec<TY, 16>(dy + i + 4, v + 4);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= gs;
      if constexpr (sizeof(TY) == 2) {
        store_vec<TY, 8>(dy + i, v);
      } else {
        store_vec<TY, 4>(dy + i, v);
        store_vec<TY, 4>(dy + i + 4, v + 4);
      }
    } else {
      for (int64_t k = i; k < n; ++k) Elem<TY>::st(dy + k, Elem<TY>::ld(dy + k) * gs);
    }
  }
}

// the fused pass of one head: Z, counts, ranks of the lane's register row x (lane & 31, the
// two lane halves holding alternate 4-column groups of every tile) and dacc += p . img
__device__ __forceinline__ void cl_fr32_head(ClTile32<4>& sh, f32x16 (&dacc)[4], const bf16x8v (&qf)[8],
                                             const int (&roff)[8], const int (&toff)[4][2], const ClArgs& a,
                                             const Geo& g, int64_t base, int x, int xsq, float thr, float& Z,
                                             int& cn, int& rk, float& pv, int spec_lo, int spec_hi,
                                             RowCursor<true, 4>& cur, int w, int lane) {
  constexpr int NW = 4, NK = 16 / NW, PT = NK + 1;  // DMAs per wave and tile: image + column bias
  const int hh = lane >> 5;
  const float it = 1.f / a.tau, c1 = it * LOG2E;
  const bool live = x < g.n;
  const int xlo = live ? xsq * g.L : -(1 << 30);  // first column of x's sequence
  const uint64_t hmask = hh ? 0xF0F0F0F0F0F0F0F0ull : 0x0F0F0F0F0F0F0F0Full;  // this half's columns
  const int ntile = (g.n + 63) / 64;
  auto stage = [&](int t) {
    const int buf = t % CL_NB32, y0 = t * 64;
    cur.stage(sh.r.img[buf], g.n, w, lane);
    glds4(y0 + lane < a.n_max ? a.colb + base + y0 + lane : &cl_ninf, sh.r.m0[buf][w]);
  };
  retire_loads();
  stage(0);
  if (ntile > 1) stage(1);
  if (ntile > 2) stage(2);
#if defined(CL_EXP) && CL_EXP >= 6
  wait_vm<0>();
  __builtin_amdgcn_s_barrier();
#endif
  for (int tI = 0; tI < ntile; ++tI) {
#if defined(CL_EXP) && CL_EXP >= 6
    // skeleton experiment: no staging / waits / barriers (the first tiles are reused)
    const int cb = tI % 3, y0 = tI * 64;
#else
    const int cb = tI % CL_NB32, y0 = tI * 64;
    if (tI + 2 < ntile) wait_vm<2 * PT>();
    else if (tI + 1 < ntile) wait_vm<PT>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (tI + 3 < ntile) stage(tI + 3);
#endif
    const unsigned char* img = sh.r.img[cb];
    const float* colb = sh.r.m0[cb][w];
    f32x16 acc[2];
#if defined(CL_PF)
    // the two image blocks' S chains interleaved (no back-to-back dependent MFMA), each
    // k-step's A fragments read one step ahead behind a compiler fence
    {
      acc[0] = f32x16{};
      acc[1] = f32x16{};
      auto rd = [&](int ib, int s2) {
        return __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(img + ib * 8192 + roff[s2]));
      };
      bf16x8v a0 = rd(0, 0), a1 = rd(1, 0);
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) {
        const int sn = s2 + 1 < 8 ? s2 + 1 : s2;
        const bf16x8v n0 = rd(0, sn), n1 = rd(1, sn);
        acc[0] = mfma32(a0, qf[s2], acc[0]);
        acc[1] = mfma32(a1, qf[s2], acc[1]);
        a0 = n0;
        a1 = n1;
        asm volatile("" ::: "memory");
      }
    }
#else
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[ib][v] = 0.f;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const bf16x8v af = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(img + ib * 8192 + roff[s]));
        acc[ib] = mfma32(af, qf[s], acc[ib]);
      }
    }
#endif
#if defined(CL_EXP) && CL_EXP >= 2
    const bool special = false;
#else
    const bool special = y0 < spec_hi && y0 + 64 > spec_lo;
#endif
    if (!special) {
      // every valid column is kept; pad / beyond-n columns are zero image rows (S = 0) with a
      // -inf bias: counted out of cn, and out of the rank when 0 > thr
      const int np = __popcll(__ballot(colb[lane] == -INFINITY) & hmask);
      cn += 32 - np;
      rk -= (0.f > thr) ? np : 0;
    }
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const float4 c4 = *reinterpret_cast<const float4*>(colb + 32 * ib + 8 * qd + 4 * hh);
        const float cv[4] = {c4.x, c4.y, c4.z, c4.w};
        if (!special) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int v = 4 * qd + j;
            const float sv = acc[ib][v];
#if defined(CL_EXP) && CL_EXP >= 5
            const float p = sv;
#elif defined(CL_EXP) && CL_EXP >= 4
            const float p = __builtin_fmaf(sv, c1, cv[j]);
#else
            const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c1, cv[j]));
#endif
#if !defined(CL_EXP) || CL_EXP < 5
            Z += p;
#endif
#if !defined(CL_EXP) || CL_EXP < 3
            rk += sv > thr ? 1 : 0;
#endif
            acc[ib][v] = p;
          }
        } else {
          int ys0 = y0;  // laundered (see cl_bwd32_head)
          asm volatile("" : "+s"(ys0));
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int v = 4 * qd + j, yl = 32 * ib + 8 * qd + 4 * hh + j, y = ys0 + yl;
            const float sv = acc[ib][v];
#if defined(CL_SP2)
            // branch-free: x's own sequence is [xlo, xlo + L); pads / beyond-n carry cv = -inf
            if (y == x) pv = sv * it;
            const bool same = (unsigned)(y - xlo) < (unsigned)g.L;
            const bool keep = live && cv[j] != -INFINITY && (!same || y == x);
            const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c1, cv[j]));
            const float p = keep ? e : 0.f;
            Z += p;
            cn += keep ? 1 : 0;
            rk += (keep && y != x && sv > thr) ? 1 : 0;
#else
            if (y == x) pv = sv * it;
            const int ysq = y < g.n ? seq_of(g, y) : -1;
            const bool keep = live && cv[j] != -INFINITY && (ysq != xsq || y == x);
            float p = 0.f;
            if (keep) {
              p = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c1, cv[j]));
              Z += p;
              cn += 1;
              rk += (y != x && sv > thr) ? 1 : 0;
            }
#endif
            acc[ib][v] = p;
          }
        }
      }
      // dacc[32 x 128] += p[32 x 32] . img[32 x 128] (as cl_bwd32_head)
#if defined(CL_PF)
      {
        const f32x16& pvv = acc[ib];
        const bf16x8v af0 = __builtin_bit_cast(bf16x8v, u32x4{pk_bf16(pvv[0], pvv[1]), pk_bf16(pvv[2], pvv[3]),
                                                              pk_bf16(pvv[4], pvv[5]), pk_bf16(pvv[6], pvv[7])});
        const bf16x8v af1 = __builtin_bit_cast(bf16x8v, u32x4{pk_bf16(pvv[8], pvv[9]), pk_bf16(pvv[10], pvv[11]),
                                                              pk_bf16(pvv[12], pvv[13]), pk_bf16(pvv[14], pvv[15])});
        const int k0 = 2 * ib * 4096, k1 = (2 * ib + 1) * 4096;
        bf16x8v b0 = tr_frag32(img, toff[0][0] + k0, toff[0][1] + k0), b1 = tr_frag32(img, toff[0][0] + k1, toff[0][1] + k1);
#pragma unroll
        for (int nd = 0; nd < 4; ++nd) {
          const int nn = nd + 1 < 4 ? nd + 1 : nd;
          const bf16x8v q0 = tr_frag32(img, toff[nn][0] + k0, toff[nn][1] + k0);
          const bf16x8v q1 = tr_frag32(img, toff[nn][0] + k1, toff[nn][1] + k1);
          dacc[nd] = mfma32(af0, b0, dacc[nd]);
          dacc[nd] = mfma32(af1, b1, dacc[nd]);
          b0 = q0;
          b1 = q1;
          asm volatile("" ::: "memory");
        }
      }
#else
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int ks = 2 * ib + hf, o = 8 * hf;
        const f32x16& pvv = acc[ib];
        const u32x4 hpk = {pk_bf16(pvv[o], pvv[o + 1]), pk_bf16(pvv[o + 2], pvv[o + 3]), pk_bf16(pvv[o + 4], pvv[o + 5]),
                           pk_bf16(pvv[o + 6], pvv[o + 7])};
        const bf16x8v af = __builtin_bit_cast(bf16x8v, hpk);
#pragma unroll
        for (int nd = 0; nd < 4; ++nd) {
          const bf16x8v bfr = tr_frag32(img, toff[nd][0] + ks * 4096, toff[nd][1] + ks * 4096);
          dacc[nd] = mfma32(af, bfr, dacc[nd]);
        }
      }
#endif
    }
  }
}

// grid ((n_max + 127) / 128, n_mb, heads): 4 waves x 32 register rows
__global__ __launch_bounds__(256, 2) void cl_fr32_k(ClArgs a0) {
  constexpr int NW = 4, XR = 32 * NW;
  __shared__ __attribute__((aligned(16))) ClTile32<NW> sh;
  __shared__ float rs_sc[NW][32], rs_w[NW][32];  // per register row: w / Z and w
  int z = blockIdx.z, mb = blockIdx.y, xb = blockIdx.x;
  if (a0.xcd_order) {
    const int per = gridDim.x * gridDim.y;
    const int lin = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), per * gridDim.z);
    z = lin / per;
    const int bid = lin - z * per;
    mb = bid / gridDim.x;
    xb = bid - mb * gridDim.x;
  }
  const ClArgs a = head_args(a0, z);
  const Geo g = geo(a, mb);
  const int x0 = xb * XR;
  if (x0 >= g.n) return;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int64_t base = (int64_t)mb * a.n_max;
  int roff[8], toff[4][2];
  frag32_offsets(roff, toff, lane);
  f32x16 dacc[4];
#pragma unroll
  for (int nd = 0; nd < 4; ++nd)
#pragma unroll
    for (int v = 0; v < 16; ++v) dacc[nd][v] = 0.f;
  const int x = x0 + 32 * w + r32;
  const bool live = x < g.n;
  bf16x8v qf[8];
  {
    const bf16_t* rp = live ? out_row(a, g, x) : nullptr;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (live) v = *reinterpret_cast<const u32x4*>(rp + 16 * s + 8 * hh);
      qf[s] = __builtin_bit_cast(bf16x8v, v);
    }
  }
  const float it = 1.f / a.tau;
  const float dg = live ? a.diag[base + x] : 0.f;
  const float thr = rank_threshold(dg, it, a.tau);
  const int xsq = live ? seq_of(g, x) : -2;
  float Z = 0.f, pv = -INFINITY;
  int cn = 0, rk = 0;
  const int spec_lo = (x0 / g.L) * g.L, spec_hi = ((min(x0 + XR, g.n) - 1) / g.L + 1) * g.L;
  RowCursor<true, 4> cur;
  cur.init(a.in_n + ((g.b0 * a.T) + g.off) * DE, a.T * DE, DE, g.L, w, lane);
  cl_fr32_head(sh, dacc, qf, roff, toff, a, g, base, x, xsq, thr, Z, cn, rk, pv, spec_lo, spec_hi, cur, w, lane);
  // the two lane halves hold the row's alternate column groups
  Z += __shfl_xor(Z, 32, 64);
  cn += __shfl_xor(cn, 32, 64);
  rk += __shfl_xor(rk, 32, 64);
  pv = fmaxf(pv, __shfl_xor(pv, 32, 64));
  const float wx = live ? a.w[base + x] : 0.f;
  if (hh == 0) {
    if (live) {
      a.lse[base + x] = cn > 0 ? it + __logf(Z) : -INFINITY;
      a.pos[base + x] = pv;
      a.cnt[base + x] = cn;
      a.rank[base + x] = rk;
    }
    rs_sc[w][r32] = (wx != 0.f && Z > 0.f) ? wx / Z : 0.f;
    rs_w[w][r32] = wx;
  }
  // epilogue (as the ROWS kernel): restage, then 16 lanes per row through F.normalize into dy
  __syncthreads();
#pragma unroll
  for (int nd = 0; nd < 4; ++nd)
#pragma unroll
    for (int v = 0; v < 16; ++v) sh.ep[w][8 * (v >> 2) + 4 * hh + (v & 3)][32 * nd + r32] = dacc[nd][v];
  __syncthreads();
  const float gs = 1.f / a.tau;  // unit upstream gradient
  const int sub = lane & 15;
#pragma unroll 1
  for (int ps = 0; ps < 8; ++ps) {
    const int rl = 4 * ps + (lane >> 4), xr = x0 + 32 * w + rl;
    const int xc = min(xr, g.n - 1);  // every lane takes part in the row reduction
    const int b = xc / g.L, t = xc - b * g.L;
    const int64_t ro = ((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head;
    const float sc = rs_sc[w][rl], wr = rs_w[w][rl];
    float inv[8];
    load_vec<bf16_t, 16>(in_row(a, g, xc) + 8 * sub, inv);
    const float4 u0 = *reinterpret_cast<const float4*>(&sh.ep[w][rl][8 * sub]);
    const float4 u1 = *reinterpret_cast<const float4*>(&sh.ep[w][rl][8 * sub + 4]);
    const float uu[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
    float gv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) gv[i] = gs * (uu[i] * sc - wr * inv[i]);
    normalize_bwd_store(gv, a.y_raw, a.y_dtype, a.y_norm[ro], a.dy, ro * DE + 8 * sub, xr < g.n);
  }
}


// ---------------------------------------------------------------- valid-row compaction (VC)
// Every logit of a pad row or a pad column is excluded (wrapper.py:175-190): a pad row has no
// loss term and no gradient, a pad column enters no row's softmax.  Training at the fixed
// shift therefore runs the S passes over the valid indices of each (mini-batch, head) only:
// m x m instead of n x n (C2 with history lengths ~ U[1, T]: m / n ~ 0.56, a third of the
// tiles).  cl_vpack_k lists the valid indices r in order (rows and columns share the index
// space: the pad flag of r is the mask of `in` token (b, t + off)), cl_vgather_k copies their
// normalised `out` / `in` rows into contiguous compact images, and the fused pass streams the
// compact `in` rows as its column tiles.  Sequences stay contiguous in compact order, so the
// same-sequence exclusion is a compact range [vcs[b], vcs[b + 1]); no column is a pad, so a
// clean tile needs no per-column bias at all.
struct VcLayout {
  int64_t m, np, cs, ridx, sh, w, cmap, pidx, R, C, total;
};
static inline VcLayout vc_layout(int64_t NH, int64_t n_mb, int64_t mbs, int64_t T, int64_t n_max) {
  auto al = [](int64_t x) { return (x + 255) / 256 * 256; };
  VcLayout L;
  int64_t o = 0;
  L.m = o; o += al(NH * n_mb * 4);
  L.np = o; o += al(n_mb * 4);
  L.cs = o; o += al(NH * n_mb * (mbs + 1) * 4);
  L.ridx = o; o += al(NH * n_mb * n_max * 4);
  L.sh = o; o += al(NH * n_mb * n_max * 4);
  L.w = o; o += al(NH * n_mb * n_max * 4);
  L.cmap = o; o += al(NH * n_mb * mbs * T * 4);
  L.pidx = o; o += al(n_mb * mbs * T * 4);
  L.R = o; o += al(NH * n_mb * n_max * DE * 2);
  L.C = o; o += al(NH * n_mb * n_max * DE * 2);
  L.total = o;
  return L;
}

// wave-level stream compaction of one sequence's positions tp in [0, T): valid(tp) in order
// -> out[k0 + rank]; returns the count.  f(tp) -> bool, emit(k, tp), miss(tp) for the rest.
template <typename F, typename E, typename M>
__device__ __forceinline__ int wave_compact(int T, int k0, int lane, F valid, E emit, M miss) {
  int k = k0;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int c = 0; c < T; c += 64) {
    const int tp = c + lane;
    const bool v = tp < T && valid(tp);
    const uint64_t bal = __ballot(v);
    if (v) emit(k + __popcll(bal & lt), tp);
    else if (tp < T) miss(tp);
    k += __popcll(bal);
  }
  return k - k0;
}

// One block per (mini-batch, head): the compact index lists, the row weights (as cl_used_k)
// and the zero dy rows the fused pass never writes (t >= L and pad rows).  The head-0 block
// also lists the mini-batch's valid physical `in` rows (the columns pass's register rows).
__global__ __launch_bounds__(256) void cl_vpack_k(ClArgs a0, float* __restrict__ w0, float loss_scale) {
  const ClArgs a = head_args(a0, blockIdx.y);
  float* wout = w0 + (int64_t)blockIdx.y * a0.head_stride;
  const int mb = blockIdx.x;
  const Geo g = geo(a, mb);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t base = (int64_t)mb * a.n_max;
  const int T = a.T, off = g.off, Bm = g.Bm;
  __shared__ int V[CL_UMAXB + 1];   // valid rows per sequence, then compact starts
  __shared__ int V2[CL_UMAXB + 1];  // head 0: valid physical `in` rows per sequence, then starts
  __shared__ int scan[256];
  __shared__ double red[256];
  const bool phys = blockIdx.y == 0;
  auto mrow = [&](int b) { return a.mask + (g.b0 + b) * a.mask_stride; };
  // pass 1: counts (one wave per sequence)
  for (int b = wv; b < Bm; b += 4) {
    const uint8_t* mr = mrow(b);
    int v = 0, v2 = 0;
    for (int c = 0; c < T; c += 64) {
      const int tp = c + lane;
      const bool ok = tp < T && mr[tp] == 0;
      v += __popcll(__ballot(ok && tp >= off));
      v2 += __popcll(__ballot(ok));
    }
    if (lane == 0) { V[b] = v; V2[b] = v2; }
  }
  __syncthreads();
  // exclusive scans over the sequences: each thread a contiguous run
  const int per = (Bm + 255) / 256;
  const int r0 = min(tid * per, Bm), r1 = min(r0 + per, Bm);
  for (int pass = 0; pass < (phys ? 2 : 1); ++pass) {
    int* A = pass ? V2 : V;
    int run = 0;
    for (int b = r0; b < r1; ++b) run += A[b];
    scan[tid] = run;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const int t = tid >= o ? scan[tid - o] : 0;
      __syncthreads();
      scan[tid] += t;
      __syncthreads();
    }
    const int total = scan[255];
    int k = scan[tid] - run;
    __syncthreads();
    for (int b = r0; b < r1; ++b) {
      const int c = A[b];
      A[b] = k;
      k += c;
    }
    if (tid == 0) A[Bm] = total;
    __syncthreads();
  }
  const int N = V[Bm];
  int* cs = a.vcs + (int64_t)mb * (a.mbs + 1);
  for (int b = tid; b <= Bm; b += 256) cs[b] = V[b];
  if (tid == 0) {
    a.vm[mb] = N;
    if (phys) a.vnp[mb] = V2[Bm];
  }
  // pass 2: the lists (one wave per sequence)
  int* cmap = a.vcmap + (int64_t)mb * a.mbs * T;
  int* pidx = a.vpidx + (int64_t)mb * a.mbs * T;
  const int L = g.L;
  for (int b = wv; b < Bm; b += 4) {
    const uint8_t* mr = mrow(b);
    int* cm = cmap + (int64_t)b * T;
    wave_compact(T, V[b], lane, [&](int tp) { return tp >= off && mr[tp] == 0; },
                 [&](int k, int tp) { a.vridx[base + k] = b * L + tp - off; cm[tp] = k; },
                 [&](int tp) { cm[tp] = -1; });
    if (phys)
      wave_compact(T, V2[b], lane, [&](int tp) { return mr[tp] == 0; },
                   [&](int k, int tp) { pidx[k] = b * T + tp; }, [&](int) {});
  }
  // row weights (cl_used_k): used = valid with a valid column outside its own sequence
  int u = 0;
  for (int b = tid; b < Bm; b += 256) {
    const int vb = V[b + 1] - V[b];
    u += (N - vb > 0) ? vb : 0;
  }
  const int U = (int)block_dsum((double)u, red);
  const float wr = U > 0 ? loss_scale / (float)U : 0.f;
  for (int r = tid; r < a.n_max; r += 256) {
    float wvv = 0.f;
    if (r < g.n) {
      const int b = seq_of(g, r);
      wvv = (!pad_of(a, g, r) && N - (V[b + 1] - V[b]) > 0) ? wr : 0.f;
    }
    wout[base + r] = wvv;
  }
  // zero dy rows (b, t, head) with t >= L or a pad index (the fused pass writes the valid ones)
  const int per_row = DE / 4;
  const int64_t cnt = (int64_t)Bm * (T + 1) * per_row;
  for (int64_t i = tid; i < cnt; i += 256) {
    const int row = (int)(i / per_row), c4 = (int)(i - (int64_t)row * per_row);
    const int b = row / (T + 1), t = row - b * (T + 1);
    if (t < L && mrow(b)[t + off] == 0) continue;
    const int64_t o = (((g.b0 + b) * (T + 1) + t) * a.NH + a.head) * DE + c4 * 4;
    if (a.y_dtype == LTHM_BF16) *reinterpret_cast<uint2*>(a.dy + o) = uint2{0u, 0u};
    else *reinterpret_cast<float4*>((float*)a.dy + o) = float4{0.f, 0.f, 0.f, 0.f};
  }
}

// compact images: vR[i] = normalised `out` row of r_i, vC[i] = normalised `in` row of r_i, and
// the positive logit diag[r_i] = out . in / tau with cl_diag_k's arithmetic (the compact forward
// reads no other diag entry).  16 lanes per row, two rows per lane group in flight.  With
// a.vnorm_out set, the `out` rows are normalised here from the raw next_token_emb (rownorm_v8_k's
// arithmetic; their norms into y_norm): the compact path never reads the other rows.
template <typename TY>
__global__ __launch_bounds__(256) void cl_vgather_k(ClArgs a0) {
  const ClArgs a = head_args(a0, blockIdx.z);
  const int mb = blockIdx.y;
  const Geo g = geo(a, mb);
  const int m = a.vm[mb];
  const int64_t base = (int64_t)mb * a.n_max;
  const int sub = threadIdx.x & 15;
  const int step = gridDim.x * 32;
  for (int i0 = blockIdx.x * 32 + (threadIdx.x >> 4); i0 < m; i0 += step) {
    int rr[2];
    u32x4 ov[2], iv[2];
    float yv[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) rr[u] = a.vridx[base + min(i0 + 16 * u, m - 1)];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (a.vnorm_out) {
        const int b = rr[u] / g.L, t = rr[u] - b * g.L;
        const int64_t ro = ((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head;
        ld8(reinterpret_cast<const TY*>(a.y_raw) + ro * DE + sub * 8, yv[u]);
      } else {
        ov[u] = *reinterpret_cast<const u32x4*>(out_row(a, g, rr[u]) + sub * 8);
      }
      iv[u] = *reinterpret_cast<const u32x4*>(in_row(a, g, rr[u]) + sub * 8);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i0 + 16 * u;
      if (a.vnorm_out) {  // rownorm_v8_k<TY, 1>
        float ss = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) ss += yv[u][k] * yv[u][k];
        const float nrm = sqrtf(group16_sum(ss));
        const float den = fmaxf(nrm, 1e-12f);
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = yv[u][k] / den;
        ov[u] = u32x4{pk_bf16(o[0], o[1]), pk_bf16(o[2], o[3]), pk_bf16(o[4], o[5]), pk_bf16(o[6], o[7])};
        if (i < m && sub == 0) {
          const int b = rr[u] / g.L, t = rr[u] - b * g.L;
          a.vnorm_out[((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head] = nrm;
        }
      }
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc = fmaf(__uint_as_float(ov[u][k] << 16), __uint_as_float(iv[u][k] << 16), acc);
        acc = fmaf(__uint_as_float(ov[u][k] & 0xffff0000u), __uint_as_float(iv[u][k] & 0xffff0000u), acc);
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) acc += __shfl_xor(acc, o, 64);
      if (i < m) {
        *reinterpret_cast<u32x4*>(a.vR + (base + i) * DE + sub * 8) = ov[u];
        *reinterpret_cast<u32x4*>(a.vC + (base + i) * DE + sub * 8) = iv[u];
        if (sub == 0) a.diag[base + rr[u]] = acc / a.tau;
      }
    }
  }
}

// backward prologue of the compact columns pass: the exp2 shift and weight of every compact
// row (cl_shift_k's values, in compact order) and, on the head-0 blocks, zero dt rows of the
// pad physical `in` rows (the columns pass writes the valid ones)
__global__ __launch_bounds__(256) void cl_vshift_k(ClArgs a0) {
  const ClArgs a = head_args(a0, blockIdx.z);
  const int mb = blockIdx.y;
  const int m = a.vm[mb];
  const int64_t base = (int64_t)mb * a.n_max;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < m; i += gridDim.x * 256) {
    const int r = a.vridx[base + i];
    const float wv = a.w[base + r];
    a.vsh[base + i] = wv != 0.f ? __log2f(wv) - a.lse[base + r] * LOG2E : -INFINITY;
    a.vw[base + i] = wv;
  }
  if (blockIdx.z != 0) return;
  const Geo g = geo(a, mb);
  const int T = a.T;
  const int per_row = DE / 4;
  const int64_t cnt = (int64_t)g.Bm * T * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * 256) {
    const int row = (int)(i / per_row), c4 = (int)(i - (int64_t)row * per_row);
    const int b = row / T, t = row - b * T;
    if (a.mask[(g.b0 + b) * a.mask_stride + t] == 0) continue;
    const int64_t o = ((g.b0 + b) * T + t) * DE + c4 * 4;
    if (a.t_dtype == LTHM_BF16) *reinterpret_cast<uint2*>((bf16_t*)a.dt + o) = uint2{0u, 0u};
    else *reinterpret_cast<float4*>((float*)a.dt + o) = float4{0.f, 0.f, 0.f, 0.f};
  }
}

// LDS of the compact fused pass: the 4-deep image ring (no per-column vector: no column is a
// pad) in a union with the epilogue restage
struct VTile {
  union {
    unsigned char img[CL_NB32][64 * 256];
    float ep[4][32][CL_EPS];
  };
};

// contiguous-row image cursor: wave w stages rows 16 w .. 16 w + 15 of tile t with four DMAs
// of 4 rows x 256 B (lane l: row 64 t + 16 w + 4 k + l / 16, slot l % 16, source chunk
// slot ^ swz32(row)); rows at or past `lim` come from the zero row.  Tiles are staged in any
// order (the compact passes visit the clean tiles first).
struct VCursor {
  const unsigned char* base;
  int row0, lim, ch0;
  __device__ __forceinline__ void init(const bf16_t* base_, int lim_, int w, int lane) {
    base = reinterpret_cast<const unsigned char*>(base_);
    row0 = 16 * w + (lane >> 4);
    lim = lim_;
    ch0 = (lane & 15) ^ (((lane >> 4) & 3) << 2);  // swz32(row) = ((row & 3) << 2) | ((row >> 2) & 3)
  }
  __device__ __forceinline__ void stage(unsigned char* img, int t, int w, int lane) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = 64 * t + row0 + 4 * k;
      const void* src = row < lim ? (const void*)(base + (int64_t)row * 256 + ((ch0 ^ k) << 4))
                                  : (const void*)(cl_zero_row + 16 * (lane & 15));
      glds16(src, img + (16 * w + 4 * k) * 256);
    }
  }
};

// the compact passes' tile order: the clean tiles first, then the special ones (the tiles of
// the register rows' own sequences [ts_lo, ts_hi], then the partial last tile tl if it lies
// past them), so that each loop runs one branch-free body
struct TileOrder {
  int ts_lo, nspan, nclean, tl, rot;
  __device__ __forceinline__ void init(int spec_lo, int spec_hi, int m, int ntile, bool last_special) {
    ts_lo = spec_lo / 64;
    const int ts_hi = (spec_hi - 1) / 64;
    nspan = ts_hi - ts_lo + 1;
    tl = (last_special && (m & 63) && ntile - 1 > ts_hi) ? ntile - 1 : -1;
    nclean = ntile - nspan - (tl >= 0 ? 1 : 0);
    rot = 0;
  }
  // step i -> tile; the clean steps optionally rotated by `rot` (spreads the blocks that share an
  // image over its tiles)
  __device__ __forceinline__ int at(int i) const {
    if (i < nclean && rot) {
      i += rot % nclean;
      if (i >= nclean) i -= nclean;
    }
    if (i < ts_lo) return i;
    if (i < nclean) return i + nspan;
    const int j = i - nclean;
    return j < nspan ? ts_lo + j : tl;
  }
};

// S^T tile of the 32x32x16 engine: acc[ib] = img rows 32 ib .. 32 ib + 31 against the register
// rows (the two chains interleaved, each k-step's A fragments read one step ahead)
__device__ __forceinline__ void s_tile32(f32x16 (&acc)[2], const unsigned char* img, const int (&roff)[8],
                                         const bf16x8v (&qf)[8]) {
  acc[0] = f32x16{};
  acc[1] = f32x16{};
  auto rd = [&](int ib, int s) {
    return __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(img + ib * 8192 + roff[s]));
  };
  bf16x8v f0 = rd(0, 0), f1 = rd(1, 0);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int sn = s + 1 < 8 ? s + 1 : s;
    const bf16x8v n0 = rd(0, sn), n1 = rd(1, sn);
    acc[0] = mfma32(f0, qf[s], acc[0]);
    acc[1] = mfma32(f1, qf[s], acc[1]);
    f0 = n0;
    f1 = n1;
  }
}

// dacc[32 x 128] += P[32 x 32] . img[32 x 128] for image block ib (k-steps 2 ib, 2 ib + 1)
__device__ __forceinline__ void pv_tile32(f32x16 (&dacc)[4], const f32x16& p, int ib, const unsigned char* img,
                                          const int (&toff)[4][2]) {
  const bf16x8v af0 = __builtin_bit_cast(bf16x8v, u32x4{pk_bf16(p[0], p[1]), pk_bf16(p[2], p[3]),
                                                        pk_bf16(p[4], p[5]), pk_bf16(p[6], p[7])});
  const bf16x8v af1 = __builtin_bit_cast(bf16x8v, u32x4{pk_bf16(p[8], p[9]), pk_bf16(p[10], p[11]),
                                                        pk_bf16(p[12], p[13]), pk_bf16(p[14], p[15])});
  const int k0 = 2 * ib * 4096, k1 = (2 * ib + 1) * 4096;
#pragma unroll
  for (int nd = 0; nd < 4; ++nd) {
    dacc[nd] = mfma32(af0, tr_frag32(img, toff[nd][0] + k0, toff[nd][1] + k0), dacc[nd]);
    dacc[nd] = mfma32(af1, tr_frag32(img, toff[nd][0] + k1, toff[nd][1] + k1), dacc[nd]);
  }
}

// Fused forward + ROWS pass over compact rows x (register rows) and compact columns y (image
// tiles) of one (mini-batch, head): as cl_fr32_k, with the clean tiles visited first in a loop
// of their own (one branch-free body), then the special ones (TileOrder).
// grid ((n_max + 127) / 128, n_mb, heads): 4 waves x 32 register rows
__global__ __launch_bounds__(256, 2) void cl_fr32v_k(ClArgs a0) {
  constexpr int NW = 4, XR = 32 * NW;
  __shared__ __attribute__((aligned(16))) VTile sh;
  __shared__ float rs_sc[NW][32], rs_w[NW][32], rs_pd[NW][32];  // per register row: w / Z, w, p of the diagonal
  int z = blockIdx.z, mb = blockIdx.y, xb = blockIdx.x;
  if (a0.xcd_order & 1) {
    // XCD-contiguous order: the row blocks of one (mini-batch, head) share an XCD's L2
    const int per = gridDim.x * gridDim.y;
    const int lin = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), per * gridDim.z);
    z = lin / per;
    const int bid = lin - z * per;
    mb = bid / gridDim.x;
    xb = bid - mb * gridDim.x;
  }
  const ClArgs a = head_args(a0, z);
  const int m = a.vm[mb];
  const int x0 = xb * XR;
  if (x0 >= m) return;
  const Geo g = geo(a, mb);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int64_t base = (int64_t)mb * a.n_max;
  const int* cs = a.vcs + (int64_t)mb * (a.mbs + 1);
  const int* ridx = a.vridx + base;
  int roff[8], toff[4][2];
  frag32_offsets(roff, toff, lane);
  f32x16 dacc[4];
#pragma unroll
  for (int nd = 0; nd < 4; ++nd) dacc[nd] = f32x16{};
  const int x = x0 + 32 * w + r32;
  const bool live = x < m;
  const int r = live ? ridx[x] : 0;
  bf16x8v qf[8];
  {
    const bf16_t* rp = a.vR + (base + (live ? x : 0)) * DE;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (live) v = *reinterpret_cast<const u32x4*>(rp + 16 * s + 8 * hh);
      qf[s] = __builtin_bit_cast(bf16x8v, v);
    }
  }
  const float it = 1.f / a.tau, c1 = it * LOG2E, csh = -c1;  // p = e^(S / tau - 1 / tau)
  const float dg = live ? a.diag[base + r] : 0.f;
  const float thr = rank_threshold(dg, it, a.tau);
  const int xsq = live ? seq_of(g, r) : 0;
  const int xlo = live ? cs[xsq] : -(1 << 30);
  const unsigned xlen = live ? (unsigned)(cs[xsq + 1] - cs[xsq]) : 0u;
  // the block's own sequences (compact ranges), where the same-sequence exclusion applies
  const int rlo = ridx[x0], rhi = ridx[min(x0 + XR, m) - 1];
  const int spec_lo = cs[seq_of(g, rlo)], spec_hi = cs[seq_of(g, rhi) + 1];
  float Z = 0.f;
  int cn = 0, rk = 0;
  const int ntile = (m + 63) / 64;
  TileOrder ord;
  ord.init(spec_lo, spec_hi, m, ntile, true);
  if (a0.xcd_order & 2) ord.rot = xb;  // the row blocks start their clean tiles at different columns
  VCursor cur;
  cur.init(a.vC + base * DE, m, w, lane);
  retire_loads();
  cur.stage(sh.img[0], ord.at(0), w, lane);
  if (ntile > 1) cur.stage(sh.img[1], ord.at(1), w, lane);
  if (ntile > 2) cur.stage(sh.img[2], ord.at(2), w, lane);
  if (ntile > 2) wait_vm<8>();
  else if (ntile > 1) wait_vm<4>();
  else wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  // software pipeline: step i's exp / sums / P . img run in the same basic block as step i + 1's
  // S MFMAs (past the last step they read a stale slot and are discarded).  At the top of step
  // i: step i + 1 landed (i + 2 may still be in flight), every wave is done with step i - 1, whose
  // ring slot takes step i + 3.
  f32x16 sacc[2];
  s_tile32(sacc, sh.img[0], roff, qf);
  auto open_step = [&](int i) {
    if (i + 2 < ntile) wait_vm<4>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (i + 3 < ntile) cur.stage(sh.img[(i + 3) % CL_NB32], ord.at(i + 3), w, lane);
  };
#if defined(CL_VX) && (CL_VX & 1)
  wait_vm<0>();  // experiment: the clean loop re-reads the staged slots (no staging / waits / barriers)
  __builtin_amdgcn_s_barrier();
#endif
  // clean tiles: no exclusion, no pad, every element kept
  for (int i = 0; i < ord.nclean; ++i) {
#if !defined(CL_VX) || !(CL_VX & 1)
    open_step(i);
#endif
    const unsigned char* img = sh.img[i % CL_NB32];
    const unsigned char* imgn = sh.img[(i + 1) % CL_NB32];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
#if defined(CL_VX) && (CL_VX & 2)
        (void)thr;  // experiment: no element work (P = S)
#else
        const float sv = sacc[ib][v];
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c1, csh));
        Z += p;
        rk += sv > thr ? 1 : 0;
        sacc[ib][v] = p;
#endif
      }
    }
    cn += 32;
    f32x16 snext[2];
    s_tile32(snext, imgn, roff, qf);
    pv_tile32(dacc, sacc[0], 0, img, toff);
    pv_tile32(dacc, sacc[1], 1, img, toff);
    sacc[0] = snext[0];
    sacc[1] = snext[1];
  }
  // special tiles: the register rows' own sequences and the partial tile.  Per lane, the kept
  // columns of row x form a 64-bit mask over the tile (x's own sequence, diagonal included, and
  // the columns >= m excluded); an excluded S becomes -inf (v_bfe_i32 + v_bfi_b32), after which
  // the clean body's operations give p = 0 and no rank.  The diagonal (always kept) enters in
  // the epilogue, from the positive logit dg.
  auto below = [](int k) { return k >= 64 ? ~0ull : (1ull << k) - 1ull; };
#if defined(CL_VX) && (CL_VX & 1)
  for (int i = ntile; i < ntile; ++i) {  // experiment: special tiles skipped
#else
  for (int i = ord.nclean; i < ntile; ++i) {
#endif
    open_step(i);
    const unsigned char* img = sh.img[i % CL_NB32];
    const unsigned char* imgn = sh.img[(i + 1) % CL_NB32];
    const int y0 = 64 * ord.at(i);
    const int lo = min(max(xlo - y0, 0), 64), hi = min(max(xlo + (int)xlen - y0, 0), 64);
    const int me = min(max(m - y0, 0), 64);
    uint64_t keep = live ? (below(lo) | (below(me) & ~below(hi))) : 0ull;
    keep >>= 4 * hh;  // bit cv of this lane's element v of block ib: cv = 32 ib + 8 (v >> 2) + (v & 3)
    const uint32_t kw[2] = {(uint32_t)keep, (uint32_t)(keep >> 32)};
    cn += __popc(kw[0] & 0x0F0F0F0Fu) + __popc(kw[1] & 0x0F0F0F0Fu);
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int msk = __builtin_amdgcn_sbfe((int)kw[ib], 8 * (v >> 2) + (v & 3), 1);
        const float sv = __uint_as_float((__float_as_uint(sacc[ib][v]) & msk) | (0xff800000u & ~msk));
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c1, csh));
        Z += p;
        rk += sv > thr ? 1 : 0;
        sacc[ib][v] = p;
      }
    }
    f32x16 snext[2];
    s_tile32(snext, imgn, roff, qf);
    pv_tile32(dacc, sacc[0], 0, img, toff);
    pv_tile32(dacc, sacc[1], 1, img, toff);
    sacc[0] = snext[0];
    sacc[1] = snext[1];
  }
  // the two lane halves hold the row's alternate column groups
  Z += __shfl_xor(Z, 32, 64);
  cn += __shfl_xor(cn, 32, 64);
  rk += __shfl_xor(rk, 32, 64);
  // the diagonal: p = e^(S_xx / tau - 1 / tau) with S_xx / tau = dg, the positive logit
  const float pd = live ? __builtin_amdgcn_exp2f((dg - it) * LOG2E) : 0.f;
  Z += pd;
  cn += live ? 1 : 0;
  const float wx = live ? a.w[base + r] : 0.f;
  if (hh == 0) {
    if (live) {
      a.lse[base + r] = it + __logf(Z);
      a.pos[base + r] = dg;
      a.cnt[base + r] = cn;
      a.rank[base + r] = rk;
    }
    rs_sc[w][r32] = (wx != 0.f && Z > 0.f) ? wx / Z : 0.f;
    rs_w[w][r32] = wx;
    rs_pd[w][r32] = pd;
  }
  // epilogue: restage, then 16 lanes per row through F.normalize into dy
  __syncthreads();
#pragma unroll
  for (int nd = 0; nd < 4; ++nd)
#pragma unroll
    for (int v = 0; v < 16; ++v) sh.ep[w][8 * (v >> 2) + 4 * hh + (v & 3)][32 * nd + r32] = dacc[nd][v];
  __syncthreads();
  const float gs = 1.f / a.tau;  // unit upstream gradient
  const int sub = lane & 15;
#pragma unroll 1
  for (int ps = 0; ps < 8; ++ps) {
    const int rl = 4 * ps + (lane >> 4), xr = x0 + 32 * w + rl;
    const int xc = min(xr, m - 1);  // every lane takes part in the row reduction
    const int rr = ridx[xc];
    const int b = rr / g.L, t = rr - b * g.L;
    const int64_t ro = ((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head;
    const float sc = rs_sc[w][rl], wr = rs_w[w][rl], pdr = rs_pd[w][rl];
    float inv[8];
    load_vec<bf16_t, 16>(a.vC + (base + xc) * DE + 8 * sub, inv);
    const float4 u0 = *reinterpret_cast<const float4*>(&sh.ep[w][rl][8 * sub]);
    const float4 u1 = *reinterpret_cast<const float4*>(&sh.ep[w][rl][8 * sub + 4]);
    const float uu[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
    float gv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) gv[i] = gs * (__builtin_fmaf(pdr, inv[i], uu[i]) * sc - wr * inv[i]);
    normalize_bwd_store(gv, a.y_raw, a.y_dtype, a.y_norm[ro], a.dy, ro * DE + 8 * sub, xr < m);
  }
}

// Columns pass over compact images: register rows = the mini-batch's valid physical `in` rows
// (the same operand for every head), image = the compact `out` rows of each head in turn, so
// dIn is summed over the heads in registers and dt is written once (as cl_bwd32_k COLS).
// grid ((mbs T + 127) / 128, n_mb)
__global__ __launch_bounds__(256, 2) void cl_bwd32v_k(ClArgs a0) {
  constexpr int NW = 4, XR = 32 * NW;
  __shared__ __attribute__((aligned(16))) ClTile32<NW> sh;
  const int per = gridDim.x * gridDim.y;
  const int lin = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, per);
  const int mb = lin / gridDim.x, xb = lin - mb * gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int T = a0.T;
  const int64_t b0 = (int64_t)mb * a0.mbs;
  const int np = a0.vnp[mb];
  const int j0 = xb * XR;
  if (j0 >= np) return;
  const int* pidx = a0.vpidx + (int64_t)mb * a0.mbs * T;
  const int j = j0 + 32 * w + r32;
  const bool pin = j < np;
  const int p = pidx[pin ? j : np - 1];
  const int pb = p / T, pt = p - pb * T;
  int roff[8], toff[4][2];
  frag32_offsets(roff, toff, lane);
  f32x16 dacc[4];
#pragma unroll
  for (int nd = 0; nd < 4; ++nd) dacc[nd] = f32x16{};
  bf16x8v qf[8];
  {
    const bf16_t* rp = a0.in_n + ((b0 + pb) * T + pt) * DE;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (pin) v = *reinterpret_cast<const u32x4*>(rp + 16 * s + 8 * hh);
      qf[s] = __builtin_bit_cast(bf16x8v, v);
    }
  }
  const int b_lo = pidx[j0] / T, b_hi = pidx[min(j0 + XR, np) - 1] / T;
  const float c1 = LOG2E / a0.tau;
  const int nrun = a0.heads_run;
#pragma unroll 1
  for (int hz = 0; hz < nrun; ++hz) {
    const ClArgs a = head_args(a0, hz);
    const int m = a.vm[mb];
    if (m == 0) continue;
    const int64_t base = (int64_t)mb * a.n_max;
    const int* cs = a.vcs + (int64_t)mb * (a.mbs + 1);
    const int xc = pin ? a.vcmap[(int64_t)mb * a.mbs * T + p] : -1;
    const bool live = xc >= 0;
    const int xlo = cs[pb];
    const unsigned xlen = (unsigned)(cs[pb + 1] - xlo);
    const int spec_lo = cs[b_lo], spec_hi = cs[b_hi + 1];
    const bool wmask = __ballot(!live) != 0ull;
    const float* shv = a.vsh + base;
    const float* wvv = a.vw + base;
    VCursor cur;
    cur.init(a.vR + base * DE, m, w, lane);
    const int ntile = (m + 63) / 64;
    TileOrder ord;
    ord.init(spec_lo, spec_hi, m, ntile, false);  // past m: shift -inf, so the partial tile is clean
    auto stage = [&](int i) {
      const int buf = i % CL_NB32, y0 = ord.at(i) * 64;
      cur.stage(sh.r.img[buf], ord.at(i), w, lane);
      const bool inr = y0 + lane < m;
      glds4(inr ? shv + y0 + lane : &cl_ninf, sh.r.m0[buf][w]);
      glds4(inr ? wvv + y0 + lane : &cl_zero_f, sh.r.m1[buf][w]);
    };
    constexpr int PT = 6;  // DMAs per wave and tile
    __syncthreads();  // the previous head's last tiles are read before this head's prologue restages the ring
    retire_loads();
    stage(0);
    if (ntile > 1) stage(1);
    if (ntile > 2) stage(2);
    auto open_step = [&](int i) {
      if (i + 2 < ntile) wait_vm<2 * PT>();
      else if (i + 1 < ntile) wait_vm<PT>();
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      if (i + 3 < ntile) stage(i + 3);
    };
    for (int i = 0; i < ord.nclean; ++i) {
      open_step(i);
      const int cb = i % CL_NB32;
      const unsigned char* img = sh.r.img[cb];
      f32x16 acc[2];
      s_tile32(acc, img, roff, qf);
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          const float4 ys = *reinterpret_cast<const float4*>(&sh.r.m0[cb][w][32 * ib + 8 * qd + 4 * hh]);
          const float yv[4] = {ys.x, ys.y, ys.z, ys.w};
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            acc[ib][4 * qd + jj] = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[ib][4 * qd + jj], c1, yv[jj]));
        }
      if (wmask && !live) {
        acc[0] = f32x16{};
        acc[1] = f32x16{};
      }
      pv_tile32(dacc, acc[0], 0, img, toff);
      pv_tile32(dacc, acc[1], 1, img, toff);
    }
    for (int i = ord.nclean; i < ntile; ++i) {
      open_step(i);
      const int cb = i % CL_NB32;
      const unsigned char* img = sh.r.img[cb];
      f32x16 acc[2];
      s_tile32(acc, img, roff, qf);
      // kept image rows of column c as a 64-bit mask over the tile: c's own sequence is excluded
      // except the diagonal (an excluded S becomes -inf, so its dS is 0); the diagonal's dS also
      // carries the -w of w (p - [r == c])
      const int y0 = 64 * ord.at(i);
      const int lo = min(max(xlo - y0, 0), 64), hi = min(max(xlo + (int)xlen - y0, 0), 64);
      auto below = [](int k) { return k >= 64 ? ~0ull : (1ull << k) - 1ull; };
      const int dd = xc - y0;
      uint64_t keep = below(lo) | ~below(hi);
      if (live && dd >= 0 && dd < 64) keep |= 1ull << dd;
      keep >>= 4 * hh;
      const uint32_t kw[2] = {(uint32_t)keep, (uint32_t)(keep >> 32)};
      int dx = dd - 4 * hh;
      asm volatile("" : "+v"(dx));
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          const float4 ys = *reinterpret_cast<const float4*>(&sh.r.m0[cb][w][32 * ib + 8 * qd + 4 * hh]);
          const float4 ws = *reinterpret_cast<const float4*>(&sh.r.m1[cb][w][32 * ib + 8 * qd + 4 * hh]);
          const float yv[4] = {ys.x, ys.y, ys.z, ys.w}, wv4[4] = {ws.x, ws.y, ws.z, ws.w};
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int v = 4 * qd + jj, cv = 8 * qd + jj;
            const int msk = __builtin_amdgcn_sbfe((int)kw[ib], cv, 1);
            const float sv = __uint_as_float((__float_as_uint(acc[ib][v]) & msk) | (0xff800000u & ~msk));
            const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(sv, c1, yv[jj]));
            const uint32_t dm = 0u - (uint32_t)(dx == 32 * ib + cv);  // the diagonal: all ones
            acc[ib][v] = e - __uint_as_float(__float_as_uint(wv4[jj]) & dm);
          }
        }
      if (wmask && !live) {
        acc[0] = f32x16{};
        acc[1] = f32x16{};
      }
      pv_tile32(dacc, acc[0], 0, img, toff);
      pv_tile32(dacc, acc[1], 1, img, toff);
    }
  }
  __syncthreads();
#pragma unroll
  for (int nd = 0; nd < 4; ++nd)
#pragma unroll
    for (int v = 0; v < 16; ++v) sh.ep[w][8 * (v >> 2) + 4 * hh + (v & 3)][32 * nd + r32] = dacc[nd][v];
  const float gs = (a0.gscale ? *a0.gscale : 1.f) / a0.tau;
  const int sub = lane & 15;
#pragma unroll 1
  for (int ps = 0; ps < 8; ++ps) {
    const int rl = 4 * ps + (lane >> 4), q = j0 + 32 * w + rl;
    const int pq = pidx[min(q, np - 1)];
    const int64_t ro = b0 * T + pq;
    float gv[8];
    const float4 u0 = *reinterpret_cast<const float4*>(&sh.ep[w][rl][8 * sub]);
    const float4 u1 = *reinterpret_cast<const float4*>(&sh.ep[w][rl][8 * sub + 4]);
    gv[0] = gs * u0.x; gv[1] = gs * u0.y; gv[2] = gs * u0.z; gv[3] = gs * u0.w;
    gv[4] = gs * u1.x; gv[5] = gs * u1.y; gv[6] = gs * u1.z; gv[7] = gs * u1.w;
    normalize_bwd_store(gv, a0.t_raw, a0.t_dtype, a0.t_norm[ro], a0.dt, ro * DE + 8 * sub, q < np);
  }
}

}  // namespace lthm

using namespace lthm;

static ClArgs cl_args(const lthm_contrastive_desc* d) {
  ClArgs a;
  a.out_n = (const bf16_t*)d->out_n; a.in_n = (const bf16_t*)d->in_n; a.mask = d->mask; a.mask_stride = d->mask_stride;
  a.B = d->B; a.T = d->T; a.NH = d->n_heads; a.head = d->head; a.mbs = d->mb_size; a.n_mb = d->n_mb; a.n_max = d->n_max;
  a.offsets = d->offsets; a.tau = d->tau;
  a.lse = d->lse; a.pos = d->pos; a.cnt = d->cnt; a.rank = d->rank; a.diag = d->diag; a.w = d->w;
  a.gscale = d->gscale;
  a.d_out = d->d_out; a.d_in = d->d_in;
  a.colb = nullptr;
  a.lq = d->logq; a.lq_stride = d->logq_stride; a.lqcol = d->logq_col;
  a.y_raw = (const bf16_t*)d->y_raw; a.y_norm = d->y_norm; a.dy = (bf16_t*)d->dy;
  a.head_stride = d->head_stride;
  a.y_dtype = d->y_dtype;
  a.heads_run = d->heads_run > 1 ? d->heads_run : 1;
  a.t_raw = d->t_raw; a.t_dtype = d->t_dtype; a.t_norm = d->t_norm; a.dt = d->dt;
  a.xcd_order = 0;
  a.vm = nullptr; a.vcs = nullptr; a.vridx = nullptr; a.vsh = nullptr; a.vw = nullptr; a.vcmap = nullptr;
  a.vR = nullptr; a.vC = nullptr; a.vpidx = nullptr; a.vnp = nullptr; a.vnorm_out = nullptr;
  if (d->vc_ws) {
    const VcLayout L = vc_layout(d->n_heads, d->n_mb, d->mb_size, d->T, d->n_max);
    char* b = (char*)d->vc_ws;
    a.vm = (int*)(b + L.m); a.vnp = (int*)(b + L.np); a.vcs = (int*)(b + L.cs); a.vridx = (int*)(b + L.ridx);
    a.vsh = (float*)(b + L.sh); a.vw = (float*)(b + L.w); a.vcmap = (int*)(b + L.cmap); a.vpidx = (int*)(b + L.pidx);
    a.vR = (bf16_t*)(b + L.R); a.vC = (bf16_t*)(b + L.C);
  }
  return a;
}

static int cl_check(const lthm_contrastive_desc* d) {
  if (!d || d->De != DE || d->B <= 0 || d->T <= 0 || d->mb_size <= 0 || d->n_mb <= 0) return 1;
  if ((int64_t)d->mb_size * d->T > d->n_max || d->n_max % 64 != 0) return 1;
  if ((int64_t)d->n_max * d->T >= (1ll << 32)) return 1;  // seq_of: c / L by one 32 x 64 multiply
  if (d->head < 0 || d->head >= d->n_heads) return 1;
  if (d->logq && (!d->logq_col || d->logq_stride < d->T)) return 1;
  return 0;
}

static int64_t cl_stats_blocks(int32_t n_max) { return (n_max + CL_SROWS - 1) / CL_SROWS; }

extern "C" int64_t lthm_contrastive_vc_ws_bytes(int64_t B, int32_t T, int32_t n_heads, int32_t mb_size, int32_t n_mb,
                                                int32_t n_max) {
  if (B <= 0 || T <= 0 || n_heads <= 0 || mb_size <= 0 || n_mb <= 0 || n_max <= 0) return -1;
  return vc_layout(n_heads, n_mb, mb_size, T, n_max).total;
}

// the compact path's preconditions (beyond cl_check and the fused-rows ones)
static bool vc_ok(const lthm_contrastive_desc* d) {
  if (!d->vc_ws) return false;
  if (!d->out_n && !(d->y_raw && d->y_norm)) return false;
  if (d->vc_ws_bytes < vc_layout(d->n_heads, d->n_mb, d->mb_size, d->T, d->n_max).total) return false;
  return d->head == 0 && d->heads_run == d->n_heads && d->head_stride == (int64_t)d->n_mb * d->n_max &&
         d->mb_size <= CL_UMAXB && (int64_t)d->mb_size * d->T <= (1ll << 30);
}

extern "C" int64_t lthm_contrastive_ws_bytes(int32_t n_mb, int32_t n_max, int32_t heads) {
  if (n_mb <= 0 || n_max <= 0 || heads <= 0) return -1;
  const int64_t hm = (int64_t)heads * n_mb;
  return hm * n_max * 4 + ((hm * n_max * 4) % 8) + hm * cl_stats_blocks(n_max) * CL_NPART * 8;
}

template <typename TX>
static void launch_rownorm(const TX* x, int64_t rows, int D, bf16_t* out, float* norms, const uint8_t* mask,
                           int64_t mgroup, int64_t mstride, hipStream_t s) {
  if (D % 8 == 0) {
    const int grid = grid_for(rows, 16, 256 * 8);
    if (D <= 128)
      hipLaunchKernelGGL((rownorm_v8_k<TX, 1>), dim3(grid), dim3(256), 0, s, x, rows, D, out, norms, mask, mgroup, mstride);
    else
      hipLaunchKernelGGL((rownorm_v8_k<TX, 2>), dim3(grid), dim3(256), 0, s, x, rows, D, out, norms, mask, mgroup, mstride);
  } else {
    hipLaunchKernelGGL((rownorm_k<TX>), dim3(grid_for(rows, 4, 256 * 8)), dim3(256), 0, s, x, rows, D, out, norms,
                       mask, mgroup, mstride);
  }
}

template <typename TX>
static void launch_rownorm_bwd(const TX* x, const float* norms, const float* g, int64_t rows, int D, bf16_t* dx_bf,
                               float* dx_f, hipStream_t s) {
  if (D % 8 == 0) {
    const int grid = grid_for(rows, 16, 256 * 8);
    if (D <= 128)
      hipLaunchKernelGGL((rownorm_bwd_v8_k<TX, 1>), dim3(grid), dim3(256), 0, s, x, norms, g, rows, D, dx_bf, dx_f);
    else
      hipLaunchKernelGGL((rownorm_bwd_v8_k<TX, 2>), dim3(grid), dim3(256), 0, s, x, norms, g, rows, D, dx_bf, dx_f);
  } else {
    hipLaunchKernelGGL((rownorm_bwd_k<TX>), dim3(grid_for(rows, 4, 256 * 8)), dim3(256), 0, s, x, norms, g, rows, D,
                       dx_bf, dx_f);
  }
}

extern "C" int lthm_rownorm(const void* x, int32_t x_dtype, int64_t rows, int32_t D, void* out_bf16, float* norms,
                            const uint8_t* row_mask, int64_t mask_group, int64_t mask_stride, void* stream) {
  LTHM_REQUIRE(rows >= 0 && D > 0 && D <= 256);
  LTHM_REQUIRE(!row_mask || (mask_group > 0 && mask_stride >= mask_group));
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (x_dtype == LTHM_BF16)
    launch_rownorm((const bf16_t*)x, rows, D, (bf16_t*)out_bf16, norms, row_mask, mask_group, mask_stride, s);
  else
    launch_rownorm((const float*)x, rows, D, (bf16_t*)out_bf16, norms, row_mask, mask_group, mask_stride, s);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_rownorm_bwd(const void* x, int32_t x_dtype, const float* norms, const float* g, int64_t rows,
                                int32_t D, void* dx_bf16, float* dx_f32, void* stream) {
  LTHM_REQUIRE(rows >= 0 && D > 0 && D <= 256);
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (x_dtype == LTHM_BF16)
    launch_rownorm_bwd((const bf16_t*)x, norms, g, rows, D, (bf16_t*)dx_bf16, dx_f32, s);
  else
    launch_rownorm_bwd((const float*)x, norms, g, rows, D, (bf16_t*)dx_bf16, dx_f32, s);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_contrastive_fwd(const lthm_contrastive_desc* d, float* stats, int32_t nstat, const int32_t* ks,
                                    int32_t nk, float loss_scale, void* stream) {
  LTHM_REQUIRE(cl_check(d) == 0 && stats && d->lse && d->pos && d->cnt && d->rank && d->diag && d->w);
  LTHM_REQUIRE(nstat >= CL_NSTAT + nk);
  // several heads per launch: no tail round per head (C2: 4096 blocks a head at 3 per CU
  // is 5.33 rounds of the 768 slots; six heads together are 32)
  const int nrun = d->heads_run > 1 ? d->heads_run : 1;
  LTHM_REQUIRE(d->head + nrun <= d->n_heads);
  LTHM_REQUIRE(nrun == 1 || d->head_stride >= (int64_t)d->n_mb * d->n_max);
  const int64_t ws = lthm_contrastive_ws_bytes(d->n_mb, d->n_max, nrun);
  LTHM_REQUIRE(d->stats_ws && d->stats_ws_bytes >= ws);
  ClArgs a = cl_args(d);
  a.colb = d->w;  // scratch until cl_rowstats_k writes the used flags
  hipStream_t s = (hipStream_t)stream;
  const int64_t hm = (int64_t)nrun * d->n_mb;
  int* hist = (int*)d->stats_ws;
  double* part = (double*)((char*)d->stats_ws + ((hm * d->n_max * 4 + 7) / 8) * 8);
  const bool fixed = 2.f / d->tau <= 80.f && !d->logq;
  const bool rows = fixed && d->y_raw && d->y_norm && d->dy && d->head == 0 && nrun == d->n_heads &&
                    d->mb_size <= CL_UMAXB && (d->y_dtype == LTHM_BF16 || d->y_dtype == LTHM_F32);
  // out_n may be null only on the compact path (its gather normalises the `out` rows it needs)
  LTHM_REQUIRE(d->out_n || (rows && vc_ok(d)));
  if (rows) a.colb = (float*)hist;  // the per-column bias lives in the histogram until the fused pass is done
  if (hipMemsetAsync(hist, 0, hm * d->n_max * 4, s) != hipSuccess) return (int)hipGetLastError();
  if (!(rows && vc_ok(d))) {  // the compact path computes the diagonal in its gather
    hipLaunchKernelGGL(cl_diag_k, dim3(64, d->n_mb, nrun), dim3(256), 0, s, a);
    LTHM_CHECK_LAUNCH();
  }
  const dim3 grid((d->n_max + CL_ROWS - 1) / CL_ROWS, d->n_mb, nrun);
  if (rows) {
    // forward + the row side of the backward in one pass (row weights from the pad mask first)
    const bool vc = vc_ok(d);
    if (d->vc_ws && !vc) return 1;
    if (vc) {
      // valid-row compaction: index lists + weights + zero dy rows, then the compact images
      hipLaunchKernelGGL(cl_vpack_k, dim3(d->n_mb, nrun), dim3(256), 0, s, a, d->w, loss_scale);
      LTHM_CHECK_LAUNCH();
      // out_n null: the gather normalises the valid `out` rows itself and writes their norms
      ClArgs ag = a;
      if (!d->out_n) ag.vnorm_out = const_cast<float*>(d->y_norm);
      const dim3 gg(std::max(1, std::min(16, d->n_max / 256)), d->n_mb, nrun);
      if (d->y_dtype == LTHM_BF16) hipLaunchKernelGGL(cl_vgather_k<bf16_t>, gg, dim3(256), 0, s, ag);
      else hipLaunchKernelGGL(cl_vgather_k<float>, gg, dim3(256), 0, s, ag);
      LTHM_CHECK_LAUNCH();
    } else {
      hipLaunchKernelGGL(cl_used_k, dim3(d->n_mb, nrun), dim3(256), 0, s, a, d->w, loss_scale);
      LTHM_CHECK_LAUNCH();
    }
    // block order: the compact pass runs XCD-contiguous (the row blocks of one (mini-batch, head)
    // share an XCD's L2: 4.97 -> 4.32 ms on tools/loss_bench.py, profiles/r04m_*); the full pass
    // keeps the plain order (3-5 % faster there, tools/ab_fr_xcd.sh)
    static const int xcd_env = getenv("LTHM_CL_FR_XCD") ? atoi(getenv("LTHM_CL_FR_XCD")) : -1;
    a.xcd_order = xcd_env >= 0 ? xcd_env : (vc ? 1 : 0);
    if (d->main_ev0 && hipEventRecord((hipEvent_t)d->main_ev0, s) != hipSuccess) return (int)hipGetLastError();
    if (vc) hipLaunchKernelGGL(cl_fr32v_k, dim3((d->n_max + 127) / 128, d->n_mb, nrun), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(cl_fr32_k, dim3((d->n_max + 127) / 128, d->n_mb, nrun), dim3(256), 0, s, a);
    LTHM_CHECK_LAUNCH();
    if (d->main_ev1 && hipEventRecord((hipEvent_t)d->main_ev1, s) != hipSuccess) return (int)hipGetLastError();
    if (hipMemsetAsync(hist, 0, hm * d->n_max * 4, s) != hipSuccess) return (int)hipGetLastError();
    a.colb = d->w;
  } else {
    // the fixed softmax shift 1/tau bounds the plain logits only: logQ takes the online max
    // fixed shift: 3 blocks per CU (3 waves per SIMD hide more of the exp / count VALU
    // latency: 0.91 -> 0.78-0.82 ms per C2 head; a 2-deep ring at 3 blocks measured the
    // same, 4 blocks spill); running shift: 2
    if (d->main_ev0 && hipEventRecord((hipEvent_t)d->main_ev0, s) != hipSuccess) return (int)hipGetLastError();
    if (fixed) hipLaunchKernelGGL((cl_fwd_k<true, 3, 3>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((cl_fwd_k<false, 3, 2>), grid, dim3(256), 0, s, a);
    LTHM_CHECK_LAUNCH();
    if (d->main_ev1 && hipEventRecord((hipEvent_t)d->main_ev1, s) != hipSuccess) return (int)hipGetLastError();
  }
  const int nblk = (int)cl_stats_blocks(d->n_max);
  hipLaunchKernelGGL(cl_rowstats_k, dim3(nblk, d->n_mb, nrun), dim3(256), 0, s, a, hist, part);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL(cl_stats_k, dim3(d->n_mb, 1, nrun), dim3(256), 0, s, a, (const int*)hist, (const double*)part,
                     nblk, stats, nstat, (const int*)ks, nk);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL(cl_wscale_k, dim3(min((d->n_max + 255) / 256, 64), d->n_mb, nrun), dim3(256), 0, s, a,
                     (const float*)stats, nstat, loss_scale);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_contrastive_bwd(const lthm_contrastive_desc* d, void* stream) {
  LTHM_REQUIRE(cl_check(d) == 0 && d->lse && d->w && d->diag);
  const int nrun = d->heads_run > 1 ? d->heads_run : 1;
  LTHM_REQUIRE(d->head + nrun <= d->n_heads);
  LTHM_REQUIRE(nrun == 1 || d->head_stride >= (int64_t)d->n_mb * d->n_max);
  const bool fused = d->y_raw && d->y_norm && d->dy && d->t_raw && d->t_norm && d->dt;
  ClArgs a = cl_args(d);
  a.colb = d->diag;  // the shift scratch (advanced per head by head_args)
  hipStream_t s = (hipStream_t)stream;
  const bool fixed = 2.f / d->tau <= 80.f && !d->logq;
  LTHM_REQUIRE(d->out_n || (fused && d->rows_done && vc_ok(d)));  // only the compact COLS pass reads no out_n
  if (fused && d->rows_done) {
    // the forward ran the ROWS side (dy for a unit upstream gradient): COLS, then dy *= gscale
    LTHM_REQUIRE(fixed && d->head == 0 && nrun == d->n_heads);
    LTHM_REQUIRE((d->y_dtype == LTHM_BF16 || d->y_dtype == LTHM_F32) &&
                 (d->t_dtype == LTHM_BF16 || d->t_dtype == LTHM_F32));
    const bool vc = vc_ok(d);
    if (d->vc_ws && !vc) return 1;
    const dim3 gcols((int)(((int64_t)d->mb_size * d->T + 127) / 128), d->n_mb, 1);
    if (vc) {
      hipLaunchKernelGGL(cl_vshift_k, dim3(std::max(1, std::min(16, d->n_max / 256)), d->n_mb, nrun), dim3(256), 0, s,
                         a);
      LTHM_CHECK_LAUNCH();
    } else {
      ClArgs ash = a;
      ash.dy = nullptr;
      ash.d_out = nullptr;  // the dy tails were zeroed by the forward
      hipLaunchKernelGGL(cl_shift_k, dim3((d->n_max + 255) / 256, d->n_mb, nrun), dim3(256), 0, s, ash);
      LTHM_CHECK_LAUNCH();
    }
    if (d->main_ev0 && hipEventRecord((hipEvent_t)d->main_ev0, s) != hipSuccess) return (int)hipGetLastError();
    if (vc) hipLaunchKernelGGL(cl_bwd32v_k, gcols, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((cl_bwd32_k<false, true, 4>), gcols, dim3(256), 0, s, a);
    LTHM_CHECK_LAUNCH();
    if (d->main_ev1 && hipEventRecord((hipEvent_t)d->main_ev1, s) != hipSuccess) return (int)hipGetLastError();
    if (d->gscale) {
      const int64_t n = (int64_t)d->B * (d->T + 1) * d->n_heads * DE;
      const dim3 gs((unsigned)std::min<int64_t>((n / 8 + 255) / 256, 2048));
      if (d->y_dtype == LTHM_BF16) hipLaunchKernelGGL(cl_dyscale_k<bf16_t>, gs, dim3(256), 0, s, (bf16_t*)d->dy, n, d->gscale);
      else hipLaunchKernelGGL(cl_dyscale_k<float>, gs, dim3(256), 0, s, (float*)d->dy, n, d->gscale);
      LTHM_CHECK_LAUNCH();
    }
    return 0;
  }
  if (fused) {
    // every head in one call: the COLS pass sums dIn over the heads and writes dt once
    LTHM_REQUIRE(d->head == 0 && nrun == d->n_heads);
    LTHM_REQUIRE((d->y_dtype == LTHM_BF16 || d->y_dtype == LTHM_F32) &&
                 (d->t_dtype == LTHM_BF16 || d->t_dtype == LTHM_F32));
    hipLaunchKernelGGL(cl_shift_k, dim3((d->n_max + 255) / 256, d->n_mb, nrun), dim3(256), 0, s, a);
    LTHM_CHECK_LAUNCH();
    // 4 waves per workgroup, two workgroups per CU (8 waves, one workgroup per CU: the same
    // time within 1% at C2, tools/prof_loss_ab.sh)
    const dim3 grows((d->n_max + 127) / 128, d->n_mb, nrun);
    const dim3 gcols((int)(((int64_t)d->mb_size * d->T + 127) / 128), d->n_mb, 1);
    if (fixed) {
      hipLaunchKernelGGL((cl_bwd32_k<true, true, 4>), grows, dim3(256), 0, s, a);
      LTHM_CHECK_LAUNCH();
      hipLaunchKernelGGL((cl_bwd32_k<false, true, 4>), gcols, dim3(256), 0, s, a);
    } else {
      hipLaunchKernelGGL((cl_bwd32_k<true, false, 4>), grows, dim3(256), 0, s, a);
      LTHM_CHECK_LAUNCH();
      hipLaunchKernelGGL((cl_bwd32_k<false, false, 4>), gcols, dim3(256), 0, s, a);
    }
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  // one head, f32 d_in accumulated (16x16x32 kernels)
  LTHM_REQUIRE(nrun == 1 && (d->d_out || d->dy) && d->d_in);
  LTHM_REQUIRE(!d->dy || (d->y_raw && d->y_norm && d->y_dtype == LTHM_BF16));
  hipLaunchKernelGGL(cl_shift_k, dim3((d->n_max + 255) / 256, d->n_mb), dim3(256), 0, s, a);
  LTHM_CHECK_LAUNCH();
  dim3 grid((d->n_max + CL_ROWS - 1) / CL_ROWS, d->n_mb);
  if (fixed) {
    hipLaunchKernelGGL((cl_bwd_k<true, true>), grid, dim3(256), 0, s, a);
    LTHM_CHECK_LAUNCH();
    hipLaunchKernelGGL((cl_bwd_k<false, true>), grid, dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((cl_bwd_k<true, false>), grid, dim3(256), 0, s, a);
    LTHM_CHECK_LAUNCH();
    hipLaunchKernelGGL((cl_bwd_k<false, false>), grid, dim3(256), 0, s, a);
  }
  LTHM_CHECK_LAUNCH();
  return 0;
}
