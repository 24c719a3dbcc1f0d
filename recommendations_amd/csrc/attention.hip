// Causal self-attention with the learned relative-position bias, forward and
// backward (commons/transformers/layers.py:13-35 RelativePositionBias, :41-61
// ScaledDotProductAttention, :247-265 MultiHeadAttention).
//
//   S[q,k] = (Q[q] . K[k]) / sqrt(E) + table[q - k + T, h]  (+ -inf for k > q)
//   P = softmax_k(S),  O = P V;  the per-row log-sum-exp is kept for backward.
//
// The LTHM encoder runs short sequences (T' = T+1 <= 257), so one workgroup
// holds a whole (batch, head) problem: K and V (bf16, padded rows) live in LDS,
// each wave walks query rows, scores stay in registers (T/64 per lane) and the
// [T, T] score matrix never touches HBM.  The backward recomputes P from the
// saved LSE in two passes (rows: dQ and the bias gradient; columns: dK, dV), so
// no T x T buffer is needed at all.
#include "common.hpp"

#include <cstdlib>

namespace lthm {

struct AttnArgs {
  const bf16_t *q, *k, *v;
  int64_t q_ts, k_ts, v_ts;  // token strides (elements)
  int64_t q_hs, k_hs, v_hs;  // head strides
  int64_t q_bs, k_bs, v_bs;  // batch strides
  bf16_t* o;                 // [B, T, H, E]
  int64_t o_ts, o_hs, o_bs;
  const float* table;        // [R, H] or null
  float* lse;                // [B, H, T]
  int T, H, causal;
  // backward
  const bf16_t* dout;
  bf16_t *dq, *dk, *dv;      // same strides as q, k, v
  float* dtable_part;        // [B, 2T+1, H] (T' <= 256) / [parts, 2T+1, H] (windowed)
  float* delta;              // [B, H, T] workspace of the windowed backward
  int B;
  const float* mask;         // additive [., ., T, T] or null (VALU kernels only)
  int64_t m_bs, m_hs, m_rs;
  int tail;                  // attn_bwd32_k: the last query as a vector pass (bwd32_tail_mode)
  // packed rows (shared pad prefix; the long-T' 32x32x16 kernels): row t of sequence b is row
  // rmap[b T + t] of q / k / v (batch strides unused); wmap the same with -1 where the row is not
  // the sequence's own (a pad of a sequence other than the chain's owner): its dO reads as zero,
  // its O / dQ are not stored, query tiles with no own row are skipped.  dK / dV of chain rows
  // (packed row < chain) go to dk_chain / dv_chain row b chain + t (token stride chain_ts).
  const int* rmap;
  const int* wmap;
  bf16_t *dk_chain, *dv_chain;
  int64_t chain_ts;
  int chain;
};

// the packed row of (b, t) through `map` (rmap / wmap), or t + the batch offset when unmapped
__device__ __forceinline__ int64_t row_of(const int* map, int64_t b, int T, int t, int64_t bs_rows) {
  return map ? (int64_t)map[b * T + t] : b * bs_rows + t;
}

// the first query tile holding a row the sequence owns (0 unless packed): tiles before it are
// pads of a sequence other than the chain's owner, whose outputs and gradients nobody reads
__device__ __forceinline__ int first_own_tile(const AttnArgs& a, int b, int T) {
  if (!a.wmap) return 0;
  const int* w = a.wmap + (int64_t)b * T;
  const int nt = (T + 31) >> 5;
  int t = 0;
  while (t < nt && w[min(32 * t + 31, T - 1)] < 0) ++t;
  return t;
}

__device__ __forceinline__ const float* mask_head(const AttnArgs& a, int b, int h) {
  return a.mask ? a.mask + (int64_t)b * a.m_bs + (int64_t)h * a.m_hs : nullptr;
}

constexpr int ROWPAD = 2;  // bf16 elements of row padding (bank spread)

template <int E>
__device__ __forceinline__ float dot_row_reg(const bf16_t* __restrict__ row_lds, const float* reg) {
  float s = 0.f;
  const uint32_t* p = reinterpret_cast<const uint32_t*>(row_lds);
#pragma unroll
  for (int e2 = 0; e2 < E / 2; ++e2) {
    const uint32_t u = p[e2];
    s = fmaf(reg[2 * e2], __uint_as_float(u << 16), s);
    s = fmaf(reg[2 * e2 + 1], __uint_as_float(u & 0xffff0000u), s);
  }
  return s;
}

template <int E>
__device__ __forceinline__ void load_rows_lds(bf16_t* dst, const bf16_t* __restrict__ src, int64_t ts, int T, int tid) {
  // E/8 chunks of 16 B per row
  constexpr int CPR = E / 8;
  for (int idx = tid; idx < T * CPR; idx += 256) {
    const int t = idx / CPR, c = idx - t * CPR;
    const u32x4 v = *reinterpret_cast<const u32x4*>(src + (int64_t)t * ts + c * 8);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst + t * (E + ROWPAD) + c * 8);
    d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3];
  }
}

template <int E>
__device__ __forceinline__ void load_row_reg(float* reg, const bf16_t* __restrict__ src) {
#pragma unroll
  for (int c = 0; c < E / 8; ++c) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(src + c * 8);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      reg[c * 8 + 2 * i] = __uint_as_float(v[i] << 16);
      reg[c * 8 + 2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
    }
  }
}

template <int E, int NK>
__global__ __launch_bounds__(256) void attn_fwd_k(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int T = a.T;
  bf16_t* Ks = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Vs = Ks + T * (E + ROWPAD);
  float* bias = reinterpret_cast<float*>(Vs + T * (E + ROWPAD));  // [2T+1]
  float* prow = bias + 2 * T + 2;                                   // [4][T]
  const int b = blockIdx.x / a.H, h = blockIdx.x - (blockIdx.x / a.H) * a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  load_rows_lds<E>(Ks, a.k + b * a.k_bs + h * a.k_hs, a.k_ts, T, tid);
  load_rows_lds<E>(Vs, a.v + b * a.v_bs + h * a.v_hs, a.v_ts, T, tid);
  for (int i = tid; i <= 2 * T; i += 256) bias[i] = a.table ? a.table[(int64_t)i * a.H + h] : 0.f;
  __syncthreads();
  const float sq = sqrtf((float)E);
  const float* mk = mask_head(a, b, h);
  float qr[E];
  for (int qi = wave; qi < T; qi += 4) {
    load_row_reg<E>(qr, a.q + b * a.q_bs + h * a.q_hs + (int64_t)qi * a.q_ts);
    float s[NK];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int k = lane + 64 * j;
      s[j] = -INFINITY;
      if (k < T && (!a.causal || k <= qi)) {
        s[j] = dot_row_reg<E>(Ks + k * (E + ROWPAD), qr) / sq + bias[qi - k + T];
        if (mk) s[j] += mk[(int64_t)qi * a.m_rs + k];
      }
      mx = fmaxf(mx, s[j]);
    }
    mx = wave_max(mx);
    float l = 0.f;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int k = lane + 64 * j;
      const float p = (s[j] == -INFINITY) ? 0.f : __expf(s[j] - mx);
      l += p;
      if (k < T) prow[wave * T + k] = p;
    }
    __builtin_amdgcn_wave_barrier();
    l = wave_sum(l);
    const float inv = 1.f / l;
    const int kmax = a.causal ? qi + 1 : T;
    for (int e = lane; e < E; e += 64) {
      float o = 0.f;
      for (int k = 0; k < kmax; ++k) o = fmaf(prow[wave * T + k], bf2f(Vs[k * (E + ROWPAD) + e]), o);
      a.o[b * a.o_bs + h * a.o_hs + (int64_t)qi * a.o_ts + e] = f2bf(o * inv);
    }
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) a.lse[((int64_t)b * a.H + h) * T + qi] = mx + __logf(l);
  }
}

template <int E, int NK>
__global__ __launch_bounds__(256) void attn_bwd_k(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int T = a.T;
  constexpr int RS = E + ROWPAD;
  bf16_t* Qs = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Ks = Qs + T * RS;
  bf16_t* Vs = Ks + T * RS;
  bf16_t* dOs = Vs + T * RS;
  float* bias = reinterpret_cast<float*>(dOs + T * RS);  // [2T+2]
  float* dbias = bias + 2 * T + 2;                        // [2T+2]
  float* lse = dbias + 2 * T + 2;                         // [T]
  float* delta = lse + T;                                 // [T]
  float* rowbuf = delta + T;                              // [4][2][T]
  const int b = blockIdx.x / a.H, h = blockIdx.x - (blockIdx.x / a.H) * a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16_t* qg = a.q + b * a.q_bs + h * a.q_hs;
  const bf16_t* kg = a.k + b * a.k_bs + h * a.k_hs;
  const bf16_t* vg = a.v + b * a.v_bs + h * a.v_hs;
  const bf16_t* og = a.o + b * a.o_bs + h * a.o_hs;
  const bf16_t* dog = a.dout + b * a.o_bs + h * a.o_hs;
  load_rows_lds<E>(Qs, qg, a.q_ts, T, tid);
  load_rows_lds<E>(Ks, kg, a.k_ts, T, tid);
  load_rows_lds<E>(Vs, vg, a.v_ts, T, tid);
  load_rows_lds<E>(dOs, dog, a.o_ts, T, tid);
  for (int i = tid; i <= 2 * T; i += 256) {
    bias[i] = a.table ? a.table[(int64_t)i * a.H + h] : 0.f;
    dbias[i] = 0.f;
  }
  for (int i = tid; i < T; i += 256) lse[i] = a.lse[((int64_t)b * a.H + h) * T + i];
  __syncthreads();
  // delta[q] = dO[q] . O[q]
  for (int qi = wave; qi < T; qi += 4) {
    float d = 0.f;
    for (int e = lane; e < E; e += 64) d += bf2f(dOs[qi * RS + e]) * bf2f(og[(int64_t)qi * a.o_ts + e]);
    d = wave_sum(d);
    if (lane == 0) delta[qi] = d;
  }
  __syncthreads();
  const float sq = sqrtf((float)E);
  const float* mk = mask_head(a, b, h);
  float r1[E], r2[E];
  float* dsrow = rowbuf + wave * 2 * T;
  float* prow = dsrow + T;
  // pass A: rows -> dQ, dbias
  for (int qi = wave; qi < T; qi += 4) {
    load_row_reg<E>(r1, qg + (int64_t)qi * a.q_ts);  // q
    load_row_reg<E>(r2, dog + (int64_t)qi * a.o_ts); // dO
    const float lq = lse[qi], dq_ = delta[qi];
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int k = lane + 64 * j;
      if (k < T) {
        float ds = 0.f;
        if (!a.causal || k <= qi) {
          const float s = dot_row_reg<E>(Ks + k * RS, r1) / sq + bias[qi - k + T] +
                          (mk ? mk[(int64_t)qi * a.m_rs + k] : 0.f);
          const float p = (s == -INFINITY) ? 0.f : __expf(s - lq);
          const float dp = dot_row_reg<E>(Vs + k * RS, r2);
          ds = p * (dp - dq_);
          atomicAdd(&dbias[qi - k + T], ds);
        }
        dsrow[k] = ds;
      }
    }
    __builtin_amdgcn_wave_barrier();
    const int kmax = a.causal ? qi + 1 : T;
    for (int e = lane; e < E; e += 64) {
      float acc = 0.f;
      for (int k = 0; k < kmax; ++k) acc = fmaf(dsrow[k], bf2f(Ks[k * RS + e]), acc);
      a.dq[b * a.q_bs + h * a.q_hs + (int64_t)qi * a.q_ts + e] = f2bf(acc / sq);
    }
    __builtin_amdgcn_wave_barrier();
  }
  // pass B: columns -> dK, dV
  for (int ki = wave; ki < T; ki += 4) {
    load_row_reg<E>(r1, kg + (int64_t)ki * a.k_ts);  // k
    load_row_reg<E>(r2, vg + (int64_t)ki * a.v_ts);  // v
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int qi = lane + 64 * j;
      if (qi < T) {
        float ds = 0.f, p = 0.f;
        if (!a.causal || ki <= qi) {
          const float s = dot_row_reg<E>(Qs + qi * RS, r1) / sq + bias[qi - ki + T] +
                          (mk ? mk[(int64_t)qi * a.m_rs + ki] : 0.f);
          p = (s == -INFINITY) ? 0.f : __expf(s - lse[qi]);
          const float dp = dot_row_reg<E>(dOs + qi * RS, r2);
          ds = p * (dp - delta[qi]);
        }
        dsrow[qi] = ds;
        prow[qi] = p;
      }
    }
    __builtin_amdgcn_wave_barrier();
    const int qmin = a.causal ? ki : 0;
    for (int e = lane; e < E; e += 64) {
      float ak = 0.f, av = 0.f;
      for (int qi = qmin; qi < T; ++qi) {
        ak = fmaf(dsrow[qi], bf2f(Qs[qi * RS + e]), ak);
        av = fmaf(prow[qi], bf2f(dOs[qi * RS + e]), av);
      }
      a.dk[b * a.k_bs + h * a.k_hs + (int64_t)ki * a.k_ts + e] = f2bf(ak / sq);
      a.dv[b * a.v_bs + h * a.v_hs + (int64_t)ki * a.v_ts + e] = f2bf(av);
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  if (a.dtable_part) {
    for (int i = tid; i <= 2 * T; i += 256) a.dtable_part[((int64_t)b * (2 * T + 1) + i) * a.H + h] = dbias[i];
  }
}

// ===========================================================================
// MFMA path (E in {32, 64, 128}): v_mfma_f32_16x16x32_bf16 tiles.
//
// Fragment layouts (wave64, 16x16x32):  A[l&15][8(l>>4)+i],  B[8(l>>4)+i][l&15],
// C[4(l>>4)+j][l&15].  Whole-head operands live in LDS "images": row-major
// [Tk, E] bf16 with 16-byte chunks XOR-swizzled so that 16 consecutive rows
// read at one chunk hit distinct banks (row-fragment reads), while
// ds_read_tr16_b64 gives the k-strided B fragments (keys / queries as k).
// Probabilities P and dS leave the C layout through a padded per-wave f32
// scratch and enter the next MFMA as bf16 hi + lo halves, so the second
// product (P.V, dS.K, P^T.dO, dS^T.Q) carries ~16 mantissa bits of P / dS.
// ===========================================================================
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int SCR_LD = 36;  // scratch row stride (floats): conflict-free C-layout writes, 16 B aligned reads

template <int E>
__device__ __forceinline__ int img_off(int row, int ch) {
  constexpr int NC = E / 8;
  constexpr int RPL = (256 / (2 * E)) > 0 ? 256 / (2 * E) : 1;  // rows per 256-byte bank line
  return row * (2 * E) + ((ch ^ ((row / RPL) & (NC - 1))) << 4);
}

// stage rows [0, Tk) of a head (row r at src + r*ts) into an image; rows >= T are zero
template <int E>
__device__ __forceinline__ void stage_img(unsigned char* img, const bf16_t* __restrict__ src, int64_t ts, int T, int Tk,
                                          int tid) {
  constexpr int NC = E / 8;
  for (int idx = tid; idx < Tk * NC; idx += 256) {
    const int r = idx / NC, c = idx - r * NC;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r < T) v = *reinterpret_cast<const u32x4*>(src + (int64_t)r * ts + c * 8);
    *reinterpret_cast<u32x4*>(img + img_off<E>(r, c)) = v;
  }
}

// the same image by LDS-DMA (global_load_lds_dwordx4): 1-KiB pieces, wave w
// issues pieces w, w + 4, ...; the DMA's lane-linear destination slot loads the
// chunk that img_off's swizzle puts there.  Rows >= T read a zero chunk.  All
// pieces of every image are in flight together; the caller retires them with
// wait_vm<0>() + __syncthreads().
__device__ __attribute__((aligned(16))) unsigned char attn_zero16[16];
template <int E>
__device__ __forceinline__ void stage_img_dma(unsigned char* img, const bf16_t* __restrict__ src, int64_t ts, int T,
                                              int Tk, int wave, int lane) {
  constexpr int NC = E / 8;                                   // 16-B chunks per row
  constexpr int RPP = 1024 / (2 * E);                         // rows per 1-KiB piece
  constexpr int RPL = (256 / (2 * E)) > 0 ? 256 / (2 * E) : 1;
  const int npieces = Tk / RPP;
  for (int d = wave; d < npieces; d += 4) {
    const int row = RPP * d + lane / NC, slot = lane % NC;
    const int ch = slot ^ ((row / RPL) & (NC - 1));
    const void* p = row < T ? (const void*)(src + (int64_t)row * ts + ch * 8) : (const void*)attn_zero16;
    glds16(p, img + d * 1024);
  }
}

// row fragment: B[k = 32s + 8(l>>4) + i][n = row0 + (l&15)] = img[row0 + (l&15)][32s + ...]
template <int E>
__device__ __forceinline__ bf16x8v img_row_frag(const unsigned char* img, int row0, int s, int lane) {
  return __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(img + img_off<E>(row0 + (lane & 15), s * 4 + (lane >> 4))));
}

// transposed fragment: B[k = kb + 8(l>>4) + i][n = nb + (l&15)] = img[kb + ...][nb + (l&15)]
template <int E>
__device__ __forceinline__ bf16x8v img_tr_frag(const unsigned char* img, int kb, int nb, int lane) {
  const int gq = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int kr = kb + 8 * gq + q;
  const int ch = (nb >> 3) + (p >> 1);
  const unsigned char* a0 = img + img_off<E>(kr, ch) + 8 * (p & 1);
  const unsigned char* a1 = img + img_off<E>(kr + 4, ch) + 8 * (p & 1);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8v, v);
}

// A fragments of 16 global rows r0 + (l&15) (zero for rows >= T)
template <int E>
__device__ __forceinline__ void glob_row_frags(bf16x8v (&f)[E / 32], const bf16_t* __restrict__ base, int64_t ts, int r0,
                                               int T, int lane) {
  const int r = r0 + (lane & 15);
#pragma unroll
  for (int s = 0; s < E / 32; ++s) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r < T) v = *reinterpret_cast<const u32x4*>(base + (int64_t)r * ts + (s * 4 + (lane >> 4)) * 8);
    f[s] = __builtin_bit_cast(bf16x8v, v);
  }
}

// C-layout pair (cols 0..15, 16..31) -> A fragment (k = 32 cols) as bf16 hi + lo
__device__ __forceinline__ void c_to_a_split(float* scr, const f32x4& c0, const f32x4& c1, int lane, bf16x8v& hi,
                                             bf16x8v& lo) {
  const int col = lane & 15, rg = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    scr[(rg + j) * SCR_LD + col] = c0[j];
    scr[(rg + j) * SCR_LD + 16 + col] = c1[j];
  }
  __builtin_amdgcn_wave_barrier();
  const float* rp = scr + (lane & 15) * SCR_LD + 8 * (lane >> 4);
  const f32x4 x0 = *reinterpret_cast<const f32x4*>(rp);
  const f32x4 x1 = *reinterpret_cast<const f32x4*>(rp + 4);
  __builtin_amdgcn_wave_barrier();
  s16x8 h, l;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float v = i < 4 ? x0[i] : x1[i - 4];
    const uint32_t u = __float_as_uint(v) & 0xffff0000u;  // truncated high half (exact remainder below)
    h[i] = (short)(u >> 16);
    l[i] = (short)f2bf(v - __uint_as_float(u));
  }
  hi = __builtin_bit_cast(bf16x8v, h);
  lo = __builtin_bit_cast(bf16x8v, l);
}

// C-layout pair (cols 0..15, 16..31 of a 16-row tile) -> 16-B bf16 row stores:
// lane l writes row r0 + (l & 15), columns 8 (l >> 4) .. + 7 of the 32 (scaled by
// `scale`); rows >= T are skipped.  One 1-KiB store instruction instead of eight
// 2-byte scatters per lane.
__device__ __forceinline__ void c_store_rows(float* scr, const f32x4& c0, const f32x4& c1, float scale, int lane,
                                             bf16_t* __restrict__ base, int64_t ts, int r0, int T) {
  const int col = lane & 15, rg = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    scr[(rg + j) * SCR_LD + col] = c0[j];
    scr[(rg + j) * SCR_LD + 16 + col] = c1[j];
  }
  __builtin_amdgcn_wave_barrier();
  const float* rp = scr + (lane & 15) * SCR_LD + 8 * (lane >> 4);
  const f32x4 x0 = *reinterpret_cast<const f32x4*>(rp);
  const f32x4 x1 = *reinterpret_cast<const f32x4*>(rp + 4);
  __builtin_amdgcn_wave_barrier();
  const int r = r0 + (lane & 15);
  if (r < T) {
    const float v[8] = {x0[0] * scale, x0[1] * scale, x0[2] * scale, x0[3] * scale,
                        x1[0] * scale, x1[1] * scale, x1[2] * scale, x1[3] * scale};
    store_vec<bf16_t, 8>(base + (int64_t)r * ts + 8 * (lane >> 4), v);
  }
}

__device__ __forceinline__ float row16_max(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Longest-processing-time assignment of the 16-row tiles of one head to the 4
// waves (the same deterministic schedule in every wave; ntiles <= 16).  With
// causal masking a query tile q0 costs ceil((q0 + 16) / 32) key blocks and a key
// tile k0 costs (Tk - (k0 & ~31)) / 32 query blocks, so the round-robin deal
// (tile t -> wave t % 4) leaves the wave holding the ragged last tile (T' = 129:
// one valid row, every key block) ~40 % behind the others.
__device__ __forceinline__ uint32_t lpt_tiles(int ntiles, int Tk, bool causal, bool key_tiles, int wave) {
  int load[4] = {0, 0, 0, 0};
  uint32_t mine = 0;
  for (int i = 0; i < ntiles; ++i) {
    const int t = key_tiles ? i : ntiles - 1 - i;  // descending cost
    const int c0 = 16 * t;
    const int nb = !causal ? Tk / 32 : key_tiles ? (Tk - (c0 & ~31)) / 32 : min(Tk, (c0 + 16 + 31) & ~31) / 32;
    int w = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j)
      if (load[j] < load[w]) w = j;
    load[w] += nb + 1;
    if (w == wave) mine |= 1u << t;
  }
  return mine;
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

template <int E>
__global__ __launch_bounds__(256) void attn_fwd_mfma_k(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NS = E / 32, NE = E / 16;
  const int T = a.T, Tk = (T + 31) & ~31, Tq = (T + 15) & ~15;
  unsigned char* Ki = smem;
  unsigned char* Vi = Ki + Tk * E * 2;
  float* bias = reinterpret_cast<float*>(Vi + Tk * E * 2);  // [2T+1], region padded to 16 B
  float* scr_all = bias + ((2 * T + 4) & ~3);                 // [4][16][SCR_LD], 16 B aligned
  const int b = blockIdx.x / a.H, h = blockIdx.x - (blockIdx.x / a.H) * a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  stage_img_dma<E>(Ki, a.k + b * a.k_bs + h * a.k_hs, a.k_ts, T, Tk, wave, lane);
  stage_img_dma<E>(Vi, a.v + b * a.v_bs + h * a.v_hs, a.v_ts, T, Tk, wave, lane);
  for (int i = tid; i <= 2 * T; i += 256) bias[i] = a.table ? a.table[(int64_t)i * a.H + h] : 0.f;
  wait_vm<0>();
  __syncthreads();
  float* scr = scr_all + wave * 16 * SCR_LD;
  const float rs = rsqrtf((float)E);
  const bf16_t* qg = a.q + b * a.q_bs + h * a.q_hs;
  const int col = lane & 15, rg = (lane >> 4) * 4;
  // the wave's tiles in ascending order; the next tile's Q fragments are loaded while
  // the current one computes
  uint32_t mine = lpt_tiles(Tq / 16, Tk, a.causal, false, wave);
  bf16x8v qn[NS];
  if (mine) glob_row_frags<E>(qn, qg, a.q_ts, 16 * __builtin_ctz(mine), T, lane);
  while (mine) {
    const int q0 = 16 * __builtin_ctz(mine);
    mine &= mine - 1;
    bf16x8v qf[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = qn[s];
    if (mine) glob_row_frags<E>(qn, qg, a.q_ts, 16 * __builtin_ctz(mine), T, lane);
    f32x4 o[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) o[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) { m[j] = -INFINITY; l[j] = 0.f; }
    const int kend = a.causal ? min(Tk, (q0 + 16 + 31) & ~31) : Tk;
    for (int k0 = 0; k0 < kend; k0 += 32) {
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        s0 = MFMA(qf[s], img_row_frag<E>(Ki, k0, s, lane), s0);
        s1 = MFMA(qf[s], img_row_frag<E>(Ki, k0 + 16, s, lane), s1);
      }
      float bm[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = q0 + rg + j;
        const int ka = k0 + col, kb = k0 + 16 + col;
        const bool va = q < T && ka < T && (!a.causal || ka <= q);
        const bool vb = q < T && kb < T && (!a.causal || kb <= q);
        s0[j] = va ? s0[j] * rs + bias[q - ka + T] : -INFINITY;
        s1[j] = vb ? s1[j] * rs + bias[q - kb + T] : -INFINITY;
        bm[j] = row16_max(fmaxf(s0[j], s1[j]));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float mn = fmaxf(m[j], bm[j]);
        const float alpha = (mn == -INFINITY) ? 1.f : __expf(m[j] - mn);
        m[j] = mn;
        const float pa = (s0[j] == -INFINITY) ? 0.f : __expf(s0[j] - mn);
        const float pb = (s1[j] == -INFINITY) ? 0.f : __expf(s1[j] - mn);
        s0[j] = pa;
        s1[j] = pb;
        l[j] = l[j] * alpha + pa + pb;
#pragma unroll
        for (int e = 0; e < NE; ++e) o[e][j] *= alpha;
      }
      bf16x8v ph, pl;
      c_to_a_split(scr, s0, s1, lane, ph, pl);
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const bf16x8v vf = img_tr_frag<E>(Vi, k0, e * 16, lane);
        o[e] = MFMA(ph, vf, o[e]);
        o[e] = MFMA(pl, vf, o[e]);
      }
    }
    bf16_t* og = a.o + b * a.o_bs + h * a.o_hs;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = q0 + rg + j;
      const float lt = row16_sum(l[j]);
      const float inv = 1.f / lt;
#pragma unroll
      for (int e = 0; e < NE; ++e) o[e][j] *= inv;
      if (q < T && col == 0) a.lse[((int64_t)b * a.H + h) * T + q] = m[j] + __logf(lt);
    }
#pragma unroll
    for (int e = 0; e < NE; e += 2) c_store_rows(scr, o[e], o[e + 1], 1.f, lane, og + e * 16, a.o_ts, q0, T);
  }
}

// Backward, one block per (head, pass): pass 0 = query tiles -> dQ and the bias
// gradient; pass 1 = key tiles -> dK and dV.
// P = exp(S - lse) is recomputed from the forward's LSE; delta = rowsum(dO * O).
// MERGED: one block per (b, h) runs the row pass and then the column pass, restaging the
// LDS images in between (the second pass's q / dO come from L2, delta is computed once)
template <int E, bool MERGED = false>
__global__ __launch_bounds__(256, 3) void attn_bwd_mfma_k(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NS = E / 32, NE = E / 16;
  const int T = a.T, Tk = (T + 31) & ~31, Tq = (T + 15) & ~15;
  unsigned char* I0 = smem;                 // pass 0: K image, pass 1: Q image
  unsigned char* I1 = I0 + Tk * E * 2;      // pass 0: V image, pass 1: dO image
  float* bias = reinterpret_cast<float*>(I1 + Tk * E * 2);  // [2T+2]
  float* dbias = bias + 2 * T + 2;                            // [2T+2]
  float* lse = dbias + 2 * T + 2;                             // [Tk]
  float* delta = lse + Tk;                                    // [Tk]
  float* scr_all = delta + Tk;                                // [4][16][SCR_LD]
  // both passes of a head are adjacent logical blocks on one XCD, dispatched together:
  // the second pass's reads of q / k / v / o / dO hit that XCD's L2
  const int lid = xcd_remap(blockIdx.x, gridDim.x), bh = MERGED ? lid : lid >> 1;
  const int b = bh / a.H, h = bh - (bh / a.H) * a.H;
  const bool rows_pass = MERGED || (lid & 1) == 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16_t* qg = a.q + b * a.q_bs + h * a.q_hs;
  const bf16_t* kg = a.k + b * a.k_bs + h * a.k_hs;
  const bf16_t* vg = a.v + b * a.v_bs + h * a.v_hs;
  const bf16_t* og = a.o + b * a.o_bs + h * a.o_hs;
  const bf16_t* dog = a.dout + b * a.o_bs + h * a.o_hs;
  if (rows_pass) {
    stage_img_dma<E>(I0, kg, a.k_ts, T, Tk, wave, lane);
    stage_img_dma<E>(I1, vg, a.v_ts, T, Tk, wave, lane);
  } else {
    stage_img_dma<E>(I0, qg, a.q_ts, T, Tk, wave, lane);
    stage_img_dma<E>(I1, dog, a.o_ts, T, Tk, wave, lane);
  }
  for (int i = tid; i < 2 * T + 2; i += 256) bias[i] = (a.table && i <= 2 * T) ? a.table[(int64_t)i * a.H + h] : 0.f;
  for (int i = tid; i < 2 * T + 2; i += 256) dbias[i] = 0.f;
  const float* lse_g = a.lse + ((int64_t)b * a.H + h) * T;
  for (int i = tid; i < Tk; i += 256) lse[i] = i < T ? lse_g[i] : 0.f;
  // delta[q] = dO[q] . O[q]: one thread per (row, 16-byte chunk), the loads of
  // four passes in flight at once, then a shuffle sum over the E/8 chunk lanes
  {
    constexpr int CPR = E / 8;
    for (int base = 0; base < Tk * CPR; base += 4 * 256) {
      u32x4 u[4], v[4];
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = base + it * 256 + tid;
        const int q = idx / CPR, c = idx - q * CPR;
        u[it] = v[it] = u32x4{0u, 0u, 0u, 0u};
        if (q < T) {
          u[it] = *reinterpret_cast<const u32x4*>(dog + (int64_t)q * a.o_ts + c * 8);
          v[it] = *reinterpret_cast<const u32x4*>(og + (int64_t)q * a.o_ts + c * 8);
        }
      }
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = base + it * 256 + tid;
        const int q = idx / CPR, c = idx - q * CPR;
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          d += __uint_as_float(u[it][i] << 16) * __uint_as_float(v[it][i] << 16) +
               __uint_as_float(u[it][i] & 0xffff0000u) * __uint_as_float(v[it][i] & 0xffff0000u);
#pragma unroll
        for (int o = 1; o < CPR; o <<= 1) d += __shfl_xor(d, o, 64);
        if (c == 0 && q < Tk) delta[q] = d;
      }
    }
  }
  wait_vm<0>();
  __syncthreads();
  float* scr = scr_all + wave * 16 * SCR_LD;
  const float rs = rsqrtf((float)E);
  const int col = lane & 15, rg = (lane >> 4) * 4;
  if (rows_pass) {
    const uint32_t mine = lpt_tiles(Tq / 16, Tk, a.causal, false, wave);
    for (int q0 = 0; q0 < Tq; q0 += 16) {
      if (!((mine >> (q0 >> 4)) & 1u)) continue;
      bf16x8v qf[NS], df[NS];
      glob_row_frags<E>(qf, qg, a.q_ts, q0, T, lane);
      glob_row_frags<E>(df, dog, a.o_ts, q0, T, lane);
      f32x4 dq[NE];
#pragma unroll
      for (int e = 0; e < NE; ++e) dq[e] = f32x4{0.f, 0.f, 0.f, 0.f};
      float lq[4], dl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) { lq[j] = lse[min(q0 + rg + j, Tk - 1)]; dl[j] = delta[min(q0 + rg + j, Tk - 1)]; }
      const int kend = a.causal ? min(Tk, (q0 + 16 + 31) & ~31) : Tk;
      for (int k0 = 0; k0 < kend; k0 += 32) {
        f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, p0 = s0, p1 = s0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          s0 = MFMA(qf[s], img_row_frag<E>(I0, k0, s, lane), s0);
          s1 = MFMA(qf[s], img_row_frag<E>(I0, k0 + 16, s, lane), s1);
          p0 = MFMA(df[s], img_row_frag<E>(I1, k0, s, lane), p0);
          p1 = MFMA(df[s], img_row_frag<E>(I1, k0 + 16, s, lane), p1);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = q0 + rg + j;
          const int ka = k0 + col, kb = k0 + 16 + col;
          const bool va = q < T && ka < T && (!a.causal || ka <= q);
          const bool vb = q < T && kb < T && (!a.causal || kb <= q);
          const float da = va ? __expf(s0[j] * rs + bias[q - ka + T] - lq[j]) * (p0[j] - dl[j]) : 0.f;
          const float db = vb ? __expf(s1[j] * rs + bias[q - kb + T] - lq[j]) * (p1[j] - dl[j]) : 0.f;
          s0[j] = da;
          s1[j] = db;
        }
        bf16x8v gh, gl;
        c_to_a_split(scr, s0, s1, lane, gh, gl);
        if (a.dtable_part) {
          // bias gradient: the tile's dS is still in the wave's scratch; lane l
          // sums diagonal r - c = l - 31 of the 16 x 32 tile, so one LDS atomic
          // per lane and tile (distinct addresses within the instruction)
          // replaces eight colliding per-element atomics
          const int dd = lane - 31;
          const int idx = q0 - k0 + T + dd;
          if (lane < 47 && idx >= 0 && idx <= 2 * T) {
            float sum = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int c = r - dd;
              if (c >= 0 && c < 32) sum += scr[r * SCR_LD + c];
            }
            atomicAdd(&dbias[idx], sum);
          }
          __builtin_amdgcn_wave_barrier();
          asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const bf16x8v kf = img_tr_frag<E>(I0, k0, e * 16, lane);
          dq[e] = MFMA(gh, kf, dq[e]);
          dq[e] = MFMA(gl, kf, dq[e]);
        }
      }
      bf16_t* dqg = a.dq + b * a.q_bs + h * a.q_hs;
#pragma unroll
      for (int e = 0; e < NE; e += 2) c_store_rows(scr, dq[e], dq[e + 1], rs, lane, dqg + e * 16, a.q_ts, q0, T);
    }
    __syncthreads();
    if (a.dtable_part)
      for (int i = tid; i <= 2 * T; i += 256) a.dtable_part[((int64_t)b * (2 * T + 1) + i) * a.H + h] = dbias[i];
  }
  if constexpr (MERGED) {
    __syncthreads();  // every wave is done with the K / V images
    stage_img_dma<E>(I0, qg, a.q_ts, T, Tk, wave, lane);
    stage_img_dma<E>(I1, dog, a.o_ts, T, Tk, wave, lane);
    wait_vm<0>();
    __syncthreads();
  }
  if (MERGED || !rows_pass) {
    const uint32_t mine = lpt_tiles(Tq / 16, Tk, a.causal, true, wave);
    for (int k0 = 0; k0 < Tq; k0 += 16) {
      if (!((mine >> (k0 >> 4)) & 1u)) continue;
      bf16x8v kf[NS], vf[NS];
      glob_row_frags<E>(kf, kg, a.k_ts, k0, T, lane);
      glob_row_frags<E>(vf, vg, a.v_ts, k0, T, lane);
      f32x4 dk[NE], dv[NE];
#pragma unroll
      for (int e = 0; e < NE; ++e) { dk[e] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[e] = dk[e]; }
      const int qbeg = a.causal ? (k0 & ~31) : 0;
      for (int q0 = qbeg; q0 < Tk; q0 += 32) {
        // transposed scores: rows = keys k0 + rg + j, cols = queries q0 + col (+16)
        f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, p0 = s0, p1 = s0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          s0 = MFMA(kf[s], img_row_frag<E>(I0, q0, s, lane), s0);
          s1 = MFMA(kf[s], img_row_frag<E>(I0, q0 + 16, s, lane), s1);
          p0 = MFMA(vf[s], img_row_frag<E>(I1, q0, s, lane), p0);
          p1 = MFMA(vf[s], img_row_frag<E>(I1, q0 + 16, s, lane), p1);
        }
        const int qa = q0 + col, qb = q0 + 16 + col;
        const float la = lse[qa], lb = lse[qb], da_ = delta[qa], db_ = delta[qb];
        f32x4 g0, g1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = k0 + rg + j;
          const bool va = k < T && qa < T && (!a.causal || k <= qa);
          const bool vb = k < T && qb < T && (!a.causal || k <= qb);
          const float pa = va ? __expf(s0[j] * rs + bias[qa - k + T] - la) : 0.f;
          const float pb = vb ? __expf(s1[j] * rs + bias[qb - k + T] - lb) : 0.f;
          g0[j] = pa * (p0[j] - da_);
          g1[j] = pb * (p1[j] - db_);
          s0[j] = pa;
          s1[j] = pb;
        }
        bf16x8v ph, pl, gh, gl;
        c_to_a_split(scr, s0, s1, lane, ph, pl);
        c_to_a_split(scr, g0, g1, lane, gh, gl);
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const bf16x8v dof = img_tr_frag<E>(I1, q0, e * 16, lane);
          dv[e] = MFMA(ph, dof, dv[e]);
          dv[e] = MFMA(pl, dof, dv[e]);
          const bf16x8v qf = img_tr_frag<E>(I0, q0, e * 16, lane);
          dk[e] = MFMA(gh, qf, dk[e]);
          dk[e] = MFMA(gl, qf, dk[e]);
        }
      }
      bf16_t* dkg = a.dk + b * a.k_bs + h * a.k_hs;
      bf16_t* dvg = a.dv + b * a.v_bs + h * a.v_hs;
#pragma unroll
      for (int e = 0; e < NE; e += 2) {
        c_store_rows(scr, dk[e], dk[e + 1], rs, lane, dkg + e * 16, a.k_ts, k0, T);
        c_store_rows(scr, dv[e], dv[e + 1], 1.f, lane, dvg + e * 16, a.v_ts, k0, T);
      }
    }
  }
}
// ===========================================================================
// Backward on 32x32x16 MFMA (E = 64, T' <= 256, no general mask): one workgroup per
// (b, h) holding K, V, Q and dO images in LDS for the whole kernel, so the rows units (dQ)
// and the columns units (dK, dV) run side by side over the 4 waves (longest first) with no
// barrier and no global read between them.  The score tiles are oriented so that every
// product after the first takes its operand straight from the accumulator
// (cdna_hip_programming.md §3): no LDS scratch round trip, no bf16 hi / lo split of P and
// dS, and the gradients leave as transposed accumulators (8-byte runs of a token's row).
//  * rows unit, query tile i: S^T[k][q] = K . Q^T and dP^T = V . dO^T, dS^T elementwise
//    (the query is the lane), dQ^T += K^T . dS^T with K read transposed; the bias gradient
//    by rotating each register across the lane half by its key offset (ds_bpermute), which
//    puts one diagonal per lane: one LDS atomic per lane and tile;
//  * columns unit, key tile j: S = Q . K^T and dP = dO . V^T, P and dS elementwise (the key
//    is the lane), dV^T += dO^T . P and dK^T += Q^T . dS with dO / Q read transposed.
// Image rows are 128 B: chunk ch of row r at slot ch ^ s(r >> 1), s(u) = ((u & 1) << 2) |
// ((u >> 1) & 3): the row-fragment reads (16 lanes, 16 rows, one chunk) and the
// transposed reads (4 rows x 4 chunks per 32 lanes) are both conflict-free.
constexpr int E_BWD32 = 64;
// cost-ladder builds of attn_bwd32_k (tools/build_variant.sh ... -DLTHM_ABW_X=n; timing only,
// wrong results): 1 skips the units (staging, delta, bias copies, partial stores only), 2 skips
// the staging loads (units on stale LDS), 3 skips the units' gradient stores
#ifndef LTHM_ABW_X
#define LTHM_ABW_X 0
#endif
typedef float f32x16 __attribute__((ext_vector_type(16)));
#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

// image of rows [0, Tk) (row r at src + r * ts; rows >= T zero) by LDS-DMA: 1-KiB pieces of
// 8 rows, the lane loading the chunk that the swizzle puts in its lane-linear slot
// map (packed rows): row r at src + map[r] * ts, a zero row where map[r] < 0
__device__ __forceinline__ void stage_img32(unsigned char* img, const bf16_t* __restrict__ src, int64_t ts, int T,
                                            int Tk, int wave, int lane, int nw, const int* map = nullptr) {
  for (int d = wave; d < Tk / 8; d += nw) {
    const int row = 8 * d + (lane >> 3), slot = lane & 7;
    const int u = row >> 1;
    const int ch = slot ^ (((u & 1) << 2) | ((u >> 1) & 3));
    const int64_t rr = row < T ? (map ? (int64_t)map[row] : (int64_t)row) : -1;
    const void* p = rr >= 0 ? (const void*)(src + rr * ts + ch * 8) : (const void*)attn_zero16;
    glds16(p, img + d * 1024);
  }
}

__device__ __forceinline__ uint32_t pk_bf16_rne(float lo, float hi) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}

// registers 8 s .. 8 s + 7 of a 32 x 32 accumulator as the bf16 A operand of k-step s
__device__ __forceinline__ bf16x8v acc_frag32(const f32x16& x, int s) {
  const int o = 8 * s;
  const u32x4 h = {pk_bf16_rne(x[o], x[o + 1]), pk_bf16_rne(x[o + 2], x[o + 3]), pk_bf16_rne(x[o + 4], x[o + 5]),
                   pk_bf16_rne(x[o + 6], x[o + 7])};
  return __builtin_bit_cast(bf16x8v, h);
}

// dot of two bf16x8 fragments in fp32
__device__ __forceinline__ float bf8_dot(const bf16x8v& x, const bf16x8v& y) {
  const u32x4 u = __builtin_bit_cast(u32x4, x), w = __builtin_bit_cast(u32x4, y);
  float d = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    d += __uint_as_float(u[i] << 16) * __uint_as_float(w[i] << 16) +
         __uint_as_float(u[i] & 0xffff0000u) * __uint_as_float(w[i] & 0xffff0000u);
  return d;
}

// the relative-position bias in log2 units, two shifted copies each way, so that the four
// entries x .. x + 3 (columns units) or x .. x - 3 (rows units) of any x are two aligned
// 8-byte reads: ext[e] = table[e - BPAD] * log2 e inside [0, 2T], 0 outside (every x a
// tile forms lies in [-30, 2T + 30]).  ne = 34 (mod 64) puts the two copies' 32-lane read
// groups on disjoint banks.
constexpr int BPAD = 32;
__host__ __device__ __forceinline__ int bias_ne(int T) { return ((2 * T + 2 * BPAD + 11 + 63) & ~63) + 34; }

__device__ __forceinline__ int a32_swz(int row) {
  const int u = row >> 1;
  return ((u & 1) << 2) | ((u >> 1) & 3);
}

// lane-constant parts of the fragment offsets: tiles start at multiples of 16 image rows, so
// the swizzle of (tile row + r) depends on r alone.  row[s]: k-step s of row r0 + (lane & 31);
// tr[nd][hi]: the transposed read of columns 32 nd .. 32 nd + 31 (see a32 layout above)
struct Frag32Off {
  int row[4];
  int tr[2][2];
};
__device__ __forceinline__ Frag32Off frag32_off(int lane) {
  const int hh = lane >> 5, r32 = lane & 31;
  Frag32Off o;
#pragma unroll
  for (int s = 0; s < 4; ++s) o.row[s] = r32 * 128 + (((2 * s + hh) ^ a32_swz(r32)) << 4);
  const int colhalf = (lane >> 4) & 1, li = lane & 15, q = li >> 2, pp = li & 3;
#pragma unroll
  for (int nd = 0; nd < 2; ++nd)
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) {
      const int row = 4 * hh + 8 * hi + q, ch = 4 * nd + 2 * colhalf + (pp >> 1);
      o.tr[nd][hi] = row * 128 + ((ch ^ a32_swz(row)) << 4) + 8 * (pp & 1);
    }
  return o;
}
__device__ __forceinline__ bf16x8v frag_at(const unsigned char* p) {
  return __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ bf16x8v tr_at(const unsigned char* lo, const unsigned char* hi) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef __attribute__((address_space(3))) unsigned char lds_u8_t;
  const s16x4 l = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds_u8_t*)lo);
  const s16x4 h = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds_u8_t*)hi);
  const s16x8 v = {l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
  return __builtin_bit_cast(bf16x8v, v);
}

// 32 x 32 transposed-gradient accumulator (row e = 32 nd + 8 g + 4 hh + j in the registers,
// column = the token r0 + (lane & 31)) stored as 8-byte runs of the token's row
// map (packed rows): token r stored at row map[r], not at all where map[r] < 0
__device__ __forceinline__ void store_accT32(const f32x16& x, float scale, bf16_t* __restrict__ base, int64_t ts,
                                             int r0, int nd, int T, int lane, const int* map = nullptr) {
  const int r = r0 + (lane & 31), hh = lane >> 5;
  if (LTHM_ABW_X == 3) return;
  // every lane takes part in the lane-half exchange below; the store is per lane
  const int64_t rr = r < T ? (map ? (int64_t)map[r] : (int64_t)r) : -1;
  // register 4 g + j holds e = 32 nd + 8 g + 4 hh + j.  Packed to bf16 pairs, then the lane halves
  // trade groups (v_permlane32_swap: the upper half of the first operand with the lower half of
  // the second): lane (t, hh) ends with e = 32 nd + 16 hh .. + 15, two 16-B stores per lane
  // instead of four 8-B ones (the stores touch half as many lines per instruction)
  uint32_t w[4][2];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    w[g][0] = pk_bf16_rne(x[4 * g] * scale, x[4 * g + 1] * scale);
    w[g][1] = pk_bf16_rne(x[4 * g + 2] * scale, x[4 * g + 3] * scale);
  }
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const auto sw = __builtin_amdgcn_permlane32_swap(w[g][q], w[g + 2][q], false, false);
      w[g][q] = sw[0];
      w[g + 2][q] = sw[1];
    }
  if (r >= T || rr < 0) return;
  bf16_t* row = base + rr * ts + 32 * nd + 16 * hh;
  // hh = 0: w[g] = e 8g .. 8g + 3 (kept), w[g + 2] = e 8g + 4 .. 8g + 7 (from the upper half);
  // hh = 1: w[g] = e 16 + 8g .. + 3 (from the lower half), w[g + 2] = e 16 + 8g + 4 .. (kept)
#pragma unroll
  for (int g = 0; g < 2; ++g)
    *reinterpret_cast<uint4*>(row + 8 * g) = uint4{w[g][0], w[g][1], w[g + 2][0], w[g + 2][1]};
}

// the wave's units over the NW waves, longest first: unit u < nt is the rows unit of query
// tile u, unit nt + j the columns unit of key tile j (cost: tiles visited + 1)
template <int NW>
__device__ __forceinline__ uint32_t lpt_units(int nt, bool causal, int wave, bool tail = false) {
  int load[NW] = {};
  uint32_t mine = 0;
  for (int c = nt; c >= 1; --c)  // descending cost; causal: rows tile c - 1 and columns tile nt - c
    for (int side = 0; side < 2; ++side) {
      const int u = side == 0 ? c - 1 : nt + (nt - c);
      const int cost = (causal ? c : nt) + 1;
      int w = 0;
#pragma unroll
      for (int j = 1; j < NW; ++j)
        if (load[j] < load[w]) w = j;
      load[w] += cost;
      if (w == wave) mine |= 1u << u;
    }
  if (tail) {  // the tail unit (bit 2 nt), about two tile visits, on the least loaded wave
    int w = 0;
#pragma unroll
    for (int j = 1; j < NW; ++j)
      if (load[j] < load[w]) w = j;
    if (w == wave) mine |= 1u << (2 * nt);
  }
  return mine;
}

// LDS: the bias copies, lse, delta and the bias gradient first, then the K, Q, dO and V
// images (rows 0 .. Timg - 1, zero from T) and a zero slack up to V's last tile.  Tile reads
// past an image's end (the last, ragged tile) land in the next image or the slack, finite
// data: the edge tiles select those elements' P and dS to zero after the products, so no
// such read reaches a gradient.
struct Bwd32Smem {
  const unsigned char *IK, *IQ, *IO, *IV;
  const float *bfw, *brv, *lse, *dlt;
  float* dbias;
  int ne;
  const float *tp, *tds;  // tail query's P and dS per key (bwd32_tail_mode), else null
};

// Causal T' = 32 n + 1 (C2: T' = 129, the history plus one token): the last query row would
// take a tile of its own, a third of the tile visits for one row.  Instead the units cover
// rows / keys [0, T' - 1) and the last query q* = T' - 1 runs as a vector pass: its P / dS
// per key into LDS (and its bias-gradient diagonal), dQ[q*] and dK / dV of key q* (only q*
// sees it) in a small extra unit, and the rank-1 terms dS[q*][k] Q[q*], P[q*][k] dO[q*]
// added to the columns units' accumulators before they store.
__host__ __device__ __forceinline__ bool bwd32_tail_mode(int T, int causal) { return causal && T > 32 && (T & 31) == 1; }

// rows unit: dQ of query tile i (and the bias gradient of its tiles)
template <bool EDGE>
__device__ __forceinline__ void rows_math(f32x16& st, const f32x16& pt, const float* bp, float lq, float dl, float c2,
                                          int kb0, int kmax) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float2 lo = *reinterpret_cast<const float2*>(bp + 8 * g);
    const float2 hi = *reinterpret_cast<const float2*>(bp + 8 * g + 2);
    const float bv[4] = {lo.x - lq, lo.y - lq, hi.x - lq, hi.y - lq};
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int v = 4 * g + jj;
      const float p = __builtin_amdgcn_exp2f(fmaf(st[v], c2, bv[jj]));
      const float ds = p * (pt[v] - dl);
      st[v] = (!EDGE || kb0 + 8 * g + jj < kmax) ? ds : 0.f;
    }
  }
}

// G: Q / dO fragments from global memory, once per query tile (the rows kernel of long T'
// holds only the K / V images); else re-read per tile from the images
// Tu: rows / keys the units cover (T', or T' - 1 in the tail mode)
template <bool G = false>
__device__ __forceinline__ void bwd32_rows(const AttnArgs& a, const Bwd32Smem& m, const Frag32Off& fo, int b, int h,
                                           int i, int lane, int Tu) {
  constexpr float L2E = 1.4426950408889634f;
  const int T = a.T, nt = (Tu + 31) >> 5, hh = lane >> 5, r32 = lane & 31;
  const float rs = rsqrtf((float)E_BWD32), c2 = rs * L2E;
  const bool ragged = (Tu & 31) != 0;
  const int q0 = 32 * i, q = q0 + r32;
  bf16x8v gq[4], gd[4];
  if constexpr (G) {
    const bool pk = a.rmap != nullptr;
    const bf16_t* qg = a.q + (pk ? 0 : b * a.q_bs) + h * a.q_hs;
    const bf16_t* dg = a.dout + (pk ? 0 : b * a.o_bs) + h * a.o_hs;
    const int64_t rq = q < Tu ? (pk ? (int64_t)a.rmap[(int64_t)b * T + q] : (int64_t)q) : 0;
    const int64_t rd = q < Tu ? (pk ? (int64_t)a.wmap[(int64_t)b * T + q] : (int64_t)q) : -1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u32x4 u = {0u, 0u, 0u, 0u}, v = u;
      if (q < Tu) u = *reinterpret_cast<const u32x4*>(qg + rq * a.q_ts + 16 * s + 8 * hh);
      if (rd >= 0) v = *reinterpret_cast<const u32x4*>(dg + rd * a.o_ts + 16 * s + 8 * hh);
      gq[s] = __builtin_bit_cast(bf16x8v, u);
      gd[s] = __builtin_bit_cast(bf16x8v, v);
    }
  }
  const float lq = m.lse[q], dl = m.dlt[q];
  const int kmax = q < Tu ? (a.causal ? q + 1 : Tu) : 0;  // keys k < kmax are live for this query
  f32x16 dq[2];
#pragma unroll
  for (int nd = 0; nd < 2; ++nd)
#pragma unroll
    for (int v = 0; v < 16; ++v) dq[nd][v] = 0.f;
  float carry = 0.f;
  const bool has_tab = a.dtable_part != nullptr;
  const int jend = a.causal ? i + 1 : nt;
  // bias of (q, k0 + 4 hh - jj) for tile 0: descending copy, 32 entries on per tile
  const int z0 = m.ne - 1 - (q - 4 * hh + T + BPAD);
  const float* bp = m.brv + (z0 & 1) * m.ne + (z0 & ~1);
  float wrap[16];  // lane constants of the diagonal rotation: 1 where register v wraps
#pragma unroll
  for (int v = 0; v < 16; ++v) wrap[v] = r32 + 4 * hh + 8 * (v >> 2) + (v & 3) >= 32 ? 1.f : 0.f;
  for (int j = 0; j < jend; ++j, bp += 32) {
    const int k0 = 32 * j;
    f32x16 st, pt;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      st[v] = 0.f;
      pt[v] = 0.f;
    }
    int qo = q0 * 128;  // laundered: the Q / dO fragments are re-read per tile, not kept live
    asm volatile("" : "+v"(qo));
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      st = MFMA32(frag_at(m.IK + k0 * 128 + fo.row[s]), G ? gq[s] : frag_at(m.IQ + qo + fo.row[s]), st);
      pt = MFMA32(frag_at(m.IV + k0 * 128 + fo.row[s]), G ? gd[s] : frag_at(m.IO + qo + fo.row[s]), pt);
    }
    // S^T[k][q]: the key k = k0 + 8 g + 4 hh + jj in register 4 g + jj, the query q in the lane
    if ((a.causal && j == i) || (ragged && (i == nt - 1 || j == nt - 1)))
      rows_math<true>(st, pt, bp, lq, dl, c2, k0 + 4 * hh, kmax);
    else
      rows_math<false>(st, pt, bp, lq, dl, c2, k0 + 4 * hh, kmax);
    if (has_tab) {
      // diagonal sums of the tile: register v rotated across the lane half by its key
      // offset puts diagonal q - k = r32 (r32 - 32 when wrapped) in lane r32
      float tot = 0.f, neg = 0.f;
      // the 16 rotation addresses are lane constants the compiler keeps live across the tiles
      // (234 / 246 VGPRs, no spill: C5 backward 3.15 -> 3.07 ms, C2 0.95 -> 0.94 ms against
      // recomputing them per tile, tools/ab_attn_lib.sh)
      const int rl = r32 + 4 * hh;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int kv = rl + 8 * (v >> 2) + (v & 3);
        const float x =
            __int_as_float(__builtin_amdgcn_ds_bpermute(((kv & 31) | (hh << 5)) << 2, __float_as_int(st[v])));
        tot += x;
        neg = fmaf(x, wrap[v], neg);
      }
      tot += __shfl_xor(tot, 32, 64);
      neg += __shfl_xor(neg, 32, 64);
      // diagonal q - k = 32 (i - j) + r32 is complete: this tile's pos, the previous tile's neg
      const int d = 32 * (i - j) + r32 + T;
      if (hh == 0 && d <= 2 * T) atomicAdd(&m.dbias[d], tot - neg + carry);
      carry = neg;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8v gf = acc_frag32(st, s);
      const unsigned char* kt = m.IK + (k0 + 16 * s) * 128;
#pragma unroll
      for (int nd = 0; nd < 2; ++nd) dq[nd] = MFMA32(tr_at(kt + fo.tr[nd][0], kt + fo.tr[nd][1]), gf, dq[nd]);
    }
  }
  if (has_tab) {
    const int d = 32 * (i - jend) + r32 + T;
    if (hh == 0 && d >= 0 && d <= 2 * T) atomicAdd(&m.dbias[d], carry);
  }
  const bool pk = G && a.wmap != nullptr;
  bf16_t* dqg = a.dq + (pk ? 0 : b * a.q_bs) + h * a.q_hs;
#pragma unroll
  for (int nd = 0; nd < 2; ++nd)
    store_accT32(dq[nd], rs, dqg, a.q_ts, q0, nd, T, lane, pk ? a.wmap + (int64_t)b * T : nullptr);
}

// columns unit: dK, dV of key tile j
template <bool EDGE>
__device__ __forceinline__ void cols_math(f32x16& sx, f32x16& px, const float* bp, const float* lse, const float* dlt,
                                          float c2, int qb0, int qlo, int span) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 l4 = *reinterpret_cast<const float4*>(lse + 8 * g);
    const float4 d4 = *reinterpret_cast<const float4*>(dlt + 8 * g);
    const float2 lo = *reinterpret_cast<const float2*>(bp + 8 * g);
    const float2 hi = *reinterpret_cast<const float2*>(bp + 8 * g + 2);
    const float bv[4] = {lo.x - l4.x, lo.y - l4.y, hi.x - l4.z, hi.y - l4.w};
    const float dv4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int v = 4 * g + jj;
      const float p = __builtin_amdgcn_exp2f(fmaf(sx[v], c2, bv[jj]));
      const float ds = p * (px[v] - dv4[jj]);
      const bool live = !EDGE || (unsigned)(qb0 + 8 * g + jj - qlo) < (unsigned)span;
      px[v] = live ? ds : 0.f;
      sx[v] = live ? p : 0.f;
    }
  }
}

// G: K / V fragments from global memory, once per key tile (the columns kernel of long T'
// holds only the Q / dO images)
template <bool G = false>
__device__ __forceinline__ void bwd32_cols(const AttnArgs& a, const Bwd32Smem& m, const Frag32Off& fo, int b, int h,
                                           int j, int lane, int Tu, int ilo = 0) {
  constexpr float L2E = 1.4426950408889634f;
  const int T = a.T, nt = (Tu + 31) >> 5, hh = lane >> 5, r32 = lane & 31;
  const float rs = rsqrtf((float)E_BWD32), c2 = rs * L2E;
  const bool ragged = (Tu & 31) != 0;
  const int k0 = 32 * j, k = k0 + r32;
  bf16x8v gk[4], gv[4];
  const bool pkd = G && a.rmap != nullptr;
  const int64_t rk = k < Tu ? (pkd ? (int64_t)a.rmap[(int64_t)b * T + k] : (int64_t)k) : 0;
  if constexpr (G) {
    const bf16_t* kg = a.k + (pkd ? 0 : b * a.k_bs) + h * a.k_hs;
    const bf16_t* vg = a.v + (pkd ? 0 : b * a.v_bs) + h * a.v_hs;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u32x4 u = {0u, 0u, 0u, 0u}, v = u;
      if (k < Tu) {
        u = *reinterpret_cast<const u32x4*>(kg + rk * a.k_ts + 16 * s + 8 * hh);
        v = *reinterpret_cast<const u32x4*>(vg + rk * a.v_ts + 16 * s + 8 * hh);
      }
      gk[s] = __builtin_bit_cast(bf16x8v, u);
      gv[s] = __builtin_bit_cast(bf16x8v, v);
    }
  }
  // live queries of this key: [qlo, T)
  const int qlo = k < Tu ? (a.causal ? k : 0) : Tu, span = Tu - qlo;
  f32x16 dk[2], dv[2];
#pragma unroll
  for (int nd = 0; nd < 2; ++nd)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      dk[nd][v] = 0.f;
      dv[nd][v] = 0.f;
    }
  const int i0 = max(a.causal ? j : 0, ilo);
  // bias of (q0 + 4 hh + jj, k): ascending copy, 32 entries on per tile
  const int e0 = 32 * i0 + 4 * hh - k + T + BPAD;
  const float* bp = m.bfw + (e0 & 1) * m.ne + (e0 & ~1);
  for (int i = i0; i < nt; ++i, bp += 32) {
    const int q0 = 32 * i;
    f32x16 sx, px;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      sx[v] = 0.f;
      px[v] = 0.f;
    }
    int ko = k0 * 128;  // laundered: the K / V fragments are re-read per tile, not kept live
    asm volatile("" : "+v"(ko));
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sx = MFMA32(frag_at(m.IQ + q0 * 128 + fo.row[s]), G ? gk[s] : frag_at(m.IK + ko + fo.row[s]), sx);
      px = MFMA32(frag_at(m.IO + q0 * 128 + fo.row[s]), G ? gv[s] : frag_at(m.IV + ko + fo.row[s]), px);
    }
    // S[q][k]: the query q = q0 + 8 g + 4 hh + jj in register 4 g + jj, the key k in the lane
    const int qb0 = q0 + 4 * hh;
    if ((a.causal && j == i) || (ragged && (i == nt - 1 || j == nt - 1)))
      cols_math<true>(sx, px, bp, m.lse + qb0, m.dlt + qb0, c2, qb0, qlo, span);
    else
      cols_math<false>(sx, px, bp, m.lse + qb0, m.dlt + qb0, c2, qb0, qlo, span);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8v pf = acc_frag32(sx, s), gf = acc_frag32(px, s);
      const unsigned char* ot = m.IO + (q0 + 16 * s) * 128;
      const unsigned char* qt = m.IQ + (q0 + 16 * s) * 128;
#pragma unroll
      for (int nd = 0; nd < 2; ++nd) {
        dv[nd] = MFMA32(tr_at(ot + fo.tr[nd][0], ot + fo.tr[nd][1]), pf, dv[nd]);
        dk[nd] = MFMA32(tr_at(qt + fo.tr[nd][0], qt + fo.tr[nd][1]), gf, dk[nd]);
      }
    }
  }
  if (m.tds) {  // tail mode: the last query's rank-1 terms (k < Tu: every lane's key is live)
    const int qs = T - 1, sw = a32_swz(qs);
    const float dsk = m.tds[k], pk = m.tp[k];
#pragma unroll
    for (int nd = 0; nd < 2; ++nd)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int e = 32 * nd + 8 * g + 4 * hh, off = qs * 128 + (((e >> 3) ^ sw) << 4) + 8 * hh;
        const uint2 qv = *reinterpret_cast<const uint2*>(m.IQ + off);
        const uint2 ov = *reinterpret_cast<const uint2*>(m.IO + off);
        const float qf[4] = {__uint_as_float(qv.x << 16), __uint_as_float(qv.x & 0xffff0000u),
                             __uint_as_float(qv.y << 16), __uint_as_float(qv.y & 0xffff0000u)};
        const float of[4] = {__uint_as_float(ov.x << 16), __uint_as_float(ov.x & 0xffff0000u),
                             __uint_as_float(ov.y << 16), __uint_as_float(ov.y & 0xffff0000u)};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          dk[nd][4 * g + jj] = fmaf(dsk, qf[jj], dk[nd][4 * g + jj]);
          dv[nd][4 * g + jj] = fmaf(pk, of[jj], dv[nd][4 * g + jj]);
        }
      }
  }
  if (pkd) {
    // a chain key's gradient is one sequence's share of the chain row's: to the chain buffer
    // (summed over the sequences afterwards), the others to their packed row (keys k >= T:
    // store_accT32 stores nothing, but every lane takes part in its lane exchange)
    const bool ch = rk < a.chain;
    bf16_t* dkg = ch ? a.dk_chain + ((int64_t)b * a.chain + k) * a.chain_ts + h * a.k_hs : a.dk + rk * a.k_ts + h * a.k_hs;
    bf16_t* dvg = ch ? a.dv_chain + ((int64_t)b * a.chain + k) * a.chain_ts + h * a.v_hs : a.dv + rk * a.v_ts + h * a.v_hs;
#pragma unroll
    for (int nd = 0; nd < 2; ++nd) {
      store_accT32(dk[nd], rs, dkg - (int64_t)(k0 + r32) * a.k_ts, a.k_ts, k0, nd, T, lane);
      store_accT32(dv[nd], 1.f, dvg - (int64_t)(k0 + r32) * a.v_ts, a.v_ts, k0, nd, T, lane);
    }
    return;
  }
  bf16_t* dkg = a.dk + b * a.k_bs + h * a.k_hs;
  bf16_t* dvg = a.dv + b * a.v_bs + h * a.v_hs;
#pragma unroll
  for (int nd = 0; nd < 2; ++nd) {
    store_accT32(dk[nd], rs, dkg, a.k_ts, k0, nd, T, lane);
    store_accT32(dv[nd], 1.f, dvg, a.v_ts, k0, nd, T, lane);
  }
}

// the tail query's vector pass (bwd32_tail_mode): P and dS of (q*, k) for every key k <= q*
// (a thread per key; dot products over the swizzled image rows), stored to tp / tds and as
// the bias gradient's diagonal q* - k (written once each, before any unit adds to it)
__device__ __forceinline__ void bwd32_tail_pass(const Bwd32Smem& m, float* tp, float* tds, float* dbias, int T, int tid,
                                                int nth, bool accum = false) {
  const float c2 = rsqrtf((float)E_BWD32) * 1.4426950408889634f;
  const int qs = T - 1, sq = a32_swz(qs);
  const float lq = m.lse[qs], dl = m.dlt[qs];
  for (int k = tid; k <= qs; k += nth) {
    const int sk = a32_swz(k);
    float sc = 0.f, dp = 0.f;
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) {
      const bf16x8v kf = frag_at(m.IK + k * 128 + ((ch ^ sk) << 4)), vf = frag_at(m.IV + k * 128 + ((ch ^ sk) << 4));
      const bf16x8v qf = frag_at(m.IQ + qs * 128 + ((ch ^ sq) << 4)), of = frag_at(m.IO + qs * 128 + ((ch ^ sq) << 4));
      sc += bf8_dot(kf, qf);
      dp += bf8_dot(vf, of);
    }
    const float p = __builtin_amdgcn_exp2f(fmaf(sc, c2, m.bfw[qs - k + T + BPAD] - lq));
    const float ds = p * (dp - dl);
    tp[k] = p;
    tds[k] = ds;
    if (accum) dbias[qs - k + T] += ds;  // the persistent kernel sums the diagonals over its batch entries
    else dbias[qs - k + T] = ds;
  }
}

// the tail unit: dQ[q*] = rs sum_k dS[q*][k] K[k] (lane = a column pair, the lane halves split
// the keys), dK[q*] = rs dS[q*][q*] Q[q*] and dV[q*] = P[q*][q*] dO[q*]
__device__ __forceinline__ void bwd32_tail_unit(const AttnArgs& a, const Bwd32Smem& m, int b, int h, int lane) {
  const float rs = rsqrtf((float)E_BWD32);
  const int T = a.T, qs = T - 1, hh = lane >> 5, c = 2 * (lane & 31);
  float a0 = 0.f, a1 = 0.f;
  for (int k = hh; k <= qs; k += 2) {
    const float d = m.tds[k];
    const uint32_t kv = *reinterpret_cast<const uint32_t*>(m.IK + k * 128 + (((c >> 3) ^ a32_swz(k)) << 4) + 2 * (c & 7));
    a0 = fmaf(d, __uint_as_float(kv << 16), a0);
    a1 = fmaf(d, __uint_as_float(kv & 0xffff0000u), a1);
  }
  a0 += __shfl_xor(a0, 32, 64);
  a1 += __shfl_xor(a1, 32, 64);
  const int off = qs * 128 + (((c >> 3) ^ a32_swz(qs)) << 4) + 2 * (c & 7);
  if (hh == 0) {
    *reinterpret_cast<uint32_t*>(a.dq + b * a.q_bs + h * a.q_hs + (int64_t)qs * a.q_ts + c) = pk_bf16_rne(rs * a0, rs * a1);
    const uint32_t qv = *reinterpret_cast<const uint32_t*>(m.IQ + off);
    const float f = rs * m.tds[qs];
    *reinterpret_cast<uint32_t*>(a.dk + b * a.k_bs + h * a.k_hs + (int64_t)qs * a.k_ts + c) =
        pk_bf16_rne(f * __uint_as_float(qv << 16), f * __uint_as_float(qv & 0xffff0000u));
  } else {
    const uint32_t ov = *reinterpret_cast<const uint32_t*>(m.IO + off);
    const float f = m.tp[qs];
    *reinterpret_cast<uint32_t*>(a.dv + b * a.v_bs + h * a.v_hs + (int64_t)qs * a.v_ts + c) =
        pk_bf16_rne(f * __uint_as_float(ov << 16), f * __uint_as_float(ov & 0xffff0000u));
  }
}

__host__ __device__ __forceinline__ int bwd32_timg(int T) { return (T + 7) & ~7; }
// float region, 16-byte multiple: bias copies, lse, delta, bias gradient, and in the tail mode
// the tail query's P / dS per key
__host__ __device__ __forceinline__ int bwd32_fbytes(int T, bool tail = false) {
  return (4 * bias_ne(T) + 2 * ((T + 31) & ~31) + ((2 * T + 1 + 3) & ~3) + (tail ? 2 * ((T + 3) & ~3) : 0)) * 4;
}

// rows past V for the last tile (Tu: the rows the units cover)
__host__ __device__ __forceinline__ int bwd32_slack(int T, int Tu) {
  const int d = ((Tu + 31) & ~31) - bwd32_timg(T);
  return d > 0 ? d : 0;
}
__host__ __device__ __forceinline__ int bwd32_slack(int T) { return bwd32_slack(T, T); }

#ifndef LTHM_BWD32_NW
#define LTHM_BWD32_NW 4  // A/B builds: tools/build_variant.sh ... -DLTHM_BWD32_NW=8
#endif
constexpr int BWD32_NW = LTHM_BWD32_NW, BWD32_WPE = 2;  // waves per (b, h); waves per SIMD the registers allow

template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(BWD32_WPE, BWD32_WPE))) void attn_bwd32_k(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr float L2E = 1.4426950408889634f;
  const int T = a.T, Tk = (T + 31) & ~31, ne = bias_ne(T), Ti = bwd32_timg(T);
  const bool tail = a.tail != 0;
  const int Tu = tail ? T - 1 : T, nt = (Tu + 31) >> 5;  // rows / keys of the units
  float* bfw = reinterpret_cast<float*>(smem);  // [2][ne] ascending copies
  float* brv = bfw + 2 * ne;                     // [2][ne] descending copies
  float* lse_s = brv + 2 * ne;                   // [Tk] lse * log2 e (0 past T)
  float* dlt_s = lse_s + Tk;                     // [Tk] delta = dO . O (0 past T)
  float* dbias = dlt_s + Tk;                     // [2T + 1]
  float* tp = dbias + ((2 * T + 1 + 3) & ~3);    // tail mode: [T] P, [T] dS of the last query
  float* tds = tp + ((T + 3) & ~3);
  unsigned char* IK = smem + bwd32_fbytes(T, tail);
  unsigned char* IQ = IK + Ti * 128;
  unsigned char* IO = IQ + Ti * 128;
  unsigned char* IV = IO + Ti * 128;
  const int bh = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bh / a.H, h = bh - (bh / a.H) * a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16_t* qg = a.q + b * a.q_bs + h * a.q_hs;
  const bf16_t* kg = a.k + b * a.k_bs + h * a.k_hs;
  const bf16_t* vg = a.v + b * a.v_bs + h * a.v_hs;
  const bf16_t* og = a.o + b * a.o_bs + h * a.o_hs;
  const bf16_t* dog = a.dout + b * a.o_bs + h * a.o_hs;
  const float* lse_g = a.lse + ((int64_t)b * a.H + h) * T;
  if (LTHM_ABW_X != 2) {
  stage_img32(IK, kg, a.k_ts, T, Ti, wave, lane, NW);
  stage_img32(IQ, qg, a.q_ts, T, Ti, wave, lane, NW);
  stage_img32(IO, dog, a.o_ts, T, Ti, wave, lane, NW);
  stage_img32(IV, vg, a.v_ts, T, Ti, wave, lane, NW);
  }
  if (LTHM_ABW_X != 2) {  // delta[q] = dO[q] . O[q]: four threads per row, every load in flight before the first use
    constexpr int RPI = 16 * NW, NIT = (256 + RPI - 1) / RPI;  // rows per iteration, iterations for Tk <= 256
    u32x4 du[NIT][2], ou[NIT][2];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int r = (tid >> 2) + RPI * it, c = (tid & 3) * 16;
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        du[it][x] = ou[it][x] = (u32x4){0u, 0u, 0u, 0u};
        if (r < T) {
          du[it][x] = *reinterpret_cast<const u32x4*>(dog + (int64_t)r * a.o_ts + c + 8 * x);
          ou[it][x] = *reinterpret_cast<const u32x4*>(og + (int64_t)r * a.o_ts + c + 8 * x);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int r = (tid >> 2) + RPI * it;
      float d = bf8_dot(__builtin_bit_cast(bf16x8v, du[it][0]), __builtin_bit_cast(bf16x8v, ou[it][0])) +
                bf8_dot(__builtin_bit_cast(bf16x8v, du[it][1]), __builtin_bit_cast(bf16x8v, ou[it][1]));
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      if ((tid & 3) == 0 && r < Tk) {
        dlt_s[r] = r < T ? d : 0.f;
        lse_s[r] = r < T ? lse_g[r] * L2E : 0.f;
      }
    }
  }
  for (int c = 0; c < 2; ++c)
    for (int y = tid; y < ne; y += 64 * NW) {
      const int xf = y + c - BPAD, xr = ne - 1 - (y + c) - BPAD;
      bfw[c * ne + y] = (a.table && xf >= 0 && xf <= 2 * T) ? a.table[(int64_t)xf * a.H + h] * L2E : 0.f;
      brv[c * ne + y] = (a.table && xr >= 0 && xr <= 2 * T) ? a.table[(int64_t)xr * a.H + h] * L2E : 0.f;
    }
  for (int i = tid; i <= 2 * T; i += 64 * NW) dbias[i] = 0.f;
  for (int i = tid; i < bwd32_slack(T, Tu) * 32; i += 64 * NW) reinterpret_cast<float*>(IV + Ti * 128)[i] = 0.f;
  wait_vm<0>();
  __syncthreads();
  const Bwd32Smem m{IK, IQ, IO, IV, bfw, brv, lse_s, dlt_s, dbias, ne, tail ? tp : nullptr, tail ? tds : nullptr};
  if (tail) {
    bwd32_tail_pass(m, tp, tds, dbias, T, tid, 64 * NW);
    __syncthreads();
  }
  const Frag32Off fo = frag32_off(lane);
  const uint32_t mine = LTHM_ABW_X == 1 ? 0u : lpt_units<NW>(nt, a.causal, wave, tail);
  // longest first: the rows unit of tile c - 1 and the columns unit of tile nt - c cost alike
  for (int c = nt; c >= 1; --c) {
    if (mine & (1u << (c - 1))) bwd32_rows(a, m, fo, b, h, c - 1, lane, Tu);
    if (mine & (1u << (2 * nt - c))) bwd32_cols(a, m, fo, b, h, nt - c, lane, Tu);
  }
  if (mine & (1u << (2 * nt))) bwd32_tail_unit(a, m, b, h, lane);
  if (a.dtable_part) {
    __syncthreads();
    for (int i = tid; i <= 2 * T; i += 64 * NW) a.dtable_part[((int64_t)b * (2 * T + 1) + i) * a.H + h] = dbias[i];
  }
}

static size_t bwd32_lds(int T, bool tail) {
  return (size_t)bwd32_fbytes(T, tail) + (size_t)(4 * bwd32_timg(T) + bwd32_slack(T, tail ? T - 1 : T)) * 128;
}

// Persistent form of attn_bwd32_k (round 5): one workgroup per CU walks the batch entries of one
// head, b = slot, slot + S, ... (S workgroups per head), with TWO image sets: while the units of
// entry b run on one set, the LDS-DMA of entry b + S fills the other, so the K / Q / dO / V
// staging (the non-persistent kernel waits on it at every workgroup start) overlaps the MFMA
// work.  The next entry's O rows and LSE ride in registers (one wave per SIMD: the whole
// register file); delta = dO . O is formed from the landed dO image.  The head's bias copies
// are staged once, and the bias gradient accumulates over the workgroup's entries in LDS: one
// partial per (slot, head) instead of one per batch entry.
__host__ __device__ __forceinline__ int bwd32p_set_bytes(int T, bool tail) {
  return (4 * bwd32_timg(T) + bwd32_slack(T, tail ? T - 1 : T)) * 128;
}
static size_t bwd32p_lds(int T, bool tail) { return (size_t)bwd32_fbytes(T, tail) + 2 * (size_t)bwd32p_set_bytes(T, tail); }

template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(1, 1))) void attn_bwd32p_k(AttnArgs a, int B,
                                                                                                  int S) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr float L2E = 1.4426950408889634f;
  constexpr int NIT = (256 + 16 * NW - 1) / (16 * NW);  // delta rows per thread (Tk <= 256)
  const int T = a.T, Tk = (T + 31) & ~31, ne = bias_ne(T), Ti = bwd32_timg(T);
  const bool tail = a.tail != 0;
  const int Tu = tail ? T - 1 : T, nt = (Tu + 31) >> 5;
  float* bfw = reinterpret_cast<float*>(smem);
  float* brv = bfw + 2 * ne;
  float* lse_s = brv + 2 * ne;
  float* dlt_s = lse_s + Tk;
  float* dbias = dlt_s + Tk;
  float* tp = dbias + ((2 * T + 1 + 3) & ~3);
  float* tds = tp + ((T + 3) & ~3);
  const int setb = bwd32p_set_bytes(T, tail);
  unsigned char* img0 = smem + bwd32_fbytes(T, tail);
  const int g = blockIdx.x, h = g % a.H, slot = g / a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the head's bias copies, the bias-gradient sums, both sets' zero slack
  for (int c = 0; c < 2; ++c)
    for (int y = tid; y < ne; y += 64 * NW) {
      const int xf = y + c - BPAD, xr = ne - 1 - (y + c) - BPAD;
      bfw[c * ne + y] = (a.table && xf >= 0 && xf <= 2 * T) ? a.table[(int64_t)xf * a.H + h] * L2E : 0.f;
      brv[c * ne + y] = (a.table && xr >= 0 && xr <= 2 * T) ? a.table[(int64_t)xr * a.H + h] * L2E : 0.f;
    }
  for (int i = tid; i <= 2 * T; i += 64 * NW) dbias[i] = 0.f;
  for (int st = 0; st < 2; ++st)
    for (int i = tid; i < bwd32_slack(T, Tu) * 32; i += 64 * NW)
      reinterpret_cast<float*>(img0 + st * setb + 4 * Ti * 128)[i] = 0.f;
  // entry b's images into set st, its O rows and LSE into registers
  u32x4 ou[NIT][2];
  float lq = 0.f;
  auto fetch = [&](int bb, int st) {
    unsigned char* IK = img0 + st * setb;
    stage_img32(IK, a.k + bb * a.k_bs + h * a.k_hs, a.k_ts, T, Ti, wave, lane, NW);
    stage_img32(IK + Ti * 128, a.q + bb * a.q_bs + h * a.q_hs, a.q_ts, T, Ti, wave, lane, NW);
    stage_img32(IK + 2 * Ti * 128, a.dout + bb * a.o_bs + h * a.o_hs, a.o_ts, T, Ti, wave, lane, NW);
    stage_img32(IK + 3 * Ti * 128, a.v + bb * a.v_bs + h * a.v_hs, a.v_ts, T, Ti, wave, lane, NW);
    const bf16_t* og = a.o + bb * a.o_bs + h * a.o_hs;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int r = (tid >> 2) + 16 * NW * it, c = (tid & 3) * 16;
#pragma unroll
      for (int x = 0; x < 2; ++x)
        ou[it][x] = r < T ? *reinterpret_cast<const u32x4*>(og + (int64_t)r * a.o_ts + c + 8 * x) : u32x4{0u, 0u, 0u, 0u};
    }
    lq = tid < T ? a.lse[((int64_t)bb * a.H + h) * T + tid] : 0.f;
  };
  const Frag32Off fo = frag32_off(lane);
  const uint32_t mine = LTHM_ABW_X == 1 ? 0u : lpt_units<NW>(nt, a.causal, wave, tail);
  if (slot < B) fetch(slot, 0);
  int st = 0;
  for (int b = slot; b < B; b += S, st ^= 1) {
    wait_vm<0>();
    __syncthreads();  // entry b landed; every wave is done with the previous entry (set st ^ 1, floats)
    unsigned char* IK = img0 + st * setb;
    unsigned char* IQ = IK + Ti * 128;
    unsigned char* IO = IQ + Ti * 128;
    unsigned char* IV = IO + Ti * 128;
    {  // delta[q] = dO[q] . O[q] from the dO image and the O rows in registers; the LSE
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int r = (tid >> 2) + 16 * NW * it, c = (tid & 3) * 16;
        const int rr = r < Ti ? r : 0;
        float d = 0.f;
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          const int ch = (c >> 3) + x;
          const bf16x8v dv = frag_at(IO + rr * 128 + ((ch ^ a32_swz(rr)) << 4));
          d += bf8_dot(dv, __builtin_bit_cast(bf16x8v, ou[it][x]));
        }
        d += __shfl_xor(d, 1, 64);
        d += __shfl_xor(d, 2, 64);
        if ((tid & 3) == 0 && r < Tk) dlt_s[r] = r < T ? d : 0.f;
      }
      if (tid < Tk) lse_s[tid] = tid < T ? lq * L2E : 0.f;
    }
    if (b + S < B) fetch(b + S, st ^ 1);  // the other set's last readers passed the barrier above
    __syncthreads();
    const Bwd32Smem m{IK, IQ, IO, IV, bfw, brv, lse_s, dlt_s, dbias, ne, tail ? tp : nullptr, tail ? tds : nullptr};
    if (tail) {
      bwd32_tail_pass(m, tp, tds, dbias, T, tid, 64 * NW, true);
      __syncthreads();
    }
    const int bh = b;  // (b, h) of this entry
    for (int c = nt; c >= 1; --c) {
      if (mine & (1u << (c - 1))) bwd32_rows(a, m, fo, bh, h, c - 1, lane, Tu);
      if (mine & (1u << (2 * nt - c))) bwd32_cols(a, m, fo, bh, h, nt - c, lane, Tu);
    }
    if (mine & (1u << (2 * nt))) bwd32_tail_unit(a, m, bh, h, lane);
  }
  if (a.dtable_part && slot < B) {
    __syncthreads();
    for (int i = tid; i <= 2 * T; i += 64 * NW) a.dtable_part[((int64_t)slot * (2 * T + 1) + i) * a.H + h] = dbias[i];
  }
}

// ===========================================================================
// Long sequences (T' > 256, e.g. the C5 config's T' = 513): the head no longer
// fits LDS whole.  A workgroup owns 64 rows (one 16-row tile per wave) and
// streams the other side through LDS in windows of AW_W rows by LDS-DMA (K/V
// for the forward and the dQ pass, Q/dO for the dK/dV pass); the online softmax
// (forward) and the register accumulators (backward) carry across windows.
// Same per-element math, bias and causal mask as the whole-head kernels above.
// delta = rowsum(dO * O) comes from attn_delta_k; the dQ pass also produces the
// bias gradient, accumulated in LDS over AW_BG batch entries per workgroup and
// written as one partial per (batch group, row block): no atomics to HBM.
// ===========================================================================
constexpr int AW_W = 128;  // window rows
constexpr int AW_R = 64;   // rows owned by a workgroup
constexpr int AW_BG = 16;  // batch entries per dQ / bias-gradient workgroup

template <int E>
__device__ __forceinline__ void fwd_kblock(const unsigned char* Ki, const unsigned char* Vi, int k0, int kimg, int q0,
                                           const bf16x8v (&qf)[E / 32], f32x4 (&o)[E / 16], float (&m)[4],
                                           float (&l)[4], const float* bias, float rs, int T, bool causal, float* scr,
                                           int lane) {
  constexpr int NS = E / 32, NE = E / 16;
  const int col = lane & 15, rg = (lane >> 4) * 4;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    s0 = MFMA(qf[s], img_row_frag<E>(Ki, kimg, s, lane), s0);
    s1 = MFMA(qf[s], img_row_frag<E>(Ki, kimg + 16, s, lane), s1);
  }
  float bm[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = q0 + rg + j;
    const int ka = k0 + col, kb = k0 + 16 + col;
    const bool va = q < T && ka < T && (!causal || ka <= q);
    const bool vb = q < T && kb < T && (!causal || kb <= q);
    s0[j] = va ? s0[j] * rs + bias[q - ka + T] : -INFINITY;
    s1[j] = vb ? s1[j] * rs + bias[q - kb + T] : -INFINITY;
    bm[j] = row16_max(fmaxf(s0[j], s1[j]));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float mn = fmaxf(m[j], bm[j]);
    const float alpha = (mn == -INFINITY) ? 1.f : __expf(m[j] - mn);
    m[j] = mn;
    const float pa = (s0[j] == -INFINITY) ? 0.f : __expf(s0[j] - mn);
    const float pb = (s1[j] == -INFINITY) ? 0.f : __expf(s1[j] - mn);
    s0[j] = pa;
    s1[j] = pb;
    l[j] = l[j] * alpha + pa + pb;
#pragma unroll
    for (int e = 0; e < NE; ++e) o[e][j] *= alpha;
  }
  bf16x8v ph, pl;
  c_to_a_split(scr, s0, s1, lane, ph, pl);
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const bf16x8v vf = img_tr_frag<E>(Vi, kimg, e * 16, lane);
    o[e] = MFMA(ph, vf, o[e]);
    o[e] = MFMA(pl, vf, o[e]);
  }
}

template <int E>
__global__ __launch_bounds__(256) void attn_fwd_win_k(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NS = E / 32, NE = E / 16;
  const int T = a.T, Tk = (T + 31) & ~31;
  unsigned char* Ki = smem;
  unsigned char* Vi = Ki + AW_W * E * 2;
  float* bias = reinterpret_cast<float*>(Vi + AW_W * E * 2);  // [2T+1], region padded to 16 B
  float* scr_all = bias + ((2 * T + 4) & ~3);
  const int b = blockIdx.x / a.H, h = blockIdx.x - (blockIdx.x / a.H) * a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.y * AW_R, q0 = r0 + wave * 16;
  const bool valid = q0 < T;
  for (int i = tid; i <= 2 * T; i += 256) bias[i] = a.table ? a.table[(int64_t)i * a.H + h] : 0.f;
  float* scr = scr_all + wave * 16 * SCR_LD;
  const float rs = rsqrtf((float)E);
  const bf16_t* kg = a.k + b * a.k_bs + h * a.k_hs;
  const bf16_t* vg = a.v + b * a.v_bs + h * a.v_hs;
  bf16x8v qf[NS];
  glob_row_frags<E>(qf, a.q + b * a.q_bs + h * a.q_hs, a.q_ts, q0, T, lane);
  f32x4 o[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) o[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) { m[j] = -INFINITY; l[j] = 0.f; }
  const int kend_blk = a.causal ? min(Tk, (r0 + AW_R + 31) & ~31) : Tk;
  const int kend = a.causal ? min(Tk, (q0 + 16 + 31) & ~31) : Tk;
  for (int w0 = 0; w0 < kend_blk; w0 += AW_W) {
    const int wr = min(AW_W, kend_blk - w0);
    __syncthreads();  // the previous window is consumed (first pass: the bias fill is done)
    stage_img_dma<E>(Ki, kg + (int64_t)w0 * a.k_ts, a.k_ts, T - w0, wr, wave, lane);
    stage_img_dma<E>(Vi, vg + (int64_t)w0 * a.v_ts, a.v_ts, T - w0, wr, wave, lane);
    wait_vm<0>();
    __syncthreads();
    if (valid)
      for (int k0 = w0; k0 < min(w0 + wr, kend); k0 += 32)
        fwd_kblock<E>(Ki, Vi, k0, k0 - w0, q0, qf, o, m, l, bias, rs, T, a.causal != 0, scr, lane);
  }
  if (!valid) return;
  const int col = lane & 15, rg = (lane >> 4) * 4;
  bf16_t* og = a.o + b * a.o_bs + h * a.o_hs;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = q0 + rg + j;
    const float lt = row16_sum(l[j]);
    const float inv = 1.f / lt;
#pragma unroll
    for (int e = 0; e < NE; ++e) o[e][j] *= inv;
    if (q < T && col == 0) a.lse[((int64_t)b * a.H + h) * T + q] = m[j] + __logf(lt);
  }
#pragma unroll
  for (int e = 0; e < NE; e += 2) c_store_rows(scr, o[e], o[e + 1], 1.f, lane, og + e * 16, a.o_ts, q0, T);
}

// delta[b, h, q] = dO[q] . O[q] (f32 over the bf16 operands).  E / 8 lanes per row, one
// 16-B chunk each, rows in (b, q, h) order -- the order of the [B, T, H, E] head-interleaved
// O / dO -- so a wave reads contiguous 128-B rows (one row per thread read 16 B per
// instruction 1 KB apart: 3.8 TB/s at C5), then a shuffle tree over the row's lanes
template <int E>
__global__ __launch_bounds__(256) void attn_delta_k(AttnArgs a) {
  constexpr int LPR = E / 8;
  static_assert(LPR >= 1 && LPR <= 64 && (LPR & (LPR - 1)) == 0, "E / 8 lanes per row");
  const int64_t n = (int64_t)a.B * a.H * a.T;
  const int64_t total = n * LPR;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int c = threadIdx.x % LPR;
  // the loop bound is uniform over the block (256 is a multiple of LPR), so every lane of a
  // wave takes part in the shuffles
  for (int64_t t0 = (int64_t)blockIdx.x * blockDim.x; t0 < total; t0 += stride) {
    const int64_t r = (t0 + threadIdx.x) / LPR;
    const int h = (int)(r % a.H);
    const int64_t bq = r / a.H;
    const int q = (int)(bq % a.T);
    const int64_t b = bq / a.T;
    float d = 0.f;
    const int64_t rr = r < n ? (a.wmap ? (int64_t)a.wmap[b * a.T + q] : (int64_t)q) : -1;
    if (rr >= 0) {
      const int64_t bo = a.wmap ? 0 : b * a.o_bs;
      const bf16_t* dp = a.dout + bo + h * a.o_hs + rr * a.o_ts + c * 8;
      const bf16_t* op = a.o + bo + h * a.o_hs + rr * a.o_ts + c * 8;
      const u32x4 u = *reinterpret_cast<const u32x4*>(dp);
      const u32x4 v = *reinterpret_cast<const u32x4*>(op);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        d += __uint_as_float(u[k] << 16) * __uint_as_float(v[k] << 16) +
             __uint_as_float(u[k] & 0xffff0000u) * __uint_as_float(v[k] & 0xffff0000u);
    }
#pragma unroll
    for (int o = LPR / 2; o >= 1; o >>= 1) d += __shfl_xor(d, o, 64);
    if (r < n && c == 0) a.delta[(b * a.H + h) * a.T + q] = d;
  }
}

// dQ (+ bias gradient) of 64 query rows, K / V streamed in windows
template <int E>
__global__ __launch_bounds__(256, 2) void attn_bwd_rows_win_k(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NS = E / 32, NE = E / 16;
  const int T = a.T, Tk = (T + 31) & ~31;
  unsigned char* I0 = smem;                 // K window
  unsigned char* I1 = I0 + AW_W * E * 2;    // V window
  float* bias = reinterpret_cast<float*>(I1 + AW_W * E * 2);  // [2T+2]
  float* dbias = bias + 2 * T + 2;                            // [2T+2]
  float* scr_all = dbias + 2 * T + 2;
  const int h = blockIdx.x % a.H, bg = blockIdx.x / a.H, rc = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = rc * AW_R, q0 = r0 + wave * 16;
  const bool valid = q0 < T;
  for (int i = tid; i < 2 * T + 2; i += 256) bias[i] = (a.table && i <= 2 * T) ? a.table[(int64_t)i * a.H + h] : 0.f;
  for (int i = tid; i < 2 * T + 2; i += 256) dbias[i] = 0.f;
  float* scr = scr_all + wave * 16 * SCR_LD;
  const float rs = rsqrtf((float)E);
  const int col = lane & 15, rg = (lane >> 4) * 4;
  const int kend_blk = a.causal ? min(Tk, (r0 + AW_R + 31) & ~31) : Tk;
  const int kend = a.causal ? min(Tk, (q0 + 16 + 31) & ~31) : Tk;
  const int b1 = min(a.B, (bg + 1) * AW_BG);
  for (int b = bg * AW_BG; b < b1; ++b) {
    const bf16_t* kg = a.k + b * a.k_bs + h * a.k_hs;
    const bf16_t* vg = a.v + b * a.v_bs + h * a.v_hs;
    bf16x8v qf[NS], df[NS];
    glob_row_frags<E>(qf, a.q + b * a.q_bs + h * a.q_hs, a.q_ts, q0, T, lane);
    glob_row_frags<E>(df, a.dout + b * a.o_bs + h * a.o_hs, a.o_ts, q0, T, lane);
    float lq[4], dl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t qi = ((int64_t)b * a.H + h) * T + min(q0 + rg + j, T - 1);
      lq[j] = a.lse[qi];
      dl[j] = a.delta[qi];
    }
    f32x4 dq[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) dq[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int w0 = 0; w0 < kend_blk; w0 += AW_W) {
      const int wr = min(AW_W, kend_blk - w0);
      __syncthreads();
      stage_img_dma<E>(I0, kg + (int64_t)w0 * a.k_ts, a.k_ts, T - w0, wr, wave, lane);
      stage_img_dma<E>(I1, vg + (int64_t)w0 * a.v_ts, a.v_ts, T - w0, wr, wave, lane);
      wait_vm<0>();
      __syncthreads();
      if (!valid) continue;
      for (int k0 = w0; k0 < min(w0 + wr, kend); k0 += 32) {
        const int ki = k0 - w0;
        f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, p0 = s0, p1 = s0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          s0 = MFMA(qf[s], img_row_frag<E>(I0, ki, s, lane), s0);
          s1 = MFMA(qf[s], img_row_frag<E>(I0, ki + 16, s, lane), s1);
          p0 = MFMA(df[s], img_row_frag<E>(I1, ki, s, lane), p0);
          p1 = MFMA(df[s], img_row_frag<E>(I1, ki + 16, s, lane), p1);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = q0 + rg + j;
          const int ka = k0 + col, kb = k0 + 16 + col;
          const bool va = q < T && ka < T && (!a.causal || ka <= q);
          const bool vb = q < T && kb < T && (!a.causal || kb <= q);
          s0[j] = va ? __expf(s0[j] * rs + bias[q - ka + T] - lq[j]) * (p0[j] - dl[j]) : 0.f;
          s1[j] = vb ? __expf(s1[j] * rs + bias[q - kb + T] - lq[j]) * (p1[j] - dl[j]) : 0.f;
        }
        bf16x8v gh, gl;
        c_to_a_split(scr, s0, s1, lane, gh, gl);
        if (a.dtable_part) {  // diagonal sums of the 16 x 32 dS tile, one LDS atomic per lane
          const int dd = lane - 31;
          const int idx = q0 - k0 + T + dd;
          if (lane < 47 && idx >= 0 && idx <= 2 * T) {
            float sum = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int c = r - dd;
              if (c >= 0 && c < 32) sum += scr[r * SCR_LD + c];
            }
            atomicAdd(&dbias[idx], sum);
          }
          __builtin_amdgcn_wave_barrier();
          asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const bf16x8v kf = img_tr_frag<E>(I0, ki, e * 16, lane);
          dq[e] = MFMA(gh, kf, dq[e]);
          dq[e] = MFMA(gl, kf, dq[e]);
        }
      }
    }
    if (valid) {
      bf16_t* dqg = a.dq + b * a.q_bs + h * a.q_hs;
#pragma unroll
      for (int e = 0; e < NE; e += 2) c_store_rows(scr, dq[e], dq[e + 1], rs, lane, dqg + e * 16, a.q_ts, q0, T);
    }
  }
  __syncthreads();
  if (a.dtable_part)
    for (int i = tid; i <= 2 * T; i += 256)
      a.dtable_part[(((int64_t)bg * gridDim.y + rc) * (2 * T + 1) + i) * a.H + h] = dbias[i];
}

// dK and dV of 64 key rows, Q / dO (+ their lse, delta) streamed in windows
template <int E>
__global__ __launch_bounds__(256, 2) void attn_bwd_cols_win_k(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NS = E / 32, NE = E / 16;
  const int T = a.T, Tk = (T + 31) & ~31;
  unsigned char* I0 = smem;                 // Q window
  unsigned char* I1 = I0 + AW_W * E * 2;    // dO window
  float* bias = reinterpret_cast<float*>(I1 + AW_W * E * 2);  // [2T+2]
  float* wl = bias + 2 * T + 2;                               // [AW_W] lse of the window rows
  float* wd = wl + AW_W;                                      // [AW_W] delta of the window rows
  float* scr_all = wd + AW_W;
  const int b = blockIdx.x / a.H, h = blockIdx.x - (blockIdx.x / a.H) * a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c0 = blockIdx.y * AW_R, k0 = c0 + wave * 16;
  const bool valid = k0 < T;
  for (int i = tid; i < 2 * T + 2; i += 256) bias[i] = (a.table && i <= 2 * T) ? a.table[(int64_t)i * a.H + h] : 0.f;
  float* scr = scr_all + wave * 16 * SCR_LD;
  const float rs = rsqrtf((float)E);
  const int col = lane & 15, rg = (lane >> 4) * 4;
  const bf16_t* qg = a.q + b * a.q_bs + h * a.q_hs;
  const bf16_t* dog = a.dout + b * a.o_bs + h * a.o_hs;
  const float* lse_g = a.lse + ((int64_t)b * a.H + h) * T;
  const float* del_g = a.delta + ((int64_t)b * a.H + h) * T;
  bf16x8v kf[NS], vf[NS];
  glob_row_frags<E>(kf, a.k + b * a.k_bs + h * a.k_hs, a.k_ts, k0, T, lane);
  glob_row_frags<E>(vf, a.v + b * a.v_bs + h * a.v_hs, a.v_ts, k0, T, lane);
  f32x4 dk[NE], dv[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) { dk[e] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[e] = dk[e]; }
  const int qbeg_blk = a.causal ? (c0 & ~31) : 0;
  const int qbeg = a.causal ? (k0 & ~31) : 0;
  for (int w0 = qbeg_blk; w0 < Tk; w0 += AW_W) {
    const int wr = min(AW_W, Tk - w0);
    __syncthreads();
    stage_img_dma<E>(I0, qg + (int64_t)w0 * a.q_ts, a.q_ts, T - w0, wr, wave, lane);
    stage_img_dma<E>(I1, dog + (int64_t)w0 * a.o_ts, a.o_ts, T - w0, wr, wave, lane);
    for (int i = tid; i < wr; i += 256) {
      wl[i] = w0 + i < T ? lse_g[w0 + i] : 0.f;
      wd[i] = w0 + i < T ? del_g[w0 + i] : 0.f;
    }
    wait_vm<0>();
    __syncthreads();
    if (!valid) continue;
    for (int q0 = max(w0, qbeg); q0 < w0 + wr; q0 += 32) {
      const int qi = q0 - w0;
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, p0 = s0, p1 = s0;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        s0 = MFMA(kf[s], img_row_frag<E>(I0, qi, s, lane), s0);
        s1 = MFMA(kf[s], img_row_frag<E>(I0, qi + 16, s, lane), s1);
        p0 = MFMA(vf[s], img_row_frag<E>(I1, qi, s, lane), p0);
        p1 = MFMA(vf[s], img_row_frag<E>(I1, qi + 16, s, lane), p1);
      }
      const int qa = q0 + col, qb = q0 + 16 + col;
      const float la = wl[qi + col], lb = wl[qi + 16 + col], da_ = wd[qi + col], db_ = wd[qi + 16 + col];
      f32x4 g0, g1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + rg + j;
        const bool va = k < T && qa < T && (!a.causal || k <= qa);
        const bool vb = k < T && qb < T && (!a.causal || k <= qb);
        const float pa = va ? __expf(s0[j] * rs + bias[qa - k + T] - la) : 0.f;
        const float pb = vb ? __expf(s1[j] * rs + bias[qb - k + T] - lb) : 0.f;
        g0[j] = pa * (p0[j] - da_);
        g1[j] = pb * (p1[j] - db_);
        s0[j] = pa;
        s1[j] = pb;
      }
      bf16x8v ph, pl, gh, gl;
      c_to_a_split(scr, s0, s1, lane, ph, pl);
      c_to_a_split(scr, g0, g1, lane, gh, gl);
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const bf16x8v dof = img_tr_frag<E>(I1, qi, e * 16, lane);
        dv[e] = MFMA(ph, dof, dv[e]);
        dv[e] = MFMA(pl, dof, dv[e]);
        const bf16x8v qf = img_tr_frag<E>(I0, qi, e * 16, lane);
        dk[e] = MFMA(gh, qf, dk[e]);
        dk[e] = MFMA(gl, qf, dk[e]);
      }
    }
  }
  if (!valid) return;
  bf16_t* dkg = a.dk + b * a.k_bs + h * a.k_hs;
  bf16_t* dvg = a.dv + b * a.v_bs + h * a.v_hs;
#pragma unroll
  for (int e = 0; e < NE; e += 2) {
    c_store_rows(scr, dk[e], dk[e + 1], rs, lane, dkg + e * 16, a.k_ts, k0, T);
    c_store_rows(scr, dv[e], dv[e + 1], 1.f, lane, dvg + e * 16, a.v_ts, k0, T);
  }
}
#undef MFMA

static size_t fwd_win_lds(int T, int E) {
  return (size_t)2 * AW_W * E * 2 + (size_t)((2 * T + 4) & ~3) * 4 + (size_t)4 * 16 * SCR_LD * 4;
}
static size_t rows_win_lds(int T, int E) {
  return (size_t)2 * AW_W * E * 2 + (size_t)(2 * T + 2) * 8 + (size_t)4 * 16 * SCR_LD * 4;
}
static size_t cols_win_lds(int T, int E) {
  return (size_t)2 * AW_W * E * 2 + (size_t)(2 * T + 2) * 4 + (size_t)2 * AW_W * 4 + (size_t)4 * 16 * SCR_LD * 4;
}
// windowed path: T' beyond what one workgroup keeps in LDS whole
static bool attn_windowed(int T) { return T > 256; }
static int attn_row_blocks(int T) { return (T + AW_R - 1) / AW_R; }
static int64_t attn_win_parts(int B, int T) { return (int64_t)((B + AW_BG - 1) / AW_BG) * attn_row_blocks(T); }
// bias-gradient partials: the windowed kernels write one per (batch group, row block), the
// 32x32 long-T' kernels one per batch entry; whichever path runs zeroes the rest
static int64_t attn_parts(int B, int T) {
  return attn_windowed(T) ? std::max<int64_t>(attn_win_parts(B, T), B) : (int64_t)B;
}
static int attn_zero_parts(const AttnArgs& a, int64_t used, int64_t parts, hipStream_t s) {
  if (!a.dtable_part || parts <= used) return 0;
  const size_t row = (size_t)(2 * a.T + 1) * a.H;
  return hipMemsetAsync(a.dtable_part + used * row, 0, (size_t)(parts - used) * row * 4, s) == hipSuccess
             ? 0
             : (int)hipErrorInvalidValue;
}

template <int E>
static int attn_launch_win(const AttnArgs& a, int B, bool bwd, hipStream_t s) {
  const unsigned nrb = (unsigned)attn_row_blocks(a.T);
  if (!bwd) {
    const size_t sh = fwd_win_lds(a.T, E);
    if (sh > 160 * 1024) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((attn_fwd_win_k<E>), dim3(B * a.H, nrb), dim3(256), sh, s, a);
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  const size_t sr = rows_win_lds(a.T, E), sc = cols_win_lds(a.T, E);
  if (sr > 160 * 1024 || sc > 160 * 1024 || !a.delta) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL((attn_delta_k<E>), dim3(grid_for((int64_t)B * a.H * a.T * (E / 8), 256, 256 * 16)), dim3(256), 0, s, a);
  LTHM_CHECK_LAUNCH();
  const unsigned nbg = (unsigned)((B + AW_BG - 1) / AW_BG);
  hipLaunchKernelGGL((attn_bwd_rows_win_k<E>), dim3(nbg * a.H, nrb), dim3(256), sr, s, a);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL((attn_bwd_cols_win_k<E>), dim3(B * a.H, nrb), dim3(256), sc, s, a);
  LTHM_CHECK_LAUNCH();
  return attn_zero_parts(a, attn_win_parts(B, a.T), attn_parts(B, a.T), s);
}

static size_t fwd_mfma_lds(int T, int E) {
  const int Tk = (T + 31) & ~31;
  return (size_t)2 * Tk * E * 2 + (size_t)((2 * T + 4) & ~3) * 4 + (size_t)4 * 16 * SCR_LD * 4;
}
static size_t bwd_mfma_lds(int T, int E) {
  const int Tk = (T + 31) & ~31;
  return (size_t)2 * Tk * E * 2 + (size_t)(2 * T + 2) * 8 + (size_t)2 * Tk * 4 + (size_t)4 * 16 * SCR_LD * 4;
}

static int attn_cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

template <int E>
static int attn_launch_mfma(const AttnArgs& a, int B, bool bwd, hipStream_t s) {
  static const bool old_bwd = getenv("LTHM_ATTN_BWD_OLD") && atoi(getenv("LTHM_ATTN_BWD_OLD"));  // A/B switch
  // LTHM_ATTN_TAIL=0: the last query of T' = 32 n + 1 in tiles like the others (A/B switch)
  static const bool no_tail = getenv("LTHM_ATTN_TAIL") && getenv("LTHM_ATTN_TAIL")[0] == '0';
  // LTHM_ATTN_BWD_P=1: the persistent double-buffered kernel instead of one workgroup per (b, h).
  // Off by default: at one wave per SIMD its units' dependency chains are exposed (C2 1.23 ms
  // against 0.91; with the loads removed it still takes 1.23, the per-(b, h) kernel 0.60:
  // profiles/r05h_ladder.log)
  static const bool no_pers = !(getenv("LTHM_ATTN_BWD_P") && getenv("LTHM_ATTN_BWD_P")[0] == '1');
  if (E == 64 && bwd && !old_bwd) {
    AttnArgs t = a;
    t.tail = !no_tail && bwd32_tail_mode(a.T, a.causal);
    const int cus = attn_cu_count();
    int S = std::min(B, std::max(1, cus / a.H));  // workgroups per head
    if (!no_pers && bwd32p_lds(a.T, t.tail) <= 160 * 1024 && B >= 2 * S && S >= 1) {
      hipLaunchKernelGGL(attn_bwd32p_k<4>, dim3(S * a.H), dim3(256), bwd32p_lds(a.T, t.tail), s, t, B, S);
      LTHM_CHECK_LAUNCH();
      // partials past the S per head were never written
      return attn_zero_parts(a, S, attn_parts(B, a.T), s);
    }
    hipLaunchKernelGGL(attn_bwd32_k<BWD32_NW>, dim3(B * a.H), dim3(64 * BWD32_NW), bwd32_lds(a.T, t.tail), s, t);
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  const size_t sh = bwd ? bwd_mfma_lds(a.T, E) : fwd_mfma_lds(a.T, E);
  if (sh > 160 * 1024) return (int)hipErrorInvalidValue;
  // backward: one block per (b, h) for both passes (C2: 0.98 -> 0.93 ms against one block per pass)
  if (bwd) hipLaunchKernelGGL((attn_bwd_mfma_k<E, true>), dim3(B * a.H), dim3(256), sh, s, a);
  else hipLaunchKernelGGL((attn_fwd_mfma_k<E>), dim3(B * a.H), dim3(256), sh, s, a);
  LTHM_CHECK_LAUNCH();
  return 0;
}

static size_t fwd_lds(int T, int E) { return (size_t)2 * T * (E + ROWPAD) * 2 + (size_t)(2 * T + 2) * 4 + (size_t)4 * T * 4; }
static size_t bwd_lds(int T, int E) {
  return (size_t)4 * T * (E + ROWPAD) * 2 + (size_t)(2 * T + 2) * 8 + (size_t)2 * T * 4 + (size_t)8 * T * 4;
}

template <int E>
static int attn_launch(const AttnArgs& a, int B, bool bwd, hipStream_t s) {
  const int nk = (a.T + 63) / 64;
  const size_t sh = bwd ? bwd_lds(a.T, E) : fwd_lds(a.T, E);
  if (sh > 160 * 1024) return (int)hipErrorInvalidValue;
  dim3 grid(B * a.H);
#define LTHM_ATTN_CASE(NKV)                                                                  \
  if (nk == NKV) {                                                                          \
    if (bwd) hipLaunchKernelGGL((attn_bwd_k<E, NKV>), grid, dim3(256), sh, s, a);            \
    else hipLaunchKernelGGL((attn_fwd_k<E, NKV>), grid, dim3(256), sh, s, a);                \
    LTHM_CHECK_LAUNCH();                                                                     \
    return 0;                                                                                \
  }
  LTHM_ATTN_CASE(1)
  LTHM_ATTN_CASE(2)
  LTHM_ATTN_CASE(3)
  LTHM_ATTN_CASE(4)
#undef LTHM_ATTN_CASE
  return (int)hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------
// Backward for long T' (E = 64, 256 < T' <= 620): the four images no longer fit together, so
// two kernels of one 8-wave workgroup per (b, h) each hold two: the rows kernel K and V
// (rows units, dQ and the bias gradient, Q / dO fragments from global once per query tile),
// the columns kernel Q and dO (columns units, dK and dV, K / V fragments from global once
// per key tile); delta = dO . O comes from attn_delta_k.  Same units as attn_bwd32_k.
__host__ __device__ __forceinline__ int bwd32l_fbytes(int T) {
  return (2 * bias_ne(T) + 2 * ((T + 31) & ~31) + ((2 * T + 1 + 3) & ~3)) * 4;
}
static size_t bwd32l_lds(int T) {
  return (size_t)bwd32l_fbytes(T) + (size_t)(2 * bwd32_timg(T) + bwd32_slack(T)) * 128;
}

template <int NW, bool ROWS>
__global__ __launch_bounds__(64 * NW) void attn_bwd32l_k(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr float L2E = 1.4426950408889634f;
  const int T = a.T, Tk = (T + 31) & ~31, nt = Tk / 32, ne = bias_ne(T), Ti = bwd32_timg(T);
  float* bias = reinterpret_cast<float*>(smem);  // [2][ne]: descending (rows) or ascending (columns) copies
  float* lse_s = bias + 2 * ne;                  // [Tk]
  float* dlt_s = lse_s + Tk;                     // [Tk]
  float* dbias = dlt_s + Tk;                     // [2T + 1] (rows)
  unsigned char* I0 = smem + bwd32l_fbytes(T);   // rows: K, columns: Q
  unsigned char* I1 = I0 + Ti * 128;             // rows: V, columns: dO
  const int bh = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bh / a.H, h = bh - (bh / a.H) * a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool pk = a.rmap != nullptr;
  const int* rm = pk ? a.rmap + (int64_t)b * T : nullptr;
  const int* wm = pk ? a.wmap + (int64_t)b * T : nullptr;
  if (ROWS) {
    stage_img32(I0, a.k + (pk ? 0 : b * a.k_bs) + h * a.k_hs, a.k_ts, T, Ti, wave, lane, NW, rm);
    stage_img32(I1, a.v + (pk ? 0 : b * a.v_bs) + h * a.v_hs, a.v_ts, T, Ti, wave, lane, NW, rm);
  } else {
    stage_img32(I0, a.q + (pk ? 0 : b * a.q_bs) + h * a.q_hs, a.q_ts, T, Ti, wave, lane, NW, rm);
    stage_img32(I1, a.dout + (pk ? 0 : b * a.o_bs) + h * a.o_hs, a.o_ts, T, Ti, wave, lane, NW, wm);
  }
  const int tl0 = first_own_tile(a, b, T);  // query tiles before tl0: no own row, skipped
  for (int c = 0; c < 2; ++c)
    for (int y = tid; y < ne; y += 64 * NW) {
      const int x = ROWS ? ne - 1 - (y + c) - BPAD : y + c - BPAD;
      bias[c * ne + y] = (a.table && x >= 0 && x <= 2 * T) ? a.table[(int64_t)x * a.H + h] * L2E : 0.f;
    }
  const int64_t rb = ((int64_t)b * a.H + h) * T;
  for (int i = tid; i < Tk; i += 64 * NW) {
    lse_s[i] = i < T ? a.lse[rb + i] * L2E : 0.f;
    dlt_s[i] = i < T ? a.delta[rb + i] : 0.f;
  }
  if (ROWS)
    for (int i = tid; i <= 2 * T; i += 64 * NW) dbias[i] = 0.f;
  for (int i = tid; i < bwd32_slack(T) * 32; i += 64 * NW) reinterpret_cast<float*>(I1 + Ti * 128)[i] = 0.f;
  wait_vm<0>();
  __syncthreads();
  const Bwd32Smem m = ROWS ? Bwd32Smem{I0, nullptr, nullptr, I1, nullptr, bias, lse_s, dlt_s, dbias, ne, nullptr, nullptr}
                           : Bwd32Smem{nullptr, I0, I1, nullptr, bias, nullptr, lse_s, dlt_s, dbias, ne, nullptr, nullptr};
  const Frag32Off fo = frag32_off(lane);
  // tiles over the waves, longest first (rows: query tile t visits t + 1 key tiles; columns:
  // key tile t visits nt - t query tiles)
  uint32_t mk[2] = {0u, 0u};  // up to 64 tiles
  {
    int load[NW] = {};
    for (int c = nt; c >= 1; --c) {
      const int t = ROWS ? c - 1 : nt - c;
      if (ROWS && t < tl0) continue;
      const int cost = (ROWS ? (a.causal ? c : nt) : nt - max(a.causal ? t : 0, tl0)) + 1;
      int w = 0;
#pragma unroll
      for (int j = 1; j < NW; ++j)
        if (load[j] < load[w]) w = j;
      load[w] += cost;
      if (w == wave) mk[t >> 5] |= 1u << (t & 31);
    }
  }
  for (int c = nt; c >= 1; --c) {
    const int t = ROWS ? c - 1 : nt - c;
    if (!((mk[t >> 5] >> (t & 31)) & 1u)) continue;
    if (ROWS) bwd32_rows<true>(a, m, fo, b, h, t, lane, T);
    else bwd32_cols<true>(a, m, fo, b, h, t, lane, T, tl0);
  }
  if (ROWS && a.dtable_part) {
    __syncthreads();
    for (int i = tid; i <= 2 * T; i += 64 * NW) a.dtable_part[((int64_t)b * (2 * T + 1) + i) * a.H + h] = dbias[i];
  }
}

// ---------------------------------------------------------------------------
// Forward on 32x32x16 MFMA (E = 64, T' up to 620, no general mask): one workgroup per
// (b, h) with the K and V images resident in LDS (2 T' x 128 B: the windowed path is not
// needed while they fit), 32-row query tiles balanced over the waves, longest first.  Per
// tile pair: S^T = K . Q^T (the query is the lane; the two lane halves hold alternate key
// groups, so the running max and sum combine with one lane swap), online softmax in log2
// units with the bias as pre-shifted log2-scaled copies (as the backward), and
// O^T += V^T . P^T with P^T straight from the accumulator as bf16 hi + lo (the split keeps
// the output within 1e-3 of the bf16-rounded fp32 reference).  O leaves as the transposed
// accumulator (8-byte runs of each query's row), lse per query.
__host__ __device__ __forceinline__ int fwd32_slack(int T) {
  const int d = ((T + 31) & ~31) - bwd32_timg(T);
  return d > 0 ? d : 0;
}
static size_t fwd32_lds(int T) {
  return (size_t)2 * bias_ne(T) * 4 + (size_t)(2 * bwd32_timg(T) + fwd32_slack(T)) * 128;
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_fwd32_k(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
  const int T = a.T, Tk = (T + 31) & ~31, nt = Tk / 32, ne = bias_ne(T), Ti = bwd32_timg(T);
  float* brv = reinterpret_cast<float*>(smem);  // [2][ne] descending copies (rows units' layout)
  unsigned char* IK = smem + 2 * ne * 4;
  unsigned char* IV = IK + Ti * 128;
  const int bh = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bh / a.H, h = bh - (bh / a.H) * a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5, r32 = lane & 31;
  const bool pk = a.rmap != nullptr;
  const int* rm = pk ? a.rmap + (int64_t)b * T : nullptr;
  const int* wm = pk ? a.wmap + (int64_t)b * T : nullptr;
  const bf16_t* qg = a.q + (pk ? 0 : b * a.q_bs) + h * a.q_hs;
  const bf16_t* kg = a.k + (pk ? 0 : b * a.k_bs) + h * a.k_hs;
  const bf16_t* vg = a.v + (pk ? 0 : b * a.v_bs) + h * a.v_hs;
  stage_img32(IK, kg, a.k_ts, T, Ti, wave, lane, NW, rm);
  stage_img32(IV, vg, a.v_ts, T, Ti, wave, lane, NW, rm);
  const int tl0 = first_own_tile(a, b, T);  // query tiles before tl0: no own row, skipped
  for (int c = 0; c < 2; ++c)
    for (int y = tid; y < ne; y += 64 * NW) {
      const int xr = ne - 1 - (y + c) - BPAD;
      brv[c * ne + y] = (a.table && xr >= 0 && xr <= 2 * T) ? a.table[(int64_t)xr * a.H + h] * L2E : 0.f;
    }
  for (int i = tid; i < fwd32_slack(T) * 32; i += 64 * NW) reinterpret_cast<float*>(IV + Ti * 128)[i] = 0.f;
  wait_vm<0>();
  __syncthreads();
  const Frag32Off fo = frag32_off(lane);
  const float c2 = rsqrtf((float)E_BWD32) * L2E;
  const bool ragged = (T & 31) != 0;
  // query tiles over the waves, longest first (cost: key tiles visited + 1)
  uint32_t lo_mask = 0, hi_mask = 0;  // up to 64 tiles
  {
    int load[NW] = {};
    for (int t = nt - 1; t >= tl0; --t) {
      const int cost = (a.causal ? t + 1 : nt) + 1;
      int w = 0;
#pragma unroll
      for (int j = 1; j < NW; ++j)
        if (load[j] < load[w]) w = j;
      load[w] += cost;
      if (w == wave) {
        if (t < 32) lo_mask |= 1u << t;
        else hi_mask |= 1u << (t - 32);
      }
    }
  }
  bf16_t* og = a.o + (pk ? 0 : b * a.o_bs) + h * a.o_hs;
  float* lse_g = a.lse + ((int64_t)b * a.H + h) * T;
  for (int q = tid; q < 32 * tl0 && q < T; q += 64 * NW) lse_g[q] = 0.f;  // skipped rows: finite, unread
  for (int t = nt - 1; t >= 0; --t) {
    if (!((t < 32 ? lo_mask >> t : hi_mask >> (t - 32)) & 1u)) continue;
    const int i = t, q0 = 32 * i, q = q0 + r32;
    bf16x8v qf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (q < T) v = *reinterpret_cast<const u32x4*>(qg + (rm ? (int64_t)rm[q] : (int64_t)q) * a.q_ts + 16 * s + 8 * hh);
      qf[s] = __builtin_bit_cast(bf16x8v, v);
    }
    f32x16 o[2];
#pragma unroll
    for (int nd = 0; nd < 2; ++nd)
#pragma unroll
      for (int v = 0; v < 16; ++v) o[nd][v] = 0.f;
    float m = -INFINITY, l = 0.f;
    const int kmax = q < T ? (a.causal ? q + 1 : T) : 0;
    const int z0 = ne - 1 - (q - 4 * hh + T + BPAD);
    const float* bp = brv + (z0 & 1) * ne + (z0 & ~1);
    const int jend = a.causal ? i + 1 : nt;
    for (int j = 0; j < jend; ++j, bp += 32) {
      const int k0 = 32 * j;
      f32x16 st;
#pragma unroll
      for (int v = 0; v < 16; ++v) st[v] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) st = MFMA32(frag_at(IK + k0 * 128 + fo.row[s]), qf[s], st);
      // S^T[k][q] -> log2-scaled logits; the key k = k0 + 8 g + 4 hh + jj in register 4 g + jj
      const bool edge = (a.causal && j == i) || (ragged && (i == nt - 1 || j == nt - 1));
      float mt = -INFINITY;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float2 blo = *reinterpret_cast<const float2*>(bp + 8 * g);
        const float2 bhi = *reinterpret_cast<const float2*>(bp + 8 * g + 2);
        const float bv[4] = {blo.x, blo.y, bhi.x, bhi.y};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int v = 4 * g + jj;
          float tv = fmaf(st[v], c2, bv[jj]);
          if (edge && !(k0 + 8 * g + 4 * hh + jj < kmax)) tv = -INFINITY;
          st[v] = tv;
          mt = fmaxf(mt, tv);
        }
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);
      const float mu = mn == -INFINITY ? 0.f : mn;  // no live key yet: every p is 0
      const float sc = __builtin_amdgcn_exp2f(m - mu);  // m = -inf: 0
      l *= sc;
#pragma unroll
      for (int nd = 0; nd < 2; ++nd)
#pragma unroll
        for (int v = 0; v < 16; ++v) o[nd][v] *= sc;
      m = mn;
      f32x16 lo;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const float p = __builtin_amdgcn_exp2f(st[v] - mu);
        l += p;
        st[v] = p;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8v hf = acc_frag32(st, s2);
        const u32x4 hb = __builtin_bit_cast(u32x4, hf);
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // the remainder p - bf16(p), exact in f32
          lo[8 * s2 + 2 * e] = st[8 * s2 + 2 * e] - __uint_as_float(hb[e] << 16);
          lo[8 * s2 + 2 * e + 1] = st[8 * s2 + 2 * e + 1] - __uint_as_float(hb[e] & 0xffff0000u);
        }
        const bf16x8v lf = acc_frag32(lo, s2);
        const unsigned char* vt = IV + (k0 + 16 * s2) * 128;
#pragma unroll
        for (int nd = 0; nd < 2; ++nd) {
          const bf16x8v vf = tr_at(vt + fo.tr[nd][0], vt + fo.tr[nd][1]);
          o[nd] = MFMA32(vf, hf, o[nd]);
          o[nd] = MFMA32(vf, lf, o[nd]);
        }
      }
    }
    l += __shfl_xor(l, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
    for (int nd = 0; nd < 2; ++nd) store_accT32(o[nd], inv, og, a.o_ts, q0, nd, T, lane, wm);
    if (hh == 0 && q < T) lse_g[q] = l > 0.f ? (m + __log2f(l)) * LN2 : -INFINITY;
  }
}

// the 32x32x16 forward: E = 64, K and V images within LDS (T' <= 620), not switched off
static bool fwd32_ok(const AttnArgs& a) {
  static const bool off = getenv("LTHM_ATTN_FWD_OLD") && atoi(getenv("LTHM_ATTN_FWD_OLD"));  // A/B switch
  return !off && fwd32_lds(a.T) <= 160 * 1024 && a.T <= 2048;
}
static int attn_launch_fwd32(const AttnArgs& a, int B, hipStream_t s) {
  const size_t sh = fwd32_lds(a.T);
  // more than 80 KiB of images: one block per CU, so 8 waves (two per SIMD)
  if (sh > 80 * 1024) hipLaunchKernelGGL(attn_fwd32_k<8>, dim3(B * a.H), dim3(512), sh, s, a);
  else hipLaunchKernelGGL(attn_fwd32_k<4>, dim3(B * a.H), dim3(256), sh, s, a);
  LTHM_CHECK_LAUNCH();
  return 0;
}

// the long-T' 32x32x16 backward (E = 64): two images of T' rows within LDS
static bool bwd32l_ok(const AttnArgs& a) {
  static const bool off = getenv("LTHM_ATTN_BWD_OLD") && atoi(getenv("LTHM_ATTN_BWD_OLD"));  // A/B switch
  return !off && a.delta && bwd32l_lds(a.T) <= 160 * 1024 && a.T <= 2048;
}
static int attn_launch_bwd32l(const AttnArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL((attn_delta_k<64>), dim3(grid_for((int64_t)B * a.H * a.T * 8, 256, 256 * 16)), dim3(256), 0, s, a);
  LTHM_CHECK_LAUNCH();
  const size_t sh = bwd32l_lds(a.T);
  hipLaunchKernelGGL((attn_bwd32l_k<8, true>), dim3(B * a.H), dim3(512), sh, s, a);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL((attn_bwd32l_k<8, false>), dim3(B * a.H), dim3(512), sh, s, a);
  LTHM_CHECK_LAUNCH();
  return attn_zero_parts(a, B, attn_parts(B, a.T), s);
}

static int attn_dispatch(const AttnArgs& a, int B, int E, bool bwd, hipStream_t s) {
  if (a.rmap) {  // packed rows: the long-T' 32x32x16 kernels only
    if (a.mask || !attn_windowed(a.T) || E != 64 || !a.wmap) return (int)hipErrorInvalidValue;
    if (!bwd) return fwd32_ok(a) ? attn_launch_fwd32(a, B, s) : (int)hipErrorInvalidValue;
    if (!a.dk_chain || !a.dv_chain || a.chain <= 0) return (int)hipErrorInvalidValue;
    return bwd32l_ok(a) ? attn_launch_bwd32l(a, B, s) : (int)hipErrorInvalidValue;
  }
  if (a.mask) {  // general additive mask: the whole-head VALU kernels
    if (a.T > 256) return (int)hipErrorInvalidValue;
    switch (E) {
      case 16: return attn_launch<16>(a, B, bwd, s);
      case 32: return attn_launch<32>(a, B, bwd, s);
      case 64: return attn_launch<64>(a, B, bwd, s);
      case 128: return attn_launch<128>(a, B, bwd, s);
      default: return (int)hipErrorInvalidValue;
    }
  }
  if (attn_windowed(a.T)) {
    if (E == 64 && !bwd && fwd32_ok(a)) return attn_launch_fwd32(a, B, s);
    if (E == 64 && bwd && bwd32l_ok(a)) return attn_launch_bwd32l(a, B, s);
    switch (E) {
      case 32: return attn_launch_win<32>(a, B, bwd, s);
      case 64: return attn_launch_win<64>(a, B, bwd, s);
      case 128: return attn_launch_win<128>(a, B, bwd, s);
      default: return (int)hipErrorInvalidValue;
    }
  }
  switch (E) {
    case 16: return attn_launch<16>(a, B, bwd, s);
    case 32: return attn_launch_mfma<32>(a, B, bwd, s);
    case 64: if (!bwd && fwd32_ok(a)) return attn_launch_fwd32(a, B, s);
             return attn_launch_mfma<64>(a, B, bwd, s);
    case 128: return attn_launch_mfma<128>(a, B, bwd, s);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace lthm

using namespace lthm;

static void fill_common(AttnArgs& a, const lthm_attn_desc* d) {
  a.q = (const bf16_t*)d->q; a.k = (const bf16_t*)d->k; a.v = (const bf16_t*)d->v;
  a.q_ts = d->q_tok_stride; a.k_ts = d->k_tok_stride; a.v_ts = d->v_tok_stride;
  a.q_hs = d->q_head_stride; a.k_hs = d->k_head_stride; a.v_hs = d->v_head_stride;
  a.q_bs = d->q_batch_stride; a.k_bs = d->k_batch_stride; a.v_bs = d->v_batch_stride;
  a.o = (bf16_t*)d->out; a.o_ts = d->o_tok_stride; a.o_hs = d->o_head_stride; a.o_bs = d->o_batch_stride;
  a.table = d->table; a.lse = d->lse; a.T = d->T; a.H = d->H; a.causal = d->causal;
  a.dout = (const bf16_t*)d->dout; a.dq = (bf16_t*)d->dq; a.dk = (bf16_t*)d->dk; a.dv = (bf16_t*)d->dv;
  a.dtable_part = d->dtable_part;
  a.delta = d->delta;
  a.B = d->B;
  a.mask = d->mask;
  a.m_bs = d->mask_batch_stride;
  a.m_hs = d->mask_head_stride;
  a.m_rs = d->mask_row_stride;
  a.rmap = d->row_map; a.wmap = d->live_map;
  a.dk_chain = (bf16_t*)d->dk_chain; a.dv_chain = (bf16_t*)d->dv_chain;
  a.chain_ts = d->chain_ts; a.chain = d->chain_rows;
}

static int check_desc(const lthm_attn_desc* d) {
  if (!d || d->B < 0 || d->T <= 0 || d->T > 4096 || d->H <= 0) return 1;
  if (d->T > 256 && d->E == 16) return 1;  // the windowed path is MFMA-only (E = 32, 64, 128)
  if (d->table && d->table_rows < 2 * d->T + 1) return 1;
  if (d->mask && (d->T > 256 || d->mask_row_stride < d->T || d->mask_batch_stride < 0 || d->mask_head_stride < 0))
    return 1;
  if ((d->q_tok_stride % 8) || (d->k_tok_stride % 8) || (d->v_tok_stride % 8) || (d->o_tok_stride % 8)) return 1;
  // 16-B rows: LDS-DMA image staging and vector row stores
  if ((d->q_head_stride % 8) || (d->k_head_stride % 8) || (d->v_head_stride % 8) || (d->o_head_stride % 8)) return 1;
  if ((d->q_batch_stride % 8) || (d->k_batch_stride % 8) || (d->v_batch_stride % 8) || (d->o_batch_stride % 8)) return 1;
  const void* ptrs[8] = {d->q, d->k, d->v, d->out, d->dout, d->dq, d->dk, d->dv};
  for (const void* p : ptrs)
    if ((uintptr_t)p % 16) return 1;
  return 0;
}

extern "C" int64_t lthm_attn_bwd_parts(int32_t B, int32_t T) { return attn_parts(B, T); }

// the packed-row dispatch's own test (attn_dispatch, a.rmap set), exported so that the caller
// unpacks instead of failing where it does not hold
extern "C" int lthm_attn_packed_ok(int32_t T, int32_t E) {
  if (T <= 0 || T > 4096 || E != 64 || !attn_windowed(T)) return 0;
  AttnArgs a{};
  a.T = T;
  a.delta = reinterpret_cast<float*>(16);  // bwd32l_ok asks only whether a delta workspace is given
  return fwd32_ok(a) && bwd32l_ok(a) ? 1 : 0;
}

extern "C" int lthm_attn_fwd(const lthm_attn_desc* d, void* stream) {
  LTHM_REQUIRE(check_desc(d) == 0 && d->lse != nullptr && d->out != nullptr);
  if (d->B == 0) return 0;
  AttnArgs a{};
  fill_common(a, d);
  return attn_dispatch(a, d->B, d->E, false, (hipStream_t)stream);
}

extern "C" int lthm_attn_bwd(const lthm_attn_desc* d, void* stream) {
  LTHM_REQUIRE(check_desc(d) == 0 && d->dout && d->dq && d->dk && d->dv);
  LTHM_REQUIRE(d->k_head_stride != 0 || d->H == 1);  // shared-KV heads: caller expands (see kernels.py)
  if (d->B == 0) return 0;
  AttnArgs a{};
  fill_common(a, d);
  return attn_dispatch(a, d->B, d->E, true, (hipStream_t)stream);
}
