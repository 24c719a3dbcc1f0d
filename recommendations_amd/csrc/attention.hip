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
};

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

// delta[b, h, q] = dO[q] . O[q] (f32 over the bf16 operands), one thread per row
template <int E>
__global__ __launch_bounds__(256) void attn_delta_k(AttnArgs a) {
  const int64_t n = (int64_t)a.B * a.H * a.T;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(i % a.T);
    const int64_t bh = i / a.T;
    const int h = (int)(bh % a.H);
    const int64_t b = bh / a.H;
    const bf16_t* dp = a.dout + b * a.o_bs + h * a.o_hs + (int64_t)q * a.o_ts;
    const bf16_t* op = a.o + b * a.o_bs + h * a.o_hs + (int64_t)q * a.o_ts;
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < E / 8; ++c) {
      const u32x4 u = *reinterpret_cast<const u32x4*>(dp + c * 8);
      const u32x4 v = *reinterpret_cast<const u32x4*>(op + c * 8);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        d += __uint_as_float(u[k] << 16) * __uint_as_float(v[k] << 16) +
             __uint_as_float(u[k] & 0xffff0000u) * __uint_as_float(v[k] & 0xffff0000u);
    }
    a.delta[i] = d;
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
static int64_t attn_parts(int B, int T) {
  return attn_windowed(T) ? (int64_t)((B + AW_BG - 1) / AW_BG) * attn_row_blocks(T) : (int64_t)B;
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
  hipLaunchKernelGGL((attn_delta_k<E>), dim3(grid_for((int64_t)B * a.H * a.T, 256, 256 * 16)), dim3(256), 0, s, a);
  LTHM_CHECK_LAUNCH();
  const unsigned nbg = (unsigned)((B + AW_BG - 1) / AW_BG);
  hipLaunchKernelGGL((attn_bwd_rows_win_k<E>), dim3(nbg * a.H, nrb), dim3(256), sr, s, a);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL((attn_bwd_cols_win_k<E>), dim3(B * a.H, nrb), dim3(256), sc, s, a);
  LTHM_CHECK_LAUNCH();
  return 0;
}

static size_t fwd_mfma_lds(int T, int E) {
  const int Tk = (T + 31) & ~31;
  return (size_t)2 * Tk * E * 2 + (size_t)((2 * T + 4) & ~3) * 4 + (size_t)4 * 16 * SCR_LD * 4;
}
static size_t bwd_mfma_lds(int T, int E) {
  const int Tk = (T + 31) & ~31;
  return (size_t)2 * Tk * E * 2 + (size_t)(2 * T + 2) * 8 + (size_t)2 * Tk * 4 + (size_t)4 * 16 * SCR_LD * 4;
}

template <int E>
static int attn_launch_mfma(const AttnArgs& a, int B, bool bwd, hipStream_t s) {
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

static int attn_dispatch(const AttnArgs& a, int B, int E, bool bwd, hipStream_t s) {
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
    case 64: return attn_launch_mfma<64>(a, B, bwd, s);
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

extern "C" int lthm_attn_fwd(const lthm_attn_desc* d, void* stream) {
  LTHM_REQUIRE(check_desc(d) == 0 && d->lse != nullptr && d->out != nullptr);
  if (d->B == 0) return 0;
  AttnArgs a;
  fill_common(a, d);
  return attn_dispatch(a, d->B, d->E, false, (hipStream_t)stream);
}

extern "C" int lthm_attn_bwd(const lthm_attn_desc* d, void* stream) {
  LTHM_REQUIRE(check_desc(d) == 0 && d->dout && d->dq && d->dk && d->dv);
  LTHM_REQUIRE(d->k_head_stride != 0 || d->H == 1);  // shared-KV heads: caller expands (see kernels.py)
  if (d->B == 0) return 0;
  AttnArgs a;
  fill_common(a, d);
  return attn_dispatch(a, d->B, d->E, true, (hipStream_t)stream);
}
