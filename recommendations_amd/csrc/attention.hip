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
  float* dtable_part;        // [B, 2T+1, H]
};

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
          const float s = dot_row_reg<E>(Ks + k * RS, r1) / sq + bias[qi - k + T];
          const float p = __expf(s - lq);
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
          const float s = dot_row_reg<E>(Qs + qi * RS, r1) / sq + bias[qi - ki + T];
          p = __expf(s - lse[qi]);
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
  switch (E) {
    case 16: return attn_launch<16>(a, B, bwd, s);
    case 32: return attn_launch<32>(a, B, bwd, s);
    case 64: return attn_launch<64>(a, B, bwd, s);
    case 128: return attn_launch<128>(a, B, bwd, s);
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
}

static int check_desc(const lthm_attn_desc* d) {
  if (!d || d->B < 0 || d->T <= 0 || d->T > 256 || d->H <= 0) return 1;
  if (d->table && d->table_rows < 2 * d->T + 1) return 1;
  if ((d->q_tok_stride % 8) || (d->k_tok_stride % 8) || (d->v_tok_stride % 8) || (d->o_tok_stride % 8)) return 1;
  return 0;
}

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
