// Small streaming kernels shared by the path: dtype casts, column sums (bias /
// LayerNorm-affine / position-bias gradients), fills.
#include "common.hpp"

namespace lthm {

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void cast_k(const TI* __restrict__ in, TO* __restrict__ out, int64_t n) {
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float v[4];
    load_vec<TI, 4 * sizeof(TI)>(in + i * 4, v);
    store_vec<TO, 4>(out + i * 4, v);
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    Elem<TO>::st(out + i, Elem<TI>::ld(in + i));
}

// ---------------------------------------------------------------- dropout
// nn.Dropout(p) (commons/transformers/layers.py:253-256, 264, 283; query_tower.py:133):
// keep element i with probability 1 - p, scale kept values by 1 / (1 - p).  The keep
// decision is a counter-based hash of (seed, i), so the backward regenerates the
// forward's mask from the seed alone (no mask tensor is stored).
__device__ __forceinline__ bool dropout_keep(uint64_t seed, int64_t i, uint32_t thresh24) {
  uint64_t z = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 40) >= thresh24;  // u = (z >> 40) / 2^24 >= p
}

// y = [res1] + [res2] + x * keep / (1 - p)
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void dropout_k(const TI* __restrict__ x, TO* __restrict__ y, int64_t n,
                                                 uint32_t thresh24, float scale, uint64_t seed,
                                                 const float* __restrict__ res1, const float* __restrict__ res2) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = dropout_keep(seed, i, thresh24) ? Elem<TI>::ld(x + i) * scale : 0.f;
    if (res1) v += res1[i];
    if (res2) v += res2[i];
    Elem<TO>::st(y + i, v);
  }
}

// x [rows, groups * cols] in place: element (r, g, c) *= keep(g * rows + r) / (1 - p)
// (the reference's token dropout: attn_dropout(ones[B, 1, T, 1]) for q, k and v)
template <typename T>
__global__ __launch_bounds__(256) void dropout_rows_k(T* __restrict__ x, int64_t rows, int cols, int groups,
                                                      uint32_t thresh24, float scale, uint64_t seed) {
  const int64_t n = rows * groups * (int64_t)cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / ((int64_t)groups * cols);
    const int g = (int)((i / cols) % groups);
    const float f = dropout_keep(seed, (int64_t)g * rows + r, thresh24) ? scale : 0.f;
    Elem<T>::st(x + i, Elem<T>::ld(x + i) * f);
  }
}

__global__ __launch_bounds__(256) void dropout_mask_k(uint8_t* __restrict__ out, int64_t n, uint32_t thresh24,
                                                      uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = dropout_keep(seed, i, thresh24) ? 1 : 0;
}

static inline uint32_t dropout_thresh(float p) {
  const double t = (double)p * 16777216.0;
  return t >= 16777216.0 ? 16777216u : (uint32_t)t;
}

// ---------------------------------------------------------------- streaming logQ
// CascadedStreamingLogQCorrectionModule (commons/layers.py:189-237, train_step as fixed
// in SURVEY §3.5 #7-8) driven the way the LTHM loss drives it (wrapper.py:126-136): for
// each mini-batch k in order, first the train_step on its non-pad ids at batch index
// batch_idx0 + k (b[h] <- (1 - alpha) b[h] + alpha (idx - a[h]); a[h] <- idx, every
// duplicate of a mini-batch computing from the pre-update state, as the reference's
// index_put does), then the correction of all its ids:
// out = -beta * min_m (-log b_m[(id + off_m) mod N]).
//
// The chain through b and a runs per bucket, and a bucket's chain depends only on WHICH
// mini-batches touched it.  So, all in parallel:
//   logq_insert_k  every (non-pad token, module) inserts its key m * N + h into an
//                  open-addressing table and sets bit k of the entry's mini-batch mask;
//   logq_apply_k   every entry keeps the bucket's state from before the call and walks its
//                  mask bits in increasing k, applying the update -- the same fp32 operations
//                  in the same order as the reference's sequence of train_steps (no
//                  contraction: __fmul_rn / __fadd_rn), so b and a come out bit-identical;
//   logq_out_k     (with out) every token's value after ITS mini-batch: untouched buckets read
//                  the table, touched ones replay their chain up to k from the saved state.
// The table holds 2x the (token, module) pairs, so probing always ends.
constexpr uint32_t LQ_EMPTY = 0xFFFFFFFFu;

__device__ __forceinline__ int64_t logq_bucket(int64_t id, int64_t off, int64_t nb) {
  const int64_t h = (int64_t)((uint64_t)id + (uint64_t)off) % nb;  // int64 wrap, then torch remainder
  return h < 0 ? h + nb : h;
}

__device__ __forceinline__ uint32_t logq_slot0(uint32_t key, uint32_t cap_mask) {
  uint32_t x = key * 0x9E3779B1u;
  x ^= x >> 15;
  x *= 0x85EBCA77u;
  x ^= x >> 13;
  return x & cap_mask;
}

struct LogqArgs {
  const int64_t* ids;
  const uint8_t* mask;
  int64_t B, ids_stride, mask_stride;
  int T, mbs, n_mod, n_w;
  const int64_t* offs;
  int64_t nb;
  float* bt;
  float* at;
  float alpha, oma, beta;
  int64_t batch_idx0;
  uint32_t* keys;   // [cap]
  uint32_t* bits;   // [cap, n_w]
  float* b0;        // [cap]
  float* a0;        // [cap]
  uint32_t cap_mask;
  float* out;
};

__device__ __forceinline__ void logq_step(float& b, float& a, float idx, float alpha, float oma) {
  // (1 - alpha) * b[h] + (alpha * (batch_idx - a[h])).float(): three rounded fp32 ops and the add
  b = __fadd_rn(__fmul_rn(oma, b), __fmul_rn(alpha, __fsub_rn(idx, a)));
  a = idx;
}

// one thread per (token, module) pair: the modules' probe chains (returning CAS round trips)
// run side by side instead of one after another per token (round 6: 7 modules on C2)
__global__ __launch_bounds__(256) void logq_insert_k(LogqArgs p) {
  const int64_t n = p.B * p.T * p.n_mod;
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t tok = i / p.n_mod;
    const int m = (int)(i - tok * p.n_mod);
    const int64_t bb = tok / p.T, t = tok - bb * p.T;
    if (p.mask && p.mask[bb * p.mask_stride + t]) continue;
    const int64_t id = p.ids[bb * p.ids_stride + t];
    const int mb = (int)(bb / p.mbs);
    const uint32_t key = (uint32_t)((int64_t)m * p.nb + logq_bucket(id, p.offs[m], p.nb));
    uint32_t s = logq_slot0(key, p.cap_mask);
    while (true) {
      const uint32_t old = atomicCAS(p.keys + s, LQ_EMPTY, key);
      if (old == LQ_EMPTY || old == key) break;
      s = (s + 1) & p.cap_mask;
    }
    atomicOr(p.bits + (int64_t)s * p.n_w + (mb >> 5), 1u << (mb & 31));
  }
}

__global__ __launch_bounds__(256) void logq_apply_k(LogqArgs p) {
  const int64_t cap = (int64_t)p.cap_mask + 1;
  for (int64_t s = blockIdx.x * (int64_t)256 + threadIdx.x; s < cap; s += (int64_t)gridDim.x * 256) {
    const uint32_t key = p.keys[s];
    if (key == LQ_EMPTY) continue;
    float b = p.bt[key], a = p.at[key];
    if (p.out) {  // the pre-call state: only logq_out_k's replays read it
      p.b0[s] = b;
      p.a0[s] = a;
    }
    for (int w = 0; w < p.n_w; ++w) {
      uint32_t m = p.bits[s * p.n_w + w];
      while (m) {
        const int k = w * 32 + __builtin_ctz(m);
        m &= m - 1;
        logq_step(b, a, (float)(p.batch_idx0 + k), p.alpha, p.oma);
      }
    }
    p.bt[key] = b;
    p.at[key] = a;
  }
}

// update = 0: the plain forward (no table; cap_mask unused)
__global__ __launch_bounds__(256) void logq_out_k(LogqArgs p, int update) {
  const int64_t n = p.B * p.T;
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t bb = i / p.T, t = i % p.T;
    const int64_t id = p.ids[bb * p.ids_stride + t];
    const int mb = (int)(bb / p.mbs);
    float q = INFINITY;
    for (int m = 0; m < p.n_mod; ++m) {
      const uint32_t key = (uint32_t)((int64_t)m * p.nb + logq_bucket(id, p.offs[m], p.nb));
      float b = p.bt[key];
      if (update) {
        uint32_t s = logq_slot0(key, p.cap_mask);
        uint32_t k0;
        while ((k0 = p.keys[s]) != LQ_EMPTY && k0 != key) s = (s + 1) & p.cap_mask;
        if (k0 == key) {  // replay this bucket's chain up to (and including) mini-batch mb
          float a = p.a0[s];
          b = p.b0[s];
          for (int w = 0; w <= (mb >> 5); ++w) {
            uint32_t bits = p.bits[(int64_t)s * p.n_w + w];
            if (w == (mb >> 5)) bits &= (mb & 31) == 31 ? 0xFFFFFFFFu : ((2u << (mb & 31)) - 1u);
            while (bits) {
              const int k = w * 32 + __builtin_ctz(bits);
              bits &= bits - 1;
              logq_step(b, a, (float)(p.batch_idx0 + k), p.alpha, p.oma);
            }
          }
        }
      }
      q = fminf(q, -logf(b));
    }
    p.out[bb * p.T + t] = -p.beta * q;
  }
}

static inline int64_t logq_cap(int64_t B, int T, int n_mod) {
  const int64_t pairs = B * (int64_t)T * n_mod;
  int64_t cap = 1024;
  while (cap < 2 * pairs) cap <<= 1;
  return cap;
}

// Multi-tensor f32 -> bf16 cast (lthm_cast_multi_bf16): a block per 1024-element
// chunk of the concatenation; the tensor is found by a search of the chunk-prefix
// table, so every lane of a chunk works on one tensor.
constexpr int CM_MT = 48;
struct CastList {
  const float* in[CM_MT];
  bf16_t* out[CM_MT];
  int64_t n[CM_MT];
  int64_t chunk_off[CM_MT + 1];  // prefix of ceil(n / 1024)
  int nt;
};
__global__ __launch_bounds__(256) void cast_multi_k(CastList L) {
  const int64_t c = blockIdx.x;
  int lo = 0, hi = L.nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.chunk_off[mid] <= c) lo = mid;
    else hi = mid - 1;
  }
  const int64_t base = (c - L.chunk_off[lo]) * 1024 + threadIdx.x * 4;
  const int64_t n = L.n[lo];
  const float* __restrict__ in = L.in[lo];
  bf16_t* __restrict__ out = L.out[lo];
  if (base + 4 <= n && ((((uintptr_t)(in + base)) | ((uintptr_t)(out + base))) & 7) == 0) {
    float v[4];
    load_vec<float, 16>(in + base, v);
    store_vec<bf16_t, 4>(out + base, v);
  } else {
    for (int64_t i = base; i < base + 4 && i < n; ++i) out[i] = f2bf(in[i]);
  }
}

// out[c] (+)= sum_r in[r*ld + c]; grid (col tiles of 64, row chunks); one atomic per column per block
template <typename T>
__global__ __launch_bounds__(256) void colsum_k(const T* __restrict__ in, int64_t rows, int64_t cols, int64_t ld,
                                               float* __restrict__ out, int64_t rows_per_block) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float acc = 0.f;
  if (c < cols) {
    // eight rows' loads in flight ahead of the (in-order) adds: 0.029 -> 0.018 ms per C2 call
#pragma unroll 8
    for (int64_t r = r0 + wave; r < r1; r += 4) acc += Elem<T>::ld(in + r * ld + c);
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < cols) {
    const float s = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    if (gridDim.y == 1) out[c] += s;
    else atomicAdd(out + c, s);
  }
}

__global__ void fill_k(float* p, float v, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

}  // namespace lthm

using namespace lthm;

extern "C" int lthm_cast(const void* in, int32_t in_dtype, void* out, int32_t out_dtype, int64_t n, void* stream) {
  LTHM_REQUIRE(n >= 0);
  if (n == 0) return 0;
  LTHM_REQUIRE(((uintptr_t)in % 8) == 0 && ((uintptr_t)out % 8) == 0);
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(n / 4 + 1, 256, 256 * 8);
  if (in_dtype == LTHM_F32 && out_dtype == LTHM_BF16)
    hipLaunchKernelGGL((cast_k<float, bf16_t>), dim3(grid), dim3(256), 0, s, (const float*)in, (bf16_t*)out, n);
  else if (in_dtype == LTHM_BF16 && out_dtype == LTHM_F32)
    hipLaunchKernelGGL((cast_k<bf16_t, float>), dim3(grid), dim3(256), 0, s, (const bf16_t*)in, (float*)out, n);
  else if (in_dtype == LTHM_F32 && out_dtype == LTHM_F32)
    hipLaunchKernelGGL((cast_k<float, float>), dim3(grid), dim3(256), 0, s, (const float*)in, (float*)out, n);
  else if (in_dtype == LTHM_BF16 && out_dtype == LTHM_BF16)
    hipLaunchKernelGGL((cast_k<bf16_t, bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)in, (bf16_t*)out, n);
  else
    return (int)hipErrorInvalidValue;
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_dropout(const void* x, int32_t x_dtype, void* y, int32_t y_dtype, int64_t n, float p,
                            uint64_t seed, const float* res1, const float* res2, void* stream) {
  LTHM_REQUIRE(n >= 0 && p >= 0.f && p < 1.f);
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(n, 256, 256 * 16);
  const uint32_t th = dropout_thresh(p);
  const float sc = 1.f / (1.f - p);
  if (x_dtype == LTHM_F32 && y_dtype == LTHM_F32)
    hipLaunchKernelGGL((dropout_k<float, float>), dim3(grid), dim3(256), 0, s, (const float*)x, (float*)y, n, th, sc,
                       seed, res1, res2);
  else if (x_dtype == LTHM_F32 && y_dtype == LTHM_BF16)
    hipLaunchKernelGGL((dropout_k<float, bf16_t>), dim3(grid), dim3(256), 0, s, (const float*)x, (bf16_t*)y, n, th,
                       sc, seed, res1, res2);
  else if (x_dtype == LTHM_BF16 && y_dtype == LTHM_F32)
    hipLaunchKernelGGL((dropout_k<bf16_t, float>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (float*)y, n, th,
                       sc, seed, res1, res2);
  else if (x_dtype == LTHM_BF16 && y_dtype == LTHM_BF16)
    hipLaunchKernelGGL((dropout_k<bf16_t, bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, n,
                       th, sc, seed, res1, res2);
  else
    return (int)hipErrorInvalidValue;
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_dropout_rows(void* x, int32_t dtype, int64_t rows, int32_t cols, int32_t groups, float p,
                                 uint64_t seed, void* stream) {
  LTHM_REQUIRE(rows >= 0 && cols > 0 && groups > 0 && p >= 0.f && p < 1.f);
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(rows * groups * (int64_t)cols, 256, 256 * 16);
  const uint32_t th = dropout_thresh(p);
  const float sc = 1.f / (1.f - p);
  if (dtype == LTHM_F32)
    hipLaunchKernelGGL((dropout_rows_k<float>), dim3(grid), dim3(256), 0, s, (float*)x, rows, cols, groups, th, sc, seed);
  else if (dtype == LTHM_BF16)
    hipLaunchKernelGGL((dropout_rows_k<bf16_t>), dim3(grid), dim3(256), 0, s, (bf16_t*)x, rows, cols, groups, th, sc,
                       seed);
  else
    return (int)hipErrorInvalidValue;
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_dropout_mask(uint8_t* out, int64_t n, float p, uint64_t seed, void* stream) {
  LTHM_REQUIRE(n >= 0 && p >= 0.f && p < 1.f);
  if (n == 0) return 0;
  hipLaunchKernelGGL(dropout_mask_k, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, out, n,
                     dropout_thresh(p), seed);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t lthm_logq_ws_bytes(int64_t B, int32_t T, int32_t mb_size, int32_t n_modules) {
  if (B < 0 || T <= 0 || mb_size <= 0 || n_modules <= 0) return -1;
  const int64_t cap = logq_cap(B, T, n_modules);
  const int64_t n_w = ((B + mb_size - 1) / mb_size + 31) / 32;
  return cap * (4 + 4 * n_w + 8) + 256;
}

extern "C" int lthm_logq_stream(const int64_t* ids, int64_t ids_stride, const uint8_t* mask, int64_t mask_stride,
                                int64_t B, int32_t T, int32_t mb_size, float* b_tables, float* a_tables,
                                const int64_t* hash_offsets, int32_t n_modules, int64_t num_buckets, float alpha,
                                int64_t batch_idx0, float beta, int32_t update, float* out, void* workspace,
                                int64_t ws_bytes, void* stream) {
  LTHM_REQUIRE(B >= 0 && T > 0 && mb_size > 0 && n_modules > 0 && num_buckets > 0);
  LTHM_REQUIRE(ids_stride >= T && (!mask || mask_stride >= T));
  LTHM_REQUIRE((int64_t)n_modules * num_buckets < (int64_t)LQ_EMPTY);  // keys m * N + h fit 32 bits
  LTHM_REQUIRE(batch_idx0 >= 0 && batch_idx0 + (B + mb_size - 1) / mb_size <= (1ll << 24));  // exact in fp32
  LTHM_REQUIRE(!update || (workspace && ws_bytes >= lthm_logq_ws_bytes(B, T, mb_size, n_modules)));
  if (B == 0 || (!update && !out)) return 0;
  hipStream_t s = (hipStream_t)stream;
  LogqArgs p{};
  p.ids = ids; p.mask = mask; p.B = B; p.ids_stride = ids_stride; p.mask_stride = mask_stride;
  p.T = T; p.mbs = mb_size; p.n_mod = n_modules; p.offs = hash_offsets; p.nb = num_buckets;
  p.bt = b_tables; p.at = a_tables; p.alpha = alpha; p.oma = (float)(1.0 - (double)alpha); p.beta = beta;
  p.batch_idx0 = batch_idx0; p.out = out;
  const int64_t n = B * (int64_t)T;
  if (update) {
    const int64_t cap = logq_cap(B, T, n_modules);
    p.n_w = (int)(((B + mb_size - 1) / mb_size + 31) / 32);
    char* w = (char*)workspace;
    p.keys = (uint32_t*)w;
    p.bits = (uint32_t*)(w + cap * 4);
    p.b0 = (float*)(w + cap * (4 + 4 * (int64_t)p.n_w));
    p.a0 = p.b0 + cap;
    p.cap_mask = (uint32_t)(cap - 1);
    if (hipMemsetAsync(p.keys, 0xFF, cap * 4, s) != hipSuccess) return (int)hipGetLastError();
    if (hipMemsetAsync(p.bits, 0, cap * 4 * (int64_t)p.n_w, s) != hipSuccess) return (int)hipGetLastError();
    hipLaunchKernelGGL(logq_insert_k, dim3(grid_for(n * n_modules, 256, 256 * 64)), dim3(256), 0, s, p);
    LTHM_CHECK_LAUNCH();
    hipLaunchKernelGGL(logq_apply_k, dim3(grid_for(cap, 256, 256 * 32)), dim3(256), 0, s, p);
    LTHM_CHECK_LAUNCH();
  }
  if (out) {
    hipLaunchKernelGGL(logq_out_k, dim3(grid_for(n, 256, 256 * 32)), dim3(256), 0, s, p, update);
    LTHM_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int lthm_cast_multi_bf16(int32_t count, float** in, void** out, const int64_t* n, void* stream) {
  LTHM_REQUIRE(count >= 0 && (count == 0 || (in && out && n)));
  for (int t0 = 0; t0 < count; t0 += CM_MT) {
    CastList L;
    L.nt = 0;
    L.chunk_off[0] = 0;
    for (int t = t0; t < count && t < t0 + CM_MT; ++t) {
      LTHM_REQUIRE(n[t] >= 0 && (n[t] == 0 || (in[t] && out[t])));
      if (n[t] == 0) continue;
      L.in[L.nt] = in[t];
      L.out[L.nt] = static_cast<bf16_t*>(out[t]);
      L.n[L.nt] = n[t];
      L.chunk_off[L.nt + 1] = L.chunk_off[L.nt] + (n[t] + 1023) / 1024;
      ++L.nt;
    }
    if (L.nt == 0) continue;
    hipLaunchKernelGGL(cast_multi_k, dim3((unsigned)L.chunk_off[L.nt]), dim3(256), 0, (hipStream_t)stream, L);
    LTHM_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int lthm_colsum(const void* in, int32_t dtype, int64_t rows, int64_t cols, int64_t ld, float* out,
                           int32_t accumulate, void* stream) {
  LTHM_REQUIRE(rows >= 0 && cols >= 0 && ld >= cols);
  hipStream_t s = (hipStream_t)stream;
  if (!accumulate && cols > 0) {
    hipLaunchKernelGGL(fill_k, dim3(grid_for(cols, 256, 1024)), dim3(256), 0, s, out, 0.f, cols);
    LTHM_CHECK_LAUNCH();
  }
  if (rows == 0 || cols == 0) return 0;
  const int64_t ctiles = (cols + 63) / 64;
  int64_t ychunks = 2048 / ctiles;
  if (ychunks < 1) ychunks = 1;
  int64_t rpb = (rows + ychunks - 1) / ychunks;
  if (rpb < 64) rpb = 64;
  const int64_t ny = (rows + rpb - 1) / rpb;
  dim3 grid((unsigned)ctiles, (unsigned)ny);
  if (dtype == LTHM_F32)
    hipLaunchKernelGGL((colsum_k<float>), grid, dim3(256), 0, s, (const float*)in, rows, cols, ld, out, rpb);
  else
    hipLaunchKernelGGL((colsum_k<bf16_t>), grid, dim3(256), 0, s, (const bf16_t*)in, rows, cols, ld, out, rpb);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_fill_f32(float* p, float v, int64_t n, void* stream) {
  LTHM_REQUIRE(n >= 0);
  if (n == 0) return 0;
  hipLaunchKernelGGL(fill_k, dim3(grid_for(n, 256, 2048)), dim3(256), 0, (hipStream_t)stream, p, v, n);
  LTHM_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- trim + activations
namespace lthm {
// first column t (of T) where some row is not padded -> *out (atomicMin); *out pre-set to T by the host wrapper
// colany[t] = 1 iff column t of mask [B, T] holds a non-pad entry
__global__ void col_any_k(const uint8_t* __restrict__ mask, int64_t B, int T, int* __restrict__ colany) {
  const int64_t n = B * T;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (mask[i] == 0) colany[i % T] = 1;
}
// out[0] = first column with a non-pad entry (T if none), out[1] = number of all-pad columns
__global__ __launch_bounds__(256) void trim_stats_k(const int* __restrict__ colany, int T, int* __restrict__ out) {
  __shared__ int s_first, s_cnt;
  if (threadIdx.x == 0) { s_first = T; s_cnt = 0; }
  __syncthreads();
  int first = T, cnt = 0;
  for (int t = threadIdx.x; t < T; t += 256) {
    if (colany[t]) first = min(first, t);
    else cnt += 1;
  }
  atomicMin(&s_first, first);
  atomicAdd(&s_cnt, cnt);
  __syncthreads();
  if (threadIdx.x == 0) { out[0] = s_first; out[1] = s_cnt; }
}
__global__ void set_int_k(int* p, int v) { *p = v; }

__device__ __forceinline__ float act_f(int act, float x) {
  if (act == LTHM_ACT_GELU) {
    const float kb = 0.7978845608028654f, kk = 0.044715f;
    return 0.5f * x * (1.f + tanhf(kb * (x + kk * x * x * x)));
  }
  return x / (1.f + expf(-1.702f * x));
}
__device__ __forceinline__ float act_g(int act, float x) {
  if (act == LTHM_ACT_GELU) {
    const float kb = 0.7978845608028654f, kk = 0.044715f;
    const float x2 = x * x, t = tanhf(kb * (x + kk * x2 * x));
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * kb * (1.f + 3.f * kk * x2);
  }
  const float s = 1.f / (1.f + expf(-1.702f * x));
  return s + 1.702f * x * s * (1.f - s);
}
template <typename T>
__global__ __launch_bounds__(256) void act_k(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ y, int64_t n, int act) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float xv = Elem<T>::ld(x + i);
    Elem<T>::st(y + i, dy ? Elem<T>::ld(dy + i) * act_g(act, xv) : act_f(act, xv));
  }
}
}  // namespace lthm

extern "C" int lthm_trim_stats(const uint8_t* mask, int64_t B, int32_t T, int32_t* work, void* stream) {
  LTHM_REQUIRE(B >= 0 && T > 0 && work != nullptr);
  hipStream_t s = (hipStream_t)stream;
  int* colany = (int*)work + 2;
  LTHM_REQUIRE(hipMemsetAsync(colany, 0, (size_t)T * sizeof(int), s) == hipSuccess);
  if (B > 0) hipLaunchKernelGGL(col_any_k, dim3(grid_for(B * T, 256, 1024)), dim3(256), 0, s, mask, B, T, colany);
  hipLaunchKernelGGL(trim_stats_k, dim3(1), dim3(256), 0, s, (const int*)colany, (int)T, (int*)work);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_activation(const void* x, const void* dy, void* y, int32_t dtype, int64_t n, int32_t act, void* stream) {
  LTHM_REQUIRE(n >= 0 && (act == LTHM_ACT_GELU || act == LTHM_ACT_QGELU));
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(n, 256, 256 * 16);
  if (dtype == LTHM_F32) hipLaunchKernelGGL((act_k<float>), dim3(grid), dim3(256), 0, s, (const float*)x, (const float*)dy, (float*)y, n, act);
  else hipLaunchKernelGGL((act_k<bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)dy, (bf16_t*)y, n, act);
  LTHM_CHECK_LAUNCH();
  return 0;
}

namespace lthm {
__global__ void quantile_map_k(const float* __restrict__ x, int64_t B, int F, const float* __restrict__ q, int nq, int shared,
                               float* __restrict__ out) {
  const int64_t n = B * F;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(i % F);
    const float* qf = q + (shared ? 0 : (int64_t)f * nq);
    const float v = x[i];
    int b = 0;
    for (int k = 0; k < nq; ++k) b += (qf[k] < v) ? 1 : 0;  // torch.bucketize(right=False)
    out[i] = (float)b / (float)(nq + 1) - 0.5f;
  }
}
}  // namespace lthm

extern "C" int lthm_quantile_map(const float* x, int64_t B, int32_t F, const float* quantiles, int32_t nq, int32_t shared,
                                 float* out, void* stream) {
  LTHM_REQUIRE(B >= 0 && F > 0 && nq > 0);
  if (B == 0) return 0;
  hipLaunchKernelGGL(quantile_map_k, dim3(grid_for(B * F, 256, 2048)), dim3(256), 0, (hipStream_t)stream, x, B, F,
                     quantiles, nq, shared, out);
  LTHM_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- BCE with logits
namespace lthm {
__global__ __launch_bounds__(256) void bce_fwd_k(const float* __restrict__ z, const float* __restrict__ y, int64_t n,
                                                 float inv_n, float* __restrict__ loss_sum) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float zi = z[i];
    acc += fmaxf(zi, 0.f) - zi * y[i] + log1pf(expf(-fabsf(zi)));
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss_sum, ((red[0] + red[1]) + (red[2] + red[3])) * inv_n);
}
__global__ __launch_bounds__(256) void bce_bwd_k(const float* __restrict__ z, const float* __restrict__ y, int64_t n,
                                                 const float* __restrict__ gscale, float inv_n, float* __restrict__ dz) {
  const float g = (gscale ? *gscale : 1.f) * inv_n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dz[i] = (1.f / (1.f + expf(-z[i])) - y[i]) * g;
}
}  // namespace lthm

// ---------------------------------------------------------------- mean squared error
// nn.MSELoss (embedding_module_gen.py:139, the reconstruction model): mean((y - x)^2),
// backward dy = 2 (y - x) g / n.  y f32 or bf16 (KShift output), x f32.
namespace lthm {
template <typename TY>
__global__ __launch_bounds__(256) void mse_fwd_k(const TY* __restrict__ y, const float* __restrict__ x, int64_t n,
                                                 float inv_n, float* __restrict__ loss_sum) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float d = Elem<TY>::ld(y + i) - x[i];
    acc = fmaf(d, d, acc);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss_sum, ((red[0] + red[1]) + (red[2] + red[3])) * inv_n);
}
template <typename TY>
__global__ __launch_bounds__(256) void mse_bwd_k(const TY* __restrict__ y, const float* __restrict__ x, int64_t n,
                                                 const float* __restrict__ gscale, float inv_n, TY* __restrict__ dy) {
  const float g = (gscale ? *gscale : 1.f) * 2.f * inv_n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    Elem<TY>::st(dy + i, (Elem<TY>::ld(y + i) - x[i]) * g);
}
}  // namespace lthm

extern "C" int lthm_mse_fwd(const void* y, int32_t y_dtype, const float* x, int64_t n, float inv_n, float* loss_sum,
                            void* stream) {
  LTHM_REQUIRE(n >= 0 && loss_sum != nullptr && (y_dtype == LTHM_F32 || y_dtype == LTHM_BF16));
  if (n == 0) return 0;
  const dim3 g(grid_for(n, 256, 1024)), b(256);
  if (y_dtype == LTHM_F32)
    hipLaunchKernelGGL(mse_fwd_k<float>, g, b, 0, (hipStream_t)stream, (const float*)y, x, n, inv_n, loss_sum);
  else
    hipLaunchKernelGGL(mse_fwd_k<bf16_t>, g, b, 0, (hipStream_t)stream, (const bf16_t*)y, x, n, inv_n, loss_sum);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_mse_bwd(const void* y, int32_t y_dtype, const float* x, int64_t n, const float* gscale, float inv_n,
                            void* dy, void* stream) {
  LTHM_REQUIRE(n >= 0 && dy != nullptr && (y_dtype == LTHM_F32 || y_dtype == LTHM_BF16));
  if (n == 0) return 0;
  const dim3 g(grid_for(n, 256, 4096)), b(256);
  if (y_dtype == LTHM_F32)
    hipLaunchKernelGGL(mse_bwd_k<float>, g, b, 0, (hipStream_t)stream, (const float*)y, x, n, gscale, inv_n, (float*)dy);
  else
    hipLaunchKernelGGL(mse_bwd_k<bf16_t>, g, b, 0, (hipStream_t)stream, (const bf16_t*)y, x, n, gscale, inv_n,
                       (bf16_t*)dy);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_bce_logits_fwd(const float* z, const float* y, int64_t n, float inv_n, float* loss_sum,
                                   void* stream) {
  LTHM_REQUIRE(n >= 0 && loss_sum != nullptr);
  if (n == 0) return 0;
  hipLaunchKernelGGL(bce_fwd_k, dim3(grid_for(n, 256, 1024)), dim3(256), 0, (hipStream_t)stream, z, y, n, inv_n,
                     loss_sum);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_bce_logits_bwd(const float* z, const float* y, int64_t n, const float* gscale, float inv_n,
                                   float* dz, void* stream) {
  LTHM_REQUIRE(n >= 0 && dz != nullptr);
  if (n == 0) return 0;
  hipLaunchKernelGGL(bce_bwd_k, dim3(grid_for(n, 256, 2048)), dim3(256), 0, (hipStream_t)stream, z, y, n, gscale,
                     inv_n, dz);
  LTHM_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- fp8 quantisation
namespace lthm {
template <typename T>
__global__ __launch_bounds__(256) void amax_k(const T* __restrict__ x, int64_t n8, unsigned* __restrict__ amax) {
  __shared__ float red[4];
  float m = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    if constexpr (sizeof(T) == 2) {
      load_vec<T, 16>(x + i * 8, v);
    } else {
      load_vec<T, 16>(x + i * 8, v);
      load_vec<T, 16>(x + i * 8 + 4, v + 4);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(amax, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}
template <typename T>
__global__ __launch_bounds__(256) void quant_fp8_k(const T* __restrict__ x, int64_t n8, const unsigned* __restrict__ amax,
                                                   uint8_t* __restrict__ q, float* __restrict__ scale) {
  const float am = __uint_as_float(*amax);
  const float s = am > 0.f ? am / 448.f : 1.f;
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale = s;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    if constexpr (sizeof(T) == 2) {
      load_vec<T, 16>(x + i * 8, v);
    } else {
      load_vec<T, 16>(x + i * 8, v);
      load_vec<T, 16>(x + i * 8 + 4, v + 4);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fminf(fmaxf(v[e] / s, -448.f), 448.f);
    u32x2 w;
    w[0] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
    w[0] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], (int)w[0], true);
    w[1] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], 0, false);
    w[1] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], (int)w[1], true);
    *reinterpret_cast<u32x2*>(q + i * 8) = w;
  }
}
}  // namespace lthm

extern "C" int lthm_quantize_fp8(const void* x, int32_t dtype, int64_t n, uint8_t* q, float* scale, int32_t* work,
                                 void* stream) {
  LTHM_REQUIRE(n >= 0 && n % 8 == 0 && q && scale && work);
  LTHM_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)q % 8) == 0);
  LTHM_REQUIRE(dtype == LTHM_F32 || dtype == LTHM_BF16);
  hipStream_t s = (hipStream_t)stream;
  LTHM_REQUIRE(hipMemsetAsync(work, 0, 4, s) == hipSuccess);
  const int64_t n8 = n / 8;
  const int grid = grid_for(n8 > 0 ? n8 : 1, 256, 256 * 8);
  if (dtype == LTHM_BF16) {
    if (n8) hipLaunchKernelGGL((amax_k<bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, n8, (unsigned*)work);
    hipLaunchKernelGGL((quant_fp8_k<bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, n8, (const unsigned*)work,
                       q, scale);
  } else {
    if (n8) hipLaunchKernelGGL((amax_k<float>), dim3(grid), dim3(256), 0, s, (const float*)x, n8, (unsigned*)work);
    hipLaunchKernelGGL((quant_fp8_k<float>), dim3(grid), dim3(256), 0, s, (const float*)x, n8, (const unsigned*)work,
                       q, scale);
  }
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_amax(const void* x, int32_t dtype, int64_t n, int32_t* amax, void* stream) {
  LTHM_REQUIRE(n >= 0 && n % 8 == 0 && amax && ((uintptr_t)x % 16) == 0);
  LTHM_REQUIRE(dtype == LTHM_F32 || dtype == LTHM_BF16);
  const int64_t n8 = n / 8;
  if (n8 == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(n8, 256, 256 * 8);
  if (dtype == LTHM_BF16)
    hipLaunchKernelGGL((amax_k<bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, n8, (unsigned*)amax);
  else
    hipLaunchKernelGGL((amax_k<float>), dim3(grid), dim3(256), 0, s, (const float*)x, n8, (unsigned*)amax);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_quantize_fp8_amax(const void* x, int32_t dtype, int64_t n, const int32_t* amax, uint8_t* q,
                                      float* scale, void* stream) {
  LTHM_REQUIRE(n >= 0 && n % 8 == 0 && q && scale && amax);
  LTHM_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)q % 8) == 0);
  LTHM_REQUIRE(dtype == LTHM_F32 || dtype == LTHM_BF16);
  hipStream_t s = (hipStream_t)stream;
  const int64_t n8 = n / 8;
  const int grid = grid_for(n8 > 0 ? n8 : 1, 256, 256 * 8);
  if (dtype == LTHM_BF16)
    hipLaunchKernelGGL((quant_fp8_k<bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, n8,
                       (const unsigned*)amax, q, scale);
  else
    hipLaunchKernelGGL((quant_fp8_k<float>), dim3(grid), dim3(256), 0, s, (const float*)x, n8,
                       (const unsigned*)amax, q, scale);
  LTHM_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- MoELinear gates / expert scaling
namespace lthm {
__global__ __launch_bounds__(256) void moe_gate_fwd_k(const float* __restrict__ logits, int64_t M, int E, float scale,
                                                      int top_k, float* __restrict__ probs) {
  for (int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
    const float* lg = logits + m * E;
    float mx = -INFINITY;
    for (int e = 0; e < E; ++e) {
      const float ge = lg[e] * scale;
      bool keep = true;
      if (top_k > 0) {  // kept iff fewer than top_k entries are strictly larger (ties stay, as torch.where(g < thr))
        int greater = 0;
        for (int j = 0; j < E; ++j) greater += (lg[j] * scale > ge) ? 1 : 0;
        keep = greater < top_k;
      }
      if (keep) mx = fmaxf(mx, ge);
      probs[m * E + e] = keep ? ge : -INFINITY;
    }
    float sum = 0.f;
    for (int e = 0; e < E; ++e) {
      const float v = probs[m * E + e];
      const float p = v == -INFINITY ? 0.f : expf(v - mx);
      probs[m * E + e] = p;
      sum += p;
    }
    const float inv = 1.f / sum;
    for (int e = 0; e < E; ++e) probs[m * E + e] *= inv;
  }
}
__global__ __launch_bounds__(256) void moe_gate_bwd_k(const float* __restrict__ probs, const float* __restrict__ dp,
                                                      int64_t M, int E, float scale, float* __restrict__ dl) {
  for (int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
    float dot = 0.f;
    for (int e = 0; e < E; ++e) dot += probs[m * E + e] * dp[m * E + e];
    for (int e = 0; e < E; ++e) dl[m * E + e] = scale * probs[m * E + e] * (dp[m * E + e] - dot);
  }
}
__global__ __launch_bounds__(256) void moe_scale_k(const bf16_t* __restrict__ H, const float* __restrict__ probs,
                                                   int64_t M, int E, int P, bf16_t* __restrict__ GH) {
  const int64_t n = M * E * P;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / ((int64_t)E * P);
    const int e = (int)((i / P) % E);
    GH[i] = f2bf(probs[m * E + e] * bf2f(H[i]));
  }
}
__device__ __forceinline__ float moe_gelu_grad(float x) {
  const float kb = 0.7978845608028654f, kk = 0.044715f;
  const float x2 = x * x, t = tanhf(kb * (x + kk * x2 * x));
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * kb * (1.f + 3.f * kk * x2);
}
// one wave per (m, e): lanes stride the P hidden units, wave-reduced dg
__global__ __launch_bounds__(256) void moe_hidden_bwd_k(const float* __restrict__ dGH, const bf16_t* __restrict__ H,
                                                        const bf16_t* __restrict__ pre, const float* __restrict__ probs,
                                                        int64_t M, int E, int P, bf16_t* __restrict__ dpre,
                                                        float* __restrict__ dg) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t w = blockIdx.x * 4 + (threadIdx.x >> 6); w < M * E; w += nw) {
    const int64_t base = w * P;  // (m, e) row segment: m * E * P + e * P
    const float pr = probs[w];
    float acc = 0.f;
    for (int p = lane; p < P; p += 64) {
      const float d = dGH[base + p];
      acc += d * bf2f(H[base + p]);
      dpre[base + p] = f2bf(pr * d * moe_gelu_grad(bf2f(pre[base + p])));
    }
    acc = wave_sum(acc);
    if (lane == 0) dg[w] = acc;
  }
}
}  // namespace lthm

extern "C" int lthm_moe_gate_fwd(const float* logits, int64_t M, int32_t E, float scale, int32_t top_k, float* probs,
                                 void* stream) {
  LTHM_REQUIRE(M >= 0 && E > 0 && E <= 64 && top_k >= 0);
  if (M == 0) return 0;
  hipLaunchKernelGGL(moe_gate_fwd_k, dim3(grid_for(M, 256, 2048)), dim3(256), 0, (hipStream_t)stream, logits, M, E,
                     scale, top_k, probs);
  LTHM_CHECK_LAUNCH();
  return 0;
}
extern "C" int lthm_moe_gate_bwd(const float* probs, const float* dprobs, int64_t M, int32_t E, float scale,
                                 float* dlogits, void* stream) {
  LTHM_REQUIRE(M >= 0 && E > 0 && E <= 64);
  if (M == 0) return 0;
  hipLaunchKernelGGL(moe_gate_bwd_k, dim3(grid_for(M, 256, 2048)), dim3(256), 0, (hipStream_t)stream, probs, dprobs,
                     M, E, scale, dlogits);
  LTHM_CHECK_LAUNCH();
  return 0;
}
extern "C" int lthm_moe_scale(const void* H, const float* probs, int64_t M, int32_t E, int32_t P, void* GH,
                              void* stream) {
  LTHM_REQUIRE(M >= 0 && E > 0 && P > 0);
  if (M == 0) return 0;
  hipLaunchKernelGGL(moe_scale_k, dim3(grid_for(M * E * P, 256, 4096)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)H, probs, M, E, P, (bf16_t*)GH);
  LTHM_CHECK_LAUNCH();
  return 0;
}
extern "C" int lthm_moe_hidden_bwd(const float* dGH, const void* H, const void* pre, const float* probs, int64_t M,
                                   int32_t E, int32_t P, void* dpre, float* dg, void* stream) {
  LTHM_REQUIRE(M >= 0 && E > 0 && P > 0);
  if (M == 0) return 0;
  hipLaunchKernelGGL(moe_hidden_bwd_k, dim3(grid_for(M * E, 4, 4096)), dim3(256), 0, (hipStream_t)stream, dGH,
                     (const bf16_t*)H, (const bf16_t*)pre, probs, M, E, P, (bf16_t*)dpre, dg);
  LTHM_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- row gather / scatter
// Token compaction (the product tower runs on the non-pad tokens only): dst row i = src row
// idx[i] (gather) or dst row idx[i] = src row i (scatter), rows of row_bytes (a multiple of 16),
// 16-B lanes, a block of 256 threads walking rows.  idx[i] < 0 gathers a zero row.
namespace lthm {
// src and dst may be the same buffer when every idx[i] is i or -1 (zeroing rows in place: each
// thread reads its 16-B chunk before it writes the same chunk), so neither is __restrict__
__global__ __launch_bounds__(256) void rows_move_k(const unsigned char* src, int64_t sld,
                                                   const int32_t* __restrict__ idx, int64_t count,
                                                   unsigned char* dst, int64_t dld, int chunks,
                                                   int scatter) {
  const int64_t total = count * chunks;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / chunks;
    const int c = (int)(e - i * chunks);
    const int32_t j = idx[i];
    if (scatter) {
      if (j >= 0)
        *reinterpret_cast<u32x4*>(dst + j * dld + 16 * c) = *reinterpret_cast<const u32x4*>(src + i * sld + 16 * c);
    } else {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (j >= 0) v = *reinterpret_cast<const u32x4*>(src + j * sld + 16 * c);
      *reinterpret_cast<u32x4*>(dst + i * dld + 16 * c) = v;
    }
  }
}
}  // namespace lthm

extern "C" int lthm_rows_move(const void* src, int64_t src_ld_bytes, const int32_t* idx, int64_t count, void* dst,
                              int64_t dst_ld_bytes, int64_t row_bytes, int32_t scatter, void* stream) {
  LTHM_REQUIRE(count >= 0 && row_bytes > 0 && row_bytes % 16 == 0 && src_ld_bytes % 16 == 0 && dst_ld_bytes % 16 == 0);
  LTHM_REQUIRE(((uintptr_t)src | (uintptr_t)dst) % 16 == 0);
  if (count == 0) return 0;
  const int chunks = (int)(row_bytes / 16);
  hipLaunchKernelGGL(rows_move_k, dim3(grid_for(count * chunks, 256, 4096)), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned char*)src, src_ld_bytes, idx, count, (unsigned char*)dst, dst_ld_bytes, chunks,
                     scatter);
  LTHM_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- shared pad prefix
// Encoder over left-padded histories (query_tower.py:99-110 after encoder.py:52's flip): with
// causal attention, no dropout and a position-0 token that is the same for every sequence, a
// pad position p of sequence b attends to positions 0 .. p only, all pads, so its state at
// every layer depends on p alone.  The encoder then runs a "packed" token set: the chain
// (positions 0 .. P of the longest prefix, once) and each sequence's positions past its pads.
//   pad_prefix_stats_k  per sequence: npad (leading mask bytes set) and whether the mask is a
//                       prefix; batch totals into stats {ok, valid, max npad, argmax}
//   pad_prefix_maps_k   full row (b, p) -> packed row (pof; pof_x: -1 at the pad rows of every
//                       sequence but the chain's owner) and packed row -> full row (fop)
//   pad_prefix_sum_k    chain row p of a packed gradient = sum over the sequences with
//                       npad >= p of their row p (fixed order: per 32-sequence chunk, then
//                       the chunks in order), the valid rows copied from their full rows
namespace lthm {
__global__ __launch_bounds__(256) void pad_prefix_stats_k(const uint8_t* __restrict__ mask, int64_t mstride, int B,
                                                          int T, int* __restrict__ npad, int* __restrict__ stats) {
  for (int b = blockIdx.x * 256 + threadIdx.x; b < B; b += gridDim.x * 256) {
    const uint8_t* m = mask + (int64_t)b * mstride;
    int n = 0;
    while (n < T && m[n]) ++n;
    bool ok = true;
    for (int t = n; t < T; ++t) ok = ok && !m[t];
    npad[b] = n;
    if (!ok) atomicAnd(stats, 0);
    atomicAdd(stats + 1, T - n);
    atomicMax(stats + 2, n);
  }
}
__global__ void pad_prefix_init_k(int* __restrict__ stats, int B) {
  if (threadIdx.x == 0) {
    stats[0] = 1;
    stats[1] = 0;
    stats[2] = 0;
    stats[3] = B;
  }
}
__global__ __launch_bounds__(256) void pad_prefix_owner_k(const int* __restrict__ npad, int B, int* __restrict__ stats) {
  for (int b = blockIdx.x * 256 + threadIdx.x; b < B; b += gridDim.x * 256)
    if (npad[b] == stats[2]) atomicMin(stats + 3, b);
}
// Tp = T + 1 positions (0 = the shared first token); voff[b] = packed row of b's first valid position
__global__ __launch_bounds__(256) void pad_prefix_maps_k(const int* __restrict__ npad, const int64_t* __restrict__ voff,
                                                         int B, int Tp, int P, int owner, int32_t* __restrict__ pof,
                                                         int32_t* __restrict__ pof_x, int32_t* __restrict__ fop) {
  const int64_t n = (int64_t)B * Tp;
  for (int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x; f < n; f += (int64_t)gridDim.x * 256) {
    const int b = (int)(f / Tp), p = (int)(f - (int64_t)b * Tp);
    const int np = npad[b];
    if (p <= np) {  // position 0 and the pads: the chain row p
      pof[f] = p;
      pof_x[f] = b == owner ? p : -1;
      if (b == owner) fop[p] = (int32_t)f;
    } else {
      const int32_t r = (int32_t)(P + 1 + voff[b] + (p - np - 1));
      pof[f] = r;
      pof_x[f] = r;
      fop[r] = (int32_t)f;
    }
  }
}
template <typename T>
__device__ __forceinline__ void ld8f(const T* p, float* v) {
  if constexpr (sizeof(T) == 2) {
    const u32x4 u = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(u[k] << 16);
      v[2 * k + 1] = __uint_as_float(u[k] & 0xffff0000u);
    }
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p), c = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
  }
}
// pass 1: grid (chain rows, sequence chunks of 32); 8 columns per thread
template <typename T>
__global__ __launch_bounds__(256) void pad_prefix_part_k(const T* __restrict__ src, int64_t ld, int W,
                                                         const int* __restrict__ npad, int B, int Tp,
                                                         float* __restrict__ part, int P) {
  const int p = blockIdx.x, ch = blockIdx.y;
  const int b0 = ch * 32, b1 = min(b0 + 32, B);
  float* out = part + ((int64_t)ch * (P + 1) + p) * W;
  for (int c = threadIdx.x * 8; c < W; c += 256 * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int b = b0; b < b1; ++b) {
      if (npad[b] < p) continue;
      float v[8];
      ld8f<T>(src + ((int64_t)b * Tp + p) * ld + c, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k];
    }
    *reinterpret_cast<float4*>(out + c) = float4{acc[0], acc[1], acc[2], acc[3]};
    *reinterpret_cast<float4*>(out + c + 4) = float4{acc[4], acc[5], acc[6], acc[7]};
  }
}
// pass 2: chain row p = the chunks' partial sums in order
template <typename T>
__global__ __launch_bounds__(256) void pad_prefix_fold_k(const float* __restrict__ part, int nch, int W, int P,
                                                         T* __restrict__ dst, int64_t ld) {
  const int64_t n = (int64_t)(P + 1) * W;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    float s = 0.f;
    for (int k = 0; k < nch; ++k) s += part[(int64_t)k * n + e];
    const int64_t r = e / W, c = e - r * W;
    if constexpr (sizeof(T) == 2) dst[r * ld + c] = f2bf(s);
    else dst[r * ld + c] = s;
  }
}
}  // namespace lthm

extern "C" int lthm_pad_prefix_stats(const uint8_t* mask, int64_t mask_stride, int32_t B, int32_t T, int32_t* npad,
                                     int32_t* stats, void* stream) {
  LTHM_REQUIRE(B > 0 && T > 0 && mask_stride >= T && mask && npad && stats);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pad_prefix_init_k, dim3(1), dim3(64), 0, s, stats, B);
  LTHM_CHECK_LAUNCH();
  const int grid = (B + 255) / 256;
  hipLaunchKernelGGL(pad_prefix_stats_k, dim3(grid), dim3(256), 0, s, mask, mask_stride, B, T, npad, stats);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL(pad_prefix_owner_k, dim3(grid), dim3(256), 0, s, (const int*)npad, B, stats);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_pad_prefix_maps(const int32_t* npad, const int64_t* voff, int32_t B, int32_t Tp, int32_t P,
                                    int32_t owner, int32_t* pof, int32_t* pof_x, int32_t* fop, void* stream) {
  LTHM_REQUIRE(B > 0 && Tp > 1 && P >= 0 && P < Tp && owner >= 0 && owner < B && (int64_t)B * Tp < (1ll << 31));
  hipLaunchKernelGGL(pad_prefix_maps_k, dim3(grid_for((int64_t)B * Tp, 256, 4096)), dim3(256), 0, (hipStream_t)stream,
                     (const int*)npad, voff, B, Tp, P, owner, pof, pof_x, fop);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t lthm_pad_prefix_ws_bytes(int32_t B, int32_t P, int32_t W) {
  if (B <= 0 || P < 0 || W <= 0) return -1;
  return (int64_t)((B + 31) / 32) * (P + 1) * W * 4;
}

extern "C" int lthm_pad_prefix_sum(const void* src, int64_t src_ld, int32_t dtype, int32_t W, const int32_t* npad,
                                   int32_t B, int32_t Tp, int32_t P, void* dst, int64_t dst_ld, void* ws,
                                   int64_t ws_bytes, void* stream) {
  LTHM_REQUIRE(src && dst && npad && W > 0 && W % 8 == 0 && B > 0 && Tp > 0 && P >= 0 && P < Tp);
  LTHM_REQUIRE(src_ld >= W && dst_ld >= W && src_ld % 8 == 0 && dst_ld % 8 == 0);
  LTHM_REQUIRE(((uintptr_t)src % 16) == 0);
  LTHM_REQUIRE(ws && ws_bytes >= lthm_pad_prefix_ws_bytes(B, P, W));
  LTHM_REQUIRE(dtype == LTHM_BF16 || dtype == LTHM_F32);
  hipStream_t s = (hipStream_t)stream;
  const int nch = (B + 31) / 32;
  float* part = (float*)ws;
  const dim3 g1(P + 1, nch);
  const int g2 = grid_for((int64_t)(P + 1) * W, 256, 2048);
  if (dtype == LTHM_BF16) {
    hipLaunchKernelGGL(pad_prefix_part_k<bf16_t>, g1, dim3(256), 0, s, (const bf16_t*)src, src_ld, W, (const int*)npad,
                       B, Tp, part, P);
    LTHM_CHECK_LAUNCH();
    hipLaunchKernelGGL(pad_prefix_fold_k<bf16_t>, dim3(g2), dim3(256), 0, s, (const float*)part, nch, W, P, (bf16_t*)dst,
                       dst_ld);
  } else {
    hipLaunchKernelGGL(pad_prefix_part_k<float>, g1, dim3(256), 0, s, (const float*)src, src_ld, W, (const int*)npad,
                       B, Tp, part, P);
    LTHM_CHECK_LAUNCH();
    hipLaunchKernelGGL(pad_prefix_fold_k<float>, dim3(g2), dim3(256), 0, s, (const float*)part, nch, W, P, (float*)dst,
                       dst_ld);
  }
  LTHM_CHECK_LAUNCH();
  return 0;
}
