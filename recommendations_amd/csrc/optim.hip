// Optimizer and gradient-transform kernels for gfx950.
//
//  * dense AdamW (torch.optim.AdamW semantics; models/lthm/sequence/wrapper.py:263-275
//    builds AdamW over every parameter) — fused, in place, fp32 master + optional
//    bf16 shadow copy for the GEMM operands;
//  * dense Adagrad (embedding_module_gen.py:97,137: Adagrad lr 0.5);
//  * sparse row-wise AdamW / Adagrad over the rows a step actually touched
//    (list produced by the KShift backward): the documented deviation for
//    100M-row tables (SURVEY.md §7 "Dense optimizer on giant tables");
//  * squared-norm reductions for cap_gradients (commons/functional.py:23) and
//    gradient clipping (accelerate_training_strategy.py:357-362).
#include "common.hpp"

namespace lthm {

__global__ __launch_bounds__(256) void adamw_k(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                               float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                                               float wd, float bc1, float bc2_sqrt, float gscale, bf16_t* __restrict__ shadow,
                                               int zero_grad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * gscale;
    float pi = p[i];
    pi = pi * (1.f - lr * wd);
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    // torch: denom = sqrt(v) / sqrt(bc2) + eps ; p -= lr / bc1 * m / denom
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - (lr / bc1) * mi / denom;
    p[i] = pi;
    if (shadow) shadow[i] = f2bf(pi);
    if (zero_grad) g[i] = 0.f;
  }
}

// Multi-tensor AdamW: up to AW_MT tensors per launch (kernel-argument pointer
// table), element i of the concatenation found by a binary search of the
// prefix offsets.  Same update as adamw_k; one launch instead of one per tensor.
constexpr int AW_MT = 48;
struct AdamWList {
  float* p[AW_MT];
  float* g[AW_MT];
  float* m[AW_MT];
  float* v[AW_MT];
  int64_t off[AW_MT + 1];
  int nt;
};
__global__ __launch_bounds__(256) void adamw_multi_k(AdamWList L, float lr, float b1, float b2, float eps, float wd,
                                                     float bc1, float bc2_sqrt, float gscale) {
  const int64_t total = L.off[L.nt];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = L.nt - 1;
    while (lo < hi) {  // largest t with off[t] <= i
      const int mid = (lo + hi + 1) >> 1;
      if (L.off[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    const int64_t j = i - L.off[lo];
    float* __restrict__ p = L.p[lo];
    float* __restrict__ m = L.m[lo];
    float* __restrict__ v = L.v[lo];
    const float gi = L.g[lo][j] * gscale;
    float pi = p[j] * (1.f - lr * wd);
    const float mi = b1 * m[j] + (1.f - b1) * gi;
    const float vi = b2 * v[j] + (1.f - b2) * gi * gi;
    m[j] = mi;
    v[j] = vi;
    const float pn = pi - (lr / bc1) * mi / (sqrtf(vi) / bc2_sqrt + eps);
    p[j] = pn;
  }
}

__global__ __launch_bounds__(256) void adagrad_k(float* __restrict__ p, float* __restrict__ g, float* __restrict__ s,
                                                 int64_t n, float clr, float eps, float wd, int zero_grad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i];
    if (wd != 0.f) gi += wd * p[i];
    const float si = s[i] + gi * gi;
    s[i] = si;
    p[i] = p[i] - clr * gi / (sqrtf(si) + eps);
    if (zero_grad) g[i] = 0.f;
  }
}

// per-element row-wise updates, shared by the per-element and the 16-byte kernels so both
// round identically
__device__ __forceinline__ float adamw_elem(float p, float g, float& m, float& v, float lr, float b1, float b2,
                                           float eps, float wd, float bc1, float bc2_sqrt) {
  p = p * (1.f - lr * wd);
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  return p - (lr / bc1) * m / (sqrtf(v) / bc2_sqrt + eps);
}
__device__ __forceinline__ float adagrad_elem(float p, float g, float& s, float clr, float eps) {
  s = s + g * g;
  return p - clr * g / (sqrtf(s) + eps);
}

// rows[0 .. *count) touched rows of a [R, D] table; the gradient row is consumed and re-zeroed,
// the row's touched flag reset.  One wave per row.
__global__ __launch_bounds__(256) void sparse_adamw_k(const int64_t* __restrict__ rows, const int64_t* __restrict__ count,
                                                      int64_t max_rows, int D, float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                      float* __restrict__ v, int32_t* __restrict__ flags, float lr, float b1,
                                                      float b2, float eps, float wd, float bc1, float bc2_sqrt,
                                                      bf16_t* __restrict__ shadow, int zero_grad) {
  const int64_t cnt = min(*count, max_rows);  // never past the row-list capacity
  // D <= 64 dividing 64: 64 / D rows per wave (all lanes busy); else one row per wave
  const int lane = threadIdx.x & 63;
  const int rpw = (D <= 64 && 64 % D == 0) ? 64 / D : 1;
  const int sub = rpw > 1 ? lane / D : 0, d0 = rpw > 1 ? lane - sub * D : lane;
  for (int64_t k = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * rpw + sub; k < cnt;
       k += (int64_t)gridDim.x * 4 * rpw) {
    const int64_t r = rows[k];
    for (int d = d0; d < D; d += 64) {
      const int64_t i = r * D + d;
      float mi = m[i], vi = v[i];
      const float pi = adamw_elem(p[i], g[i], mi, vi, lr, b1, b2, eps, wd, bc1, bc2_sqrt);
      m[i] = mi;
      v[i] = vi;
      p[i] = pi;
      if (shadow) shadow[i] = f2bf(pi);
      if (zero_grad) g[i] = 0.f;
    }
    if (flags && d0 == 0) flags[r] = 0;
  }
}

// 16-byte form of sparse_adamw_k / sparse_adagrad_k for D % 4 == 0 with D / 4 dividing 64:
// D / 4 lanes per row, 256 / D rows per wave (C4's D = 32: 8 rows, each array's row one
// 128-B access by 8 lanes), the next row index loaded before the current row's update,
// so a wave keeps several rows of every array in flight (the row-per-wave form is
// latency-bound: one row's loads at a time behind the index load).  Same per-element
// arithmetic, bit-identical results.
__device__ __forceinline__ void ld4f(const float* p, float (&v)[4]) {
  const float4 t = *reinterpret_cast<const float4*>(p);
  v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}
__device__ __forceinline__ void st4f(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ void st4bf(bf16_t* p, const float (&v)[4]) {
  u32x2 w;
  w[0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  w[1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *reinterpret_cast<u32x2*>(p) = w;
}

// ZG: re-zero each consumed gradient row (off when the next backward overwrites a row's first
// touch: the K = 1 first-touch tables, lthm_sparse_*_ex keep_grad)
template <bool ADAM, bool ZG>
__global__ __launch_bounds__(256) void sparse_opt_v4_k(const int64_t* __restrict__ rows, const int64_t* __restrict__ count,
                                                       int64_t max_rows, int D, float* __restrict__ p,
                                                       float* __restrict__ g, float* __restrict__ m,
                                                       float* __restrict__ v, int32_t* __restrict__ flags, float lr,
                                                       float b1, float b2, float eps, float wd, float bc1,
                                                       float bc2_sqrt, bf16_t* __restrict__ shadow) {
  const int64_t cnt = min(*count, max_rows);
  const int lane = threadIdx.x & 63;
  const int L = D >> 2, rpw = 64 / L;
  const int sub = lane / L, d0 = (lane - sub * L) * 4;
  const int64_t stride = (int64_t)gridDim.x * 4 * rpw;
  int64_t k = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * rpw + sub;
  int64_t r = k < cnt ? rows[k] : 0;
  for (; k < cnt; k += stride) {
    const int64_t kn = k + stride;
    const int64_t rn = kn < cnt ? rows[kn] : 0;  // the next row index in flight
    const int64_t i = r * D + d0;
    float gi[4], pi[4], mi[4];
    ld4f(g + i, gi);
    ld4f(p + i, pi);
    ld4f(m + i, mi);  // ADAM: first moment; Adagrad: the state sum
    if constexpr (ADAM) {
      float vi[4];
      ld4f(v + i, vi);
#pragma unroll
      for (int e = 0; e < 4; ++e) pi[e] = adamw_elem(pi[e], gi[e], mi[e], vi[e], lr, b1, b2, eps, wd, bc1, bc2_sqrt);
      st4f(v + i, vi);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) pi[e] = adagrad_elem(pi[e], gi[e], mi[e], lr, eps);
    }
    st4f(m + i, mi);
    st4f(p + i, pi);
    if (shadow) st4bf(shadow + i, pi);
    if constexpr (ZG) {
      const float z[4] = {0.f, 0.f, 0.f, 0.f};
      st4f(g + i, z);
    }
    if (flags && d0 == 0) flags[r] = 0;
    r = rn;
  }
}

static bool sparse_v4_ok(int D, const void* a, const void* b, const void* c, const void* d, const void* sh) {
  if (D % 4 != 0 || D > 256 || 64 % (D / 4) != 0) return false;
  for (const void* q : {a, b, c, d})
    if (q && ((uintptr_t)q % 16) != 0) return false;
  return !sh || ((uintptr_t)sh % 8) == 0;
}

__global__ __launch_bounds__(256) void sparse_adagrad_k(const int64_t* __restrict__ rows, const int64_t* __restrict__ count,
                                                        int64_t max_rows, int D, float* __restrict__ p, float* __restrict__ g, float* __restrict__ s,
                                                        int32_t* __restrict__ flags, float clr, float eps,
                                                        bf16_t* __restrict__ shadow, int zero_grad) {
  const int64_t cnt = min(*count, max_rows);  // never past the row-list capacity
  const int lane = threadIdx.x & 63;
  const int rpw = (D <= 64 && 64 % D == 0) ? 64 / D : 1;
  const int sub = rpw > 1 ? lane / D : 0, d0 = rpw > 1 ? lane - sub * D : lane;
  for (int64_t k = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * rpw + sub; k < cnt;
       k += (int64_t)gridDim.x * 4 * rpw) {
    const int64_t r = rows[k];
    for (int d = d0; d < D; d += 64) {
      const int64_t i = r * D + d;
      float si = s[i];
      const float pi = adagrad_elem(p[i], g[i], si, clr, eps);
      s[i] = si;
      p[i] = pi;
      if (shadow) shadow[i] = f2bf(pi);
      if (zero_grad) g[i] = 0.f;
    }
    if (flags && d0 == 0) flags[r] = 0;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void sumsq_k(const T* __restrict__ x, int64_t n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = Elem<T>::ld(x + i);
    s += v * v;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, red[0] + red[1] + red[2] + red[3]);
}

// y = x * (1 / (sqrt(ss) + add_eps))  or, for clipping, x * min(1, max_norm / (sqrt(ss) + 1e-6))
template <typename T>
__global__ __launch_bounds__(256) void scale_by_norm_k(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                       const float* __restrict__ ss, float add_eps, float max_norm) {
  const float nrm = sqrtf(*ss);
  float sc;
  if (max_norm > 0.f) sc = fminf(1.f, max_norm / (nrm + 1e-6f));
  else sc = 1.f / (nrm + add_eps);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (max_norm > 0.f) Elem<T>::st(y + i, Elem<T>::ld(x + i) * sc);
    else Elem<T>::st(y + i, Elem<T>::ld(x + i) / (nrm + add_eps));
  }
}

}  // namespace lthm

using namespace lthm;

extern "C" int lthm_adamw(float* p, float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                          float eps, float weight_decay, int64_t step, float grad_scale, void* bf16_shadow,
                          int32_t zero_grad, void* stream) {
  LTHM_REQUIRE(n >= 0 && step >= 1);
  if (n == 0) return 0;
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2 = 1.f - powf(beta2, (float)step);
  hipLaunchKernelGGL(adamw_k, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, beta1,
                     beta2, eps, weight_decay, bc1, sqrtf(bc2), grad_scale, (bf16_t*)bf16_shadow, zero_grad);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_adamw_multi(int32_t count, float** p, float** g, float** m, float** v,
                                const int64_t* n, float lr, float beta1, float beta2, float eps, float weight_decay,
                                int64_t step, float grad_scale, void* stream) {
  LTHM_REQUIRE(count >= 0 && step >= 1 && (count == 0 || (p && g && m && v && n)));
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2 = 1.f - powf(beta2, (float)step);
  for (int t0 = 0; t0 < count; t0 += AW_MT) {
    AdamWList L;
    L.nt = 0;
    L.off[0] = 0;
    for (int t = t0; t < count && t < t0 + AW_MT; ++t) {
      LTHM_REQUIRE(n[t] >= 0 && (n[t] == 0 || (p[t] && g[t] && m[t] && v[t])));
      if (n[t] == 0) continue;
      L.p[L.nt] = p[t]; L.g[L.nt] = g[t]; L.m[L.nt] = m[t]; L.v[L.nt] = v[t];
      L.off[L.nt + 1] = L.off[L.nt] + n[t];
      ++L.nt;
    }
    if (L.nt == 0) continue;
    hipLaunchKernelGGL(adamw_multi_k, dim3(grid_for(L.off[L.nt], 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream,
                       L, lr, beta1, beta2, eps, weight_decay, bc1, sqrtf(bc2), grad_scale);
    LTHM_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int lthm_adagrad(float* p, float* g, float* state_sum, int64_t n, float lr, float lr_decay, float eps,
                            float weight_decay, int64_t step, int32_t zero_grad, void* stream) {
  LTHM_REQUIRE(n >= 0 && step >= 1);
  if (n == 0) return 0;
  const float clr = lr / (1.f + (float)(step - 1) * lr_decay);
  hipLaunchKernelGGL(adagrad_k, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream, p, g, state_sum, n, clr,
                     eps, weight_decay, zero_grad);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_sparse_adamw_ex(const int64_t* rows, const int64_t* count, int64_t max_rows, int32_t D, float* p,
                                    float* g, float* m, float* v, int32_t* flags, float lr, float beta1, float beta2,
                                    float eps, float weight_decay, int64_t step, void* bf16_shadow, int32_t keep_grad,
                                    void* stream) {
  LTHM_REQUIRE(D > 0 && step >= 1 && max_rows >= 0);
  if (max_rows == 0) return 0;
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2 = 1.f - powf(beta2, (float)step);
  if (sparse_v4_ok(D, p, g, m, v, bf16_shadow)) {
    const int rpw = 256 / D;
    const dim3 grid(grid_for((max_rows + rpw - 1) / rpw, 4, 256 * 16));
    if (keep_grad)
      hipLaunchKernelGGL((sparse_opt_v4_k<true, false>), grid, dim3(256), 0, (hipStream_t)stream, rows, count, max_rows, D,
                         p, g, m, v, flags, lr, beta1, beta2, eps, weight_decay, bc1, sqrtf(bc2), (bf16_t*)bf16_shadow);
    else
      hipLaunchKernelGGL((sparse_opt_v4_k<true, true>), grid, dim3(256), 0, (hipStream_t)stream, rows, count, max_rows, D,
                         p, g, m, v, flags, lr, beta1, beta2, eps, weight_decay, bc1, sqrtf(bc2), (bf16_t*)bf16_shadow);
  } else {
    hipLaunchKernelGGL(sparse_adamw_k, dim3(grid_for(max_rows, 4, 256 * 16)), dim3(256), 0, (hipStream_t)stream, rows, count, max_rows, D,
                       p, g, m, v, flags, lr, beta1, beta2, eps, weight_decay, bc1, sqrtf(bc2), (bf16_t*)bf16_shadow,
                       keep_grad ? 0 : 1);
  }
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_sparse_adamw(const int64_t* rows, const int64_t* count, int64_t max_rows, int32_t D, float* p, float* g,
                                 float* m, float* v, int32_t* flags, float lr, float beta1, float beta2, float eps,
                                 float weight_decay, int64_t step, void* bf16_shadow, void* stream) {
  return lthm_sparse_adamw_ex(rows, count, max_rows, D, p, g, m, v, flags, lr, beta1, beta2, eps, weight_decay, step,
                              bf16_shadow, 0, stream);
}

extern "C" int lthm_sparse_adagrad_ex(const int64_t* rows, const int64_t* count, int64_t max_rows, int32_t D, float* p,
                                      float* g, float* state_sum, int32_t* flags, float lr, float lr_decay, float eps,
                                      int64_t step, void* bf16_shadow, int32_t keep_grad, void* stream) {
  LTHM_REQUIRE(D > 0 && step >= 1 && max_rows >= 0);
  if (max_rows == 0) return 0;
  const float clr = lr / (1.f + (float)(step - 1) * lr_decay);
  if (sparse_v4_ok(D, p, g, state_sum, nullptr, bf16_shadow)) {
    const int rpw = 256 / D;
    const dim3 grid(grid_for((max_rows + rpw - 1) / rpw, 4, 256 * 16));
    if (keep_grad)
      hipLaunchKernelGGL((sparse_opt_v4_k<false, false>), grid, dim3(256), 0, (hipStream_t)stream, rows, count, max_rows,
                         D, p, g, state_sum, nullptr, flags, clr, 0.f, 0.f, eps, 0.f, 1.f, 1.f, (bf16_t*)bf16_shadow);
    else
      hipLaunchKernelGGL((sparse_opt_v4_k<false, true>), grid, dim3(256), 0, (hipStream_t)stream, rows, count, max_rows,
                         D, p, g, state_sum, nullptr, flags, clr, 0.f, 0.f, eps, 0.f, 1.f, 1.f, (bf16_t*)bf16_shadow);
  } else {
    hipLaunchKernelGGL(sparse_adagrad_k, dim3(grid_for(max_rows, 4, 256 * 16)), dim3(256), 0, (hipStream_t)stream, rows, count,
                       max_rows, D, p, g, state_sum, flags, clr, eps, (bf16_t*)bf16_shadow, keep_grad ? 0 : 1);
  }
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_sparse_adagrad(const int64_t* rows, const int64_t* count, int64_t max_rows, int32_t D, float* p,
                                   float* g, float* state_sum, int32_t* flags, float lr, float lr_decay, float eps,
                                   int64_t step, void* bf16_shadow, void* stream) {
  return lthm_sparse_adagrad_ex(rows, count, max_rows, D, p, g, state_sum, flags, lr, lr_decay, eps, step, bf16_shadow,
                                0, stream);
}

extern "C" int lthm_sumsq(const void* x, int32_t dtype, int64_t n, float* out_accum, void* stream) {
  LTHM_REQUIRE(n >= 0);
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(n, 256, 1024);
  if (dtype == LTHM_F32) hipLaunchKernelGGL((sumsq_k<float>), dim3(grid), dim3(256), 0, s, (const float*)x, n, out_accum);
  else hipLaunchKernelGGL((sumsq_k<bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, n, out_accum);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_scale_by_norm(const void* x, void* y, int32_t dtype, int64_t n, const float* sumsq, float add_eps,
                                  float max_norm, void* stream) {
  LTHM_REQUIRE(n >= 0);
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(n, 256, 256 * 16);
  if (dtype == LTHM_F32)
    hipLaunchKernelGGL((scale_by_norm_k<float>), dim3(grid), dim3(256), 0, s, (const float*)x, (float*)y, n, sumsq, add_eps, max_norm);
  else
    hipLaunchKernelGGL((scale_by_norm_k<bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, n, sumsq, add_eps, max_norm);
  LTHM_CHECK_LAUNCH();
  return 0;
}
