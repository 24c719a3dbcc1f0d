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

// rows[0 .. *count) touched rows of a [R, D] table; the gradient row is consumed and re-zeroed,
// the row's touched flag reset.  One wave per row.
__global__ __launch_bounds__(256) void sparse_adamw_k(const int64_t* __restrict__ rows, const int64_t* __restrict__ count,
                                                      int64_t max_rows, int D, float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                      float* __restrict__ v, int32_t* __restrict__ flags, float lr, float b1,
                                                      float b2, float eps, float wd, float bc1, float bc2_sqrt,
                                                      bf16_t* __restrict__ shadow) {
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
      const float gi = g[i];
      float pi = p[i] * (1.f - lr * wd);
      const float mi = b1 * m[i] + (1.f - b1) * gi;
      const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
      m[i] = mi;
      v[i] = vi;
      pi = pi - (lr / bc1) * mi / (sqrtf(vi) / bc2_sqrt + eps);
      p[i] = pi;
      if (shadow) shadow[i] = f2bf(pi);
      g[i] = 0.f;
    }
    if (d0 == 0) flags[r] = 0;
  }
}

__global__ __launch_bounds__(256) void sparse_adagrad_k(const int64_t* __restrict__ rows, const int64_t* __restrict__ count,
                                                        int64_t max_rows, int D, float* __restrict__ p, float* __restrict__ g, float* __restrict__ s,
                                                        int32_t* __restrict__ flags, float clr, float eps,
                                                        bf16_t* __restrict__ shadow) {
  const int64_t cnt = min(*count, max_rows);  // never past the row-list capacity
  const int lane = threadIdx.x & 63;
  const int rpw = (D <= 64 && 64 % D == 0) ? 64 / D : 1;
  const int sub = rpw > 1 ? lane / D : 0, d0 = rpw > 1 ? lane - sub * D : lane;
  for (int64_t k = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * rpw + sub; k < cnt;
       k += (int64_t)gridDim.x * 4 * rpw) {
    const int64_t r = rows[k];
    for (int d = d0; d < D; d += 64) {
      const int64_t i = r * D + d;
      const float gi = g[i];
      const float si = s[i] + gi * gi;
      s[i] = si;
      const float pi = p[i] - clr * gi / (sqrtf(si) + eps);
      p[i] = pi;
      if (shadow) shadow[i] = f2bf(pi);
      g[i] = 0.f;
    }
    if (d0 == 0) flags[r] = 0;
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

extern "C" int lthm_sparse_adamw(const int64_t* rows, const int64_t* count, int64_t max_rows, int32_t D, float* p, float* g,
                                 float* m, float* v, int32_t* flags, float lr, float beta1, float beta2, float eps,
                                 float weight_decay, int64_t step, void* bf16_shadow, void* stream) {
  LTHM_REQUIRE(D > 0 && step >= 1 && max_rows >= 0);
  if (max_rows == 0) return 0;
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2 = 1.f - powf(beta2, (float)step);
  hipLaunchKernelGGL(sparse_adamw_k, dim3(grid_for(max_rows, 4, 256 * 16)), dim3(256), 0, (hipStream_t)stream, rows, count, max_rows, D,
                     p, g, m, v, flags, lr, beta1, beta2, eps, weight_decay, bc1, sqrtf(bc2), (bf16_t*)bf16_shadow);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_sparse_adagrad(const int64_t* rows, const int64_t* count, int64_t max_rows, int32_t D, float* p,
                                   float* g, float* state_sum, int32_t* flags, float lr, float lr_decay, float eps,
                                   int64_t step, void* bf16_shadow, void* stream) {
  LTHM_REQUIRE(D > 0 && step >= 1 && max_rows >= 0);
  if (max_rows == 0) return 0;
  const float clr = lr / (1.f + (float)(step - 1) * lr_decay);
  hipLaunchKernelGGL(sparse_adagrad_k, dim3(grid_for(max_rows, 4, 256 * 16)), dim3(256), 0, (hipStream_t)stream, rows, count,
                     max_rows, D, p, g, state_sum, flags, clr, eps, (bf16_t*)bf16_shadow);
  LTHM_CHECK_LAUNCH();
  return 0;
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
