// Vector-feature layers around the MFMA GEMM (reference commons/transformers/layers.py):
//   SimhashVectorIndexer          :426-437  sign bits of x @ projection_mat packed into an int64
//   CosineLinear                  :517-525  normalize(x) @ normalize(W)^T
//   LearnableCosineVectorEmbedding:531-566  gaussian bins of CosineLinear(x) -> Linear
//   ProbabilityVectorEmbedding    :572-595  gaussian bins of a scalar -> Linear
// The output Linear of the two embeddings is the bf16 MFMA GEMM (gemm.hip); everything
// here is f32 and HBM-bound: every kernel streams its rows once with nothing re-read
// but the few-KiB projection / mean operands, which stay in L1 / L2.
#include "common.hpp"

namespace lthm {

// ---- row projections --------------------------------------------------------------
// z[r, j] = s_r * sum_k x[r, k] W[j, k], W[j, k] at w[j * ldj + k * ldk].
// Lane layout: PP = pow2 >= min(P, 64) lanes per row, 64 / PP rows per wave; blockIdx.y
// walks 64-column groups when P > 64 (cosine only).  The x row is read as f32x4 when
// dim % 4 == 0 (all lanes of a row share the address: one fetch per sub-group).
//   mode 0: bits[r] = sum_j (z[r, j] > 0) << j        (SimHash, s_r = 1, P <= 64)
//   mode 1: out[r, j] = z[r, j] / max(|x_r|, 1e-12)    (cosine; W already row-normalised)
__global__ __launch_bounds__(256) void rowproj_fwd_k(const float* __restrict__ x, int64_t rows, int dim,
                                                     const float* __restrict__ w, int64_t ldj, int64_t ldk, int P,
                                                     int PP, int mode, void* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int sub = lane / PP, j = blockIdx.y * 64 + (lane % PP);
  const int rpw = 64 / PP;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const bool jok = j < P;
  const float* wj = w + (int64_t)(jok ? j : 0) * ldj;
  for (int64_t r0 = wave * rpw; r0 < rows; r0 += nwaves * rpw) {
    const int64_t r = r0 + sub;
    const bool rok = r < rows;
    const float* xr = x + (rok ? r : 0) * (int64_t)dim;
    float acc = 0.f, ss = 0.f;
    int k = 0;
    if ((dim & 3) == 0) {
      for (; k < dim; k += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(xr + k);
        acc = fmaf(v[0], wj[(int64_t)k * ldk], acc);
        acc = fmaf(v[1], wj[(int64_t)(k + 1) * ldk], acc);
        acc = fmaf(v[2], wj[(int64_t)(k + 2) * ldk], acc);
        acc = fmaf(v[3], wj[(int64_t)(k + 3) * ldk], acc);
        ss = fmaf(v[0], v[0], fmaf(v[1], v[1], fmaf(v[2], v[2], fmaf(v[3], v[3], ss))));
      }
    }
    for (; k < dim; ++k) {
      const float v = xr[k];
      acc = fmaf(v, wj[(int64_t)k * ldk], acc);
      ss = fmaf(v, v, ss);
    }
    if (mode == 0) {
      const uint64_t m = __ballot(rok && jok && acc > 0.f);
      if (rok && (lane % PP) == 0) {
        const uint64_t bits = PP == 64 ? m : ((m >> (sub * PP)) & ((1ull << PP) - 1));
        reinterpret_cast<int64_t*>(out)[r] = (int64_t)bits;
      }
    } else if (rok && jok) {
      reinterpret_cast<float*>(out)[r * P + j] = acc / fmaxf(sqrtf(ss), 1e-12f);
    }
  }
}

// ---- F.normalize rows (f32) and its backward ----------------------------------------
// One wave per row.  fwd: y = x / max(|x|, eps).  bwd: with the incoming gradient g
// (given, or g = dz @ W_hat for CosineLinear's x side: g[k] = sum_j dz[r, j] W_hat[j, k]),
//   dx = (g - y (y . g)) / |x|   if |x| > eps,   g / eps otherwise.
// g is staged in dx itself (each lane re-reads only what it wrote), rinv[r] = 1 / max(|x|, eps)
// is kept for the weight-gradient kernel.
__device__ __forceinline__ float row_sumsq(const float* __restrict__ xr, int dim, int lane) {
  float ss = 0.f;
  for (int k = lane; k < dim; k += 64) ss = fmaf(xr[k], xr[k], ss);
  return wave_sum(ss);
}

__global__ __launch_bounds__(256) void l2norm_rows_k(const float* __restrict__ x, int64_t rows, int dim,
                                                     float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < rows; r += nwaves) {
    const float* xr = x + r * dim;
    const float inv = 1.f / fmaxf(sqrtf(row_sumsq(xr, dim, lane)), 1e-12f);
    for (int k = lane; k < dim; k += 64) y[r * dim + k] = xr[k] * inv;
  }
}

__global__ __launch_bounds__(256) void l2norm_rows_bwd_k(const float* __restrict__ x, int64_t rows, int dim,
                                                         const float* __restrict__ g, const float* __restrict__ dz,
                                                         const float* __restrict__ what, int P,
                                                         float* __restrict__ dx, float* __restrict__ rinv) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < rows; r += nwaves) {
    const float* xr = x + r * dim;
    float* dxr = dx + r * dim;
    const float n = sqrtf(row_sumsq(xr, dim, lane));
    const float inv = 1.f / fmaxf(n, 1e-12f);
    float dot = 0.f;
    for (int k = lane; k < dim; k += 64) {
      float gk;
      if (dz) {
        gk = 0.f;
        for (int jj = 0; jj < P; ++jj) gk = fmaf(dz[r * P + jj], what[(int64_t)jj * dim + k], gk);
      } else {
        gk = g[r * dim + k];
      }
      dxr[k] = gk;
      dot = fmaf(xr[k] * inv, gk, dot);
    }
    dot = wave_sum(dot);
    if (n > 1e-12f) {
      for (int k = lane; k < dim; k += 64) dxr[k] = (dxr[k] - xr[k] * inv * dot) * inv;
    } else {
      for (int k = lane; k < dim; k += 64) dxr[k] = dxr[k] * inv;
    }
    if (rinv && lane == 0) rinv[r] = inv;
  }
}

// ---- CosineLinear weight side: dW_hat[j, k] += sum_r dz[r, j] x[r, k] rinv[r] -----
// Block = 256 threads x 8 (j, k) elements each (a 2048-element slice of [P, dim], slice =
// blockIdx.y); blockIdx.x takes a contiguous row range.  x reads are coalesced along k.
__global__ __launch_bounds__(256) void cosine_wgrad_k(const float* __restrict__ dz, const float* __restrict__ x,
                                                      const float* __restrict__ rinv, int64_t rows, int P, int dim,
                                                      int64_t rows_per_block, float* __restrict__ dwhat) {
  constexpr int E = 8;
  const int64_t nel = (int64_t)P * dim;
  const int64_t e0 = (int64_t)blockIdx.y * 256 * E + threadIdx.x;
  const int64_t rs = (int64_t)blockIdx.x * rows_per_block;
  const int64_t re = rs + rows_per_block < rows ? rs + rows_per_block : rows;
  float acc[E];
  int jj[E], kk[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    acc[e] = 0.f;
    const int64_t el = e0 + (int64_t)e * 256;
    jj[e] = el < nel ? (int)(el / dim) : -1;
    kk[e] = el < nel ? (int)(el % dim) : 0;
  }
  for (int64_t r = rs; r < re; ++r) {
    const float s = rinv[r];
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (jj[e] >= 0) acc[e] = fmaf(dz[r * P + jj[e]], x[r * dim + kk[e]] * s, acc[e]);
  }
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (jj[e] >= 0 && re > rs) atomicAdd(dwhat + (int64_t)jj[e] * dim + kk[e], acc[e]);
}

// ---- gaussian bins ------------------------------------------------------------------
// One thread per (row, projection) pair i = r * P + p with value v = z[i]:
//   a[b]  = exp(((-0.5 (v - mean[p, b])) (v - mean[p, b])) / sigma2)      (:562-563, :592-593)
//   top_k : keep a[b] iff fewer than k bins are strictly larger (== a[b] >= k-th largest,
//           the reference's torch.where(act < thresh, 0, act), :565-568)
//   out   = a / max(|a|, 1e-12) over the bins                                    (:569)
// NBM (16 / 32 / 64) bounds the bin count so the bins stay in registers.
template <int NBM>
__device__ __forceinline__ float gauss_bins(float v, const float* __restrict__ mp, int nb, float s2, int topk,
                                            float (&a)[NBM], float (&dd)[NBM]) {
#pragma unroll
  for (int b = 0; b < NBM; ++b) {
    const float d = b < nb ? v - mp[b] : 0.f;
    dd[b] = d;
    a[b] = b < nb ? expf(((-0.5f * d) * d) / s2) : 0.f;
  }
  if (topk > 0 && topk < nb) {
    float keep[NBM];
#pragma unroll
    for (int b = 0; b < NBM; ++b) {
      int gt = 0;
#pragma unroll
      for (int c = 0; c < NBM; ++c) gt += (c < nb && a[c] > a[b]) ? 1 : 0;
      keep[b] = gt < topk ? a[b] : 0.f;
    }
#pragma unroll
    for (int b = 0; b < NBM; ++b) a[b] = keep[b];
  }
  float ss = 0.f;
#pragma unroll
  for (int b = 0; b < NBM; ++b) ss = fmaf(a[b], a[b], ss);
  return sqrtf(ss);
}

template <int NBM>
__global__ __launch_bounds__(256) void gauss_bins_fwd_k(const float* __restrict__ z, int64_t n, int P,
                                                        const float* __restrict__ mean, int nb, float s2, int topk,
                                                        void* __restrict__ out, int out_bf16) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(i % P);
    float a[NBM], dd[NBM];
    const float inv = 1.f / fmaxf(gauss_bins<NBM>(z[i], mean + (int64_t)p * nb, nb, s2, topk, a, dd), 1e-12f);
    if (out_bf16) {
      bf16_t* o = reinterpret_cast<bf16_t*>(out) + i * nb;
#pragma unroll
      for (int b = 0; b < NBM; ++b)
        if (b < nb) o[b] = f2bf(a[b] * inv);
    } else {
      float* o = reinterpret_cast<float*>(out) + i * nb;
#pragma unroll
      for (int b = 0; b < NBM; ++b)
        if (b < nb) o[b] = a[b] * inv;
    }
  }
}

// bwd: with y = a / |a| and incoming g over the bins,
//   g_a = (g - y (y . g)) / |a|  (|a| > eps; g / eps otherwise), zero on top-k-dropped bins,
//   g_d = g_a a (-d / sigma2);   dz[i] = sum_b g_d;   dmean[p, b] -= sum_rows g_d
// dmean is reduced in LDS per block (P * nb <= 4096) before one global atomic per entry.
template <int NBM>
__global__ __launch_bounds__(256) void gauss_bins_bwd_k(const float* __restrict__ z, int64_t n, int P,
                                                        const float* __restrict__ mean, int nb, float s2, int topk,
                                                        const void* __restrict__ gout, int g_bf16,
                                                        float* __restrict__ dz, float* __restrict__ dmean) {
  extern __shared__ float red[];
  const int nm = P * nb;
  const bool lds = nm <= 4096;
  if (lds) {
    for (int t = threadIdx.x; t < nm; t += blockDim.x) red[t] = 0.f;
    __syncthreads();
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(i % P);
    float a[NBM], dd[NBM], g[NBM];
    const float nrm = gauss_bins<NBM>(z[i], mean + (int64_t)p * nb, nb, s2, topk, a, dd);
    const float inv = 1.f / fmaxf(nrm, 1e-12f);
    float dot = 0.f;
#pragma unroll
    for (int b = 0; b < NBM; ++b) {
      g[b] = b < nb ? (g_bf16 ? bf2f(reinterpret_cast<const bf16_t*>(gout)[i * nb + b])
                              : reinterpret_cast<const float*>(gout)[i * nb + b])
                    : 0.f;
      dot = fmaf(a[b] * inv, g[b], dot);
    }
    float dzi = 0.f;
#pragma unroll
    for (int b = 0; b < NBM; ++b) {
      if (b < nb) {
        const float ga = nrm > 1e-12f ? (g[b] - a[b] * inv * dot) * inv : g[b] * inv;
        // a[b] == 0 on dropped bins (and exp underflow), which zeroes their gradient
        const float gd = ga * a[b] * (-dd[b] / s2);
        dzi += gd;
        if (lds)
          atomicAdd(red + p * nb + b, -gd);
        else
          atomicAdd(dmean + (int64_t)p * nb + b, -gd);
      }
    }
    if (dz) dz[i] = dzi;
  }
  if (lds) {
    __syncthreads();
    for (int t = threadIdx.x; t < nm; t += blockDim.x)
      if (red[t] != 0.f) atomicAdd(dmean + t, red[t]);
  }
}

}  // namespace lthm

using namespace lthm;

static int rowproj_pp(int P) {
  int pp = 1;
  while (pp < P && pp < 64) pp <<= 1;
  return pp;
}

extern "C" int lthm_rowproj_fwd(const float* x, int64_t rows, int32_t dim, const float* w, int64_t ldj, int64_t ldk,
                                int32_t P, int32_t mode, void* out, void* stream) {
  LTHM_REQUIRE(rows >= 0 && dim > 0 && P > 0 && (mode == 0 || mode == 1) && x && w && out);
  LTHM_REQUIRE(mode == 1 || P <= 64);
  LTHM_REQUIRE(((uintptr_t)x % 16) == 0 || (dim & 3) != 0);
  if (rows == 0) return 0;
  const int pp = rowproj_pp(P), rpw = 64 / pp;
  const int64_t waves = (rows + rpw - 1) / rpw;
  const int gx = (int)(waves < 4096 * 4 ? (waves + 3) / 4 : 4096);
  hipLaunchKernelGGL(rowproj_fwd_k, dim3(gx, (P + 63) / 64), dim3(256), 0, (hipStream_t)stream, x, rows, dim, w, ldj,
                     ldk, P, pp, mode, out);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_l2norm_rows(const float* x, int64_t rows, int32_t dim, float* y, void* stream) {
  LTHM_REQUIRE(rows >= 0 && dim > 0 && x && y);
  if (rows == 0) return 0;
  hipLaunchKernelGGL(l2norm_rows_k, dim3(grid_for(rows * 64, 256, 4096)), dim3(256), 0, (hipStream_t)stream, x, rows,
                     dim, y);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_l2norm_rows_bwd(const float* x, int64_t rows, int32_t dim, const float* g, const float* dz,
                                    const float* w_hat, int32_t P, float* dx, float* rinv, void* stream) {
  LTHM_REQUIRE(rows >= 0 && dim > 0 && x && dx && ((g != nullptr) != (dz != nullptr)));
  LTHM_REQUIRE(dz == nullptr || (w_hat != nullptr && P > 0));
  if (rows == 0) return 0;
  hipLaunchKernelGGL(l2norm_rows_bwd_k, dim3(grid_for(rows * 64, 256, 4096)), dim3(256), 0, (hipStream_t)stream, x,
                     rows, dim, g, dz, w_hat, P, dx, rinv);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_cosine_wgrad(const float* dz, const float* x, const float* rinv, int64_t rows, int32_t P,
                                 int32_t dim, float* dw_hat, void* stream) {
  LTHM_REQUIRE(rows >= 0 && P > 0 && dim > 0 && dz && x && rinv && dw_hat);
  if (rows == 0) return 0;
  const int64_t nel = (int64_t)P * dim;
  const int gy = (int)((nel + 2047) / 2048);
  LTHM_REQUIRE(gy <= 65535);
  // ~1024 blocks in total, at least 64 rows per block
  int64_t gx = (1024 + gy - 1) / gy;
  int64_t rpb = (rows + gx - 1) / gx;
  if (rpb < 64) rpb = 64;
  gx = (rows + rpb - 1) / rpb;
  hipLaunchKernelGGL(cosine_wgrad_k, dim3((unsigned)gx, gy), dim3(256), 0, (hipStream_t)stream, dz, x, rinv, rows, P,
                     dim, rpb, dw_hat);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_gauss_bins_fwd(const float* z, int64_t n, int32_t P, const float* mean, int32_t nb, float sigma2,
                                   int32_t top_k, void* out, int32_t out_dtype, void* stream) {
  LTHM_REQUIRE(n >= 0 && P > 0 && nb > 0 && nb <= 64 && sigma2 > 0.f && top_k >= 0 && z && mean && out);
  LTHM_REQUIRE(out_dtype == LTHM_F32 || out_dtype == LTHM_BF16);
  if (n == 0) return 0;
  const int bf = out_dtype == LTHM_BF16;
  const dim3 g(grid_for(n, 256, 4096)), b(256);
  hipStream_t s = (hipStream_t)stream;
  if (nb <= 16)
    hipLaunchKernelGGL(gauss_bins_fwd_k<16>, g, b, 0, s, z, n, P, mean, nb, sigma2, top_k, out, bf);
  else if (nb <= 32)
    hipLaunchKernelGGL(gauss_bins_fwd_k<32>, g, b, 0, s, z, n, P, mean, nb, sigma2, top_k, out, bf);
  else
    hipLaunchKernelGGL(gauss_bins_fwd_k<64>, g, b, 0, s, z, n, P, mean, nb, sigma2, top_k, out, bf);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_gauss_bins_bwd(const float* z, int64_t n, int32_t P, const float* mean, int32_t nb, float sigma2,
                                   int32_t top_k, const void* gout, int32_t g_dtype, float* dz, float* dmean,
                                   void* stream) {
  LTHM_REQUIRE(n >= 0 && P > 0 && nb > 0 && nb <= 64 && sigma2 > 0.f && top_k >= 0 && z && mean && gout && dmean);
  LTHM_REQUIRE(g_dtype == LTHM_F32 || g_dtype == LTHM_BF16);
  if (n == 0) return 0;
  const int bf = g_dtype == LTHM_BF16;
  const size_t shm = (size_t)P * nb <= 4096 ? (size_t)P * nb * sizeof(float) : 0;
  const dim3 g(grid_for(n, 256, 1024)), b(256);
  hipStream_t s = (hipStream_t)stream;
  if (nb <= 16)
    hipLaunchKernelGGL(gauss_bins_bwd_k<16>, g, b, shm, s, z, n, P, mean, nb, sigma2, top_k, gout, bf, dz, dmean);
  else if (nb <= 32)
    hipLaunchKernelGGL(gauss_bins_bwd_k<32>, g, b, shm, s, z, n, P, mean, nb, sigma2, top_k, gout, bf, dz, dmean);
  else
    hipLaunchKernelGGL(gauss_bins_bwd_k<64>, g, b, shm, s, z, n, P, mean, nb, sigma2, top_k, gout, bf, dz, dmean);
  LTHM_CHECK_LAUNCH();
  return 0;
}
