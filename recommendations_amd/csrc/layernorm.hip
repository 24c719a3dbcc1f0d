// LayerNorm forward/backward (commons/transformers/layers.py:142-149, eps 1e-5).
//
// One wave per row, the row held in registers (D/64 values per lane, D <= 1024);
// for D % 4 == 0 each lane owns 4 consecutive columns per 256-column chunk
// (16-byte f32 / 8-byte bf16 accesses).  The forward writes y in bf16 (the GEMM operand) plus the
// per-row mean / rstd; the backward fuses the residual-gradient sums of the
// double-residual encoder (x + block(x), models/lthm/sequence/query_tower.py:
// 132-137) and emits both the f32 residual gradient and its bf16 copy for the
// next GEMM, plus per-block partial sums for dweight / dbias.
#include "common.hpp"

namespace lthm {

template <int NPL, typename TY>
__global__ __launch_bounds__(256) void ln_fwd_k(const float* __restrict__ x, int64_t M, int D, const float* __restrict__ w,
                                                const float* __restrict__ b, TY* __restrict__ y, float* __restrict__ mean,
                                                float* __restrict__ rstd, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = wave; r < M; r += nw) {
    const float* xr = x + r * D;
    float v[NPL];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int c = lane + 64 * i;
      v[i] = (c < D) ? xr[c] : 0.f;
      s += v[i];
    }
    s = wave_sum(s);
    const float mu = s / (float)D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int c = lane + 64 * i;
      const float d = (c < D) ? v[i] - mu : 0.f;
      q += d * d;
    }
    q = wave_sum(q);
    const float rs = 1.f / sqrtf(q / (float)D + eps);
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        float o = (v[i] - mu) * rs * w[c];
        if (b) o += b[c];
        Elem<TY>::st(y + r * D + c, o);
      }
    }
    if (lane == 0) {
      mean[r] = mu;
      rstd[r] = rs;
    }
  }
}

template <int NPL, typename TDY>
__global__ __launch_bounds__(256) void ln_bwd_k(const TDY* __restrict__ dy, const float* __restrict__ x, int64_t M, int D,
                                                const float* __restrict__ w, const float* __restrict__ mean,
                                                const float* __restrict__ rstd, const float* __restrict__ res1,
                                                const float* __restrict__ res2, float* __restrict__ dx,
                                                bf16_t* __restrict__ dx_bf16, float* __restrict__ dw_part,
                                                float* __restrict__ db_part) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t wave = blockIdx.x * 4 + wv;
  const int64_t nw = (int64_t)gridDim.x * 4;
  float dwa[NPL], dba[NPL];
#pragma unroll
  for (int i = 0; i < NPL; ++i) { dwa[i] = 0.f; dba[i] = 0.f; }
  for (int64_t r = wave; r < M; r += nw) {
    const float mu = mean[r], rs = rstd[r];
    float g[NPL], xh[NPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        const float d = Elem<TDY>::ld(dy + r * D + c);
        xh[i] = (x[r * D + c] - mu) * rs;
        g[i] = d * w[c];
        dwa[i] += d * xh[i];
        dba[i] += d;
      } else {
        xh[i] = 0.f;
        g[i] = 0.f;
      }
      s1 += g[i];
      s2 += g[i] * xh[i];
    }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        float o = rs * (g[i] - s1 - xh[i] * s2);
        if (res1) o += res1[r * D + c];
        if (res2) o += res2[r * D + c];
        dx[r * D + c] = o;
        if (dx_bf16) dx_bf16[r * D + c] = f2bf(o);
      }
    }
  }
  // block partials for dweight / dbias
  __shared__ float red[4][1024];
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = lane + 64 * i;
    if (c < D) red[wv][c] = dwa[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) dw_part[(int64_t)blockIdx.x * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = lane + 64 * i;
    if (c < D) red[wv][c] = dba[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) db_part[(int64_t)blockIdx.x * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

// ---- vectorised variants (D % 4 == 0): lane owns columns 4(lane + 64k) .. +3,
// so every access is one 16-byte (f32) or 8-byte (bf16) transaction per lane.
template <typename T>
__device__ __forceinline__ void ld4(const T* p, float (&v)[4]) { load_vec<T, 4 * (int)sizeof(T)>(p, v); }

template <int NK, typename TY>
__global__ __launch_bounds__(256) void ln_fwd_v4_k(const float* __restrict__ x, int64_t M, int D,
                                                   const float* __restrict__ w, const float* __restrict__ b,
                                                   TY* __restrict__ y, float* __restrict__ mean,
                                                   float* __restrict__ rstd, float eps, unsigned* __restrict__ amax) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  float wv[NK][4], bv[NK][4];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = (lane + 64 * k) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) { wv[k][i] = 0.f; bv[k][i] = 0.f; }
    if (c < D) {
      ld4(w + c, wv[k]);
      if (b) ld4(b + c, bv[k]);
    }
  }
  float amx = 0.f;  // max |y| of this lane's stores, as stored (amax)
  for (int64_t r = wave; r < M; r += nw) {
    const float* xr = x + r * D;
    float v[NK][4];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c = (lane + 64 * k) * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[k][i] = 0.f;
      if (c < D) ld4(xr + c, v[k]);
#pragma unroll
      for (int i = 0; i < 4; ++i) s += v[k][i];
    }
    s = wave_sum(s);
    const float mu = s / (float)D;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c = (lane + 64 * k) * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = (c < D) ? v[k][i] - mu : 0.f;
        q += d * d;
      }
    }
    q = wave_sum(q);
    const float rs = 1.f / sqrtf(q / (float)D + eps);
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c < D) {
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (v[k][i] - mu) * rs * wv[k][i] + bv[k][i];
        store_vec<TY, 4>(y + r * D + c, o);
        if (amax)
#pragma unroll
          for (int i = 0; i < 4; ++i) amx = fmaxf(amx, fabsf(sizeof(TY) == 2 ? bf2f(f2bf(o[i])) : o[i]));
      }
    }
    if (lane == 0) {
      mean[r] = mu;
      rstd[r] = rs;
    }
  }
  if (amax) {
    amx = wave_max(amx);
    if (lane == 0) atomicMax(amax, __float_as_uint(amx));
  }
}

template <int NK, typename TDY>
__global__ __launch_bounds__(256) void ln_bwd_v4_k(const TDY* __restrict__ dy, const float* __restrict__ x, int64_t M,
                                                   int D, const float* __restrict__ w, const float* __restrict__ mean,
                                                   const float* __restrict__ rstd, const float* __restrict__ res1,
                                                   const float* __restrict__ res2, float* __restrict__ dx,
                                                   bf16_t* __restrict__ dx_bf16, float* __restrict__ dw_part,
                                                   float* __restrict__ db_part, int res1_twice) {
  const int lane = threadIdx.x & 63;
  const int wv_ = threadIdx.x >> 6;
  const int64_t wave = blockIdx.x * 4 + wv_;
  const int64_t nw = (int64_t)gridDim.x * 4;
  float wgt[NK][4], dwa[NK][4], dba[NK][4];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = (lane + 64 * k) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) { wgt[k][i] = 0.f; dwa[k][i] = 0.f; dba[k][i] = 0.f; }
    if (c < D) ld4(w + c, wgt[k]);
  }
  for (int64_t r = wave; r < M; r += nw) {
    const float mu = mean[r], rs = rstd[r];
    float g[NK][4], xh[NK][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c = (lane + 64 * k) * 4;
      float d[4] = {0.f, 0.f, 0.f, 0.f}, xv[4] = {0.f, 0.f, 0.f, 0.f};
      if (c < D) {
        ld4(dy + r * D + c, d);
        ld4(x + r * D + c, xv);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xh[k][i] = (c < D) ? (xv[i] - mu) * rs : 0.f;
        g[k][i] = d[i] * wgt[k][i];
        dwa[k][i] += d[i] * xh[k][i];
        dba[k][i] += d[i];
        s1 += g[k][i];
        s2 += g[k][i] * xh[k][i];
      }
    }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c < D) {
        float o[4], r1[4] = {0.f, 0.f, 0.f, 0.f}, r2[4] = {0.f, 0.f, 0.f, 0.f};
        if (res1) ld4(res1 + r * D + c, r1);
        if (res2) ld4(res2 + r * D + c, r2);
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = rs * (g[k][i] - s1 - xh[k][i] * s2) + r1[i] + r2[i];
        if (dx_bf16) store_vec<bf16_t, 4>(dx_bf16 + r * D + c, o);
        if (res1_twice) {  // the f32 output carries res1 once more (the next LayerNorm's two residuals)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] += r1[i];
        }
        store_vec<float, 4>(dx + r * D + c, o);
      }
    }
  }
  __shared__ float red[4][1024];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = (lane + 64 * k) * 4;
    if (c < D)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wv_][c + i] = dwa[k][i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) dw_part[(int64_t)blockIdx.x * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = (lane + 64 * k) * 4;
    if (c < D)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wv_][c + i] = dba[k][i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) db_part[(int64_t)blockIdx.x * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

template <int NPL>
static int ln_fwd_launch(const float* x, int64_t M, int D, const float* w, const float* b, void* y, int ydt, float* mean,
                         float* rstd, hipStream_t s) {
  const int grid = grid_for(M, 4, 256 * 8);
  if (ydt == LTHM_BF16)
    hipLaunchKernelGGL((ln_fwd_k<NPL, bf16_t>), dim3(grid), dim3(256), 0, s, x, M, D, w, b, (bf16_t*)y, mean, rstd, 1e-5f);
  else
    hipLaunchKernelGGL((ln_fwd_k<NPL, float>), dim3(grid), dim3(256), 0, s, x, M, D, w, b, (float*)y, mean, rstd, 1e-5f);
  LTHM_CHECK_LAUNCH();
  return 0;
}

template <int NPL>
static int ln_bwd_launch(const void* dy, int dydt, const float* x, int64_t M, int D, const float* w, const float* mean,
                         const float* rstd, const float* res1, const float* res2, float* dx, bf16_t* dxb, float* part,
                         int nblk, hipStream_t s) {
  float* dwp = part;
  float* dbp = part + (int64_t)nblk * D;
  if (dydt == LTHM_BF16)
    hipLaunchKernelGGL((ln_bwd_k<NPL, bf16_t>), dim3(nblk), dim3(256), 0, s, (const bf16_t*)dy, x, M, D, w, mean, rstd, res1,
                       res2, dx, dxb, dwp, dbp);
  else
    hipLaunchKernelGGL((ln_bwd_k<NPL, float>), dim3(nblk), dim3(256), 0, s, (const float*)dy, x, M, D, w, mean, rstd, res1,
                       res2, dx, dxb, dwp, dbp);
  LTHM_CHECK_LAUNCH();
  return 0;
}

}  // namespace lthm

using namespace lthm;

static int ln_fwd(const float* x, int64_t M, int32_t D, const float* w, const float* b, void* y, int32_t y_dtype,
                  float* mean, float* rstd, unsigned* amax, void* stream) {
  LTHM_REQUIRE(M >= 0 && D > 0 && D <= 1024 && w != nullptr);
  if (M == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (D % 4 == 0) {
    const int grid = grid_for(M, 4, 256 * 8);
#define LTHM_LN_FWD_V4(NK)                                                                                     \
    if (D <= 256 * NK) {                                                                                       \
      if (y_dtype == LTHM_BF16)                                                                                \
        hipLaunchKernelGGL((ln_fwd_v4_k<NK, bf16_t>), dim3(grid), dim3(256), 0, s, x, M, D, w, b, (bf16_t*)y,   \
                           mean, rstd, 1e-5f, amax);                                                                 \
      else                                                                                                     \
        hipLaunchKernelGGL((ln_fwd_v4_k<NK, float>), dim3(grid), dim3(256), 0, s, x, M, D, w, b, (float*)y,     \
                           mean, rstd, 1e-5f, amax);                                                                 \
      LTHM_CHECK_LAUNCH();                                                                                     \
      return 0;                                                                                                \
    }
    LTHM_LN_FWD_V4(1)
    LTHM_LN_FWD_V4(2)
    LTHM_LN_FWD_V4(4)
#undef LTHM_LN_FWD_V4
  }
  // D % 4 != 0: the scalar kernel, then amax in a pass over y
  LTHM_REQUIRE(!amax || (M * D) % 8 == 0);
  const int npl = (D + 63) / 64;
  int rc;
  if (npl <= 1) rc = ln_fwd_launch<1>(x, M, D, w, b, y, y_dtype, mean, rstd, s);
  else if (npl <= 2) rc = ln_fwd_launch<2>(x, M, D, w, b, y, y_dtype, mean, rstd, s);
  else if (npl <= 4) rc = ln_fwd_launch<4>(x, M, D, w, b, y, y_dtype, mean, rstd, s);
  else if (npl <= 8) rc = ln_fwd_launch<8>(x, M, D, w, b, y, y_dtype, mean, rstd, s);
  else rc = ln_fwd_launch<16>(x, M, D, w, b, y, y_dtype, mean, rstd, s);
  if (rc || !amax) return rc;
  return lthm_amax(y, y_dtype, M * D, reinterpret_cast<int32_t*>(amax), stream);
}

extern "C" int lthm_layernorm_fwd(const float* x, int64_t M, int32_t D, const float* w, const float* b, void* y,
                                  int32_t y_dtype, float* mean, float* rstd, void* stream) {
  return ln_fwd(x, M, D, w, b, y, y_dtype, mean, rstd, nullptr, stream);
}

extern "C" int lthm_layernorm_fwd_amax(const float* x, int64_t M, int32_t D, const float* w, const float* b, void* y,
                                       int32_t y_dtype, float* mean, float* rstd, int32_t* amax, void* stream) {
  LTHM_REQUIRE(amax != nullptr);
  return ln_fwd(x, M, D, w, b, y, y_dtype, mean, rstd, reinterpret_cast<unsigned*>(amax), stream);
}

extern "C" int lthm_layernorm_bwd_blocks(int64_t M) { return grid_for(M, 4, 256 * 4); }

static int ln_bwd(const void* dy, int32_t dy_dtype, const float* x, int64_t M, int32_t D, const float* w,
                  const float* mean, const float* rstd, const float* res1, const float* res2, float* dx,
                  void* dx_bf16, float* partials, int res1_twice, void* stream) {
  LTHM_REQUIRE(M >= 0 && D > 0 && D <= 1024 && w != nullptr && partials != nullptr);
  LTHM_REQUIRE(!res1_twice || (res1 != nullptr && D % 4 == 0));
  if (M == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int nblk = grid_for(M, 4, 256 * 4);
  bf16_t* xb = (bf16_t*)dx_bf16;
  if (D % 4 == 0) {
    float* dwp = partials;
    float* dbp = partials + (int64_t)nblk * D;
#define LTHM_LN_BWD_V4(NK)                                                                                     \
    if (D <= 256 * NK) {                                                                                       \
      if (dy_dtype == LTHM_BF16)                                                                               \
        hipLaunchKernelGGL((ln_bwd_v4_k<NK, bf16_t>), dim3(nblk), dim3(256), 0, s, (const bf16_t*)dy, x, M, D, w, \
                           mean, rstd, res1, res2, dx, xb, dwp, dbp, res1_twice);                              \
      else                                                                                                     \
        hipLaunchKernelGGL((ln_bwd_v4_k<NK, float>), dim3(nblk), dim3(256), 0, s, (const float*)dy, x, M, D, w,  \
                           mean, rstd, res1, res2, dx, xb, dwp, dbp, res1_twice);                              \
      LTHM_CHECK_LAUNCH();                                                                                     \
      return 0;                                                                                                \
    }
    LTHM_LN_BWD_V4(1)
    LTHM_LN_BWD_V4(2)
    LTHM_LN_BWD_V4(4)
#undef LTHM_LN_BWD_V4
  }
  const int npl = (D + 63) / 64;
  if (npl <= 1) return ln_bwd_launch<1>(dy, dy_dtype, x, M, D, w, mean, rstd, res1, res2, dx, xb, partials, nblk, s);
  if (npl <= 2) return ln_bwd_launch<2>(dy, dy_dtype, x, M, D, w, mean, rstd, res1, res2, dx, xb, partials, nblk, s);
  if (npl <= 4) return ln_bwd_launch<4>(dy, dy_dtype, x, M, D, w, mean, rstd, res1, res2, dx, xb, partials, nblk, s);
  if (npl <= 8) return ln_bwd_launch<8>(dy, dy_dtype, x, M, D, w, mean, rstd, res1, res2, dx, xb, partials, nblk, s);
  return ln_bwd_launch<16>(dy, dy_dtype, x, M, D, w, mean, rstd, res1, res2, dx, xb, partials, nblk, s);
}

extern "C" int lthm_layernorm_bwd(const void* dy, int32_t dy_dtype, const float* x, int64_t M, int32_t D, const float* w,
                                  const float* mean, const float* rstd, const float* res1, const float* res2, float* dx,
                                  void* dx_bf16, float* partials, void* stream) {
  return ln_bwd(dy, dy_dtype, x, M, D, w, mean, rstd, res1, res2, dx, dx_bf16, partials, 0, stream);
}

extern "C" int lthm_layernorm_bwd_ex(const void* dy, int32_t dy_dtype, const float* x, int64_t M, int32_t D,
                                     const float* w, const float* mean, const float* rstd, const float* res1,
                                     const float* res2, float* dx, void* dx_bf16, float* partials, int32_t flags,
                                     void* stream) {
  LTHM_REQUIRE((flags & ~1) == 0);
  return ln_bwd(dy, dy_dtype, x, M, D, w, mean, rstd, res1, res2, dx, dx_bf16, partials, flags & 1, stream);
}
