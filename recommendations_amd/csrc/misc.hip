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
  if (c < cols)
    for (int64_t r = r0 + wave; r < r1; r += 4) acc += Elem<T>::ld(in + r * ld + c);
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
