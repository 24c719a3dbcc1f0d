// Row-wise AdamW layout probe (C4 shape: 64M rows x D 32 f32, ~4.06M unique random rows per
// step): the update's time with p / g / m / v as four [P, D] arrays (the current layout), with the
// private state interleaved as [P, 3, D] (g, m, v) beside p, and with the gradient zero-store
// dropped (the first-touch backward overwrites a row's gradient).  Timing probe only.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/slp tools/probes/sparse_layout_probe.hip && /tmp/slp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ float adamw_e(float p, float g, float& m, float& v) {
  m = 0.9f * m + 0.1f * g;
  v = 0.999f * v + 0.001f * g * g;
  return p - 1e-3f * (m / (sqrtf(v) + 1e-8f) + 0.01f * p);
}

// SPLIT: four arrays; ZG: store g = 0; RPL: rows per lane group in flight
template <bool ZG, int RPL>
__global__ __launch_bounds__(256) void upd_split(const int64_t* __restrict__ rows, int64_t cnt, float* __restrict__ p,
                                                 float* __restrict__ g, float* __restrict__ m, float* __restrict__ v) {
  const int lane = threadIdx.x & 63, sub = lane >> 3, d0 = (lane & 7) * 4;
  const int64_t stride = (int64_t)gridDim.x * 4 * 8 * RPL;
  for (int64_t k0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 * RPL + sub; k0 < cnt; k0 += stride) {
    int64_t r[RPL];
    float4 P[RPL], G[RPL], M[RPL], V[RPL];
#pragma unroll
    for (int u = 0; u < RPL; ++u) r[u] = k0 + 8 * u < cnt ? rows[k0 + 8 * u] : -1;
#pragma unroll
    for (int u = 0; u < RPL; ++u) {
      if (r[u] < 0) continue;
      const int64_t i = r[u] * 32 + d0;
      G[u] = *(const float4*)(g + i); P[u] = *(const float4*)(p + i);
      M[u] = *(const float4*)(m + i); V[u] = *(const float4*)(v + i);
    }
#pragma unroll
    for (int u = 0; u < RPL; ++u) {
      if (r[u] < 0) continue;
      const int64_t i = r[u] * 32 + d0;
      P[u].x = adamw_e(P[u].x, G[u].x, M[u].x, V[u].x);
      P[u].y = adamw_e(P[u].y, G[u].y, M[u].y, V[u].y);
      P[u].z = adamw_e(P[u].z, G[u].z, M[u].z, V[u].z);
      P[u].w = adamw_e(P[u].w, G[u].w, M[u].w, V[u].w);
      *(float4*)(m + i) = M[u]; *(float4*)(v + i) = V[u]; *(float4*)(p + i) = P[u];
      if (ZG) *(float4*)(g + i) = float4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// interleaved private state s = [P][3][32] (g, m, v) beside p [P][32]
template <bool ZG, int RPL>
__global__ __launch_bounds__(256) void upd_ilv(const int64_t* __restrict__ rows, int64_t cnt, float* __restrict__ p,
                                               float* __restrict__ s) {
  const int lane = threadIdx.x & 63, sub = lane >> 3, d0 = (lane & 7) * 4;
  const int64_t stride = (int64_t)gridDim.x * 4 * 8 * RPL;
  for (int64_t k0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 * RPL + sub; k0 < cnt; k0 += stride) {
    int64_t r[RPL];
    float4 P[RPL], G[RPL], M[RPL], V[RPL];
#pragma unroll
    for (int u = 0; u < RPL; ++u) r[u] = k0 + 8 * u < cnt ? rows[k0 + 8 * u] : -1;
#pragma unroll
    for (int u = 0; u < RPL; ++u) {
      if (r[u] < 0) continue;
      const int64_t i = r[u] * 96 + d0;
      G[u] = *(const float4*)(s + i); M[u] = *(const float4*)(s + i + 32); V[u] = *(const float4*)(s + i + 64);
      P[u] = *(const float4*)(p + r[u] * 32 + d0);
    }
#pragma unroll
    for (int u = 0; u < RPL; ++u) {
      if (r[u] < 0) continue;
      const int64_t i = r[u] * 96 + d0;
      P[u].x = adamw_e(P[u].x, G[u].x, M[u].x, V[u].x);
      P[u].y = adamw_e(P[u].y, G[u].y, M[u].y, V[u].y);
      P[u].z = adamw_e(P[u].z, G[u].z, M[u].z, V[u].z);
      P[u].w = adamw_e(P[u].w, G[u].w, M[u].w, V[u].w);
      if (ZG) *(float4*)(s + i) = float4{0.f, 0.f, 0.f, 0.f};
      *(float4*)(s + i + 32) = M[u]; *(float4*)(s + i + 64) = V[u];
      *(float4*)(p + r[u] * 32 + d0) = P[u];
    }
  }
}

int main() {
  const int64_t P = 64ll * 1000000, D = 32;
  const int64_t n = 4194304;  // 65,536 x 64 lookups
  std::mt19937_64 rng(7);
  std::vector<int64_t> ids(n);
  for (auto& x : ids) x = (int64_t)(rng() % P);
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  std::shuffle(ids.begin(), ids.end(), rng);  // touched-row list order: random
  const int64_t cnt = (int64_t)ids.size();
  printf("unique rows %lld\n", (long long)cnt);
  int64_t* rows;
  float *p, *g, *m, *v, *s;
  CK(hipMalloc(&rows, cnt * 8));
  CK(hipMemcpy(rows, ids.data(), cnt * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&p, P * D * 4)); CK(hipMalloc(&g, P * D * 4)); CK(hipMalloc(&m, P * D * 4)); CK(hipMalloc(&v, P * D * 4));
  CK(hipMemset(p, 0, P * D * 4)); CK(hipMemset(g, 0, P * D * 4)); CK(hipMemset(m, 0, P * D * 4)); CK(hipMemset(v, 0, P * D * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes_per_row, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    printf("%-28s %.4f ms  %.2f TB/s (%.0f B/row)\n", name, ms, bytes_per_row * cnt / (ms * 1e-3) / 1e12, bytes_per_row);
    return 0;
  };
  const int grid = 256 * 16;
  timeit("split zg rpl1", 8 + 4 * 128 + 4 * 128, [&] { upd_split<true, 1><<<grid, 256>>>(rows, cnt, p, g, m, v); });
  timeit("split zg rpl2", 8 + 4 * 128 + 4 * 128, [&] { upd_split<true, 2><<<grid, 256>>>(rows, cnt, p, g, m, v); });
  timeit("split nozg rpl1", 8 + 4 * 128 + 3 * 128, [&] { upd_split<false, 1><<<grid, 256>>>(rows, cnt, p, g, m, v); });
  timeit("split nozg rpl2", 8 + 4 * 128 + 3 * 128, [&] { upd_split<false, 2><<<grid, 256>>>(rows, cnt, p, g, m, v); });
  CK(hipFree(g)); CK(hipFree(m)); CK(hipFree(v));
  CK(hipMalloc(&s, P * D * 4 * 3));
  CK(hipMemset(s, 0, P * D * 4 * 3));
  timeit("ilv zg rpl1", 8 + 4 * 128 + 4 * 128, [&] { upd_ilv<true, 1><<<grid, 256>>>(rows, cnt, p, s); });
  timeit("ilv zg rpl2", 8 + 4 * 128 + 4 * 128, [&] { upd_ilv<true, 2><<<grid, 256>>>(rows, cnt, p, s); });
  timeit("ilv nozg rpl1", 8 + 4 * 128 + 3 * 128, [&] { upd_ilv<false, 1><<<grid, 256>>>(rows, cnt, p, s); });
  timeit("ilv nozg rpl2", 8 + 4 * 128 + 3 * 128, [&] { upd_ilv<false, 2><<<grid, 256>>>(rows, cnt, p, s); });
  // sorted row list (the same rows in address order)
  std::sort(ids.begin(), ids.end());
  CK(hipMemcpy(rows, ids.data(), cnt * 8, hipMemcpyHostToDevice));
  timeit("ilv nozg rpl2 sorted", 8 + 4 * 128 + 3 * 128, [&] { upd_ilv<false, 2><<<grid, 256>>>(rows, cnt, p, s); });
  return 0;
}
