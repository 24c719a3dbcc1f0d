// Write-pattern probe: how fast can [M, N] bf16 GEMM-shaped outputs be written to HBM
// in 128 x 128 tiles (16-B stores, 256 threads), by tile order, against full-row writes?
// Built by tools/write_probe.py (hipcc -shared), timed with HIP events.
#include <hip/hip_runtime.h>
#include <stdint.h>

// one 128 x 128 bf16 tile per workgroup; order 0: row-panel major (the 8 column tiles of
// a row panel are consecutive block ids), 1: column-tile major
__global__ __launch_bounds__(256) void tile_write_k(uint4* out, int64_t M, int64_t N, int order, int reps) {
  const int64_t tn = N / 128, tm = M / 128;
  const int64_t id = blockIdx.x;
  const int64_t pm = order == 0 ? id / tn : id % tm;
  const int64_t pn = order == 0 ? id % tn : id / tm;
  const int t = threadIdx.x;
  const uint4 v = {(uint32_t)t, 1u, 2u, 3u};
  for (int r = 0; r < reps; ++r)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t row = pm * 128 + (t >> 4) + 16 * i;
      const int64_t col = pn * 128 + (t & 15) * 8;
      out[(row * N + col) / 8] = v;
    }
}

// full rows: each workgroup writes 16 whole rows (N bf16 each)
__global__ __launch_bounds__(256) void row_write_k(uint4* out, int64_t M, int64_t N) {
  const int64_t row0 = (int64_t)blockIdx.x * 16;
  const int64_t chunks = N / 8;
  const uint4 v = {(uint32_t)threadIdx.x, 1u, 2u, 3u};
  for (int64_t c = threadIdx.x; c < 16 * chunks; c += 256) {
    const int64_t r = row0 + c / chunks, cc = c % chunks;
    out[r * chunks + cc] = v;
  }
}

// persistent grid-stride over 128 x 128 tiles (tile = w + grid * i), order as tile_write_k
__global__ __launch_bounds__(256) void tile_write_persist_k(uint4* out, int64_t M, int64_t N, int order) {
  const int64_t tn = N / 128, tm = M / 128, nt = tn * tm;
  const int t = threadIdx.x;
  const uint4 v = {(uint32_t)t, 1u, 2u, 3u};
  for (int64_t id = blockIdx.x; id < nt; id += gridDim.x) {
    const int64_t pm = order == 0 ? id / tn : id % tm;
    const int64_t pn = order == 0 ? id % tn : id / tm;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t row = pm * 128 + (t >> 4) + 16 * i;
      const int64_t col = pn * 128 + (t & 15) * 8;
      out[(row * N + col) / 8] = v;
    }
  }
}

extern "C" int probe_tile(void* out, int64_t M, int64_t N, int order, void* s) {
  hipLaunchKernelGGL(tile_write_k, dim3((unsigned)((M / 128) * (N / 128))), dim3(256), 0, (hipStream_t)s,
                     (uint4*)out, M, N, order, 1);
  return (int)hipGetLastError();
}
extern "C" int probe_rows(void* out, int64_t M, int64_t N, void* s) {
  hipLaunchKernelGGL(row_write_k, dim3((unsigned)(M / 16)), dim3(256), 0, (hipStream_t)s, (uint4*)out, M, N);
  return (int)hipGetLastError();
}
extern "C" int probe_persist(void* out, int64_t M, int64_t N, int order, int grid, void* s) {
  hipLaunchKernelGGL(tile_write_persist_k, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)s, (uint4*)out, M, N,
                     order);
  return (int)hipGetLastError();
}
