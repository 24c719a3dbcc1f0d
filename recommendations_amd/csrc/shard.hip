// Row-sharded KShift lookup routing (C3: the 100M-row item table row-sharded over the
// data-parallel ranks; commons/layers.py:152-185 for the row math).
//
// Global row r lives on rank r % W at local index r / W.  A lookup of N ids x K shifts:
//  1. shard_dedup_k: per workgroup, SR_NP (row, pair) keys sorted in LDS (bitonic), runs of
//     equal rows collapsed to one request (the negative-id collapse of the arithmetic shift
//     sends ~half of all shifted rows to row P-1: one request per workgroup instead of
//     thousands); each unique row gets its owner and a rank inside (workgroup, owner);
//  2. shard_offsets_k: per owner, an exclusive scan of the per-workgroup counts, the
//     per-owner totals (the all_to_all send counts, on the device) and the owner bases;
//  3. shard_scatter_k: the unique rows into an owner-major send buffer, and for every
//     (id, shift) pair the position of its row's value in the returned buffer;
//  4. (exchange: all_to_all of the row ids, the owners gather, all_to_all of the rows back)
//  5. shard_gather_k: an owner's rows by local index r / W;
// then lthm_gather_pool sums each id's K rows in order (bit-identical to the unsharded
// KShift forward).  Requests are deduplicated per workgroup, not globally: a row that two
// workgroups both request is sent twice (the values are copies; the result is unchanged).
#include "common.hpp"

namespace lthm {

constexpr int SR_NP = 2048;  // (row, pair) keys per workgroup
constexpr int SR_PB = 11;    // bits of the pair index inside a key
constexpr int SR_MAXW = 256; // owners: shard_dedup_k counts per owner in __shared__ s_own[SR_MAXW]

__global__ __launch_bounds__(256) void shard_dedup_k(const int64_t* __restrict__ ids, int64_t n_pairs, int K,
                                                     int64_t P, int W, int64_t* __restrict__ u_row,
                                                     int32_t* __restrict__ u_slot, int32_t* __restrict__ u_cnt,
                                                     int32_t* __restrict__ blk_cnt, int32_t* __restrict__ inv_local) {
  __shared__ uint64_t keys[SR_NP];
  __shared__ int s_own[SR_MAXW];
  __shared__ int s_wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * SR_NP;
  const int np = (int)min((int64_t)SR_NP, n_pairs - base);
  for (int o = tid; o < W; o += 256) s_own[o] = 0;
  for (int p = tid; p < SR_NP; p += 256) {
    uint64_t key = ~0ull;
    if (p < np) {
      const int64_t g = base + p;
      const int64_t item = g / K;
      const int c = (int)(g - item * K);
      key = ((uint64_t)kshift_row(ids[item], c, P) << SR_PB) | (uint64_t)p;
    }
    keys[p] = key;
  }
  __syncthreads();
  for (int k = 2; k <= SR_NP; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = tid; t < SR_NP / 2; t += 256) {
        const int i0 = 2 * t - (t & (j - 1)), i1 = i0 + j;
        const bool up = (i0 & k) == 0;
        const uint64_t a = keys[i0], b = keys[i1];
        if ((a > b) == up) { keys[i0] = b; keys[i1] = a; }
      }
      __syncthreads();
    }
  }
  // run heads over the sorted keys (8 consecutive positions per thread), block exclusive scan
  constexpr int PER = SR_NP / 256;
  int cnt = 0;
  unsigned hmask = 0u;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int p = tid * PER + q;
    const bool h = p < np && (p == 0 || (keys[p] >> SR_PB) != (keys[p - 1] >> SR_PB));
    hmask |= (h ? 1u : 0u) << q;
    cnt += h ? 1 : 0;
  }
  int incl = cnt;
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  int woff = 0;
  for (int w = 0; w < wave; ++w) woff += s_wsum[w];
  int seg = woff + incl - cnt - 1;  // index of the run the position before this thread's first belongs to
  const int64_t ub = (int64_t)blockIdx.x * SR_NP;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int p = tid * PER + q;
    if (p >= np) break;
    const uint64_t key = keys[p];
    if (hmask & (1u << q)) {
      ++seg;
      const int64_t row = (int64_t)(key >> SR_PB);
      const int owner = (int)(row % W);
      u_row[ub + seg] = row;
      u_slot[ub + seg] = (owner << 16) | atomicAdd(&s_own[owner], 1);
    }
    inv_local[base + (int)(key & (SR_NP - 1))] = seg;
  }
  __syncthreads();
  for (int o = tid; o < W; o += 256) blk_cnt[(int64_t)blockIdx.x * W + o] = s_own[o];
  if (tid == 255) u_cnt[blockIdx.x] = woff + incl;
}

// one workgroup: per owner, blk_off[b][o] = sum of blk_cnt[b' < b][o]; send_cnt[o] = the
// owner's total; owner_base[o] = the totals of the owners before it
__global__ __launch_bounds__(256) void shard_offsets_k(const int32_t* __restrict__ blk_cnt, int nblk, int W,
                                                       int32_t* __restrict__ blk_off, int64_t* __restrict__ send_cnt,
                                                       int64_t* __restrict__ owner_base) {
  __shared__ int s_sum[256];
  __shared__ int64_t s_tot;
  const int tid = threadIdx.x;
  const int per = (nblk + 255) / 256;
  const int b0 = min(tid * per, nblk), b1 = min(b0 + per, nblk);
  int64_t run_base = 0;
  for (int o = 0; o < W; ++o) {
    int c = 0;
    for (int b = b0; b < b1; ++b) c += blk_cnt[(int64_t)b * W + o];
    s_sum[tid] = c;
    __syncthreads();
    for (int s = 1; s < 256; s <<= 1) {  // inclusive Hillis-Steele scan
      const int v = tid >= s ? s_sum[tid - s] : 0;
      __syncthreads();
      s_sum[tid] += v;
      __syncthreads();
    }
    int off = s_sum[tid] - c;
    for (int b = b0; b < b1; ++b) {
      blk_off[(int64_t)b * W + o] = off;
      off += blk_cnt[(int64_t)b * W + o];
    }
    if (tid == 255) {
      send_cnt[o] = s_sum[255];
      owner_base[o] = run_base;
      s_tot = run_base + s_sum[255];
    }
    __syncthreads();
    run_base = s_tot;
    __syncthreads();
  }
  if (tid == 0) owner_base[W] = run_base;  // the total request count
}

__global__ __launch_bounds__(256) void shard_scatter_k(const int64_t* __restrict__ u_row,
                                                       const int32_t* __restrict__ u_slot,
                                                       const int32_t* __restrict__ u_cnt,
                                                       const int32_t* __restrict__ blk_off,
                                                       const int64_t* __restrict__ owner_base, int W,
                                                       const int32_t* __restrict__ inv_local, int64_t n_pairs,
                                                       int64_t* __restrict__ send_rows, int64_t* __restrict__ inv) {
  __shared__ int64_t u_pos[SR_NP];
  const int tid = threadIdx.x;
  const int64_t ub = (int64_t)blockIdx.x * SR_NP;
  const int nu = u_cnt[blockIdx.x];
  for (int u = tid; u < nu; u += 256) {
    const int sl = u_slot[ub + u];
    const int o = sl >> 16;
    const int64_t pos = owner_base[o] + blk_off[(int64_t)blockIdx.x * W + o] + (sl & 0xffff);
    send_rows[pos] = u_row[ub + u];
    u_pos[u] = pos;
  }
  __syncthreads();
  const int np = (int)min((int64_t)SR_NP, n_pairs - ub);
  for (int p = tid; p < np; p += 256) inv[ub + p] = u_pos[inv_local[ub + p]];
}

// out[i] = shard[rows[i] / W] for i < *count (rows of rb bytes, 16-B vectors)
__global__ __launch_bounds__(256) void shard_gather_k(const unsigned char* __restrict__ shard, int64_t n_local,
                                                      int rb, const int64_t* __restrict__ rows,
                                                      const int64_t* __restrict__ count, int64_t cap, int W,
                                                      unsigned char* __restrict__ out) {
  const int64_t n = count ? min(*count, cap) : cap;
  const int vpr = rb / 16;
  const int64_t total = n * vpr;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / vpr;
    const int v = (int)(i - r * vpr);
    const int64_t loc = rows[r] / W;
    u32x4 val = {0u, 0u, 0u, 0u};
    if (loc >= 0 && loc < n_local) val = *reinterpret_cast<const u32x4*>(shard + loc * rb + v * 16);
    *reinterpret_cast<u32x4*>(out + r * rb + v * 16) = val;
  }
}

}  // namespace lthm

using namespace lthm;

extern "C" int64_t lthm_shard_route_ws_bytes(int64_t n_pairs, int32_t world) {
  if (n_pairs < 0 || world <= 0) return -1;
  const int64_t nblk = (n_pairs + SR_NP - 1) / SR_NP;
  // u_row (8) + u_slot (4) + inv_local (4) per key slot, u_cnt + blk_cnt + blk_off per workgroup
  return nblk * SR_NP * 16 + nblk * 4 + 2 * nblk * world * 4 + 64;
}

extern "C" int lthm_shard_route(const int64_t* ids, int64_t n_items, int32_t K, int64_t P, int32_t world,
                                int64_t* send_rows, int64_t* send_counts, int64_t* owner_base, int64_t* inv,
                                void* workspace, int64_t ws_bytes, void* stream) {
  LTHM_REQUIRE(n_items >= 0 && K > 0 && K <= 64 && P > 0 && world > 0 && world <= SR_MAXW);
  LTHM_REQUIRE(P <= (1ll << (64 - SR_PB - 1)));
  const int64_t n_pairs = n_items * K;
  LTHM_REQUIRE(workspace && ws_bytes >= lthm_shard_route_ws_bytes(n_pairs, world));
  hipStream_t s = (hipStream_t)stream;
  if (n_pairs == 0) {
    if (hipMemsetAsync(send_counts, 0, world * 8, s) != hipSuccess) return (int)hipGetLastError();
    if (hipMemsetAsync(owner_base, 0, (world + 1) * 8, s) != hipSuccess) return (int)hipGetLastError();
    return 0;
  }
  const int64_t nblk = (n_pairs + SR_NP - 1) / SR_NP;
  LTHM_REQUIRE(nblk < (1ll << 31));
  char* w = (char*)workspace;
  int64_t* u_row = (int64_t*)w;
  int32_t* u_slot = (int32_t*)(w + nblk * SR_NP * 8);
  int32_t* inv_local = (int32_t*)(w + nblk * SR_NP * 12);
  int32_t* u_cnt = (int32_t*)(w + nblk * SR_NP * 16);
  int32_t* blk_cnt = u_cnt + nblk;
  int32_t* blk_off = blk_cnt + nblk * world;
  hipLaunchKernelGGL(shard_dedup_k, dim3((int)nblk), dim3(256), 0, s, ids, n_pairs, K, P, world, u_row, u_slot, u_cnt,
                     blk_cnt, inv_local);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL(shard_offsets_k, dim3(1), dim3(256), 0, s, (const int32_t*)blk_cnt, (int)nblk, world, blk_off,
                     send_counts, owner_base);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL(shard_scatter_k, dim3((int)nblk), dim3(256), 0, s, (const int64_t*)u_row, (const int32_t*)u_slot,
                     (const int32_t*)u_cnt, (const int32_t*)blk_off, (const int64_t*)owner_base, world,
                     (const int32_t*)inv_local, n_pairs, send_rows, inv);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_shard_gather(const void* shard, int64_t n_local, int32_t row_bytes, const int64_t* rows,
                                 const int64_t* count, int64_t cap, int32_t world, void* out, void* stream) {
  LTHM_REQUIRE(n_local >= 0 && row_bytes > 0 && row_bytes % 16 == 0 && cap >= 0 && world > 0);
  if (cap == 0) return 0;
  const int64_t work = cap * (row_bytes / 16);
  hipLaunchKernelGGL(shard_gather_k, dim3(grid_for(work, 256, 256 * 16)), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned char*)shard, n_local, row_bytes, rows, count, cap, world, (unsigned char*)out);
  LTHM_CHECK_LAUNCH();
  return 0;
}
