// Fused dedup + row-wise Adagrad of a KShift table (include/lthm.h lthm_kshift_adagrad_fused).
//
// The item-embedding generator trains its KShift tables with `loss.backward(); optim.step()` and
// torch.optim.Adagrad, nothing between the two (embedding_module_gen.py:137,151-153 and :97-99
// for the mask model), so the table's gradient never has to exist as a tensor: each touched
// row's gradient is formed and consumed by its Adagrad update in one pass.
//
//   kag_prep_k       per item: the pooled-sum gradient g_i (the KShift backward's step 1:
//                    dy / sqrt(K), dy, or the F.normalize backward) into a compact [n, D]
//                    buffer; the K (row, item) pairs of the item as 32-bit keys / values
//   radix sort       hipcub::DeviceRadixSort::SortPairs (stable: a row's pairs stay in item
//                    order), rows as keys over the bits F * P needs
//   kag_heads_k      segment heads of the sorted rows, compacted by hipcub::DeviceSelect::Flagged
//   kag_apply_k      one lane group per row (segment) of <= KAG_CH pairs: the row's W / state
//                    loads issued first, the g_i of its pairs summed in sorted order (loads four
//                    pairs ahead), the update s += g g; W -= clr g / (sqrt(s) + eps) stored;
//                    longer rows are listed
//   kag_long_*       rows of > KAG_CH pairs (the reference's arithmetic-shift quirk sends the
//                    shifted rows of every negative id to row P - 1: about half the pairs of
//                    hashed ids) in chunks of KAG_CH pairs over the whole grid, the chunk sums
//                    combined by one workgroup in 16 contiguous groups, the group sums in order
//
// Every sum runs in a fixed order, so the result is deterministic; oracle/ref.py
// (kshift_adagrad_ref) restates the order and the unfused f32 update.  Nothing here is
// atomic on the table: each row is written by exactly one lane group.
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "common.hpp"

namespace lthm {

constexpr int KAG_CH = 256;  // pairs per chunk; rows with more pairs take the long path
constexpr int KAG_LW = 16;   // waves of the long-row combine workgroup

// per item (LPI lanes each, 64 / LPI items per wave, grid-stride): g_i and the item's K (row,
// item) pairs; LPI >= K and D <= 4 LPI (column d = lane + LPI q)
template <typename TY, typename TO, int LPI>
__global__ __launch_bounds__(256) void kag_prep_k(const int64_t* __restrict__ ids, int64_t n_items, int F,
                                                  const TY* __restrict__ dY, const TO* __restrict__ out,
                                                  const float* __restrict__ norms, int64_t P, int D, int K, int mode,
                                                  float scale, float* __restrict__ g, uint32_t* __restrict__ keys,
                                                  uint32_t* __restrict__ vals) {
  constexpr int IPW = 64 / LPI;
  const int l = threadIdx.x % LPI, slot = (threadIdx.x & 63) / LPI;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * IPW; base < n_items; base += nw * IPW) {
    const int64_t it = base + slot;
    if (it >= n_items) continue;  // a whole lane group: its shuffles stay inside the group
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int d = l + LPI * q;
      const float dy = d < D ? Elem<TY>::ld(dY + it * D + d) : 0.f;
      v[q] = mode == LTHM_KSHIFT_SCALE ? dy / scale : dy;
    }
    if (mode == LTHM_KSHIFT_NORMALIZE) {
      // g = (dy - y (y . dy)) / max(|x|, eps): kshift_bwd_dense_k's arithmetic
      float dot = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = l + LPI * q;
        if (d < D) dot += Elem<TO>::ld(out + it * D + d) * v[q];
      }
      dot = group_sum<LPI>(dot);
      const float nrm = norms[it];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = l + LPI * q;
        if (d < D) v[q] = nrm > 1e-12f ? (v[q] - Elem<TO>::ld(out + it * D + d) * dot) / nrm : v[q] / 1e-12f;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int d = l + LPI * q;
      if (d < D) g[it * D + d] = v[q];
    }
    if (l < K) {
      const int64_t row = (F > 1 ? (it % F) * P : 0) + kshift_row(ids[it], l, P);
      keys[it * K + l] = (uint32_t)row;
      vals[it * K + l] = (uint32_t)it;
    }
  }
}

__global__ __launch_bounds__(256) void kag_heads_k(const uint32_t* __restrict__ skeys, int64_t N,
                                                   uint8_t* __restrict__ heads) {
  for (int64_t j = blockIdx.x * 256ll + threadIdx.x; j < N; j += (int64_t)gridDim.x * 256)
    heads[j] = (j == 0 || skeys[j] != skeys[j - 1]) ? 1 : 0;
}

// column slots of a lane: slot q of lane gl covers columns (gl + LG q) CW .. + CW - 1 (CW = 4: one
// 16-B access, D % 4 == 0), none past D
template <int CW>
__device__ __forceinline__ void kag_ld(const float* __restrict__ p, int c0, int D, float* v) {
  if constexpr (CW == 4) {
    const f32x4 x = c0 < D ? *reinterpret_cast<const f32x4*>(p + c0) : f32x4{0.f, 0.f, 0.f, 0.f};
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  } else {
    v[0] = c0 < D ? p[c0] : 0.f;
  }
}
template <int CW>
__device__ __forceinline__ void kag_st(float* __restrict__ p, int c0, int D, const float* v) {
  if (c0 >= D) return;
  if constexpr (CW == 4) *reinterpret_cast<f32x4*>(p + c0) = f32x4{v[0], v[1], v[2], v[3]};
  else p[c0] = v[0];
}

// acc += g[item] over the lane's column slots for the pairs [j0, j1) in order: eight pairs' g
// rows in flight, the next eight pairs' items loaded one batch ahead (a long chunk is then one
// memory latency per eight pairs, not two per pair group), a tail of < 8 pairs one by one
template <int LG, int NQ, int CW>
__device__ __forceinline__ void kag_sum(const uint32_t* __restrict__ svals, const float* __restrict__ g, int D,
                                        int gl, uint32_t j0, uint32_t j1, float (&acc)[NQ * CW]) {
  uint32_t j = j0;
  if (j + 8 <= j1) {
    uint32_t nv[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) nv[p] = svals[j + p];
    for (; j + 8 <= j1; j += 8) {
      uint32_t cur[8];
#pragma unroll
      for (int p = 0; p < 8; ++p) cur[p] = nv[p];
      if (j + 16 <= j1) {
#pragma unroll
        for (int p = 0; p < 8; ++p) nv[p] = svals[j + 8 + p];
      }
      float x[8][NQ * CW];
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const float* gr = g + (int64_t)cur[p] * D;
#pragma unroll
        for (int q = 0; q < NQ; ++q) kag_ld<CW>(gr, (gl + LG * q) * CW, D, x[p] + q * CW);
      }
#pragma unroll
      for (int p = 0; p < 8; ++p)
#pragma unroll
        for (int e = 0; e < NQ * CW; ++e) acc[e] = __fadd_rn(acc[e], x[p][e]);
    }
  }
  for (; j < j1; ++j) {
    const float* gr = g + (int64_t)svals[j] * D;
    float x[NQ * CW];
#pragma unroll
    for (int q = 0; q < NQ; ++q) kag_ld<CW>(gr, (gl + LG * q) * CW, D, x + q * CW);
#pragma unroll
    for (int e = 0; e < NQ * CW; ++e) acc[e] = __fadd_rn(acc[e], x[e]);
  }
}

// correctly rounded f32 square root: v_sqrt_f32 is within 1 ulp; its neighbours' exact
// residuals x - s' s (one fma each) pick the rounded root
__device__ __forceinline__ float kag_sqrt_rn(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float dn = __int_as_float(__float_as_int(s) - 1), up = __int_as_float(__float_as_int(s) + 1);
  const float vp = __builtin_fmaf(-dn, s, x), vs = __builtin_fmaf(-up, s, x);
  const float r = vp <= 0.f ? dn : s;
  return vs > 0.f ? up : r;
}

// torch.optim.Adagrad's element update (lr_decay in clr, no weight decay), every operation
// rounded on its own (no contraction into fma): s = s + g * g ; W = W - (clr * g) / (sqrt(s) + eps)
__device__ __forceinline__ void kag_update(float& w, float& s, float gr, float clr, float eps) {
#pragma clang fp contract(off)
  const float gg = gr * gr;
  s = s + gg;
  const float den = kag_sqrt_rn(s) + eps;
  const float num = clr * gr;
  w = w - num / den;
}

// one LG-lane group per segment (grid-stride); segments of more than KAG_CH pairs are listed
template <int LG, int NQ, int CW>
__global__ __launch_bounds__(256) void kag_apply_k(const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ svals,
                                                   const uint32_t* __restrict__ starts, const int* __restrict__ nseg_p,
                                                   int64_t N, const float* __restrict__ g, int D, float* __restrict__ W,
                                                   float* __restrict__ S, float clr, float eps,
                                                   uint32_t* __restrict__ longlist, int* __restrict__ nlong) {
  const int nseg = *nseg_p;
  const int gl = threadIdx.x % LG;
  const int64_t ngrp = (int64_t)gridDim.x * (256 / LG);
  int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LG;
  // the next segment's bounds are loaded one iteration ahead (the grid-stride loop is a chain
  // of dependent loads: bounds -> row and items -> W / state / gradients)
  uint32_t n0 = 0, n1 = 0;
  if (u < nseg) {
    n0 = starts[u];
    n1 = u + 1 < nseg ? starts[u + 1] : (uint32_t)N;
  }
  for (; u < nseg; u += ngrp) {
    const uint32_t s0 = n0, s1 = n1;
    const int64_t un = u + ngrp;
    if (un < nseg) {
      n0 = starts[un];
      n1 = un + 1 < nseg ? starts[un + 1] : (uint32_t)N;
    }
    if (s1 - s0 > (uint32_t)KAG_CH) {
      if (gl == 0) longlist[atomicAdd(nlong, 1)] = (uint32_t)u;
      continue;
    }
    const int64_t row = skeys[s0];
    float* wr = W + row * D;
    float* sr = S + row * D;
    float w[NQ * CW], s[NQ * CW], acc[NQ * CW];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      kag_ld<CW>(wr, (gl + LG * q) * CW, D, w + q * CW);
      kag_ld<CW>(sr, (gl + LG * q) * CW, D, s + q * CW);
    }
#pragma unroll
    for (int e = 0; e < NQ * CW; ++e) acc[e] = 0.f;
    kag_sum<LG, NQ, CW>(svals, g, D, gl, s0, s1, acc);
#pragma unroll
    for (int e = 0; e < NQ * CW; ++e) kag_update(w[e], s[e], acc[e], clr, eps);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      kag_st<CW>(sr, (gl + LG * q) * CW, D, s + q * CW);
      kag_st<CW>(wr, (gl + LG * q) * CW, D, w + q * CW);
    }
  }
}

// one workgroup: chunk counts of the listed long segments -> exclusive prefix lpref[0 .. nl]
__global__ __launch_bounds__(1024) void kag_long_prep_k(const uint32_t* __restrict__ starts, const int* __restrict__ nseg_p,
                                                        int64_t N, const uint32_t* __restrict__ longlist,
                                                        const int* __restrict__ nlong, uint32_t* __restrict__ lpref) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t base;
  const int nseg = *nseg_p, nl = *nlong;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) base = 0;
  __syncthreads();
  for (int i0 = 0; i0 < nl; i0 += 1024) {
    const int i = i0 + tid;
    uint32_t m = 0;
    if (i < nl) {
      const uint32_t u = longlist[i];
      const uint32_t s0 = starts[u], s1 = (int)u + 1 < nseg ? starts[u + 1] : (uint32_t)N;
      m = (s1 - s0 + KAG_CH - 1) / KAG_CH;
    }
    uint32_t incl = m;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(incl, o, 64);
      if (lane >= o) incl += x;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t woff = base;
    for (int w = 0; w < wave; ++w) woff += wsum[w];
    if (i < nl) lpref[i] = woff + incl - m;
    __syncthreads();
    if (tid == 1023) base = woff + incl;
    __syncthreads();
  }
  if (tid == 0) lpref[nl] = base;
}

// chunk c of the long segments (grid-stride, one LG-lane group per chunk): its pairs' sum
template <int LG, int NQ, int CW>
__global__ __launch_bounds__(256) void kag_chunk_k(const uint32_t* __restrict__ svals, const uint32_t* __restrict__ starts,
                                                   const int* __restrict__ nseg_p, int64_t N,
                                                   const uint32_t* __restrict__ longlist, const int* __restrict__ nlong,
                                                   const uint32_t* __restrict__ lpref, const float* __restrict__ g, int D,
                                                   float* __restrict__ part) {
  const int nseg = *nseg_p, nl = *nlong;
  if (nl == 0) return;
  const uint32_t nch = lpref[nl];
  const int gl = threadIdx.x % LG;
  const int64_t ngrp = (int64_t)gridDim.x * (256 / LG);
  for (int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LG; c < nch; c += ngrp) {
    int lo = 0, hi = nl - 1;  // the last i with lpref[i] <= c
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (lpref[mid] <= (uint32_t)c) lo = mid;
      else hi = mid - 1;
    }
    const uint32_t u = longlist[lo];
    const uint32_t send = (int)u + 1 < nseg ? starts[u + 1] : (uint32_t)N;
    const uint32_t s0 = starts[u] + ((uint32_t)c - lpref[lo]) * KAG_CH;
    const uint32_t s1 = min(s0 + (uint32_t)KAG_CH, send);
    float acc[NQ * CW];
#pragma unroll
    for (int e = 0; e < NQ * CW; ++e) acc[e] = 0.f;
    kag_sum<LG, NQ, CW>(svals, g, D, gl, s0, s1, acc);
#pragma unroll
    for (int q = 0; q < NQ; ++q) kag_st<CW>(part + c * D, (gl + LG * q) * CW, D, acc + q * CW);
  }
}

// one workgroup per long segment (grid-stride): wave w sums the chunk sums
// [w m / 16, (w + 1) m / 16) in order, wave 0 the 16 group sums in order, then the update
__global__ __launch_bounds__(64 * KAG_LW) void kag_long_apply_k(const uint32_t* __restrict__ skeys,
                                                                const uint32_t* __restrict__ starts,
                                                                const uint32_t* __restrict__ longlist,
                                                                const int* __restrict__ nlong,
                                                                const uint32_t* __restrict__ lpref,
                                                                const float* __restrict__ part, int D,
                                                                float* __restrict__ W, float* __restrict__ S, float clr,
                                                                float eps) {
  __shared__ float red[KAG_LW][256];
  const int nl = *nlong;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = blockIdx.x; i < nl; i += gridDim.x) {
    const uint32_t b = lpref[i];
    const int64_t m = lpref[i + 1] - b;
    const int64_t c0 = wave * m / KAG_LW, c1 = (wave + 1) * m / KAG_LW;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t c = c0;
    for (; c + 4 <= c1; c += 4) {
      float x[4][4];
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int d = lane + 64 * q;
          x[p][q] = d < D ? part[(b + c + p) * (int64_t)D + d] : 0.f;
        }
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = __fadd_rn(acc[q], x[p][q]);
    }
    for (; c < c1; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = lane + 64 * q;
        acc[q] = __fadd_rn(acc[q], d < D ? part[(b + c) * (int64_t)D + d] : 0.f);
      }
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][lane + 64 * q] = acc[q];
    __syncthreads();
    if (wave == 0) {
      const int64_t row = skeys[starts[longlist[i]]];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = lane + 64 * q;
        if (d >= D) continue;
        float t = 0.f;
        for (int w = 0; w < KAG_LW; ++w) t = __fadd_rn(t, red[w][d]);
        float wv = W[row * D + d], sv = S[row * D + d];
        kag_update(wv, sv, t, clr, eps);
        S[row * D + d] = sv;
        W[row * D + d] = wv;
      }
    }
    __syncthreads();  // red is reused by the next segment
  }
}

// workspace layout (256-B aligned sections)
struct KagLayout {
  size_t cnt, g, keys, vals, skeys, svals, heads, starts, longlist, lpref, part, sort_tmp, sel_tmp, total;
  size_t sort_bytes, sel_bytes;
};

static size_t kag_al(size_t x) { return (x + 255) & ~(size_t)255; }

static int kag_layout(int64_t n_items, int K, int D, int end_bit, KagLayout* L) {
  const int64_t N = n_items * K;
  const int64_t nlong_max = N / (KAG_CH + 1) + 1, nch_max = 2 * (N / KAG_CH) + 2;
  size_t sort_bytes = 0, sel_bytes = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)N, 0, end_bit,
                                         (hipStream_t)0) != hipSuccess)
    return -1;
  if (hipcub::DeviceSelect::Flagged(nullptr, sel_bytes, hipcub::CountingInputIterator<uint32_t>(0),
                                    (const uint8_t*)nullptr, (uint32_t*)nullptr, (int*)nullptr, (int)N,
                                    (hipStream_t)0) != hipSuccess)
    return -1;
  size_t o = 0;
  L->cnt = o;      o += kag_al(4 * sizeof(int));
  L->g = o;        o += kag_al((size_t)n_items * D * 4);
  L->keys = o;     o += kag_al((size_t)N * 4);
  L->vals = o;     o += kag_al((size_t)N * 4);
  L->skeys = o;    o += kag_al((size_t)N * 4);
  L->svals = o;    o += kag_al((size_t)N * 4);
  L->heads = o;    o += kag_al((size_t)N);
  L->starts = o;   o += kag_al((size_t)N * 4);
  L->longlist = o; o += kag_al((size_t)nlong_max * 4);
  L->lpref = o;    o += kag_al((size_t)(nlong_max + 1) * 4);
  L->part = o;     o += kag_al((size_t)nch_max * D * 4);
  L->sort_tmp = o; o += kag_al(sort_bytes);
  L->sel_tmp = o;  o += kag_al(sel_bytes);
  L->total = o;
  L->sort_bytes = sort_bytes;
  L->sel_bytes = sel_bytes;
  return 0;
}

static int kag_cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

template <int LG, int NQ, int CW>
static int kag_launch_groups(const KagLayout& L, unsigned char* w, int64_t N, int D, float* W, float* S, float clr,
                             float eps, hipStream_t s) {
  const uint32_t* skeys = (const uint32_t*)(w + L.skeys);
  const uint32_t* svals = (const uint32_t*)(w + L.svals);
  const uint32_t* starts = (const uint32_t*)(w + L.starts);
  const int* cnt = (const int*)(w + L.cnt);
  const float* g = (const float*)(w + L.g);
  uint32_t* longlist = (uint32_t*)(w + L.longlist);
  uint32_t* lpref = (uint32_t*)(w + L.lpref);
  float* part = (float*)(w + L.part);
  // workgroups per CU of the row / chunk passes (latency-bound: more groups in flight);
  // LTHM_KAG_BPC overrides (A/B, profiles/r06p/: 8 / 16 / 32 per CU -> 0.658 / 0.602 / 0.592 ms per
  // generator step)
  static const int bpc = getenv("LTHM_KAG_BPC") ? atoi(getenv("LTHM_KAG_BPC")) : 32;
  const int cap = kag_cu_count() * (bpc > 0 ? bpc : 32);
  const int gpb = 256 / LG;
  hipLaunchKernelGGL((kag_apply_k<LG, NQ, CW>), dim3(grid_for(N, gpb, cap)), dim3(256), 0, s, skeys, svals, starts, cnt, N,
                     g, D, W, S, clr, eps, longlist, (int*)(cnt + 1));
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL(kag_long_prep_k, dim3(1), dim3(1024), 0, s, starts, cnt, N, (const uint32_t*)longlist, cnt + 1,
                     lpref);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL((kag_chunk_k<LG, NQ, CW>), dim3(grid_for(2 * (N / KAG_CH) + 2, gpb, cap)), dim3(256), 0, s, svals,
                     starts, cnt, N, (const uint32_t*)longlist, cnt + 1, (const uint32_t*)lpref, g, D, part);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL(kag_long_apply_k, dim3(grid_for(N / (KAG_CH + 1) + 1, 1, kag_cu_count() * 2)),
                     dim3(64 * KAG_LW), 0, s, skeys, starts, (const uint32_t*)longlist, cnt + 1,
                     (const uint32_t*)lpref, (const float*)part, D, W, S, clr, eps);
  LTHM_CHECK_LAUNCH();
  return 0;
}

static int kag_end_bit(int64_t rows) {
  int b = 1;
  while (b < 32 && ((int64_t)1 << b) < rows) ++b;
  return b;
}

}  // namespace lthm

using namespace lthm;

extern "C" int64_t lthm_kshift_adagrad_ws_bytes(int64_t n_items, int32_t K, int32_t D) {
  if (n_items < 0 || K <= 0 || K > 64 || D <= 0 || D > 256 || n_items * K >= ((int64_t)1 << 31)) return -1;
  KagLayout L;
  if (kag_layout(n_items, K, D, 32, &L) != 0) return -1;
  return (int64_t)L.total;
}

extern "C" int lthm_kshift_adagrad_fused(const int64_t* ids, int64_t n, int32_t F, const void* dY, int32_t dy_dtype,
                                         const void* out, int32_t out_dtype, const float* norms, int64_t P, int32_t D,
                                         int32_t K, int32_t mode, float* W, float* state_sum, float clr, float eps,
                                         void* workspace, int64_t ws_bytes, void* stream) {
  LTHM_REQUIRE(P > 0 && K > 0 && K <= 64 && D > 0 && D <= 256 && n >= 0 && F >= 1);
  LTHM_REQUIRE(mode >= 0 && mode <= 2);
  LTHM_REQUIRE(mode != LTHM_KSHIFT_NORMALIZE || (out != nullptr && norms != nullptr));
  LTHM_REQUIRE((int64_t)F * P <= ((int64_t)1 << 32));
  const int64_t items = n * (int64_t)F, N = items * K;
  LTHM_REQUIRE(N < ((int64_t)1 << 31));
  if (items == 0) return 0;
  LTHM_REQUIRE(ids && dY && W && state_sum && workspace);
  LTHM_REQUIRE(((uintptr_t)workspace & 255) == 0);
  const int end_bit = kag_end_bit((int64_t)F * P);
  KagLayout L;
  LTHM_REQUIRE(kag_layout(items, K, D, end_bit, &L) == 0);
  LTHM_REQUIRE(ws_bytes >= (int64_t)L.total);
  hipStream_t s = (hipStream_t)stream;
  unsigned char* w = (unsigned char*)workspace;
  LTHM_REQUIRE(hipMemsetAsync(w + L.cnt, 0, 4 * sizeof(int), s) == hipSuccess);
  const float scale = (float)__builtin_sqrt((double)K);
  float* g = (float*)(w + L.g);
  uint32_t* keys = (uint32_t*)(w + L.keys);
  uint32_t* vals = (uint32_t*)(w + L.vals);
  // lanes per item: >= K and >= D / 4, a power of two in [16, 64]
  const int need = K > (D + 3) / 4 ? K : (D + 3) / 4;
  const int lpi = need <= 16 ? 16 : need <= 32 ? 32 : 64;
  const int pg = grid_for(items, 4 * (64 / lpi), kag_cu_count() * 16);
#define KAG_PREP_L(TY, TO, LPI)                                                                                   \
  hipLaunchKernelGGL((kag_prep_k<TY, TO, LPI>), dim3(pg), dim3(256), 0, s, ids, items, F, (const TY*)dY,           \
                     (const TO*)out, norms, P, D, K, mode, scale, g, keys, vals)
#define KAG_PREP(TY, TO)                      \
  do {                                        \
    if (lpi == 16) KAG_PREP_L(TY, TO, 16);    \
    else if (lpi == 32) KAG_PREP_L(TY, TO, 32); \
    else KAG_PREP_L(TY, TO, 64);              \
  } while (0)
  const int od = out ? out_dtype : LTHM_F32;
  if (dy_dtype == LTHM_F32 && od == LTHM_F32) KAG_PREP(float, float);
  else if (dy_dtype == LTHM_F32 && od == LTHM_BF16) KAG_PREP(float, bf16_t);
  else if (dy_dtype == LTHM_BF16 && od == LTHM_F32) KAG_PREP(bf16_t, float);
  else if (dy_dtype == LTHM_BF16 && od == LTHM_BF16) KAG_PREP(bf16_t, bf16_t);
  else return (int)hipErrorInvalidValue;
#undef KAG_PREP
#undef KAG_PREP_L
  LTHM_CHECK_LAUNCH();
  uint32_t* skeys = (uint32_t*)(w + L.skeys);
  uint32_t* svals = (uint32_t*)(w + L.svals);
  size_t sb = L.sort_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(w + L.sort_tmp, sb, (const uint32_t*)keys, skeys, (const uint32_t*)vals, svals,
                                         (int)N, 0, end_bit, s) != hipSuccess)
    return (int)hipErrorLaunchFailure;
  uint8_t* heads = (uint8_t*)(w + L.heads);
  hipLaunchKernelGGL(kag_heads_k, dim3(grid_for(N, 256, kag_cu_count() * 8)), dim3(256), 0, s, (const uint32_t*)skeys, N,
                     heads);
  LTHM_CHECK_LAUNCH();
  size_t selb = L.sel_bytes;
  if (hipcub::DeviceSelect::Flagged(w + L.sel_tmp, selb, hipcub::CountingInputIterator<uint32_t>(0),
                                    (const uint8_t*)heads, (uint32_t*)(w + L.starts), (int*)(w + L.cnt), (int)N,
                                    s) != hipSuccess)
    return (int)hipErrorLaunchFailure;
  // lane groups sized to the row: 16-B column slots when D % 4 == 0 and W / state_sum are 16-B
  // aligned (D / 4 lanes rounded up to a power of two: D = 32 -> 8 lanes, 8 rows per wave in
  // flight), else one column per slot
  if (D % 4 == 0 && ((uintptr_t)W % 16) == 0 && ((uintptr_t)state_sum % 16) == 0) {
    if (D <= 4) return kag_launch_groups<1, 1, 4>(L, w, N, D, W, state_sum, clr, eps, s);
    if (D <= 8) return kag_launch_groups<2, 1, 4>(L, w, N, D, W, state_sum, clr, eps, s);
    if (D <= 16) return kag_launch_groups<4, 1, 4>(L, w, N, D, W, state_sum, clr, eps, s);
    if (D <= 32) return kag_launch_groups<8, 1, 4>(L, w, N, D, W, state_sum, clr, eps, s);
    if (D <= 64) return kag_launch_groups<16, 1, 4>(L, w, N, D, W, state_sum, clr, eps, s);
    if (D <= 128) return kag_launch_groups<32, 1, 4>(L, w, N, D, W, state_sum, clr, eps, s);
    return kag_launch_groups<64, 1, 4>(L, w, N, D, W, state_sum, clr, eps, s);
  }
  if (D <= 4) return kag_launch_groups<4, 1, 1>(L, w, N, D, W, state_sum, clr, eps, s);
  if (D <= 8) return kag_launch_groups<8, 1, 1>(L, w, N, D, W, state_sum, clr, eps, s);
  if (D <= 16) return kag_launch_groups<16, 1, 1>(L, w, N, D, W, state_sum, clr, eps, s);
  if (D <= 32) return kag_launch_groups<32, 1, 1>(L, w, N, D, W, state_sum, clr, eps, s);
  if (D <= 64) return kag_launch_groups<64, 1, 1>(L, w, N, D, W, state_sum, clr, eps, s);
  if (D <= 128) return kag_launch_groups<64, 2, 1>(L, w, N, D, W, state_sum, clr, eps, s);
  return kag_launch_groups<64, 4, 1>(L, w, N, D, W, state_sum, clr, eps, s);
}
