// KShift / Flat embedding gather+pool (forward) and LDS-dedup segmented
// backward for gfx950.
//
// Reference semantics: commons/layers.py:125-185 (KShiftEmbedding),
// commons/layers.py:44-61 (FlatEmbedding = K 1, mode NONE / NORMALIZE).
//
// Forward layout: one item (id, feature) is served by a group of LPR lanes;
// lane j of the group owns bytes [j*VB, (j+1)*VB) of every table row, so each
// of the K row reads is one fully coalesced 16-byte-per-lane access.  The K row
// indices of an item are computed once (spread over the group's lanes) and
// staged in LDS, so the 64-bit remainder is not repeated per lane.
#include "common.hpp"

namespace lthm {

constexpr int KS_BLOCK = 256;
constexpr int KS_ROWS_LDS = 1024;  // int64 row slots per wave

__global__ __launch_bounds__(256) void kshift_rows_k(const int64_t* __restrict__ ids, int64_t n,
                                                     int64_t P, int K, int64_t* __restrict__ rows) {
  int64_t total = n * K;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t i = t / K;
    int c = (int)(t - i * K);
    rows[t] = kshift_row(ids[i], c, P);
  }
}

template <typename TW, typename TO, int VB>
__global__ __launch_bounds__(KS_BLOCK) void kshift_fwd_k(
    const int64_t* __restrict__ ids, int64_t n_items, int F, const TW* __restrict__ W, int64_t P,
    int D, int K, int mode, float scale, TO* __restrict__ out, float* __restrict__ norms, int LPR_LOG2,
    const int64_t* __restrict__ xrows) {
  constexpr int NE = VB / (int)sizeof(TW);  // elements per lane
  __shared__ int64_t rows_lds[KS_BLOCK / 64][KS_ROWS_LDS];
  const int LPR = 1 << LPR_LOG2;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int gl = lane & (LPR - 1);        // lane inside group
  const int gi = lane >> LPR_LOG2;        // group (item) inside wave
  const int IPW = 64 >> LPR_LOG2;         // items per wave
  const int IPB = IPW * (KS_BLOCK / 64);  // items per block iteration

  for (int64_t base = (int64_t)blockIdx.x * IPB; base < n_items; base += (int64_t)gridDim.x * IPB) {
    const int64_t item = base + wave * IPW + gi;
    const bool valid = item < n_items;
    int64_t id = 0, rbase = 0;
    if (valid && xrows == nullptr) {
      id = ids[item];
      rbase = (F > 1) ? (int64_t)(item % F) * P : 0;
    }
    // rows for this item (computed, or explicit rows [n, K] for gathered buffers),
    // spread over the group's lanes
    for (int c = gl; c < K; c += LPR)
      rows_lds[wave][gi * K + c] = !valid ? 0 : (xrows ? xrows[item * K + c] : rbase + kshift_row(id, c, P));
    __syncthreads();
    float acc[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) acc[e] = 0.f;
    if (valid) {
      const TW* colp = W + (size_t)gl * NE;
      int c = 0;
      // issue 8 row loads ahead, then add in order c = 0..K-1 (bit-exact order): with the
      // table far past the Infinity Cache every load is an HBM miss, so the depth of
      // independent loads per lane sets the achieved bandwidth
      for (; c + 8 <= K; c += 8) {
        float v[8][NE];
#pragma unroll
        for (int u = 0; u < 8; ++u) load_vec<TW, VB>(colp + rows_lds[wave][gi * K + c + u] * D, v[u]);
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[e] = (c == 0) ? v[0][e] : acc[e] + v[0][e];
#pragma unroll
        for (int u = 1; u < 8; ++u)
#pragma unroll
          for (int e = 0; e < NE; ++e) acc[e] += v[u][e];
      }
      for (; c + 4 <= K; c += 4) {
        float v0[NE], v1[NE], v2[NE], v3[NE];
        const int64_t r0 = rows_lds[wave][gi * K + c], r1 = rows_lds[wave][gi * K + c + 1];
        const int64_t r2 = rows_lds[wave][gi * K + c + 2], r3 = rows_lds[wave][gi * K + c + 3];
        load_vec<TW, VB>(colp + r0 * D, v0);
        load_vec<TW, VB>(colp + r1 * D, v1);
        load_vec<TW, VB>(colp + r2 * D, v2);
        load_vec<TW, VB>(colp + r3 * D, v3);
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[e] = (c == 0) ? v0[e] : acc[e] + v0[e];
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[e] += v1[e];
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[e] += v2[e];
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[e] += v3[e];
      }
      for (; c < K; ++c) {
        float v0[NE];
        load_vec<TW, VB>(colp + rows_lds[wave][gi * K + c] * D, v0);
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[e] = (c == 0) ? v0[e] : acc[e] + v0[e];
      }
    }
    if (mode == LTHM_KSHIFT_NORMALIZE) {
      float ss = 0.f;
#pragma unroll
      for (int e = 0; e < NE; ++e) ss += acc[e] * acc[e];
      for (int o = LPR >> 1; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      const float nrm = sqrtf(ss);
      const float den = fmaxf(nrm, 1e-12f);
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[e] = acc[e] / den;
      if (valid && norms != nullptr && gl == 0) norms[item] = nrm;
    } else if (mode == LTHM_KSHIFT_SCALE) {
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[e] = acc[e] / scale;
    }
    if (valid) store_vec<TO, NE>(out + item * D + (size_t)gl * NE, acc);
    __syncthreads();
  }
}

// Register-row form of kshift_fwd_k (round 6) for 16-B lane vectors and K = KT in {4, 8, 16}:
// the LPR lanes of an item's group compute its K rows (lane gl: shifts c = gl + LPR j) and every
// lane reads them across the group (ds_bpermute), so no LDS staging and no workgroup barrier sit
// between two items, and the K row loads of an item issue back to back, held as raw 16-B vectors
// (4 registers each) until the in-order sum.  Waves walk the items independently (grid-stride over
// wave iterations of 64 / LPR items); the next iteration's id load is issued before this
// iteration's row loads retire.  Same arithmetic as kshift_fwd_k: f32 sum in the order
// c = 0 .. K - 1, then / sqrt(K) or / max(|v|, 1e-12).
// LTHM_KS_NT=1 (A/B build): the row loads non-temporal (read-once rows of a table far past the caches)
#ifndef LTHM_KS_NT
#define LTHM_KS_NT 0
#endif
template <typename TW, typename TO, int KT, int LPR>
__global__ __launch_bounds__(KS_BLOCK) void kshift_fwd_reg_k(const int64_t* __restrict__ ids, int64_t n_items, int F,
                                                           const TW* __restrict__ W, int64_t P, int D, int mode,
                                                           float scale, TO* __restrict__ out,
                                                           float* __restrict__ norms) {
  constexpr int NE = 16 / (int)sizeof(TW);  // elements per lane
  constexpr int IPW = 64 / LPR;             // items per wave iteration
  constexpr int KJ = (KT + LPR - 1) / LPR;  // rows computed per lane
  const int lane = threadIdx.x & 63;
  const int gl = lane & (LPR - 1), gb = lane & ~(LPR - 1), gi = lane / LPR;
  const int64_t nwaves = (int64_t)gridDim.x * (KS_BLOCK / 64);
  int64_t w = (int64_t)blockIdx.x * (KS_BLOCK / 64) + (threadIdx.x >> 6);
  int64_t item = w * IPW + gi;
  int64_t id = item < n_items ? ids[item] : 0;
  const TW* colp = W + (size_t)gl * NE;
  for (; w * IPW < n_items; w += nwaves) {  // wave-uniform
    const bool valid = item < n_items;
    const int64_t rbase = (valid && F > 1) ? (int64_t)(item % F) * P : 0;
    uint32_t rlo[KJ], rhi[KJ];
#pragma unroll
    for (int j = 0; j < KJ; ++j) {
      const int c = gl + LPR * j;
      const int64_t r = (valid && c < KT) ? rbase + kshift_row(id, c, P) : 0;
      rlo[j] = (uint32_t)r;
      rhi[j] = (uint32_t)((uint64_t)r >> 32);
    }
    const int64_t nitem = item + nwaves * IPW;
    const int64_t nid = nitem < n_items ? ids[nitem] : 0;  // in flight behind this item's rows
    u32x4 raw[KT];
#pragma unroll
    for (int c = 0; c < KT; ++c) {
      const int src = gb + (c % LPR);
      const uint64_t r = ((uint64_t)(uint32_t)__shfl((int)rhi[c / LPR], src, 64) << 32) |
                         (uint32_t)__shfl((int)rlo[c / LPR], src, 64);
#if LTHM_KS_NT
      raw[c] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(colp + (int64_t)r * D));
#else
      raw[c] = *reinterpret_cast<const u32x4*>(colp + (int64_t)r * D);
#endif
    }
    float acc[NE];
#pragma unroll
    for (int c = 0; c < KT; ++c) {
      float v[NE];
      if constexpr (sizeof(TW) == 4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = __uint_as_float(raw[c][e]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[2 * i] = __uint_as_float(raw[c][i] << 16);
          v[2 * i + 1] = __uint_as_float(raw[c][i] & 0xffff0000u);
        }
      }
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[e] = c == 0 ? v[e] : acc[e] + v[e];
    }
    if (mode == LTHM_KSHIFT_NORMALIZE) {
      float ss = 0.f;
#pragma unroll
      for (int e = 0; e < NE; ++e) ss += acc[e] * acc[e];
#pragma unroll
      for (int o = LPR >> 1; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      const float nrm = sqrtf(ss);
      const float den = fmaxf(nrm, 1e-12f);
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[e] = acc[e] / den;
      if (valid && norms != nullptr && gl == 0) norms[item] = nrm;
    } else if (mode == LTHM_KSHIFT_SCALE) {
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[e] = acc[e] / scale;
    }
    if (valid) store_vec<TO, NE>(out + item * D + (size_t)gl * NE, acc);
    item = nitem;
    id = nid;
  }
}

// ---------------------------------------------------------------------------
// Backward: LDS-staged dedup + wave-segmented reduction + one f32 add per
// unique row per workgroup.
// ---------------------------------------------------------------------------
#ifndef LTHM_KSB_X
#define LTHM_KSB_X 0  // cost-ladder builds of kshift_bwd_dense_k (tools/build_variant.sh; wrong results)
#endif
constexpr int KB_NP = 2048;            // max (row, item) pairs per workgroup
constexpr int KB_G_FLOATS = 16384;     // LDS budget for per-item gradients (64 KiB)

template <typename TY, typename TO>
__global__ __launch_bounds__(256) void kshift_bwd_dense_k(
    const int64_t* __restrict__ ids, int64_t n_items, int F, const TY* __restrict__ dY,
    const TO* __restrict__ out, const float* __restrict__ norms, int64_t P, int D, int K, int mode,
    float scale, int CH, int NP2, float* __restrict__ dW, int32_t* __restrict__ flags, int64_t* __restrict__ list,
    unsigned long long* __restrict__ count) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* keys = reinterpret_cast<uint64_t*>(smem);                   // NP2
  float* g = reinterpret_cast<float*>(smem + (size_t)KB_NP * 8);        // CH * D
  int* segs = reinterpret_cast<int*>(smem + (size_t)KB_NP * 8 + (size_t)KB_G_FLOATS * 4);  // NP2+1
  __shared__ int s_nseg;
  __shared__ int s_wsum[4];
  __shared__ int s_nnew;                    // rows this block touched first (sparse mode)
  __shared__ unsigned long long s_base;
  __shared__ int64_t s_new[KB_NP];

  const int tid = threadIdx.x;
  for (int64_t base = (int64_t)blockIdx.x * CH; base < n_items; base += (int64_t)gridDim.x * CH) {
    const int nit = (int)min((int64_t)CH, n_items - base);
    // 1) per-item input gradient g = d(out)/d(sum) applied to dY
    for (int t = tid; t < nit * D; t += 256) {
      const int it = t / D;
      const int d = t - it * D;
      float dy = Elem<TY>::ld(dY + (base + it) * D + d);
      float v;
      if (mode == LTHM_KSHIFT_SCALE) v = dy / scale;
      else v = dy;
      g[it * D + d] = v;
    }
    __syncthreads();
    if (mode == LTHM_KSHIFT_NORMALIZE) {
      // g = (dy - y (y . dy)) / max(|x|, eps)  (eps branch: dy / eps)
      const int wave = tid >> 6, lane = tid & 63;
      for (int it = wave; it < nit; it += 4) {
        float dot = 0.f;
        for (int d = lane; d < D; d += 64) dot += Elem<TO>::ld(out + (base + it) * D + d) * g[it * D + d];
        dot = wave_sum(dot);
        const float nrm = norms[base + it];
        for (int d = lane; d < D; d += 64) {
          const float dy = g[it * D + d];
          g[it * D + d] = (nrm > 1e-12f) ? (dy - Elem<TO>::ld(out + (base + it) * D + d) * dot) / nrm
                                         : dy / 1e-12f;
        }
      }
    }
    // 2) (row, pair) keys
    const int np = nit * K;
    for (int p = tid; p < NP2; p += 256) {
      uint64_t key = ~0ull;
      if (p < np) {
        const int it = p / K;
        const int c = p - it * K;
        const int64_t item = base + it;
        const int64_t row = ((F > 1) ? (int64_t)(item % F) * P : 0) + kshift_row(ids[item], c, P);
        key = ((uint64_t)row << 12) | (uint64_t)p;
      }
      keys[p] = key;
    }
    __syncthreads();
    // 3) bitonic sort of NP2 keys in LDS (LTHM_KSB_X=1 cost-ladder build: skipped, timing only)
    for (int k = 2; k <= (LTHM_KSB_X == 1 ? 1 : NP2); k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int t = tid; t < NP2 / 2; t += 256) {
          const int i0 = 2 * t - (t & (j - 1));
          const int i1 = i0 + j;
          const bool up = ((i0 & k) == 0);
          uint64_t a = keys[i0], b = keys[i1];
          if ((a > b) == up) { keys[i0] = b; keys[i1] = a; }
        }
        __syncthreads();
      }
    }
    // 4) segment heads -> compact segment starts (block exclusive scan)
    const int PER = NP2 / 256;  // NP2 >= 256 guaranteed by host
    int hflag[KB_NP / 256];
    int cnt = 0;
    for (int q = 0; q < PER; ++q) {
      const int p = tid * PER + q;
      int h = 0;
      if (p < np) h = (p == 0) || ((keys[p] >> 12) != (keys[p - 1] >> 12));
      hflag[q] = h;
      cnt += h;
    }
    // wave inclusive scan of cnt
    const int lane = tid & 63, wave = tid >> 6;
    int incl = cnt;
    for (int o = 1; o < 64; o <<= 1) {
      int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wave; ++w) woff += s_wsum[w];
    if (tid == 255) s_nseg = woff + incl;
    int pos = woff + incl - cnt;
    for (int q = 0; q < PER; ++q) {
      if (hflag[q]) segs[pos++] = tid * PER + q;
    }
    __syncthreads();
    const int nseg = s_nseg;
    if (tid == 0) {
      segs[nseg] = np;
      s_nnew = 0;
    }
    __syncthreads();
    // 5) one group of lanes per segment: ordered sum, then one f32 add per column
    const int LPR = (D >= 64) ? 64 : D;    // lanes per segment (1 float each per pass)
    const int gpw = 64 / LPR;
    const int grp = (tid >> 6) * gpw + (lane / LPR);
    const int ngrp = 4 * gpw;
    const int gl = lane % LPR;
    for (int s = grp; s < nseg; s += ngrp) {
      const int s0 = segs[s], s1 = segs[s + 1];
      const int64_t row = (int64_t)(keys[s0] >> 12);
      for (int d = gl; d < D; d += LPR) {
        float acc = 0.f;
        for (int p = s0; p < s1; ++p) {
          const int it = (int)(keys[p] & 0xfff) / K;
          acc += g[it * D + d];
        }
        if (LTHM_KSB_X != 2) atomicAdd(dW + row * D + d, acc);  // LTHM_KSB_X=2: no row adds (timing only)
      }
    }
    // touched-row flags: every segment's first-touch test with its returning atomic issued side
    // by side (up to KB_NP / 256 per thread in flight), not one per lane group inside the segment
    // loop above, where each waited for its return before the group's next segment
    if (flags != nullptr) {
      constexpr int FQ = KB_NP / 256;
      int64_t rr[FQ];
      int old[FQ];
#pragma unroll
      for (int q = 0; q < FQ; ++q) {
        const int s = tid + 256 * q;
        rr[q] = s < nseg ? (int64_t)(keys[segs[s]] >> 12) : -1;
      }
#pragma unroll
      for (int q = 0; q < FQ; ++q) old[q] = rr[q] >= 0 ? atomicExch(flags + rr[q], 1) : 1;
#pragma unroll
      for (int q = 0; q < FQ; ++q)
        if (old[q] == 0) s_new[atomicAdd(&s_nnew, 1)] = rr[q];
    }
    __syncthreads();
    if (flags != nullptr) {
      // one global reservation per block instead of one same-address atomic per row
      if (tid == 0) s_base = s_nnew ? atomicAdd(count, (unsigned long long)s_nnew) : 0ull;
      __syncthreads();
      for (int i = tid; i < s_nnew; i += 256) list[s_base + i] = s_new[i];
      __syncthreads();
    }
  }
}

static int pick_vb(int D, int esz, int* lpr_log2) {
  const int bytes = D * esz;
  int vb = 16;
  while (vb > esz && (bytes % vb != 0)) vb >>= 1;
  while (bytes / vb > 64) return -1;
  const int lpr = bytes / vb;
  if (lpr & (lpr - 1)) return -1;
  int l2 = 0;
  while ((1 << l2) < lpr) ++l2;
  *lpr_log2 = l2;
  return vb;
}

// ---------------------------------------------------------------------------
// Item-embedding artifact (embedding_module_gen.py:32-41, consumed at
// encoder.py:25-29): out = KShift_K(id; W) * sigmoid(MLP(KShift_Km(id; Wm))),
// MLP = Linear(Dm, H1) -> QuickGELU -> Linear(H1, 1) (commons/layers.py:65-81,
// the mask model of embedding_module_gen.py:79-87).  One pass: the group of LPR
// lanes that pools the item's D-wide row sum also pools its Dm-wide mask rows
// (every lane of the group reads the same 16-B mask vectors: one coalesced
// request), evaluates the H1 hidden units strided over the group, reduces the
// logit by shuffles and scales its own slice of the pooled row.  The MLP
// weights sit in LDS.  Main-table pooling keeps the in-order c = 0..K-1 sum.
// ---------------------------------------------------------------------------
constexpr int IA_MAX_DM = 16;
constexpr int IA_MAX_H1 = 256;

template <typename TW, typename TO, int VB>
__global__ __launch_bounds__(KS_BLOCK) void item_artifact_fwd_k(
    const int64_t* __restrict__ ids, int64_t n, const TW* __restrict__ W, int64_t P, int D, int K, int mode,
    float scale, const float* __restrict__ Wm, int64_t Pm, int Dm, int Km, float mscale,
    const float* __restrict__ W1, const float* __restrict__ b1, int H1, const float* __restrict__ w2,
    const float* __restrict__ b2, TO* __restrict__ out, int LPR_LOG2) {
  constexpr int NE = VB / (int)sizeof(TW);
  __shared__ int64_t rows_lds[KS_BLOCK / 64][KS_ROWS_LDS / 2];
  __shared__ int64_t mrows_lds[KS_BLOCK / 64][KS_ROWS_LDS / 2];
  __shared__ float w1_lds[IA_MAX_H1 * IA_MAX_DM];
  __shared__ float b1_lds[IA_MAX_H1], w2_lds[IA_MAX_H1];
  for (int i = threadIdx.x; i < H1 * Dm; i += KS_BLOCK) w1_lds[i] = W1[i];
  for (int i = threadIdx.x; i < H1; i += KS_BLOCK) {
    b1_lds[i] = b1[i];
    w2_lds[i] = w2[i];
  }
  const float bias2 = b2[0];
  const int LPR = 1 << LPR_LOG2;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int gl = lane & (LPR - 1);
  const int gi = lane >> LPR_LOG2;
  const int IPW = 64 >> LPR_LOG2;
  const int IPB = IPW * (KS_BLOCK / 64);
  __syncthreads();

  for (int64_t base = (int64_t)blockIdx.x * IPB; base < n; base += (int64_t)gridDim.x * IPB) {
    const int64_t item = base + wave * IPW + gi;
    const bool valid = item < n;
    const int64_t id = valid ? ids[item] : 0;
    for (int c = gl; c < K; c += LPR) rows_lds[wave][gi * K + c] = valid ? kshift_row(id, c, P) : 0;
    for (int c = gl; c < Km; c += LPR) mrows_lds[wave][gi * Km + c] = valid ? kshift_row(id, c, Pm) : 0;
    __syncthreads();
    float acc[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) acc[e] = 0.f;
    float logit = 0.f;
    if (valid) {
      const TW* colp = W + (size_t)gl * NE;
      for (int c = 0; c < K; c += 2) {
        float v0[NE], v1[NE];
        load_vec<TW, VB>(colp + rows_lds[wave][gi * K + c] * D, v0);
        if (c + 1 < K) load_vec<TW, VB>(colp + rows_lds[wave][gi * K + c + 1] * D, v1);
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[e] = (c == 0) ? v0[e] : acc[e] + v0[e];
        if (c + 1 < K) {
#pragma unroll
          for (int e = 0; e < NE; ++e) acc[e] += v1[e];
        }
      }
      // mask vector m [Dm] (every lane of the group, same addresses), in-order sum
      float m[IA_MAX_DM];
#pragma unroll
      for (int d = 0; d < IA_MAX_DM; ++d) m[d] = 0.f;
      for (int c = 0; c < Km; ++c) {
        const float* mr = Wm + mrows_lds[wave][gi * Km + c] * Dm;
#pragma unroll
        for (int d4 = 0; d4 < IA_MAX_DM / 4; ++d4)
          if (d4 * 4 < Dm) {
            const float4 v = *(const float4*)(mr + d4 * 4);
            if (c == 0) {
              m[d4 * 4] = v.x; m[d4 * 4 + 1] = v.y; m[d4 * 4 + 2] = v.z; m[d4 * 4 + 3] = v.w;
            } else {
              m[d4 * 4] += v.x; m[d4 * 4 + 1] += v.y; m[d4 * 4 + 2] += v.z; m[d4 * 4 + 3] += v.w;
            }
          }
      }
#pragma unroll
      for (int d = 0; d < IA_MAX_DM; ++d) m[d] = m[d] / mscale;
      // hidden units strided over the group: QuickGELU(W1 m + b1) . w2
      float part = 0.f;
      for (int j = gl; j < H1; j += LPR) {
        float h = b1_lds[j];
        const float* wr = w1_lds + j * Dm;
#pragma unroll
        for (int d = 0; d < IA_MAX_DM; ++d)
          if (d < Dm) h = fmaf(wr[d], m[d], h);
        const float qg = h / (1.f + __expf(-1.702f * h));
        part = fmaf(w2_lds[j], qg, part);
      }
      for (int o = LPR >> 1; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
      logit = part + bias2;
    }
    if (mode == LTHM_KSHIFT_NORMALIZE) {
      float ss = 0.f;
#pragma unroll
      for (int e = 0; e < NE; ++e) ss += acc[e] * acc[e];
      for (int o = LPR >> 1; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      const float den = fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[e] = acc[e] / den;
    } else if (mode == LTHM_KSHIFT_SCALE) {
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[e] = acc[e] / scale;
    }
    const float gate = 1.f / (1.f + __expf(-logit));
#pragma unroll
    for (int e = 0; e < NE; ++e) acc[e] = gate * acc[e];
    if (valid) store_vec<TO, NE>(out + item * D + (size_t)gl * NE, acc);
    __syncthreads();
  }
}

template <typename TW, typename TO>
static int launch_item_artifact(const int64_t* ids, int64_t n, const void* W, int64_t P, int D, int K, int mode,
                                const float* Wm, int64_t Pm, int Dm, int Km, const float* W1, const float* b1,
                                int H1, const float* w2, const float* b2, void* out, hipStream_t s) {
  int l2 = 0;
  const int vb = pick_vb(D, (int)sizeof(TW), &l2);
  LTHM_REQUIRE(vb > 0);
  const int ipw = 64 >> l2;
  LTHM_REQUIRE(ipw * K <= KS_ROWS_LDS / 2 && ipw * Km <= KS_ROWS_LDS / 2);
  const int ipb = ipw * (KS_BLOCK / 64);
  const int grid = grid_for(n, ipb, 256 * 16);
  const float scale = (float)__builtin_sqrt((double)K);
  const float mscale = (float)__builtin_sqrt((double)Km);
#define IA_LAUNCH(V)                                                                                         \
  hipLaunchKernelGGL((item_artifact_fwd_k<TW, TO, V>), dim3(grid), dim3(KS_BLOCK), 0, s, ids, n, (const TW*)W, \
                     P, D, K, mode, scale, Wm, Pm, Dm, Km, mscale, W1, b1, H1, w2, b2, (TO*)out, l2)
  if (vb == 16)
    IA_LAUNCH(16);
  else if (vb == 8)
    IA_LAUNCH(8);
  else if (vb == 4)
    IA_LAUNCH(4);
  else
    return (int)hipErrorInvalidValue;
#undef IA_LAUNCH
  LTHM_CHECK_LAUNCH();
  return 0;
}

// K = 1 (flat lookups: FlatEmbedding, the C4 ranker's table-batched tables): one row per item,
// so a lane group takes KS1_U consecutive items at once -- their ids, rows and row loads all in
// flight before the first store (the general kernel holds one row load per lane between two
// barriers).  Same per-item arithmetic (the row, /1 or L2-normalised), no LDS.
constexpr int KS1_U = 8;
// element offset of item (b, f) = item of a [B, F, D] output / gradient whose F x D row block has
// leading dimension ld (ld = F D: contiguous; larger: the block sits inside a wider row, e.g. the
// ranker's MLP input [dense | F D table rows], round 6)
__device__ __forceinline__ int64_t k1_item_off(int64_t item, int F, int D, int64_t ld) {
  if (ld == (int64_t)F * D) return item * D;
  const int64_t b = item / F;
  return b * ld + (item - b * F) * D;
}
template <typename TW, typename TO, int VB>
__global__ __launch_bounds__(KS_BLOCK) void kshift_fwd_k1_k(const int64_t* __restrict__ ids, int64_t n_items, int F,
                                                          const TW* __restrict__ W, int64_t P, int D, int mode,
                                                          TO* __restrict__ out, float* __restrict__ norms,
                                                          int LPR_LOG2, int64_t out_ld) {
  constexpr int NE = VB / (int)sizeof(TW);
  const int LPR = 1 << LPR_LOG2;
  const int lane = threadIdx.x & 63;
  const int gl = lane & (LPR - 1);
  const int64_t groups = (int64_t)gridDim.x * (KS_BLOCK >> LPR_LOG2);
  const int64_t group = (int64_t)blockIdx.x * (KS_BLOCK >> LPR_LOG2) + (threadIdx.x >> LPR_LOG2);
  for (int64_t base = group * KS1_U; base < n_items; base += groups * KS1_U) {
    int64_t rows[KS1_U];
#pragma unroll
    for (int u = 0; u < KS1_U; ++u) {
      const int64_t item = base + u;
      rows[u] = item < n_items ? ((F > 1) ? (int64_t)(item % F) * P : 0) + kshift_row(ids[item], 0, P) : -1;
    }
    float v[KS1_U][NE];
#pragma unroll
    for (int u = 0; u < KS1_U; ++u) {
      if (rows[u] >= 0) load_vec<TW, VB>(W + rows[u] * D + (size_t)gl * NE, v[u]);
      else {
#pragma unroll
        for (int e = 0; e < NE; ++e) v[u][e] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < KS1_U; ++u) {
      if (mode == LTHM_KSHIFT_NORMALIZE) {
        float ss = 0.f;
#pragma unroll
        for (int e = 0; e < NE; ++e) ss += v[u][e] * v[u][e];
        for (int o = LPR >> 1; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
        const float nrm = sqrtf(ss);
        const float den = fmaxf(nrm, 1e-12f);
#pragma unroll
        for (int e = 0; e < NE; ++e) v[u][e] = v[u][e] / den;
        if (rows[u] >= 0 && norms != nullptr && gl == 0) norms[base + u] = nrm;
      } else if (mode == LTHM_KSHIFT_SCALE) {
#pragma unroll
        for (int e = 0; e < NE; ++e) v[u][e] = v[u][e] / 1.f;
      }
      if (rows[u] >= 0) store_vec<TO, NE>(out + k1_item_off(base + u, F, D, out_ld) + (size_t)gl * NE, v[u]);
    }
  }
}

template <typename TW, typename TO>
static int launch_fwd(const int64_t* ids, int64_t n_items, int F, const void* W, int64_t P, int D, int K,
                      int mode, void* out, float* norms, hipStream_t s, const int64_t* xrows = nullptr,
                      int64_t out_ld = 0) {
  if (out_ld == 0) out_ld = (int64_t)F * D;
  const bool strided = out_ld != (int64_t)F * D;  // only the K = 1 kernel writes strided rows
  int l2 = 0;
  const int vb = pick_vb(D, (int)sizeof(TW), &l2);
  LTHM_REQUIRE(vb > 0);
  // TO vector width must divide: elements per lane NE = vb / sizeof(TW)
  const int ipw = 64 >> l2;
  LTHM_REQUIRE(ipw * K <= KS_ROWS_LDS);
  const int ipb = ipw * (KS_BLOCK / 64);
  const int grid = grid_for(n_items, ipb, 256 * 32);
  const float scale = (float)__builtin_sqrt((double)K);
  static const bool k1_off = getenv("LTHM_KSHIFT_K1") && getenv("LTHM_KSHIFT_K1")[0] == '0';  // A/B
  LTHM_REQUIRE(!strided || (K == 1 && xrows == nullptr && !k1_off && out_ld >= (int64_t)F * D));
  if (K == 1 && xrows == nullptr && !k1_off) {
    const int g1 = grid_for(n_items, ipb * KS1_U, 256 * 32);
    if (vb == 16)
      hipLaunchKernelGGL((kshift_fwd_k1_k<TW, TO, 16>), dim3(g1), dim3(KS_BLOCK), 0, s, ids, n_items, F, (const TW*)W,
                         P, D, mode, (TO*)out, norms, l2, out_ld);
    else if (vb == 8)
      hipLaunchKernelGGL((kshift_fwd_k1_k<TW, TO, 8>), dim3(g1), dim3(KS_BLOCK), 0, s, ids, n_items, F, (const TW*)W,
                         P, D, mode, (TO*)out, norms, l2, out_ld);
    else if (vb == 4)
      hipLaunchKernelGGL((kshift_fwd_k1_k<TW, TO, 4>), dim3(g1), dim3(KS_BLOCK), 0, s, ids, n_items, F, (const TW*)W,
                         P, D, mode, (TO*)out, norms, l2, out_ld);
    else
      return (int)hipErrorInvalidValue;
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  // register-row gather: 16-B lane vectors, K 4 / 8 / 16, 4 .. 32 lanes per row (LTHM_KSHIFT_REG=1: on)
  static const bool reg_on = getenv("LTHM_KSHIFT_REG") && getenv("LTHM_KSHIFT_REG")[0] == '1';
  if (reg_on && xrows == nullptr && vb == 16 && (K == 16 || K == 8 || K == 4) && l2 >= 2 && l2 <= 5) {
    const int lpr = 1 << l2;
    // waves: enough iterations per wave to amortise the first id load, capped at 32 blocks per CU
    const int64_t iters = (n_items + (64 / lpr) - 1) / (64 / lpr);
    const int gr = grid_for(iters, 4 * 2, 256 * 32);
#define KSR_LAUNCH(KT_, LPR_)                                                                                       \
  hipLaunchKernelGGL((kshift_fwd_reg_k<TW, TO, KT_, LPR_>), dim3(gr), dim3(KS_BLOCK), 0, s, ids, n_items, F,     \
                     (const TW*)W, P, D, mode, scale, (TO*)out, norms)
#define KSR_LPR(KT_)            \
  switch (lpr) {                \
    case 4: KSR_LAUNCH(KT_, 4); break;   \
    case 8: KSR_LAUNCH(KT_, 8); break;   \
    case 16: KSR_LAUNCH(KT_, 16); break; \
    default: KSR_LAUNCH(KT_, 32); break; \
  }
    if (K == 16) {
      KSR_LPR(16)
    } else if (K == 8) {
      KSR_LPR(8)
    } else {
      KSR_LPR(4)
    }
#undef KSR_LPR
#undef KSR_LAUNCH
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  if (vb == 16)
    hipLaunchKernelGGL((kshift_fwd_k<TW, TO, 16>), dim3(grid), dim3(KS_BLOCK), 0, s, ids, n_items, F,
                       (const TW*)W, P, D, K, mode, scale, (TO*)out, norms, l2, xrows);
  else if (vb == 8)
    hipLaunchKernelGGL((kshift_fwd_k<TW, TO, 8>), dim3(grid), dim3(KS_BLOCK), 0, s, ids, n_items, F,
                       (const TW*)W, P, D, K, mode, scale, (TO*)out, norms, l2, xrows);
  else if (vb == 4)
    hipLaunchKernelGGL((kshift_fwd_k<TW, TO, 4>), dim3(grid), dim3(KS_BLOCK), 0, s, ids, n_items, F,
                       (const TW*)W, P, D, K, mode, scale, (TO*)out, norms, l2, xrows);
  else
    return (int)hipErrorInvalidValue;
  LTHM_CHECK_LAUNCH();
  return 0;
}

// K = 1 (FlatEmbedding / table-batched flat lookups, e.g. the C4 ranker) with a
// plain or /sqrt(K) output: every item touches one row, so the LDS dedup and
// sort buy nothing for uniform ids.  A row's D columns map to D consecutive lanes
// (64 / D items per wave instruction, each f32 atomic instruction covering
// whole rows).  The first lane of an item marks the row touched; a block
// collects its newly touched rows of a K1_CHUNK-item chunk in LDS and reserves
// their list slots with ONE global atomic (a same-address atomic per wave
// serialises at one L2 channel).
constexpr int K1_CHUNK = 1024;
template <typename TY>
__global__ __launch_bounds__(256) void kshift_bwd_k1_k(const int64_t* __restrict__ ids, int64_t n_items, int F,
                                                       const TY* __restrict__ dY, int64_t P, int D,
                                                       float* __restrict__ dW, int32_t* __restrict__ flags,
                                                       int64_t* __restrict__ list,
                                                       unsigned long long* __restrict__ count) {
  __shared__ int64_t s_new[K1_CHUNK];
  __shared__ int s_nnew;
  __shared__ unsigned long long s_base;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ipw = 64 / D;  // items per wave instruction
  const int il = lane / D, d = lane - il * D;
  for (int64_t c0 = (int64_t)blockIdx.x * K1_CHUNK; c0 < n_items; c0 += (int64_t)gridDim.x * K1_CHUNK) {
    if (tid == 0) s_nnew = 0;
    __syncthreads();
    const int64_t c1 = min(n_items, c0 + K1_CHUNK);
    for (int64_t b = c0 + (int64_t)wave * ipw; b < c1; b += 4 * ipw) {
      const int64_t item = b + il;
      if (item < c1) {
        const int64_t row = ((F > 1) ? (int64_t)(item % F) * P : 0) + kshift_row(ids[item], 0, P);
        atomicAdd(dW + row * D + d, Elem<TY>::ld(dY + item * D + d));  // /sqrt(K) = 1 for the scale mode
        if (flags != nullptr && d == 0 && atomicExch(flags + row, 1) == 0) s_new[atomicAdd(&s_nnew, 1)] = row;
      }
    }
    __syncthreads();
    if (flags != nullptr) {
      if (tid == 0) s_base = s_nnew ? atomicAdd(count, (unsigned long long)s_nnew) : 0ull;
      __syncthreads();
      for (int i = tid; i < s_nnew; i += 256) list[s_base + i] = s_new[i];
    }
    __syncthreads();
  }
}

// The same K = 1 backward with the row gradients STORED instead of added where a row is touched
// the first time since the optimizer last cleared its flag (round 5): the first item of a row
// (the one whose flag exchange returned 0) writes the row with plain 16-lane-per-row stores,
// every other item of a touched row goes to a duplicate list; kshift_bwd_k1_dup_k then adds the
// duplicates' rows with f32 atomics, after every first store has landed (kernel boundary).
// Uniform ids over 64M rows (C4) are ~97 % first touches, so the f32 atomic traffic (the
// chip-wide ~1.3 TB/s float-atomic rate, MI355X_MICROARCH.md) becomes plain row stores.
template <typename TY>
__global__ __launch_bounds__(256) void kshift_bwd_k1_first_k(const int64_t* __restrict__ ids, int64_t n_items, int F,
                                                             const TY* __restrict__ dY, int64_t P, int D,
                                                             float* __restrict__ dW, uint32_t* __restrict__ bits,
                                                             int64_t* __restrict__ list,
                                                             unsigned long long* __restrict__ count,
                                                             int64_t* __restrict__ dups,
                                                             unsigned long long* __restrict__ ndup, int64_t dy_ld) {
  __shared__ int64_t s_new[K1_CHUNK];
  __shared__ int64_t s_dup[K1_CHUNK];
  __shared__ int s_nnew, s_ndup;
  __shared__ unsigned long long s_base, s_dbase;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // copy phase: VEC columns per lane (16-B f32 stores where D % 4 == 0), LPI lanes per item
  const int VEC = (D % 4 == 0) ? 4 : 1, LPI = D / VEC, ipw = 64 / LPI;
  const int il = lane / LPI, c = (lane - il * LPI) * VEC;
  const uint64_t lt = (1ull << lane) - 1ull;  // lanes below this one
  for (int64_t c0 = (int64_t)blockIdx.x * K1_CHUNK; c0 < n_items; c0 += (int64_t)gridDim.x * K1_CHUNK) {
    if (tid == 0) s_nnew = s_ndup = 0;
    __syncthreads();
    const int64_t c1 = min(n_items, c0 + K1_CHUNK);
    for (int64_t base = c0 + (int64_t)wave * 64; base < c1; base += 256) {
      // 64 items per wave, one per lane: the 64 bitmap atomics of the wave in flight together
      // (per item, serially, the atomic's round trip bounded the kernel)
      const int64_t item = base + lane;
      const bool ok = item < c1;
      const int64_t row = ok ? ((F > 1) ? (int64_t)(item % F) * P : 0) + kshift_row(ids[item], 0, P) : 0;
      int prev = 1;
      if (ok) {  // the row's bit of the touched-row bitmap (F * P bits: an Infinity-Cache-sized array)
        const uint32_t bit = 1u << (row & 31);
        prev = (atomicOr(bits + (row >> 5), bit) & bit) ? 1 : 0;
      }
      const bool isnew = ok && prev == 0, isdup = ok && prev != 0;
      const uint64_t mnew = __ballot(isnew), mdup = __ballot(isdup);
      int bn = 0, bd = 0;
      if (lane == 0) {
        bn = atomicAdd(&s_nnew, (int)__popcll(mnew));
        bd = atomicAdd(&s_ndup, (int)__popcll(mdup));
      }
      bn = __shfl(bn, 0, 64);
      bd = __shfl(bd, 0, 64);
      if (isnew) s_new[bn + __popcll(mnew & lt)] = row;
      if (isdup) s_dup[bd + __popcll(mdup & lt)] = item;
      // first touches: the row's gradient IS this item's (plain stores; repeats: kshift_bwd_k1_dup_k)
      const uint32_t rlo = (uint32_t)row, rhi = (uint32_t)((uint64_t)row >> 32);
#pragma unroll 4
      for (int s0 = 0; s0 < 64; s0 += ipw) {
        const int src = s0 + il;
        const int64_t r = (int64_t)(((uint64_t)(uint32_t)__shfl((int)rhi, src, 64) << 32) | (uint32_t)__shfl((int)rlo, src, 64));
        const int pv = __shfl(prev, src, 64);
        const int64_t it = base + src;
        if (it < c1 && pv == 0) {
          if (VEC == 4) {
            float g[4];
            load_vec<TY, 4 * (int)sizeof(TY)>(dY + k1_item_off(it, F, D, dy_ld) + c, g);
            *reinterpret_cast<f32x4*>(dW + r * D + c) = f32x4{g[0], g[1], g[2], g[3]};
          } else {
            dW[r * D + c] = Elem<TY>::ld(dY + k1_item_off(it, F, D, dy_ld) + c);
          }
        }
      }
    }
    __syncthreads();
    if (tid == 0) {
      s_base = s_nnew ? atomicAdd(count, (unsigned long long)s_nnew) : 0ull;
      s_dbase = s_ndup ? atomicAdd(ndup, (unsigned long long)s_ndup) : 0ull;
    }
    __syncthreads();
    for (int i = tid; i < s_nnew; i += 256) list[s_base + i] = s_new[i];
    for (int i = tid; i < s_ndup; i += 256) dups[s_dbase + i] = s_dup[i];
    __syncthreads();
  }
}

template <typename TY>
__global__ __launch_bounds__(256) void kshift_bwd_k1_dup_k(const int64_t* __restrict__ ids, int F,
                                                           const TY* __restrict__ dY, int64_t P, int D,
                                                           float* __restrict__ dW, const int64_t* __restrict__ dups,
                                                           const unsigned long long* __restrict__ ndup, int64_t dy_ld) {
  const int64_t nd = (int64_t)*ndup;
  const int lane = threadIdx.x & 63;
  const int ipw = 64 / D, il = lane / D, d = lane - il * D;
  for (int64_t b = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * ipw; b < nd; b += (int64_t)gridDim.x * 4 * ipw) {
    if (b + il < nd) {
      const int64_t item = dups[b + il];
      const int64_t row = ((F > 1) ? (int64_t)(item % F) * P : 0) + kshift_row(ids[item], 0, P);
      atomicAdd(dW + row * D + d, Elem<TY>::ld(dY + k1_item_off(item, F, D, dy_ld) + d));
    }
  }
}

template <typename TY, typename TO>
static int launch_bwd(const int64_t* ids, int64_t n_items, int F, const void* dY, const void* out,
                      const float* norms, int64_t P, int D, int K, int mode, float* dW, int32_t* flags,
                      int64_t* list, unsigned long long* count, hipStream_t s, int64_t* dups = nullptr,
                      unsigned long long* ndup = nullptr, int64_t dy_ld = 0) {
  if (dy_ld == 0) dy_ld = (int64_t)F * D;
  if (K == 1 && mode != LTHM_KSHIFT_NORMALIZE && D <= 64 && 64 % D == 0 && flags && dups && ndup) {
    LTHM_REQUIRE(hipMemsetAsync(ndup, 0, sizeof(unsigned long long), s) == hipSuccess);
    hipLaunchKernelGGL((kshift_bwd_k1_first_k<TY>), dim3(grid_for(n_items, K1_CHUNK, 256 * 8)), dim3(256), 0, s, ids,
                       n_items, F, (const TY*)dY, P, D, dW, reinterpret_cast<uint32_t*>(flags), list, count, dups, ndup,
                       dy_ld);
    LTHM_CHECK_LAUNCH();
    hipLaunchKernelGGL((kshift_bwd_k1_dup_k<TY>), dim3(1024), dim3(256), 0, s, ids, F, (const TY*)dY, P, D, dW,
                       (const int64_t*)dups, (const unsigned long long*)ndup, dy_ld);
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  LTHM_REQUIRE(dy_ld == (int64_t)F * D);  // strided gradients: the first-touch path only
  if (K == 1 && mode != LTHM_KSHIFT_NORMALIZE && D <= 64 && 64 % D == 0) {
    hipLaunchKernelGGL((kshift_bwd_k1_k<TY>), dim3(grid_for(n_items, K1_CHUNK, 256 * 8)), dim3(256), 0, s, ids,
                       n_items, F, (const TY*)dY, P, D, dW, flags, list, count);
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  int ch = KB_NP / K;
  if (ch * D > KB_G_FLOATS) ch = KB_G_FLOATS / D;
  LTHM_REQUIRE(ch >= 1);
  int np2 = 256;
  while (np2 < ch * K) np2 <<= 1;
  const float scale = (float)__builtin_sqrt((double)K);
  const size_t shmem = (size_t)KB_NP * 8 + (size_t)KB_G_FLOATS * 4 + (size_t)(KB_NP + 1) * 4;
  const int grid = grid_for(n_items, ch, 256 * 8);
  hipLaunchKernelGGL((kshift_bwd_dense_k<TY, TO>), dim3(grid), dim3(256), shmem, s, ids, n_items, F,
                     (const TY*)dY, (const TO*)out, norms, P, D, K, mode, scale, ch, np2, dW, flags, list, count);
  LTHM_CHECK_LAUNCH();
  return 0;
}

}  // namespace lthm

using namespace lthm;

extern "C" {

int lthm_abi_version(void) { return LTHM_ABI_VERSION; }

int lthm_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int lthm_kshift_rows(const int64_t* ids, int64_t n, int64_t P, int32_t K, int64_t* rows, void* stream) {
  LTHM_REQUIRE(P > 0 && K > 0 && K <= 64 && n >= 0);
  if (n == 0) return 0;
  hipLaunchKernelGGL(kshift_rows_k, dim3(grid_for(n * K, 256)), dim3(256), 0, (hipStream_t)stream, ids, n,
                     P, K, rows);
  LTHM_CHECK_LAUNCH();
  return 0;
}

static int kshift_fwd_impl(const int64_t* ids, int64_t n_items, int F, const void* W, int w_dtype, int64_t P,
                           int D, int K, int mode, void* out, int out_dtype, float* norms, void* stream,
                           const int64_t* xrows = nullptr, int64_t out_ld = 0) {
  LTHM_REQUIRE(P > 0 && K > 0 && K <= 64 && D > 0 && n_items >= 0 && F >= 1);
  LTHM_REQUIRE(mode >= 0 && mode <= 2);
  if (n_items == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (w_dtype == LTHM_F32 && out_dtype == LTHM_F32)
    return launch_fwd<float, float>(ids, n_items, F, W, P, D, K, mode, out, norms, s, xrows, out_ld);
  if (w_dtype == LTHM_F32 && out_dtype == LTHM_BF16)
    return launch_fwd<float, bf16_t>(ids, n_items, F, W, P, D, K, mode, out, norms, s, xrows, out_ld);
  if (w_dtype == LTHM_BF16 && out_dtype == LTHM_F32)
    return launch_fwd<bf16_t, float>(ids, n_items, F, W, P, D, K, mode, out, norms, s, xrows, out_ld);
  if (w_dtype == LTHM_BF16 && out_dtype == LTHM_BF16)
    return launch_fwd<bf16_t, bf16_t>(ids, n_items, F, W, P, D, K, mode, out, norms, s, xrows, out_ld);
  return (int)hipErrorInvalidValue;
}

int lthm_kshift_fwd(const int64_t* ids, int64_t n, const void* W, int32_t w_dtype, int64_t P, int64_t row_base,
                    int32_t D, int32_t K, int32_t mode, void* out, int32_t out_dtype, float* norms, void* stream) {
  const void* Wb = W;
  if (row_base != 0) {
    const size_t esz = (w_dtype == LTHM_F32) ? 4 : 2;
    Wb = (const void*)((const char*)W + (size_t)row_base * D * esz);
  }
  return kshift_fwd_impl(ids, n, 1, Wb, w_dtype, P, D, K, mode, out, out_dtype, norms, stream);
}

int lthm_kshift_fwd_multi(const int64_t* ids, int64_t n, int32_t F, const void* W, int32_t w_dtype, int64_t P,
                          int32_t D, int32_t K, int32_t mode, void* out, int32_t out_dtype, float* norms,
                          void* stream) {
  return kshift_fwd_impl(ids, n * (int64_t)F, F, W, w_dtype, P, D, K, mode, out, out_dtype, norms, stream);
}

int lthm_kshift_fwd_multi_ld(const int64_t* ids, int64_t n, int32_t F, const void* W, int32_t w_dtype, int64_t P,
                             int32_t D, int32_t K, int32_t mode, void* out, int32_t out_dtype, int64_t out_ld,
                             float* norms, void* stream) {
  LTHM_REQUIRE(out_ld >= (int64_t)F * D && (out_ld == (int64_t)F * D || K == 1));
  return kshift_fwd_impl(ids, n * (int64_t)F, F, W, w_dtype, P, D, K, mode, out, out_dtype, norms, stream, nullptr,
                         out_ld);
}

int lthm_gather_pool(const int64_t* rows, int64_t n, int32_t K, const void* W, int32_t w_dtype, int64_t R, int32_t D,
                     int32_t mode, void* out, int32_t out_dtype, float* norms, void* stream) {
  LTHM_REQUIRE(rows != nullptr || n == 0);
  return kshift_fwd_impl(nullptr, n, 1, W, w_dtype, R, D, K, mode, out, out_dtype, norms, stream, rows);
}

int lthm_kshift_bwd_dense(const int64_t* ids, int64_t n, int32_t F, const void* dY, int32_t dy_dtype,
                          const void* out, int32_t out_dtype, const float* norms, int64_t P, int32_t D, int32_t K,
                          int32_t mode, float* dW, void* stream) {
  return lthm_kshift_bwd_sparse(ids, n, F, dY, dy_dtype, out, out_dtype, norms, P, D, K, mode, dW, nullptr, nullptr,
                                nullptr, stream);
}

int lthm_kshift_bwd_sparse(const int64_t* ids, int64_t n, int32_t F, const void* dY, int32_t dy_dtype,
                           const void* out, int32_t out_dtype, const float* norms, int64_t P, int32_t D, int32_t K,
                           int32_t mode, float* dW, int32_t* flags, int64_t* list, int64_t* count, void* stream) {
  LTHM_REQUIRE((flags == nullptr) == (list == nullptr) && (list == nullptr) == (count == nullptr));
  LTHM_REQUIRE(P > 0 && K > 0 && K <= 64 && D > 0 && n >= 0 && F >= 1);
  LTHM_REQUIRE(mode >= 0 && mode <= 2);
  LTHM_REQUIRE(mode != LTHM_KSHIFT_NORMALIZE || (out != nullptr && norms != nullptr));
  const int64_t items = n * (int64_t)F;
  if (items == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (dy_dtype == LTHM_F32 && out_dtype == LTHM_F32)
    return launch_bwd<float, float>(ids, items, F, dY, out, norms, P, D, K, mode, dW, flags, list, (unsigned long long*)count, s);
  if (dy_dtype == LTHM_BF16 && out_dtype == LTHM_BF16)
    return launch_bwd<bf16_t, bf16_t>(ids, items, F, dY, out, norms, P, D, K, mode, dW, flags, list, (unsigned long long*)count, s);
  if (dy_dtype == LTHM_F32 && out_dtype == LTHM_BF16)
    return launch_bwd<float, bf16_t>(ids, items, F, dY, out, norms, P, D, K, mode, dW, flags, list, (unsigned long long*)count, s);
  if (dy_dtype == LTHM_BF16 && out_dtype == LTHM_F32)
    return launch_bwd<bf16_t, float>(ids, items, F, dY, out, norms, P, D, K, mode, dW, flags, list, (unsigned long long*)count, s);
  return (int)hipErrorInvalidValue;
}

int lthm_kshift_bwd_sparse_first_ld(const int64_t* ids, int64_t n, int32_t F, const void* dY, int32_t dy_dtype,
                                    int64_t dy_ld, int64_t P, int32_t D, float* dW, int32_t* flags, int64_t* list,
                                    int64_t* count, int64_t* dup_ws, int64_t dup_cap, void* stream);

int lthm_kshift_bwd_sparse_first(const int64_t* ids, int64_t n, int32_t F, const void* dY, int32_t dy_dtype,
                                 int64_t P, int32_t D, float* dW, int32_t* flags, int64_t* list, int64_t* count,
                                 int64_t* dup_ws, int64_t dup_cap, void* stream) {
  return lthm_kshift_bwd_sparse_first_ld(ids, n, F, dY, dy_dtype, (int64_t)F * D, P, D, dW, flags, list, count,
                                         dup_ws, dup_cap, stream);
}

int lthm_kshift_bwd_sparse_first_ld(const int64_t* ids, int64_t n, int32_t F, const void* dY, int32_t dy_dtype,
                                    int64_t dy_ld, int64_t P, int32_t D, float* dW, int32_t* flags, int64_t* list,
                                    int64_t* count, int64_t* dup_ws, int64_t dup_cap, void* stream) {
  LTHM_REQUIRE(dy_ld >= (int64_t)F * D && (dy_ld % 4 == 0 || D % 4 != 0));
  LTHM_REQUIRE(P > 0 && D > 0 && D <= 64 && 64 % D == 0 && n >= 0 && F >= 1);
  LTHM_REQUIRE(dW && flags && list && count && dup_ws && (dy_dtype == LTHM_F32 || dy_dtype == LTHM_BF16));
  const int64_t items = n * (int64_t)F;
  LTHM_REQUIRE(dup_cap >= items + 1);
  // the first-touch rows are copied as f32x4 stores from 4-element dY vectors
  const int esz = dy_dtype == LTHM_F32 ? 4 : 2;
  LTHM_REQUIRE(D % 4 != 0 || (((uintptr_t)dW % 16) == 0 && ((uintptr_t)dY % (4 * esz)) == 0));
  if (items == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  unsigned long long* ndup = (unsigned long long*)dup_ws;  // dup_ws[0]: the count, then the items
  if (dy_dtype == LTHM_F32)
    return launch_bwd<float, float>(ids, items, F, dY, nullptr, nullptr, P, D, 1, LTHM_KSHIFT_SCALE, dW, flags, list,
                                    (unsigned long long*)count, s, dup_ws + 1, ndup, dy_ld);
  return launch_bwd<bf16_t, float>(ids, items, F, dY, nullptr, nullptr, P, D, 1, LTHM_KSHIFT_SCALE, dW, flags, list,
                                   (unsigned long long*)count, s, dup_ws + 1, ndup, dy_ld);
}

int lthm_item_artifact_fwd(const int64_t* ids, int64_t n, const void* W, int32_t w_dtype, int64_t P, int32_t D,
                           int32_t K, int32_t mode, const float* Wm, int64_t Pm, int32_t Dm, int32_t Km,
                           const float* W1, const float* b1, int32_t H1, const float* w2, const float* b2, void* out,
                           int32_t out_dtype, void* stream) {
  LTHM_REQUIRE(P > 0 && K > 0 && K <= 64 && D > 0 && n >= 0 && mode >= 0 && mode <= 2);
  LTHM_REQUIRE(Pm > 0 && Km > 0 && Km <= 64 && Dm > 0 && Dm <= IA_MAX_DM && Dm % 4 == 0);
  LTHM_REQUIRE(H1 > 0 && H1 <= IA_MAX_H1 && W1 && b1 && w2 && b2 && Wm);
  LTHM_REQUIRE(((uintptr_t)Wm % 16) == 0);
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (w_dtype == LTHM_F32 && out_dtype == LTHM_F32)
    return launch_item_artifact<float, float>(ids, n, W, P, D, K, mode, Wm, Pm, Dm, Km, W1, b1, H1, w2, b2, out, s);
  if (w_dtype == LTHM_BF16 && out_dtype == LTHM_F32)
    return launch_item_artifact<bf16_t, float>(ids, n, W, P, D, K, mode, Wm, Pm, Dm, Km, W1, b1, H1, w2, b2, out, s);
  if (w_dtype == LTHM_F32 && out_dtype == LTHM_BF16)
    return launch_item_artifact<float, bf16_t>(ids, n, W, P, D, K, mode, Wm, Pm, Dm, Km, W1, b1, H1, w2, b2, out, s);
  if (w_dtype == LTHM_BF16 && out_dtype == LTHM_BF16)
    return launch_item_artifact<bf16_t, bf16_t>(ids, n, W, P, D, K, mode, Wm, Pm, Dm, Km, W1, b1, H1, w2, b2, out, s);
  return (int)hipErrorInvalidValue;
}

}  // extern "C"
