// LTHM tower kernels for gfx950:
//   * product tower forward (models/lthm/sequence/product_tower.py:43-62) fused
//     into one wave-per-token kernel: norm + pad mask, L2 normalise, emb_mapper
//     Linear(Din -> Dout), the 6 CosineVectorEmbedding modules
//     (commons/transformers/layers.py:462-471: normalise, project, bucketize,
//     EmbeddingBag-sum), the norm-histogram embedding and the masked fill;
//   * LDS-privatised small-table gradient (EmbeddingBag / nn.Embedding backward
//     for tables of <= a few thousand rows: CVE tables, time / action / position
//     tables, outcome conditioning);
//   * query-tower token assembly (models/lthm/sequence/query_tower.py:89-111)
//     and outcome conditioning (:118-122);
//   * history flip (models/lthm/sequence/encoder.py:52-54, 60-61).
#include <algorithm>

#include "common.hpp"

namespace lthm {

// ------------------------------------------------------------------ flip
__global__ void flip_k(const int64_t* __restrict__ in, int64_t* __restrict__ out, int64_t B, int T) {
  const int64_t n = B * T;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / T;
    const int t = (int)(i - b * T);
    out[b * T + (T - 1 - t)] = in[i];
  }
}

// ------------------------------------------------------------------ product tower
struct PTArgs {
  lthm_ptower_desc d;
};

template <typename TX, typename TT, int OPL>
__global__ __launch_bounds__(256) void ptower_fwd_k(lthm_ptower_desc d, int total_idx) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Din = d.Din, Dout = d.Dout;
  float* wT = reinterpret_cast<float*>(smem);            // [Din][Dout]
  float* proj = wT + Din * Dout;                          // concatenated [Din][nproj_j]
  float* grids = proj + d.proj_total;                     // concatenated
  float* xs = grids + d.grid_total;                       // [4][2][Din]
  uint16_t* rbuf = reinterpret_cast<uint16_t*>(xs + 8 * Din);  // [4][total_idx]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (!d.cve_only)
    for (int i = tid; i < Din * Dout; i += 256) {
      const int o = i / Din, k = i - o * Din;
      wT[k * Dout + o] = d.w_map[i];
    }
  for (int i = tid; i < d.proj_total; i += 256) proj[i] = d.proj[i];
  for (int i = tid; i < d.grid_total; i += 256) grids[i] = d.grids[i];
  __syncthreads();
  // OPL outputs per lane; lanes with lane*OPL >= Dout idle (Dout < 64 or not a multiple of 64)
  const bool lane_on = lane * OPL < Dout;
  const int lcol = lane_on ? lane * OPL : 0;
  float* xw = xs + wave * 2 * Din;
  float* xw2 = xw + Din;
  uint16_t* rw = rbuf + wave * total_idx;
  const TT* tab = reinterpret_cast<const TT*>(d.tables);
  const TT* hist = reinterpret_cast<const TT*>(d.hist);
  for (int64_t tok = (int64_t)blockIdx.x * 4 + wave; tok < d.n; tok += (int64_t)gridDim.x * 4) {
    // norm, mask, normalise (product_tower.py:47-51); Din <= 256: up to 4 elements per lane
    float xv[4], ss = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = lane + 64 * k;
      xv[k] = (i < Din) ? Elem<TX>::ld(reinterpret_cast<const TX*>(d.x) + tok * Din + i) : 0.f;
      ss += xv[k] * xv[k];
    }
    const float nrm = sqrtf(wave_sum(ss));
    const bool masked = !d.cve_only && ((nrm < d.norm_threshold) || (d.ids[tok] == 0));
    float xn[4], ss2 = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      xn[k] = xv[k] / fmaxf(nrm, 1e-12f);
      ss2 += xn[k] * xn[k];
    }
    // CosineVectorEmbedding re-normalises its already normalised input (layers.py:464)
    const float den2 = d.cve_only ? 1.f : fmaxf(sqrtf(wave_sum(ss2)), 1e-12f);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = lane + 64 * k;
      if (i < Din) {
        xw[i] = xn[k];
        xw2[i] = d.cve_only ? xn[k] : xn[k] / den2;
        if (d.xn_out) reinterpret_cast<bf16_t*>(d.xn_out)[tok * Din + i] = f2bf(xn[k]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    // bucket rows for all modules: lane handles (module, projection) pairs
    int base = 0;
    for (int j = 0; j < d.n_mod; ++j) {
      const int np = d.mod_nproj[j], nb = d.mod_nbins[j];
      const float* pj = proj + d.mod_proj_off[j];
      const float* gj = grids + d.mod_grid_off[j];
      for (int p = lane; p < np; p += 64) {
        float z = 0.f;
        for (int i = 0; i < Din; ++i) z = fmaf(xw2[i], pj[i * np + p], z);
        int bk = 0;
        for (int q = 0; q < nb; ++q) bk += (gj[q] < z) ? 1 : 0;  // bucketize(right=False)
        const int row = d.mod_row_off[j] + (nb + 1) * p + bk;
        rw[base + p] = (uint16_t)row;
      }
      base += np;
    }
    int hbin = -1;
    if (d.norm_bins > 0) {
      float f = floorf(nrm * (float)d.norm_bins);  // HistogramEmbedding(0, 1, nbins): uniform bins, clamped
      hbin = (int)fminf(fmaxf(f, 0.f), (float)(d.norm_bins - 1));
      if (lane == 0) rw[base] = (uint16_t)(d.cve_rows + hbin);
    }
    __builtin_amdgcn_wave_barrier();
    // emb_mapper Linear
    float acc[OPL];
    for (int q = 0; q < OPL; ++q) {
      const int o = lcol + q;
      float s = 0.f;
      if (!d.cve_only) {
        s = d.b_map ? d.b_map[o] : 0.f;
        for (int i = 0; i < Din; ++i) s = fmaf(xw[i], wT[i * Dout + o], s);
      }
      acc[q] = s;
    }
    // EmbeddingBag sums, module by module, then add (product_tower.py:53-54)
    int rb = 0;
    for (int j = 0; j < d.n_mod; ++j) {
      const int np = d.mod_nproj[j];
      float bag[OPL];
      for (int q = 0; q < OPL; ++q) bag[q] = 0.f;
      int p = 0;
      for (; p + 4 <= np; p += 4) {
        float v0[OPL], v1[OPL], v2[OPL], v3[OPL];
        const TT* r0 = tab + (int64_t)rw[rb + p] * Dout + lcol;
        const TT* r1 = tab + (int64_t)rw[rb + p + 1] * Dout + lcol;
        const TT* r2 = tab + (int64_t)rw[rb + p + 2] * Dout + lcol;
        const TT* r3 = tab + (int64_t)rw[rb + p + 3] * Dout + lcol;
        for (int q = 0; q < OPL; ++q) { v0[q] = Elem<TT>::ld(r0 + q); v1[q] = Elem<TT>::ld(r1 + q);
                                        v2[q] = Elem<TT>::ld(r2 + q); v3[q] = Elem<TT>::ld(r3 + q); }
        for (int q = 0; q < OPL; ++q) bag[q] = (((bag[q] + v0[q]) + v1[q]) + v2[q]) + v3[q];
      }
      for (; p < np; ++p) {
        const TT* r0 = tab + (int64_t)rw[rb + p] * Dout + lcol;
        for (int q = 0; q < OPL; ++q) bag[q] += Elem<TT>::ld(r0 + q);
      }
      for (int q = 0; q < OPL; ++q) acc[q] += bag[q];
      rb += np;
    }
    if (hbin >= 0) {
      const TT* hr = hist + (int64_t)hbin * Dout + lcol;
      for (int q = 0; q < OPL; ++q) acc[q] += Elem<TT>::ld(hr + q);
    }
    if (!lane_on) {
    } else if (d.emb_dtype == LTHM_F32) {
      float* eo = reinterpret_cast<float*>(d.emb_out) + tok * Dout + lcol;
      for (int q = 0; q < OPL; ++q) eo[q] = masked ? 0.f : acc[q];
    } else {
      bf16_t* eo = reinterpret_cast<bf16_t*>(d.emb_out) + tok * Dout + lcol;
      for (int q = 0; q < OPL; ++q) eo[q] = f2bf(masked ? 0.f : acc[q]);
    }
    if (lane == 0 && d.mask_out) d.mask_out[tok] = masked ? 1 : 0;
    if (d.rows_out) {
      for (int i = lane; i < total_idx; i += 64) d.rows_out[tok * total_idx + i] = masked ? (uint16_t)0xffff : rw[i];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// swizzled row-major [rows, D] bf16 LDS image (16-byte chunks XOR row group) and
// its ds_read_tr16_b64 fragment B[k = 8(lane>>4) + i][n = nb + (lane&15)]
template <int D>
__device__ __forceinline__ int ct_swz(int row) {
  constexpr int NC = D / 8;
  if constexpr (NC >= 16) {
    // bit permutation r0 -> b1, r1 -> b2, r2 -> b0 (r3, r4 stay): a transposed read's 32-lane
    // half (rows kb + {0..3, 8..11} or kb + {4..7, 12..15}, two adjacent chunks) then covers
    // 16 distinct 16-byte slots (64 banks); plain r & (NC - 1) gave 8, a 2-way conflict
    return (((row & 3) << 1) | ((row >> 2) & 1) | (row & 24)) & (NC - 1);
  } else {
    constexpr int RPL = (256 / (2 * D)) > 0 ? 256 / (2 * D) : 1;
    return (row / RPL) & (NC - 1);
  }
}
template <int D>
__device__ __forceinline__ int ct_off(int row, int ch) {
  return row * (2 * D) + ((ch ^ ct_swz<D>(row)) << 4);
}

template <int D>
__device__ __forceinline__ bf16x8v ct_tr_frag(const unsigned char* img, int nb, int lane) {
  const int gq = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int kr = 8 * gq + q;
  const int ch = (nb >> 3) + (p >> 1);
  const unsigned char* a0 = img + ct_off<D>(kr, ch) + 8 * (p & 1);
  const unsigned char* a1 = img + ct_off<D>(kr + 4, ch) + 8 * (p & 1);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8v, v);
}

// ------------------------------------------------------------------ product-tower bucket rows
// Per token: norm, pad mask, x / |x| (bf16 copy for the mapper's weight
// gradient), CVE input normalised once more (layers.py:464), histogram row.
// Per (token, projection): z = xn2 . R[:, p] (f32, sequential FMAs), bucketize
// (right = False) -> table row.  Phase 1 runs a thread per token; phase 2 a
// thread per projection with its R column and grid in registers, streaming the
// chunk's xn2 vectors from LDS as broadcast reads.
constexpr int PR_TOK = 256;
constexpr int PR_DMAX = 64;  // Din <= 64 (registers sized by the DM = 32 / 64 instance)
constexpr int PR_NBMAX = 32;
constexpr int PR_UNROLL = 2;  // tokens per phase-2 step (4 spills at 3 waves per SIMD)

template <typename TX, int DM>
__global__ __launch_bounds__(256, 3) void ptower_rows_k(lthm_ptower_desc d, int total) {
  constexpr int LD = DM + 4;
  __shared__ __attribute__((aligned(16))) float xs2[PR_TOK * LD];
  __shared__ uint8_t msk[PR_TOK];
  const int tid = threadIdx.x;
  const int Din = d.Din;
  // this thread's projection (threads >= #projections only run phase 1)
  int nb = 0, rbase = 0, mine = 0;
  float Rc[DM], gr[PR_NBMAX];
  {
    int base = 0;
    for (int m = 0; m < d.n_mod; ++m) {
      const int npm = d.mod_nproj[m];
      if (tid >= base && tid < base + npm) {
        const int p = tid - base;
        mine = 1;
        nb = d.mod_nbins[m];
        rbase = d.mod_row_off[m] + (nb + 1) * p;
#pragma unroll
        for (int i = 0; i < DM; ++i) Rc[i] = (i < Din) ? d.proj[d.mod_proj_off[m] + i * npm + p] : 0.f;
#pragma unroll
        for (int q = 0; q < PR_NBMAX; ++q) gr[q] = (q < nb) ? d.grids[d.mod_grid_off[m] + q] : INFINITY;
      }
      base += npm;
    }
  }
  const TX* x = reinterpret_cast<const TX*>(d.x);
  const bool full = Din == DM;  // the chunk's x rows stage through LDS with lane-linear loads
  for (int64_t t0 = (int64_t)blockIdx.x * PR_TOK; t0 < d.n; t0 += (int64_t)gridDim.x * PR_TOK) {
    const int cnt = (int)min((int64_t)PR_TOK, d.n - t0);
    if (full) {
      // [cnt, DM] contiguous elements: consecutive lanes read consecutive elements
      const TX* xc = x + t0 * DM;
      for (int e = tid; e < cnt * DM; e += 256) xs2[(e / DM) * LD + (e % DM)] = Elem<TX>::ld(xc + e);
      __syncthreads();
    }
    {
      const int64_t t = t0 + tid;
      if (t < d.n) {
        float v[DM];
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < DM; ++i) {
          v[i] = (i < Din) ? (full ? xs2[tid * LD + i] : Elem<TX>::ld(x + t * Din + i)) : 0.f;
          ss += v[i] * v[i];
        }
        const float nrm = sqrtf(ss);
        const bool masked = (nrm < d.norm_threshold) || (d.ids[t] == 0);
        const float den = fmaxf(nrm, 1e-12f);
        float ss2 = 0.f;
#pragma unroll
        for (int i = 0; i < DM; ++i) {
          v[i] = v[i] / den;
          ss2 += v[i] * v[i];
        }
        if (d.xn_out) {
          bf16_t* xo = reinterpret_cast<bf16_t*>(d.xn_out) + t * Din;
          if (full) {
#pragma unroll
            for (int i = 0; i < DM; i += 8) store_vec<bf16_t, 8>(xo + i, v + i);
          } else {
#pragma unroll
            for (int i = 0; i < DM; ++i)
              if (i < Din) xo[i] = f2bf(v[i]);
          }
        }
        const float den2 = fmaxf(sqrtf(ss2), 1e-12f);
#pragma unroll
        for (int i = 0; i < DM; ++i)
          if (i < Din) xs2[tid * LD + i] = v[i] / den2;
        msk[tid] = masked ? 1 : 0;
        if (d.mask_out) d.mask_out[t] = masked ? 1 : 0;
        if (d.norm_bins > 0) {
          const float f = floorf(nrm * (float)d.norm_bins);  // HistogramEmbedding(0, 1, nbins), clamped
          const int hbin = (int)fminf(fmaxf(f, 0.f), (float)(d.norm_bins - 1));
          d.rows_out[t * total + (total - 1)] = masked ? (uint16_t)0xffff : (uint16_t)(d.cve_rows + hbin);
        }
      }
    }
    __syncthreads();
    if (mine) {
      // PU tokens per step: independent FMA chains (each in the sequential i order
      // of the one-token form) keep the broadcast LDS reads in flight
      constexpr int PU = PR_UNROLL;
      int tt = 0;
      for (; tt + PU <= cnt; tt += PU) {
        float z[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) z[u] = 0.f;
#pragma unroll
        for (int i = 0; i < DM; i += 4) {
          if (i < Din) {
#pragma unroll
            for (int u = 0; u < PU; ++u) {
              const f32x4 q = *reinterpret_cast<const f32x4*>(xs2 + (tt + u) * LD + i);
              z[u] = fmaf(q[0], Rc[i], z[u]);
              z[u] = fmaf(q[1], Rc[i + 1], z[u]);
              z[u] = fmaf(q[2], Rc[i + 2], z[u]);
              z[u] = fmaf(q[3], Rc[i + 3], z[u]);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < PU; ++u) {
          int bk = 0;
#pragma unroll
          for (int q = 0; q < PR_NBMAX; ++q) bk += (gr[q] < z[u]) ? 1 : 0;  // bucketize(right=False)
          d.rows_out[(t0 + tt + u) * total + tid] = msk[tt + u] ? (uint16_t)0xffff : (uint16_t)(rbase + bk);
        }
      }
      for (; tt < cnt; ++tt) {
        const float* xr = xs2 + tt * LD;
        float z = 0.f;
#pragma unroll
        for (int i = 0; i < DM; i += 4) {
          if (i < Din) {
            const f32x4 q = *reinterpret_cast<const f32x4*>(xr + i);
            z = fmaf(q[0], Rc[i], z);
            z = fmaf(q[1], Rc[i + 1], z);
            z = fmaf(q[2], Rc[i + 2], z);
            z = fmaf(q[3], Rc[i + 3], z);
          }
        }
        int bk = 0;
#pragma unroll
        for (int q = 0; q < PR_NBMAX; ++q) bk += (gr[q] < z) ? 1 : 0;  // bucketize(right=False)
        d.rows_out[(t0 + tt) * total + tid] = msk[tt] ? (uint16_t)0xffff : (uint16_t)(rbase + bk);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ product-tower embedding on MFMA
// emb[t, :] = b + W xn[t] + sum_s Tab[rows[t, s], :]   (rows from the FULL = false pass)
// The bag sums are a one-hot GEMM  onehot[t, k] . Tab[k, :]  over all R table
// rows k (exactly 0/1 in bf16, Tab bf16, f32 accumulation).  The block first
// turns its tokens' bucket rows into a per-token bitmask over the R rows (one
// LDS OR per (token, slot)); an A fragment (8 consecutive k of one token) is
// then one byte of that mask expanded through a 256-entry LDS table of bf16
// 0/1 octets.  Tab streams through LDS in 32-row slabs read with
// ds_read_tr16_b64.  Block = 8 waves = 128 tokens x D columns (D = 16 NF <= 256);
// for even NF a wave owns 32 tokens x D/2 columns, so every B fragment read
// from LDS feeds two MFMAs (LDS traffic per MFMA halved).  The mapper Linear
// (Din <= 64) runs on the MFMA as bf16 hi/lo splits.
constexpr int PE_TOK = 128;
constexpr int PE_MAXR = 4096;  // table rows

__host__ __device__ constexpr int pe_rbw(int R32) { return R32 / 32 + 1; }  // odd dword stride: no bank repeats

// DMA (D = 128 / 256): the slabs stream by LDS-DMA through a 4-deep ring instead of the
// register-staged double buffer: ring slots 0-1 sit where the double buffer was, slots
// 2-3 reuse the mapper's wN / xs staging once the mapper products are done, so up to
// three slabs are in flight behind the MFMAs (counted vmcnt + raw barrier per slab).
__device__ __attribute__((aligned(16))) unsigned char pt_zero16[16];

template <typename TX, int NF, bool DMA = false>
__global__ __launch_bounds__(512) void ptower_emb_mfma_k(lthm_ptower_desc d, int total, int R) {
  constexpr int D = 16 * NF;
  constexpr int CH = (NF % 2 == 0) ? 2 : 1;  // column halves
  constexpr int MT = CH;                     // 16-token tiles per wave
  constexpr int NFW = NF / CH;               // 16-column fragments per wave
  constexpr int TG = 8 / CH;                 // token groups
  constexpr int SLAB = 32 * D * 2;           // one 32-row bf16 slab
  constexpr int PD = (32 * D / 8 + 511) / 512;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // wN / xs rows padded to Din + 4 floats: the 16 rows a ds_read_b128 lane group reads start
  // on 16 distinct 16-B slots (Din = 32: the 128-B pitch put them on 2, an 8-way conflict)
  const int Din = d.Din, DinP = Din + 4;
  unsigned char* slab = smem;                                            // [2][SLAB]
  float* wN = reinterpret_cast<float*>(smem + 2 * SLAB);                // [D][DinP] (nn.Linear layout)
  float* xs = wN + DinP * D;                                            // [PE_TOK][DinP]
  uint2* lut = reinterpret_cast<uint2*>(xs + PE_TOK * DinP);            // [16][32]: nibble -> four bf16 0/1
  uint32_t* bits = reinterpret_cast<uint32_t*>(lut + 512);              // [PE_TOK][RBW]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int R32 = (R + 31) & ~31;
  const int RBW = pe_rbw(R32);
  const int64_t t0 = (int64_t)blockIdx.x * PE_TOK;
  // Dout > 256: blockIdx.y picks a 256-wide column slice of the ldt = Dout wide rows
  const int ldt = D * (int)gridDim.y, col0 = D * (int)blockIdx.y;
  const bf16_t* tab = reinterpret_cast<const bf16_t*>(d.tables) + col0;
  // ---- per-block staging: mapper weights, 0/1 octet table, row bitmask, normalised x
  for (int i = tid; i < Din * D; i += 512) wN[(i / Din) * DinP + i % Din] = d.w_map[(int64_t)col0 * Din + i];
  {
    // A fragment = two nibble lookups; 32 copies of the 16-entry table, copy = lane & 31, entry
    // n at n * 256 B + 8 copy: a 32-lane ds_read_b64 group covers all 64 banks whatever the
    // nibbles (the 256-entry octet table read with ds_read_b128 hit random banks)
    const int n = tid >> 5;
    lut[tid] = uint2{((n & 1) ? 0x3F80u : 0u) | ((n & 2) ? 0x3F800000u : 0u),
                     ((n & 4) ? 0x3F80u : 0u) | ((n & 8) ? 0x3F800000u : 0u)};
  }
  for (int i = tid; i < PE_TOK * RBW; i += 512) bits[i] = 0u;
  __syncthreads();
  {
    // the block's rows are one contiguous run of nv uint16: 16-B loads, all of a thread's
    // chunks in flight before the first LDS OR (was one dependent 2-byte load per OR)
    const int64_t nt = min((int64_t)PE_TOK, d.n - t0);
    const int nv = (int)nt * total;
    const uint16_t* src = d.rows_out + t0 * total;
    if (((uintptr_t)src & 15) == 0) {
      constexpr int PASS = 9;  // 9 x 512 x 8 = 36864 >= PE_TOK * total for total <= 257 (nproj <= 256)
      u32x4 v[PASS];
#pragma unroll
      for (int q = 0; q < PASS; ++q) {
        const int c = tid + 512 * q;
        v[q] = c * 8 < nv ? *reinterpret_cast<const u32x4*>(src + c * 8) : u32x4{0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
      }
#pragma unroll
      for (int q = 0; q < PASS; ++q) {
        const int c = tid + 512 * q;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = c * 8 + e;
          const int k = (int)((v[q][e >> 1] >> (16 * (e & 1))) & 0xffffu);
          if (i < nv && k < R) {
            const int tt = i / total;
            atomicOr(bits + tt * RBW + (k >> 5), 1u << (k & 31));
          }
        }
      }
    } else {
      for (int i = tid; i < nv; i += 512) {
        const int k = src[i];
        if (k < R) atomicOr(bits + (i / total) * RBW + (k >> 5), 1u << (k & 31));
      }
    }
  }
  {
    // xn = x / max(|x|, 1e-12): 8 lanes per token
    const TX* x = reinterpret_cast<const TX*>(d.x);
    for (int tb = w * 8 + (lane >> 3); tb < PE_TOK; tb += 64) {
      const int64_t t = t0 + tb;
      float v[8];
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = (lane & 7) + 8 * i;
        v[i] = (t < d.n && c < Din) ? Elem<TX>::ld(x + t * Din + c) : 0.f;
        ss += v[i] * v[i];
      }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) ss += __shfl_xor(ss, o, 64);
      const float den = fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = (lane & 7) + 8 * i;
        if (c < Din) xs[tb * DinP + c] = v[i] / den;
      }
    }
  }
  // ---- slab pipeline
  u32x4 pf[PD];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int q = 0; q < PD; ++q) {
      const int idx = tid + 512 * q;
      const int r = idx / (D / 8), c = idx - r * (D / 8);
      pf[q] = u32x4{0u, 0u, 0u, 0u};
      if (idx < 32 * D / 8 && k0 + r < R) pf[q] = *reinterpret_cast<const u32x4*>(tab + (int64_t)(k0 + r) * ldt + c * 8);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < PD; ++q) {
      const int idx = tid + 512 * q;
      const int r = idx / (D / 8), c = idx - r * (D / 8);
      if (idx < 32 * D / 8) *reinterpret_cast<u32x4*>(slab + buf * SLAB + ct_off<D>(r, c)) = pf[q];
    }
  };
  // DMA slab k0 / 32 into ring slot `slot`: piece p = 1 KiB = 512 / D rows; lane l lands at
  // row p (512 / D) + l / NC, slot l % NC, so it loads chunk slot ^ ct_swz(row) (ct_off)
  constexpr int NC = D / 8;
  constexpr int DPW = DMA ? D / 128 : 1;  // DMAs per wave and slab (16 or 8 pieces over 8 waves)
  auto ring = [&](int slot) -> unsigned char* {
    return slot < 2 ? slab + slot * SLAB : reinterpret_cast<unsigned char*>(wN) + (slot - 2) * SLAB;
  };
  auto issue = [&](int sl) {
    const int k0 = sl * 32;
    unsigned char* img = ring(sl & 3);
#pragma unroll
    for (int q = 0; q < DPW; ++q) {
      const int pc = w + 8 * q;
      const int row = pc * (512 / D) + lane / NC;
      const int ch = (lane % NC) ^ ct_swz<D>(row);
      const void* src = k0 + row < R ? (const void*)(tab + (int64_t)(k0 + row) * ldt + ch * 8) : (const void*)pt_zero16;
      glds16(src, img + pc * 1024);
    }
  };
  const int nslab = R32 / 32;
  if constexpr (DMA) {
    issue(0);
    if (nslab > 1) issue(1);
    __syncthreads();  // (drains the two slab DMAs with the staging loads)
  } else {
    fetch(0);
    store(0);
    __syncthreads();
  }
  const int tg = w % TG, chh = w / TG;
  const int nb0 = chh * NFW * 16;  // first column of this wave
  f32x4 acc[MT][NFW];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int f = 0; f < NFW; ++f) acc[mt][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  // mapper xn . W^T on MFMA: f32 operands split into bf16 hi + lo, three products
  // (hi.hi + hi.lo + lo.hi) keep ~16 mantissa bits
  auto split8 = [](const float* p, int valid, bf16x8v& hi, bf16x8v& lo) {
    s16x8 h, l;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = i < valid ? p[i] : 0.f;
      const uint32_t u = __float_as_uint(v) & 0xffff0000u;
      h[i] = (short)(u >> 16);
      l[i] = (short)f2bf(v - __uint_as_float(u));
    }
    hi = __builtin_bit_cast(bf16x8v, h);
    lo = __builtin_bit_cast(bf16x8v, l);
  };
  for (int k0 = 0; k0 < Din; k0 += 32) {
    const int kb = k0 + 8 * (lane >> 4);
    const int valid = max(0, min(8, Din - kb));
    bf16x8v xh[MT], xl[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) split8(xs + (tg * 16 * MT + mt * 16 + (lane & 15)) * DinP + kb, valid, xh[mt], xl[mt]);
#pragma unroll
    for (int f = 0; f < NFW; ++f) {
      bf16x8v wh, wl;
      split8(wN + (nb0 + f * 16 + (lane & 15)) * DinP + kb, valid, wh, wl);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[mt][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh[mt], wh, acc[mt][f], 0, 0, 0);
        acc[mt][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh[mt], wl, acc[mt][f], 0, 0, 0);
        acc[mt][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xl[mt], wh, acc[mt][f], 0, 0, 0);
      }
    }
  }
  // this lane's mask bytes: token row tl(mt), byte (k0 >> 3) + (lane >> 4)
  const unsigned char* mb[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
    mb[mt] = reinterpret_cast<const unsigned char*>(bits + (tg * 16 * MT + mt * 16 + (lane & 15)) * RBW) + (lane >> 4);
  if constexpr (DMA) {
    __syncthreads();  // every wave is done with wN / xs: ring slots 2-3 take them over
    if (nslab > 2) issue(2);
    if (nslab > 3) issue(3);
  }
  for (int sI = 0; sI < nslab; ++sI) {
    const int cur = sI & 1, k0 = sI * 32;
    const bool more = sI + 1 < nslab;
    const unsigned char* img;
    if constexpr (DMA) {
      // slabs issued: 0 .. min(nslab - 1, sI + 2) (sI = 0: .. 3); slab sI must have landed
      const int pend = min(nslab - 1, sI == 0 ? 3 : sI + 2) - sI;
      if (pend >= 3) wait_vm<3 * DPW>();
      else if (pend == 2) wait_vm<2 * DPW>();
      else if (pend == 1) wait_vm<DPW>();
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();  // also: every wave is done with slot (sI - 1) & 3
      if (sI >= 1 && sI + 3 < nslab) issue(sI + 3);
      img = ring(sI & 3);
    } else {
      if (more) fetch(k0 + 32);
      img = slab + cur * SLAB;
    }
    bf16x8v af[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const unsigned v = mb[mt][k0 >> 3];
      const uint2 lo = lut[(v & 15) * 32 + (lane & 31)], hi = lut[(v >> 4) * 32 + (lane & 31)];
      af[mt] = __builtin_bit_cast(bf16x8v, u32x4{lo.x, lo.y, hi.x, hi.y});
    }
#pragma unroll
    for (int f = 0; f < NFW; ++f) {
      const bf16x8v bf = ct_tr_frag<D>(img, nb0 + f * 16, lane);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        acc[mt][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bf, acc[mt][f], 0, 0, 0);
    }
    if constexpr (!DMA) {
      if (more) store(cur ^ 1);
      __syncthreads();
    }
  }
  // ---- epilogue: + bias, mask fill, bf16 store
  bf16_t* eo = reinterpret_cast<bf16_t*>(d.emb_out);
  float bias[NFW];
#pragma unroll
  for (int f = 0; f < NFW; ++f) bias[f] = d.b_map ? d.b_map[col0 + nb0 + f * 16 + (lane & 15)] : 0.f;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tb = tg * 16 * MT + mt * 16 + 4 * (lane >> 4) + j;
      const int64_t t = t0 + tb;
      if (t >= d.n) continue;
      const bool masked = d.mask_out[t] != 0;
#pragma unroll
      for (int f = 0; f < NFW; ++f)
        eo[t * ldt + col0 + nb0 + f * 16 + (lane & 15)] = f2bf(masked ? 0.f : acc[mt][f][j] + bias[f]);
    }
}

// ------------------------------------------------------------------ small-table gradient
// dW[rows[t, i]] += dY[t] for every token t and index slot i (0xffff = skip).
// The slots are grouped into segments (e.g. a run of CosineVectorEmbedding
// projections whose rows form one contiguous range).  Grid: (64-column groups,
// segments, token chunks).  A block privatises its segment's [rows, 64] slice in
// LDS.  One wave walks one token at a time: its 64 lanes hold the token's 64
// dY columns, the slot row indices are loaded one per lane and broadcast with
// v_readlane into SGPRs, so every slot costs one return-less ds_add_f32 over 64
// consecutive banks (no LDS round trip on the critical path).  Chunk z writes
// its slice with plain stores into part[z] (or adds it to dW when there is one
// chunk); seg_tab_reduce_k then folds the chunks into dW in a fixed order, so
// no global atomics are used and the cross-chunk sum is deterministic.
constexpr int ST_CG = 64;
constexpr int ST_MAXSEG = 64;
struct SegTab {
  int nseg;
  int slot0[ST_MAXSEG], nslot[ST_MAXSEG], row0[ST_MAXSEG], nrow[ST_MAXSEG];
};

template <typename TY>
__global__ __launch_bounds__(256) void seg_tab_bwd_k(const uint16_t* __restrict__ rows, int nidx, const TY* __restrict__ dY,
                                                    int64_t ldy, int64_t n, int D, float* __restrict__ dst,
                                                    int64_t zstride, int direct, int64_t tok_per_block, SegTab st) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* acc = reinterpret_cast<float*>(smem);  // [R][64]
  const int seg = blockIdx.y;
  const int s0 = st.slot0[seg], ns = st.nslot[seg], r0 = st.row0[seg], R = st.nrow[seg];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < R * ST_CG; i += 256) acc[i] = 0.f;
  __syncthreads();
  const int col = blockIdx.x * ST_CG + lane;
  const bool cv = col < D;
  const int64_t t0 = (int64_t)blockIdx.z * tok_per_block;
  const int64_t t1 = min(n, t0 + tok_per_block);
  float* accl = acc + lane;
  for (int64_t t = t0 + wave; t < t1; t += 8) {
    // two tokens per iteration (t, t+4): both loads are in flight before the adds
    const int64_t u = t + 4;
    const bool uv = u < t1;
    const float va = cv ? Elem<TY>::ld(dY + t * ldy + col) : 0.f;
    const float vb = (cv && uv) ? Elem<TY>::ld(dY + u * ldy + col) : 0.f;
    const int ra = lane < ns ? (int)rows[t * nidx + s0 + lane] : 0xffff;
    const int rb = (lane < ns && uv) ? (int)rows[u * nidx + s0 + lane] : 0xffff;
    for (int i = 0; i < ns; ++i) {
      const int r = __builtin_amdgcn_readlane(ra, i) - r0;
      if ((unsigned)r < (unsigned)R) atomicAdd(accl + r * ST_CG, va);
    }
    if (uv) {
      for (int i = 0; i < ns; ++i) {
        const int r = __builtin_amdgcn_readlane(rb, i) - r0;
        if ((unsigned)r < (unsigned)R) atomicAdd(accl + r * ST_CG, vb);
      }
    }
  }
  __syncthreads();
  float* out = dst + (direct ? 0 : (int64_t)blockIdx.z * zstride);
  for (int i = tid; i < R * ST_CG; i += 256) {
    const int rr = i / ST_CG, cc = i - rr * ST_CG;
    const int cl = blockIdx.x * ST_CG + cc;
    if (cl < D) {
      float* p = out + (int64_t)(r0 + rr) * D + cl;
      if (direct) *p += acc[i];
      else *p = acc[i];
    }
  }
}

// dW[r, :] += sum_z part[z, r, :] over the rows of every segment (z ascending).
__global__ __launch_bounds__(256) void seg_tab_reduce_k(const float* __restrict__ part, int64_t zstride, int nz, int D,
                                                       float* __restrict__ dW, SegTab st) {
  const int seg = blockIdx.y;
  const int64_t base = (int64_t)st.row0[seg] * D;
  const int64_t cnt = (int64_t)st.nrow[seg] * D;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * 256) {
    float s = 0.f;
    for (int z = 0; z < nz; ++z) s += part[z * zstride + base + i];
    dW[base + i] += s;
  }
}

// ------------------------------------------------------------------ CVE table gradient on MFMA
// For tables laid out like the CosineVectorEmbedding modules (module j: slots
// [slot0_j, +nslot_j), slot s owning rows [row0_j + (s - slot0_j)*rps_j, +rps_j)):
//     dW[m, :] += sum_t [rows[t, s(m)] == m] * dY[t, :]
// is a one-hot GEMM  dW[M, D] = A[M, tokens] . dY[tokens, D]  with A built on
// the fly (one compare per element; A is exactly 0/1 in bf16 and dY is bf16, so
// every product is exact and only the f32 summation order differs from a
// scatter-add).  Block = 8 waves = 128 table rows (one 16-row MFMA tile per
// wave) x all D columns; tokens stream through LDS 32 at a time, double-buffered
// (dY as a swizzled [32, D] image read with ds_read_tr16_b64, bucket ids
// transposed to [slot][token]).  Token chunks (blockIdx.z) write f32 partials
// that seg_tab_reduce_k folds in a fixed order.  Replaces the LDS-atomic scatter
// for this layout: LDS float atomics sustain ~1 slot-update per ~190 CU cycles.
constexpr int CT_MAXTILE = 64;
constexpr int CT_ROWS = 128;   // rows per tile (8 waves x 16)
constexpr int CT_KT = 32;      // tokens per k-step
// bucket-id tile row pitch (uint16): 40 instead of 32 puts the 16 slots a wave's
// transposed 2-byte stores hit at once on 16 distinct banks (32: 4 banks, 16-way)
constexpr int CT_RTLD = CT_KT + 8;
constexpr int CT_MAXSL = 128;  // slots covering one tile
struct CveTiles {
  int ntile;
  int row0[CT_MAXTILE], nrow[CT_MAXTILE], sfirst[CT_MAXTILE], nsl[CT_MAXTILE];
  int mrow0[CT_MAXTILE], mslot0[CT_MAXTILE], rps[CT_MAXTILE];
};

// F32: dY is f32, staged as bf16 hi and lo images (two MFMAs per fragment, ~16
// mantissa bits).  GEN: slots are not tied to row ranges (e.g. a slot that
// holds either an action row or the pad row); A[m, t] counts the slots of the
// token whose row is m (<= CT_GENMAX slots, exact small integers in bf16).
constexpr int CT_GENMAX = 8;
template <int D, bool F32, bool GEN>
__global__ __launch_bounds__(512) void cve_tab_bwd_k(const uint16_t* __restrict__ rows, int nidx,
                                                    const void* __restrict__ dYv, int64_t ldy, int64_t n,
                                                    float* __restrict__ dst, int64_t zstride, int direct,
                                                    int64_t tok_per_block, CveTiles ct) {
  constexpr int NF = D / 16;
  constexpr int EPC = F32 ? 4 : 8;              // dY elements per 16-byte chunk
  constexpr int NCH = D / EPC;                  // 16-byte chunks per dY row
  constexpr int IMG = CT_KT * D * 2;            // one bf16 dY image
  constexpr int RTB = CT_MAXSL * CT_RTLD * 2;   // bucket-id tile bytes
  constexpr int BUF = (F32 ? 2 : 1) * IMG + RTB;
  constexpr int PD = (CT_KT * NCH + 511) / 512;
  constexpr int PR = (CT_KT * CT_MAXSL + 511) / 512;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // XCD-aware order: the row tiles of one token chunk get consecutive logical ids,
  // i.e. land on the same XCD, so the chunk's dY streams from HBM once and the
  // other tiles read it from that XCD's L2 (not once per tile)
  const int nbl = (int)(gridDim.x * gridDim.z);
  const int lid = xcd_remap((int)(blockIdx.x + gridDim.x * blockIdx.z), nbl);
  const int tile = lid % (int)gridDim.x;
  const int zc = lid / (int)gridDim.x;
  const int row0 = ct.row0[tile], nrow = ct.nrow[tile], sfirst = ct.sfirst[tile], nsl = ct.nsl[tile];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t t0 = (int64_t)zc * tok_per_block;
  const int64_t t1 = min(n, t0 + tok_per_block);
  // for even NF a wave owns 32 table rows (two 16-row MFMA tiles) x D/2 columns, so
  // every dY fragment read from LDS feeds two MFMAs
  constexpr int CH = (NF % 2 == 0) ? 2 : 1;
  constexpr int MT = CH, NFW = NF / CH, RG = 8 / CH;
  const int rgp = wave % RG, nb0 = (wave / RG) * NFW * 16;
  int mrow[MT], ls[MT];
  bool mvalid[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int ml = rgp * 16 * MT + mt * 16 + (lane & 15);
    mvalid[mt] = ml < nrow;
    mrow[mt] = row0 + ml;
    ls[mt] = (!GEN && mvalid[mt]) ? ct.mslot0[tile] + (mrow[mt] - ct.mrow0[tile]) / ct.rps[tile] - sfirst : 0;
  }
  f32x4 acc[MT][NFW];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int f = 0; f < NFW; ++f) acc[mt][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 pd[PD];
  uint16_t pr[PR];
  auto fetch = [&](int64_t tb) {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      const int idx = tid + 512 * k;
      const int r = idx / NCH, c = idx - r * NCH;
      pd[k] = u32x4{0u, 0u, 0u, 0u};
      if (idx < CT_KT * NCH && tb + r < t1) {
        if constexpr (F32) pd[k] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const float*>(dYv) + (tb + r) * ldy + c * 4);
        else pd[k] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(dYv) + (tb + r) * ldy + c * 8);
      }
    }
#pragma unroll
    for (int k = 0; k < PR; ++k) {
      const int idx = tid + 512 * k;
      const int r = idx / nsl, s = idx - r * nsl;
      pr[k] = 0xffff;
      if (idx < CT_KT * nsl && tb + r < t1) pr[k] = rows[(tb + r) * nidx + sfirst + s];
    }
  };
  auto store = [&](int buf) {
    unsigned char* img = smem + buf * BUF;
    uint16_t* rt = reinterpret_cast<uint16_t*>(img + (F32 ? 2 : 1) * IMG);
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      const int idx = tid + 512 * k;
      const int r = idx / NCH, c = idx - r * NCH;
      if (idx < CT_KT * NCH) {
        if constexpr (F32) {
          u32x2 hi, lo;
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // hi = RNE bf16, lo = RNE bf16 of the remainder (<= 2^-18 rel.)
            const float v0 = __uint_as_float(pd[k][2 * h]), v1 = __uint_as_float(pd[k][2 * h + 1]);
            const bf16_t h0 = f2bf(v0), h1 = f2bf(v1);
            hi[h] = (uint32_t)h0 | ((uint32_t)h1 << 16);
            lo[h] = (uint32_t)f2bf(v0 - bf2f(h0)) | ((uint32_t)f2bf(v1 - bf2f(h1)) << 16);
          }
          const int off = ct_off<D>(r, c >> 1) + 8 * (c & 1);
          *reinterpret_cast<u32x2*>(img + off) = hi;
          *reinterpret_cast<u32x2*>(img + IMG + off) = lo;
        } else {
          *reinterpret_cast<u32x4*>(img + ct_off<D>(r, c)) = pd[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < PR; ++k) {
      const int idx = tid + 512 * k;
      const int r = idx / nsl, s = idx - r * nsl;
      if (idx < CT_KT * nsl) rt[s * CT_RTLD + r] = pr[k];
    }
  };
  const int64_t nsteps = (t1 - t0 + CT_KT - 1) / CT_KT;
  if (nsteps > 0) {
    fetch(t0);
    store(0);
  }
  __syncthreads();
  for (int64_t st = 0; st < nsteps; ++st) {
    const int cur = (int)(st & 1);
    if (st + 1 < nsteps) fetch(t0 + (st + 1) * CT_KT);  // global loads in flight during the MFMAs
    const unsigned char* img = smem + cur * BUF;
    const uint16_t* rt = reinterpret_cast<const uint16_t*>(img + (F32 ? 2 : 1) * IMG);
    bf16x8v af[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      s16x8 a;
      if constexpr (GEN) {
        int cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int sl = 0; sl < CT_GENMAX; ++sl) {
          if (sl < nsl) {
            const u32x4 rv = *reinterpret_cast<const u32x4*>(rt + sl * CT_RTLD + 8 * (lane >> 4));
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const uint32_t rr = (i & 1) ? (rv[i >> 1] >> 16) : (rv[i >> 1] & 0xffffu);
              cnt[i] += ((int)rr == mrow[mt]) ? 1 : 0;
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = mvalid[mt] ? (short)f2bf((float)cnt[i]) : (short)0;
      } else {
        const u32x4 rv = *reinterpret_cast<const u32x4*>(rt + ls[mt] * CT_RTLD + 8 * (lane >> 4));
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t rr = (i & 1) ? (rv[i >> 1] >> 16) : (rv[i >> 1] & 0xffffu);
          a[i] = (mvalid[mt] && (int)rr == mrow[mt]) ? (short)0x3F80 : (short)0;
        }
      }
      af[mt] = __builtin_bit_cast(bf16x8v, a);
    }
#pragma unroll
    for (int f = 0; f < NFW; ++f) {
      const bf16x8v bh = ct_tr_frag<D>(img, nb0 + f * 16, lane);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bh, acc[mt][f], 0, 0, 0);
      if constexpr (F32) {
        const bf16x8v bl = ct_tr_frag<D>(img + IMG, nb0 + f * 16, lane);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          acc[mt][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bl, acc[mt][f], 0, 0, 0);
      }
    }
    if (st + 1 < nsteps) store(cur ^ 1);
    __syncthreads();
  }
  float* out = dst + (direct ? 0 : (int64_t)zc * zstride);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rl = rgp * 16 * MT + mt * 16 + 4 * (lane >> 4) + j;
      if (rl < nrow) {
        float* p = out + (int64_t)(row0 + rl) * D + nb0 + (lane & 15);
#pragma unroll
        for (int f = 0; f < NFW; ++f) {
          if (direct) p[f * 16] += acc[mt][f][j];
          else p[f * 16] = acc[mt][f][j];
        }
      }
    }
}

// ------------------------------------------------------------------ token assembly
// x0[b, 0]   = wpe[T] (+ ctx[b])
// x0[b, t+1] = (mask ? pad : P[b,t] + act[lab] + hod[.] + how[.] + dow[.]) + wpe[T-1-t]
template <typename TP, bool VEC>
__global__ __launch_bounds__(256) void tokens_fwd_k(lthm_tokens_desc d) {
  // A wave takes 64 rows at a time: lane l first derives the table indices of row r0 + l
  // (the label / timestamp loads and the 64-bit floor-div / mod chains of all 64 rows in
  // parallel), then the wave assembles the rows one after the other with those indices
  // read back by lane broadcast, 64 columns per instruction.
  const int T = d.T_full - d.trim, Tp = T + 1, D = d.d;
  const int64_t rows = d.B * Tp;
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4 * 64;
  for (int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64; r0 < rows; r0 += wstride) {
    const int64_t r = r0 + lane;
    int kind = 0;  // 0: context token (tp == 0), 1: pad, 2: item token
    int ia = 0, ih = 0, iw = 0, idw = 0, wrow = 0;
    int64_t b = 0, src = 0;
    if (r < rows) {
      b = r / Tp;
      const int tp = (int)(r - b * Tp);
      uint16_t ri[5] = {0xffff, 0xffff, 0xffff, 0xffff, 0xffff};
      wrow = T - tp;  // pos = seq_len - arange(0, seq_len + 1)
      ri[4] = (uint16_t)(d.off_wpe + wrow);
      if (tp > 0) {
        const int64_t g = b * d.T_full + d.trim + (tp - 1);
        if (d.mask[g] != 0) {
          kind = 1;
          ri[0] = (uint16_t)d.off_pad;
        } else {
          kind = 2;
          ia = (int)pymod64(d.labels[g], 4);
          const int64_t ts = d.ts[g];
          ih = (int)pymod64(floordiv64(ts, d.div_hod), d.mod_hod);
          iw = (int)pymod64(floordiv64(ts, d.div_how), d.mod_how);
          idw = (int)pymod64(floordiv64(ts, d.div_dow), d.mod_dow);
          ri[0] = (uint16_t)(d.off_act + ia);
          ri[1] = (uint16_t)(d.off_hod + ih);
          ri[2] = (uint16_t)(d.off_how + iw);
          ri[3] = (uint16_t)(d.off_dow + idw);
          src = b * T + (tp - 1);
        }
      }
      if (d.rows_out) {
#pragma unroll
        for (int i = 0; i < 5; ++i) d.rows_out[r * 5 + i] = ri[i];
      }
    }
    const int nr = (int)min((int64_t)64, rows - r0);
    if (VEC) {  // D == 256
      // 4 rows per step, every load of the 4 rows issued before the first store; lane l owns
      // columns 4 l .. 4 l + 3 (16-B table / x0 accesses, 8-B bf16 P accesses)
      const int c = 4 * lane;
      for (int k0 = 0; k0 < nr; k0 += 4) {
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = min(k0 + u, nr - 1);
          const int kk = __shfl(kind, k, 64), wr = __shfl(wrow, k, 64);
          const int a0 = __shfl(ia, k, 64), a1 = __shfl(ih, k, 64), a2 = __shfl(iw, k, 64), a3 = __shfl(idw, k, 64);
          const int64_t bk = (int64_t)__shfl((int)b, k, 64);
          const int64_t sk = ((int64_t)__shfl((int)(src >> 32), k, 64) << 32) | (uint32_t)__shfl((int)src, k, 64);
          f32x4 x;
          if (kk == 0) {
            x = d.ctx ? *reinterpret_cast<const f32x4*>(d.ctx + bk * 256 + c) : f32x4{0.f, 0.f, 0.f, 0.f};
          } else if (kk == 1) {
            x = *reinterpret_cast<const f32x4*>(d.pad + c);
          } else {
            if constexpr (sizeof(TP) == 2) {
              const u32x2 w = *reinterpret_cast<const u32x2*>(reinterpret_cast<const bf16_t*>(d.P) + sk * 256 + c);
              x = f32x4{__uint_as_float(w[0] << 16), __uint_as_float(w[0] & 0xffff0000u),
                        __uint_as_float(w[1] << 16), __uint_as_float(w[1] & 0xffff0000u)};
            } else {
              x = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(d.P) + sk * 256 + c);
            }
            // the same left-to-right sum as the scalar path: P + act + hod + how + dow
            x = x + *reinterpret_cast<const f32x4*>(d.act + a0 * 256 + c);
            x = x + *reinterpret_cast<const f32x4*>(d.hod + a1 * 256 + c);
            x = x + *reinterpret_cast<const f32x4*>(d.how + a2 * 256 + c);
            x = x + *reinterpret_cast<const f32x4*>(d.dow + a3 * 256 + c);
          }
          v[u] = x + *reinterpret_cast<const f32x4*>(d.wpe + (int64_t)wr * 256 + c);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (k0 + u < nr) *reinterpret_cast<f32x4*>(d.x0 + (r0 + k0 + u) * 256 + c) = v[u];
      }
      continue;
    }
    for (int k = 0; k < nr; ++k) {
      const int kk = __shfl(kind, k, 64), wr = __shfl(wrow, k, 64);
      const int a0 = __shfl(ia, k, 64), a1 = __shfl(ih, k, 64), a2 = __shfl(iw, k, 64), a3 = __shfl(idw, k, 64);
      const int64_t bk = (int64_t)__shfl((int)b, k, 64);
      const int64_t sk = ((int64_t)__shfl((int)(src >> 32), k, 64) << 32) | (uint32_t)__shfl((int)src, k, 64);
      const int64_t rk = r0 + k;
      for (int c = lane; c < D; c += 64) {
        float v;
        if (kk == 0) {
          v = d.ctx ? d.ctx[bk * D + c] : 0.f;
        } else if (kk == 1) {
          v = d.pad[c];
        } else {
          v = Elem<TP>::ld(reinterpret_cast<const TP*>(d.P) + sk * D + c);
          v = v + d.act[a0 * D + c] + d.hod[a1 * D + c] + d.how[a2 * D + c] + d.dow[a3 * D + c];
        }
        v = v + d.wpe[(int64_t)wr * D + c];
        d.x0[rk * D + c] = v;
      }
    }
  }
}

// dP[b, t] = mask ? 0 : dx0[b, t+1] (bf16), dctx[b] = dx0[b, 0]
__global__ __launch_bounds__(256) void tokens_bwd_k(lthm_tokens_desc d, const float* __restrict__ dx0, bf16_t* __restrict__ dP,
                                                    float* __restrict__ dctx) {
  const int T = d.T_full - d.trim, Tp = T + 1, D = d.d;
  const int64_t rows = d.B * Tp;
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    const int64_t b = r / Tp;
    const int tp = (int)(r - b * Tp);
    if (tp == 0) {
      if (dctx)
        for (int c = lane; c < D; c += 64) dctx[b * D + c] = dx0[r * D + c];
      continue;
    }
    const bool masked = d.mask[b * d.T_full + d.trim + tp - 1] != 0;
    if ((D & 3) == 0 && (((uintptr_t)dx0 | (uintptr_t)dP) & 15) == 0) {  // uniform: 16-B reads, 8-B writes
      for (int c = 4 * lane; c < D; c += 256) {
        const f32x4 v = masked ? f32x4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(dx0 + r * D + c);
        *reinterpret_cast<u32x2*>(dP + (b * T + tp - 1) * D + c) = u32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
      }
    } else {
      for (int c = lane; c < D; c += 64) dP[(b * T + tp - 1) * D + c] = f2bf(masked ? 0.f : dx0[r * D + c]);
    }
  }
}

// out[b, t'] = bf16(x[b, t'] + oc[outcome(b, t')]);  outcome = label of token t' (t' < T), future (t' = T)
__global__ __launch_bounds__(256) void outcome_fwd_k(const float* __restrict__ x, const int64_t* __restrict__ labels, int64_t B,
                                                     int T_full, int trim, int64_t future, const float* __restrict__ oc,
                                                     int noc, int D, bf16_t* __restrict__ out, uint16_t* __restrict__ rows) {
  const int T = T_full - trim, Tp = T + 1;
  const int64_t nrow = B * Tp;
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < nrow; r += (int64_t)gridDim.x * 4) {
    const int64_t b = r / Tp;
    const int tp = (int)(r - b * Tp);
    const int64_t lab = (tp < T) ? labels[b * T_full + trim + tp] : future;
    const int64_t o = pymod64(lab, noc);
    if ((D & 3) == 0 && (((uintptr_t)x | (uintptr_t)oc | (uintptr_t)out) & 15) == 0) {  // uniform
      for (int c = 4 * lane; c < D; c += 256) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(x + r * D + c) + *reinterpret_cast<const f32x4*>(oc + o * D + c);
        *reinterpret_cast<u32x2*>(out + r * D + c) = u32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
      }
    } else {
      for (int c = lane; c < D; c += 64) out[r * D + c] = f2bf(x[r * D + c] + oc[o * D + c]);
    }
    if (lane == 0 && rows) rows[r] = (uint16_t)o;
  }
}

}  // namespace lthm

using namespace lthm;

extern "C" int lthm_flip_tokens(const int64_t* in, int64_t* out, int64_t B, int32_t T, void* stream) {
  LTHM_REQUIRE(B >= 0 && T >= 0 && in != out);
  if (B * T == 0) return 0;
  hipLaunchKernelGGL(flip_k, dim3(grid_for(B * T, 256)), dim3(256), 0, (hipStream_t)stream, in, out, B, T);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_product_tower_fwd(const lthm_ptower_desc* d, void* stream) {
  LTHM_REQUIRE(d && d->n >= 0 && d->Din > 0 && d->Din <= 256 && d->n_mod >= 0 && d->n_mod <= LTHM_MAX_CVE);
  LTHM_REQUIRE(d->Dout > 0 && d->Dout <= 512);
  if (d->n == 0) return 0;
  int total = 0;
  for (int j = 0; j < d->n_mod; ++j) total += d->mod_nproj[j];
  total += d->norm_bins > 0 ? 1 : 0;
  LTHM_REQUIRE(total <= 1024);
  const size_t sh = (size_t)(d->Din * d->Dout + d->proj_total + d->grid_total + 8 * d->Din) * 4 + (size_t)4 * total * 2 + 16;
  LTHM_REQUIRE(sh <= 160 * 1024);
  const int grid = grid_for(d->n, 4, 256 * 8);
  hipStream_t s = (hipStream_t)stream;
  const int opl = d->Dout <= 64 ? 1 : d->Dout <= 128 ? 2 : d->Dout <= 256 ? 4 : 8;
  LTHM_REQUIRE(d->Dout % opl == 0);
  // MFMA path: per-token pass (rows, mask) + one-hot GEMM for the bag sums
  const int R = d->cve_rows + (d->norm_bins > 0 ? d->norm_bins : 0);
  const int R32 = (R + 31) & ~31;
  const int Dm = d->Dout;
  const int nsl = (Dm > 256 && Dm % 256 == 0) ? Dm / 256 : 1;  // 256-wide column slices (grid.y)
  const int Ds = Dm / nsl;
  const size_t sh_mfma = (size_t)2 * 32 * Ds * 2 + (size_t)(d->Din + 4) * Ds * 4 + (size_t)PE_TOK * (d->Din + 4) * 4 +
                         (size_t)512 * 8 + (size_t)PE_TOK * pe_rbw(R32) * 4;
  int maxnb = 0, nproj = 0;
  for (int j = 0; j < d->n_mod; ++j) {
    maxnb = std::max(maxnb, d->mod_nbins[j]);
    nproj += d->mod_nproj[j];
  }
  const bool mfma = !d->cve_only && d->tab_dtype == LTHM_BF16 && d->emb_dtype == LTHM_BF16 && d->rows_out &&
                    d->mask_out && d->ids && (Ds == 16 || Ds == 32 || Ds == 64 || Ds == 128 || Ds == 256) && nsl <= 4 && R > 0 &&
                    R <= PE_MAXR && sh_mfma <= 160 * 1024 && d->Din <= PR_DMAX && d->Din % 4 == 0 &&
                    maxnb <= PR_NBMAX && nproj <= 256;
  if (mfma) {
    const dim3 g1((unsigned)std::min<int64_t>((d->n + PR_TOK - 1) / PR_TOK, 4096));
    if (d->Din <= 32) {
      if (d->x_dtype == LTHM_BF16) hipLaunchKernelGGL((ptower_rows_k<bf16_t, 32>), g1, dim3(256), 0, s, *d, total);
      else hipLaunchKernelGGL((ptower_rows_k<float, 32>), g1, dim3(256), 0, s, *d, total);
    } else {
      if (d->x_dtype == LTHM_BF16) hipLaunchKernelGGL((ptower_rows_k<bf16_t, 64>), g1, dim3(256), 0, s, *d, total);
      else hipLaunchKernelGGL((ptower_rows_k<float, 64>), g1, dim3(256), 0, s, *d, total);
    }
    LTHM_CHECK_LAUNCH();
    const dim3 g2((unsigned)((d->n + PE_TOK - 1) / PE_TOK), (unsigned)nsl);
    // the 4-deep DMA ring needs the mapper staging (wN + xs) to hold two 32-row slabs
    const bool dma = (Ds == 128 || Ds == 256) &&
                     (size_t)(d->Din + 4) * Ds * 4 + (size_t)PE_TOK * (d->Din + 4) * 4 >= (size_t)2 * 32 * Ds * 2;
#define LTHM_PT_EMB(TX)                                                                                     \
  switch (Ds) {                                                                                             \
    case 16: hipLaunchKernelGGL((ptower_emb_mfma_k<TX, 1>), g2, dim3(512), sh_mfma, s, *d, total, R); break;  \
    case 32: hipLaunchKernelGGL((ptower_emb_mfma_k<TX, 2>), g2, dim3(512), sh_mfma, s, *d, total, R); break;  \
    case 64: hipLaunchKernelGGL((ptower_emb_mfma_k<TX, 4>), g2, dim3(512), sh_mfma, s, *d, total, R); break;  \
    case 128:                                                                                               \
      if (dma) hipLaunchKernelGGL((ptower_emb_mfma_k<TX, 8, true>), g2, dim3(512), sh_mfma, s, *d, total, R);   \
      else hipLaunchKernelGGL((ptower_emb_mfma_k<TX, 8>), g2, dim3(512), sh_mfma, s, *d, total, R);             \
      break;                                                                                                \
    default:                                                                                                \
      if (dma) hipLaunchKernelGGL((ptower_emb_mfma_k<TX, 16, true>), g2, dim3(512), sh_mfma, s, *d, total, R);  \
      else hipLaunchKernelGGL((ptower_emb_mfma_k<TX, 16>), g2, dim3(512), sh_mfma, s, *d, total, R);            \
      break;                                                                                                \
  }
    if (d->x_dtype == LTHM_BF16) { LTHM_PT_EMB(bf16_t) } else { LTHM_PT_EMB(float) }
#undef LTHM_PT_EMB
    LTHM_CHECK_LAUNCH();
    return 0;
  }
#define LTHM_PT(TX, TT)                                                                                   \
  if (opl == 1) hipLaunchKernelGGL((ptower_fwd_k<TX, TT, 1>), dim3(grid), dim3(256), sh, s, *d, total);    \
  else if (opl == 2) hipLaunchKernelGGL((ptower_fwd_k<TX, TT, 2>), dim3(grid), dim3(256), sh, s, *d, total); \
  else if (opl == 4) hipLaunchKernelGGL((ptower_fwd_k<TX, TT, 4>), dim3(grid), dim3(256), sh, s, *d, total); \
  else hipLaunchKernelGGL((ptower_fwd_k<TX, TT, 8>), dim3(grid), dim3(256), sh, s, *d, total);
  LTHM_REQUIRE(opl == 1 || opl == 2 || opl == 4 || opl == 8);
  if (d->x_dtype == LTHM_BF16 && d->tab_dtype == LTHM_BF16) { LTHM_PT(bf16_t, bf16_t) }
  else if (d->x_dtype == LTHM_F32 && d->tab_dtype == LTHM_F32) { LTHM_PT(float, float) }
  else if (d->x_dtype == LTHM_BF16 && d->tab_dtype == LTHM_F32) { LTHM_PT(bf16_t, float) }
  else { LTHM_PT(float, bf16_t) }
#undef LTHM_PT
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_segmented_table_bwd(const uint16_t* rows, int32_t nidx, int32_t nseg, const int32_t* seg_slot0,
                                        const int32_t* seg_nslot, const int32_t* seg_row0, const int32_t* seg_nrow,
                                        const void* dY, int32_t dy_dtype, int64_t ldy, int64_t n, int32_t D, float* dW,
                                        void* workspace, int64_t workspace_bytes, void* stream) {
  LTHM_REQUIRE(n >= 0 && nidx > 0 && D > 0 && nseg > 0 && nseg <= ST_MAXSEG);
  if (n == 0) return 0;
  SegTab st;
  st.nseg = nseg;
  int maxr = 1, rtot = 0;
  for (int i = 0; i < nseg; ++i) {
    st.slot0[i] = seg_slot0[i]; st.nslot[i] = seg_nslot[i]; st.row0[i] = seg_row0[i]; st.nrow[i] = seg_nrow[i];
    LTHM_REQUIRE(st.slot0[i] >= 0 && st.nslot[i] > 0 && st.nslot[i] <= 64 && st.slot0[i] + st.nslot[i] <= nidx &&
                 st.nrow[i] > 0 && st.row0[i] >= 0);
    if (st.nrow[i] > maxr) maxr = st.nrow[i];
    if (st.row0[i] + st.nrow[i] > rtot) rtot = st.row0[i] + st.nrow[i];
  }
  // row ranges must be disjoint: every (row, column) has exactly one owner block per chunk
  for (int i = 0; i < nseg; ++i)
    for (int j = i + 1; j < nseg; ++j)
      LTHM_REQUIRE(st.row0[i] + st.nrow[i] <= st.row0[j] || st.row0[j] + st.nrow[j] <= st.row0[i]);
  const size_t sh = (size_t)maxr * ST_CG * 4;
  LTHM_REQUIRE(sh <= 160 * 1024);
  const int gx = (D + ST_CG - 1) / ST_CG;
  // enough token chunks for ~4 blocks per CU, each chunk >= 512 tokens,
  // bounded by the partial-buffer workspace
  const int64_t zbytes = (int64_t)rtot * D * 4;
  int64_t gz = (1024 + (int64_t)gx * nseg - 1) / ((int64_t)gx * nseg);
  gz = std::min<int64_t>(gz, (n + 511) / 512);
  gz = std::min<int64_t>(gz, workspace ? workspace_bytes / zbytes : (int64_t)1);
  if (gz < 2) gz = 1;
  int64_t tpb = (n + gz - 1) / gz;
  gz = (n + tpb - 1) / tpb;
  const int direct = gz == 1;
  float* dst = direct ? dW : (float*)workspace;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(gx, nseg, (unsigned)gz);
  const int64_t zs = (int64_t)rtot * D;
  if (dy_dtype == LTHM_F32)
    hipLaunchKernelGGL((seg_tab_bwd_k<float>), grid, dim3(256), sh, s, rows, nidx, (const float*)dY, ldy, n, D, dst, zs,
                       direct, tpb, st);
  else
    hipLaunchKernelGGL((seg_tab_bwd_k<bf16_t>), grid, dim3(256), sh, s, rows, nidx, (const bf16_t*)dY, ldy, n, D, dst,
                       zs, direct, tpb, st);
  LTHM_CHECK_LAUNCH();
  if (!direct) {
    const int bx = (int)std::min<int64_t>(((int64_t)maxr * D + 255) / 256, 256);
    hipLaunchKernelGGL(seg_tab_reduce_k, dim3(bx, nseg), dim3(256), 0, s, (const float*)workspace, zs, (int)gz, D, dW,
                       st);
    LTHM_CHECK_LAUNCH();
  }
  return 0;
}

static int lthm_tower_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

// resident 512-thread blocks per CU of one cve_tab_bwd_k form (registers and LDS), cached
template <int DD>
static int cve_tab_bpc_d(bool f32, bool gen, size_t sh) {
  static int cache[4] = {0, 0, 0, 0};
  int& c = cache[(f32 ? 2 : 0) + (gen ? 1 : 0)];
  if (c == 0) {
    int b = 0;
    hipError_t e;
    if (f32 && gen) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, cve_tab_bwd_k<DD, true, true>, 512, sh);
    else if (f32) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, cve_tab_bwd_k<DD, true, false>, 512, sh);
    else if (gen) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, cve_tab_bwd_k<DD, false, true>, 512, sh);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, cve_tab_bwd_k<DD, false, false>, 512, sh);
    c = (e == hipSuccess && b > 0) ? b : 1;
  }
  return c;
}
static int cve_tab_blocks_per_cu(int D, bool f32, bool gen, size_t sh) {
  switch (D) {
    case 16: return cve_tab_bpc_d<16>(f32, gen, sh);
    case 32: return cve_tab_bpc_d<32>(f32, gen, sh);
    case 64: return cve_tab_bpc_d<64>(f32, gen, sh);
    case 128: return cve_tab_bpc_d<128>(f32, gen, sh);
    default: return cve_tab_bpc_d<256>(f32, gen, sh);
  }
}

static int launch_table_mfma(const uint16_t* rows, int32_t nidx, CveTiles& ct, SegTab& st, int rtot, bool gen,
                             const void* dY, int32_t dy_dtype, int64_t ldy, int64_t n, int32_t D, float* dW,
                             void* workspace, int64_t workspace_bytes, hipStream_t s) {
  const int nt = ct.ntile;
  const int64_t zbytes = (int64_t)rtot * D * 4;
  const bool f32 = dy_dtype == LTHM_F32;
  const size_t sh = 2 * ((f32 ? 2 : 1) * (size_t)CT_KT * D * 2 + (size_t)CT_MAXSL * CT_RTLD * 2);
  // one round of blocks: ntile x gz <= CUs x resident blocks per CU (the D = 256 forms hold
  // ~200 VGPRs, i.e. one 512-thread block per CU).  522 blocks for 256 slots ran three
  // rounds, the last with ten blocks.
  const int bpc = cve_tab_blocks_per_cu(D, f32, gen, sh);
  int64_t gz = std::max<int64_t>(1, (int64_t)lthm_tower_cus() * bpc / nt);
  gz = std::min<int64_t>(gz, (n + 1023) / 1024);
  gz = std::min<int64_t>(gz, workspace ? workspace_bytes / zbytes : (int64_t)1);
  if (gz < 2) gz = 1;
  int64_t tpb = (n + gz - 1) / gz;
  tpb = (tpb + CT_KT - 1) / CT_KT * CT_KT;
  gz = (n + tpb - 1) / tpb;
  const int direct = gz == 1;
  float* dst = direct ? dW : (float*)workspace;
  dim3 grid(nt, 1, (unsigned)gz);
  const int64_t zs = zbytes / 4;
#define LTHM_TAB_CASE(DD)                                                                                            \
  case DD:                                                                                                           \
    if (f32 && gen) hipLaunchKernelGGL((cve_tab_bwd_k<DD, true, true>), grid, dim3(512), sh, s, rows, nidx, dY, ldy, n, dst, zs, direct, tpb, ct); \
    else if (f32) hipLaunchKernelGGL((cve_tab_bwd_k<DD, true, false>), grid, dim3(512), sh, s, rows, nidx, dY, ldy, n, dst, zs, direct, tpb, ct); \
    else if (gen) hipLaunchKernelGGL((cve_tab_bwd_k<DD, false, true>), grid, dim3(512), sh, s, rows, nidx, dY, ldy, n, dst, zs, direct, tpb, ct); \
    else hipLaunchKernelGGL((cve_tab_bwd_k<DD, false, false>), grid, dim3(512), sh, s, rows, nidx, dY, ldy, n, dst, zs, direct, tpb, ct); \
    break;
  switch (D) {
    LTHM_TAB_CASE(16)
    LTHM_TAB_CASE(32)
    LTHM_TAB_CASE(64)
    LTHM_TAB_CASE(128)
    LTHM_TAB_CASE(256)
    default: return (int)hipErrorInvalidValue;
  }
#undef LTHM_TAB_CASE
  LTHM_CHECK_LAUNCH();
  if (!direct) {
    const int bx = (int)std::min<int64_t>(((int64_t)CT_ROWS * D + 255) / 256, 256);
    hipLaunchKernelGGL(seg_tab_reduce_k, dim3(bx, nt), dim3(256), 0, s, (const float*)workspace, zs, (int)gz, D, dW, st);
    LTHM_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int lthm_cve_table_bwd(const uint16_t* rows, int32_t nidx, int32_t nmod, const int32_t* mod_slot0,
                                  const int32_t* mod_nslot, const int32_t* mod_row0, const int32_t* mod_rps,
                                  const void* dY, int32_t dy_dtype, int64_t ldy, int64_t n, int32_t D, float* dW,
                                  void* workspace, int64_t workspace_bytes, void* stream) {
  LTHM_REQUIRE(n >= 0 && nidx > 0 && nmod > 0 && nmod <= 16 && (dy_dtype == LTHM_F32 || dy_dtype == LTHM_BF16));
  LTHM_REQUIRE(D == 16 || D == 32 || D == 64 || D == 128 || D == 256);
  if (n == 0) return 0;
  CveTiles ct;
  SegTab st;  // the same row ranges, for the partial-sum fold
  int nt = 0, rtot = 0;
  for (int j = 0; j < nmod; ++j) {
    const int s0 = mod_slot0[j], ns = mod_nslot[j], r0 = mod_row0[j], rps = mod_rps[j];
    LTHM_REQUIRE(s0 >= 0 && ns > 0 && s0 + ns <= nidx && r0 >= 0 && rps > 0 && (int64_t)ns * rps < 65535);
    for (int k = 0; k < j; ++k)  // module row ranges are disjoint
      LTHM_REQUIRE(r0 + ns * rps <= mod_row0[k] || mod_row0[k] + mod_nslot[k] * mod_rps[k] <= r0);
    const int tot = ns * rps;
    for (int r = 0; r < tot; r += CT_ROWS) {
      LTHM_REQUIRE(nt < CT_MAXTILE);
      const int nr = std::min(CT_ROWS, tot - r);
      ct.row0[nt] = r0 + r;
      ct.nrow[nt] = nr;
      ct.sfirst[nt] = s0 + r / rps;
      ct.nsl[nt] = (r + nr - 1) / rps - r / rps + 1;
      LTHM_REQUIRE(ct.nsl[nt] <= CT_MAXSL);
      ct.mrow0[nt] = r0;
      ct.mslot0[nt] = s0;
      ct.rps[nt] = rps;
      st.row0[nt] = r0 + r;
      st.nrow[nt] = nr;
      st.slot0[nt] = 0;
      st.nslot[nt] = 1;
      ++nt;
    }
    rtot = std::max(rtot, r0 + tot);
  }
  ct.ntile = nt;
  st.nseg = nt;
  return launch_table_mfma(rows, nidx, ct, st, rtot, false, dY, dy_dtype, ldy, n, D, dW, workspace, workspace_bytes,
                           (hipStream_t)stream);
}

extern "C" int lthm_table_bwd_mfma(const uint16_t* rows, int32_t nidx, int32_t R, const void* dY, int32_t dy_dtype,
                                   int64_t ldy, int64_t n, int32_t D, float* dW, void* workspace,
                                   int64_t workspace_bytes, void* stream) {
  LTHM_REQUIRE(n >= 0 && nidx > 0 && nidx <= CT_GENMAX && R > 0 && R < 0xffff &&
               (dy_dtype == LTHM_F32 || dy_dtype == LTHM_BF16));
  LTHM_REQUIRE(D == 16 || D == 32 || D == 64 || D == 128 || D == 256);
  LTHM_REQUIRE((R + CT_ROWS - 1) / CT_ROWS <= CT_MAXTILE);
  if (n == 0) return 0;
  CveTiles ct;
  SegTab st;
  int nt = 0;
  for (int r = 0; r < R; r += CT_ROWS) {
    const int nr = std::min(CT_ROWS, R - r);
    ct.row0[nt] = r;
    ct.nrow[nt] = nr;
    ct.sfirst[nt] = 0;
    ct.nsl[nt] = nidx;
    ct.mrow0[nt] = 0;
    ct.mslot0[nt] = 0;
    ct.rps[nt] = 1;
    st.row0[nt] = r;
    st.nrow[nt] = nr;
    st.slot0[nt] = 0;
    st.nslot[nt] = 1;
    ++nt;
  }
  ct.ntile = nt;
  st.nseg = nt;
  return launch_table_mfma(rows, nidx, ct, st, R, true, dY, dy_dtype, ldy, n, D, dW, workspace, workspace_bytes,
                           (hipStream_t)stream);
}

extern "C" int lthm_small_table_bwd(const uint16_t* rows, int32_t nidx, const void* dY, int32_t dy_dtype, int64_t ldy,
                                    int64_t n, int32_t R, int32_t D, float* dW, void* workspace,
                                    int64_t workspace_bytes, void* stream) {
  LTHM_REQUIRE(R > 0 && R < 0xffff && nidx <= 64);
  const int32_t s0 = 0, ns = nidx, r0 = 0, nr = R;
  return lthm_segmented_table_bwd(rows, nidx, 1, &s0, &ns, &r0, &nr, dY, dy_dtype, ldy, n, D, dW, workspace,
                                  workspace_bytes, stream);
}

extern "C" int lthm_tokens_fwd(const lthm_tokens_desc* d, void* stream) {
  LTHM_REQUIRE(d && d->B >= 0 && d->T_full > 0 && d->trim >= 0 && d->trim < d->T_full && d->d > 0);
  if (d->B == 0) return 0;
  const int64_t rows = d->B * (d->T_full - d->trim + 1);
  hipStream_t s = (hipStream_t)stream;
  // the D = 256 path reads 16-B table chunks: every operand base 16-B aligned (rows are 1 KiB)
  bool vec = d->d == 256;
  for (const void* q : {(const void*)d->act, (const void*)d->hod, (const void*)d->how, (const void*)d->dow,
                        (const void*)d->wpe, (const void*)d->pad, (const void*)d->ctx, (const void*)d->x0, d->P})
    vec = vec && ((uintptr_t)q % 16) == 0;
  if (d->p_dtype == LTHM_BF16) {
    if (vec) hipLaunchKernelGGL((tokens_fwd_k<bf16_t, true>), dim3(grid_for(rows, 256, 256 * 8)), dim3(256), 0, s, *d);
    else hipLaunchKernelGGL((tokens_fwd_k<bf16_t, false>), dim3(grid_for(rows, 256, 256 * 8)), dim3(256), 0, s, *d);
  } else {
    if (vec) hipLaunchKernelGGL((tokens_fwd_k<float, true>), dim3(grid_for(rows, 256, 256 * 8)), dim3(256), 0, s, *d);
    else hipLaunchKernelGGL((tokens_fwd_k<float, false>), dim3(grid_for(rows, 256, 256 * 8)), dim3(256), 0, s, *d);
  }
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_tokens_bwd(const lthm_tokens_desc* d, const float* dx0, void* dP, float* dctx, void* stream) {
  LTHM_REQUIRE(d && d->B >= 0);
  if (d->B == 0) return 0;
  const int64_t rows = d->B * (d->T_full - d->trim + 1);
  hipLaunchKernelGGL(tokens_bwd_k, dim3(grid_for(rows, 4, 256 * 8)), dim3(256), 0, (hipStream_t)stream, *d, dx0,
                     (bf16_t*)dP, dctx);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_outcome_fwd(const float* x, const int64_t* labels, int64_t B, int32_t T_full, int32_t trim,
                                int64_t future, const float* table, int32_t n_outcomes, int32_t D, void* out,
                                uint16_t* rows, void* stream) {
  LTHM_REQUIRE(B >= 0 && T_full > 0 && trim >= 0 && trim < T_full && n_outcomes > 0);
  if (B == 0) return 0;
  const int64_t nrow = B * (T_full - trim + 1);
  hipLaunchKernelGGL(outcome_fwd_k, dim3(grid_for(nrow, 4, 256 * 8)), dim3(256), 0, (hipStream_t)stream, x, labels, B,
                     T_full, trim, future, table, n_outcomes, D, (bf16_t*)out, rows);
  LTHM_CHECK_LAUNCH();
  return 0;
}
