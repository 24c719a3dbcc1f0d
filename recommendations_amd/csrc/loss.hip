// Fused in-batch contrastive loss of the LTHM wrapper
// (models/lthm/sequence/wrapper.py:114-245), forward + backward, for gfx950.
//
// Per mini-batch of <= 32 sequences and per lookahead head i with offset o
// (drawn per mini-batch, wrapper.py:147-153):
//   rows r = (b, t), t < L = T - o:   out_r = normalize(next_token_emb[b, t, i])
//   cols c = (b', t'):                in_c  = normalize(current_token_emb[b', t' + o])
//   logits = out . in^T / tau, -inf where same sequence & r != c, or col/row pad;
//   rows kept iff not pad and >= 1 finite negative; CE(logits, r) averaged.
// The [n, n] logits (n <= 32 T) are never written: transposed 64 x 32 tiles
// S^T = img . regrows^T are produced by bf16 MFMA (K = 128) from LDS-staged
// column tiles and reduced on the fly to per-row (sum-exp, finite count, rank
// of the positive).  The backward recomputes each tile from the saved LSE; dS
// is already in the A-operand lanes of the second MFMA, so the row kernel
// accumulates dOut and the column kernel (roles swapped) dIn in registers —
// no atomics, no LDS round trip, no T^2 buffer.
// The argsort / topk metrics (wrapper.py:228-238) become the in-kernel rank
// count #{c != r : logit[r, c] > logit[r, r]}.
#include "common.hpp"

namespace lthm {

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int DE = 128;  // product_emb_dim (model/lthm.yaml:22)

__device__ __forceinline__ int ks_off256(int row, int ch) {
  return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

// ---------------------------------------------------------------- row normalisation
// out[r] = bf16(x[r] / max(|x[r]|, 1e-12)), norms[r] = |x[r]|   (F.normalize, wrapper.py:118-119)
template <typename TX>
__global__ __launch_bounds__(256) void rownorm_k(const TX* __restrict__ x, int64_t rows, int D, bf16_t* __restrict__ out,
                                                 float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    float v[4];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      v[i] = (c < D) ? Elem<TX>::ld(x + r * D + c) : 0.f;
      ss += v[i] * v[i];
    }
    const float nrm = sqrtf(wave_sum(ss));
    const float den = fmaxf(nrm, 1e-12f);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      if (c < D) out[r * D + c] = f2bf(v[i] / den);
    }
    if (lane == 0) norms[r] = nrm;
  }
}

// dx[r] = (g - y (y . g)) / max(|x|, eps)  with y = x / |x|  (eps branch: g / eps)
template <typename TX>
__global__ __launch_bounds__(256) void rownorm_bwd_k(const TX* __restrict__ x, const float* __restrict__ norms,
                                                     const float* __restrict__ g, int64_t rows, int D,
                                                     bf16_t* __restrict__ dx_bf, float* __restrict__ dx_f) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    const float nrm = norms[r];
    float y[4], gv[4];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      y[i] = (c < D) ? Elem<TX>::ld(x + r * D + c) / fmaxf(nrm, 1e-12f) : 0.f;
      gv[i] = (c < D) ? g[r * D + c] : 0.f;
      dot += y[i] * gv[i];
    }
    dot = wave_sum(dot);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      if (c < D) {
        const float o = (nrm > 1e-12f) ? (gv[i] - y[i] * dot) / nrm : gv[i] / 1e-12f;
        if (dx_bf) dx_bf[r * D + c] = f2bf(o);
        if (dx_f) dx_f[r * D + c] = o;
      }
    }
  }
}

// ---------------------------------------------------------------- arguments and geometry
struct ClArgs {
  const bf16_t* out_n;  // [B, Tp, NH, DE]
  const bf16_t* in_n;   // [B, T, DE]
  const uint8_t* mask;  // [B, mask_stride] (already offset by trim)
  int64_t mask_stride;
  int64_t B;
  int T, NH, head, mbs, n_mb, n_max;
  const int* offsets;   // [n_mb, NH]
  float tau;
  float* lse; float* pos; int* cnt; int* rank;  // [n_mb, n_max]  (this head)
  float* diag;                                     // [n_mb, n_max]
  const float* w;                                  // [n_mb, n_max] row weights (bwd)
  const float* gscale;                             // device scalar dL (bwd)
  float* d_out;                                    // f32 [B, Tp, NH, DE]
  float* d_in;                                     // f32 [B, T, DE] (accumulated)
};

struct Geo {
  int L, off, Bm, n;
  int64_t b0;
};

__device__ __forceinline__ Geo geo(const ClArgs& a, int mb) {
  Geo g;
  g.off = a.offsets[mb * a.NH + a.head];
  g.L = a.T - g.off;
  g.b0 = (int64_t)mb * a.mbs;
  g.Bm = (int)min((int64_t)a.mbs, a.B - g.b0);
  g.n = g.L > 0 ? g.Bm * g.L : 0;
  return g;
}
__device__ __forceinline__ const bf16_t* out_row(const ClArgs& a, const Geo& g, int r) {
  const int b = r / g.L, t = r - (r / g.L) * g.L;
  return a.out_n + (((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head) * DE;
}
__device__ __forceinline__ const bf16_t* in_row(const ClArgs& a, const Geo& g, int c) {
  const int b = c / g.L, t = c - (c / g.L) * g.L;
  return a.in_n + ((g.b0 + b) * a.T + t + g.off) * DE;
}
__device__ __forceinline__ bool pad_of(const ClArgs& a, const Geo& g, int c) {
  const int b = c / g.L, t = c - (c / g.L) * g.L;
  return a.mask[(g.b0 + b) * a.mask_stride + t + g.off] != 0;
}

__device__ __forceinline__ bf16x8v row_frag(const unsigned char* img, int row, int chunk) {
  return __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(img + ks_off256(row, chunk)));
}
// transposed (k = image row) fragment: B[k = kb + 8*(lane>>4) + j][n = nb + (lane&15)]
__device__ __forceinline__ bf16x8v tr_frag(const unsigned char* img, int kb, int nb, int lane) {
  const int gq = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int kr = kb + 8 * gq + q;
  const int ch = (nb >> 3) + (p >> 1);
  const unsigned char* a0 = img + ks_off256(kr, ch) + 8 * (p & 1);
  const unsigned char* a1 = img + ks_off256(kr + 4, ch) + 8 * (p & 1);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8v, v);
}

// load this wave's 16 register rows as 4 k32 A fragments
template <typename RowFn>
__device__ __forceinline__ void reg_frags(bf16x8v (&f)[4], int lane, int cnt, int rbase, RowFn rowp) {
  const int r = rbase + (lane & 15);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r < cnt) v = *reinterpret_cast<const u32x4*>(rowp(r) + (s * 4 + (lane >> 4)) * 8);
    f[s] = __builtin_bit_cast(bf16x8v, v);
  }
}

// diag[r] = out_r . in_r / tau (fp32 dot of the bf16 operands), per (mb, row)
__global__ __launch_bounds__(256) void cl_diag_k(ClArgs a) {
  const int mb = blockIdx.y;
  const Geo g = geo(a, mb);
  const int lane = threadIdx.x & 63;
  for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < g.n; r += gridDim.x * 4) {
    const bf16_t* o = out_row(a, g, r);
    const bf16_t* i = in_row(a, g, r);
    float s = bf2f(o[lane]) * bf2f(i[lane]) + bf2f(o[lane + 64]) * bf2f(i[lane + 64]);
    s = wave_sum(s);
    if (lane == 0) a.diag[(int64_t)mb * a.n_max + r] = s / a.tau;
  }
}

// ---------------------------------------------------------------- stats (one block per mini-batch)
// per (mb): used rows, mean CE, weights w_r = used / (U * n_mb_total); metrics.
// stats[mb][*] = {loss, used, sum_negatives, min_negatives, sum_rank, median_rank, hits@k...}
__global__ __launch_bounds__(256) void cl_stats_k(ClArgs a, float* __restrict__ stats, int nstat, const int* __restrict__ ks,
                                                  int nk, float loss_scale, float* __restrict__ wout) {
  __shared__ int srank[4096];
  __shared__ float red[256];
  __shared__ int ired[256];
  const int mb = blockIdx.x;
  const Geo g = geo(a, mb);
  const int tid = threadIdx.x;
  float ls = 0.f, neg = 0.f, rks = 0.f;
  int used = 0, mneg = 0x7fffffff;
  const int64_t base = (int64_t)mb * a.n_max;
  for (int r = tid; r < g.n; r += 256) {
    const int nn = a.cnt[base + r] - 1;
    const bool u = !pad_of(a, g, r) && nn > 0;
    if (u) {
      ls += a.lse[base + r] - a.pos[base + r];
      neg += (float)nn;
      rks += (float)a.rank[base + r];
      used += 1;
      mneg = min(mneg, nn);
    }
  }
  // block reductions
  auto fsum = [&](float v) {
    red[tid] = v; __syncthreads();
    for (int s = 128; s > 0; s >>= 1) { if (tid < s) red[tid] += red[tid + s]; __syncthreads(); }
    const float t = red[0]; __syncthreads(); return t;
  };
  auto isum = [&](int v) {
    ired[tid] = v; __syncthreads();
    for (int s = 128; s > 0; s >>= 1) { if (tid < s) ired[tid] += ired[tid + s]; __syncthreads(); }
    const int t = ired[0]; __syncthreads(); return t;
  };
  auto imin = [&](int v) {
    ired[tid] = v; __syncthreads();
    for (int s = 128; s > 0; s >>= 1) { if (tid < s) ired[tid] = min(ired[tid], ired[tid + s]); __syncthreads(); }
    const int t = ired[0]; __syncthreads(); return t;
  };
  const float Ls = fsum(ls), Ns = fsum(neg), Rs = fsum(rks);
  const int U = isum(used), Mn = imin(mneg);
  const float wr = U > 0 ? loss_scale / (float)U : 0.f;
  for (int r = tid; r < a.n_max; r += 256) {
    float wv = 0.f;
    if (r < g.n) {
      const int nn = a.cnt[base + r] - 1;
      if (!pad_of(a, g, r) && nn > 0) wv = wr;
    }
    wout[base + r] = wv;
  }
  // median of the used ranks: bitonic sort in LDS (n <= 4096)
  int n2 = 1;
  while (n2 < g.n) n2 <<= 1;
  for (int i = tid; i < n2; i += 256) {
    int v = 0x7fffffff;
    if (i < g.n) {
      const int nn = a.cnt[base + i] - 1;
      if (!pad_of(a, g, i) && nn > 0) v = a.rank[base + i];
    }
    srank[i] = v;
  }
  __syncthreads();
  for (int k = 2; k <= n2; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = tid; t < n2 / 2; t += 256) {
        const int i0 = 2 * t - (t & (j - 1)), i1 = i0 + j;
        const bool up = (i0 & k) == 0;
        const int x = srank[i0], y = srank[i1];
        if ((x > y) == up) { srank[i0] = y; srank[i1] = x; }
      }
      __syncthreads();
    }
  // hits@k: rank < min(k, min negatives)
  float* st = stats + (int64_t)mb * nstat;
  for (int q = 0; q < nk; ++q) {
    const int kq = min(ks[q], Mn);
    int h = 0;
    for (int r = tid; r < g.n; r += 256) {
      const int nn = a.cnt[base + r] - 1;
      if (!pad_of(a, g, r) && nn > 0 && a.rank[base + r] < kq) h += 1;
    }
    h = isum(h);
    if (tid == 0) st[7 + q] = U > 0 ? (float)h / (float)U : 0.f;
  }
  if (tid == 0) {
    st[0] = U > 0 ? Ls / (float)U : 0.f;
    st[1] = (float)U;
    st[2] = U > 0 ? Ns / (float)U : 0.f;
    st[3] = (float)(U > 0 ? Mn : 0);
    st[4] = U > 0 ? Rs / (float)U : 0.f;
    // torch.quantile(0.5): linear interpolation between the two middle order statistics
    float med = 0.f;
    if (U > 0) {
      const float p = 0.5f * (float)(U - 1);
      const int lo = (int)floorf(p);
      const int hi = min(lo + 1, U - 1);
      med = (float)srank[lo] + (p - (float)lo) * (float)(srank[hi] - srank[lo]);
    }
    st[5] = med;
    st[6] = (float)g.off;
  }
}

// ---------------------------------------------------------------- tile engine
// 128 register rows per block (each wave: 32 rows = two 16-row MFMA tiles),
// 64-row column tiles staged through LDS with register prefetch (one barrier
// per tile), per-tile column metadata in LDS.  Rows are L2-normalised, so every
// logit lies in [-1/tau, 1/tau] (up to bf16 rounding): with 2/tau <= 80 the
// softmax shift is the constant 1/tau (no running max, exp never under- or
// overflows); smaller tau falls back to a per-tile online max.
constexpr int CL_ROWS = 128;

struct ClTile {
  unsigned char img[2][64 * 256];
  int seq[2][64];     // sequence id of each tile row (-1: beyond n)
  float lse[2][64];   // COLS pass: LSE of the image rows
  float w[2][64];     // COLS pass: weights of the image rows
  uint8_t pad[2][64];
};

template <typename RowFn>
__device__ __forceinline__ void cl_fetch(u32x4 (&pf)[4], int tid, int cnt, RowFn rowp) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int idx = tid + 256 * k;
    const int row = idx >> 4, ch = idx & 15;
    pf[k] = u32x4{0u, 0u, 0u, 0u};
    if (row < cnt) pf[k] = *reinterpret_cast<const u32x4*>(rowp(row) + ch * 8);
  }
}
__device__ __forceinline__ void cl_store(unsigned char* img, int tid, const u32x4 (&pf)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int idx = tid + 256 * k;
    *reinterpret_cast<u32x4*>(img + ks_off256(idx >> 4, idx & 15)) = pf[k];
  }
}

// transposed-k fragment: B[k][n = nb + (lane&15)] with k = 0..3 -> image rows
// kb + 4(lane>>4) + k and k = 4..7 -> rows kb + 16 + 4(lane>>4) + k-4, i.e. the k
// order in which a transposed S^T tile's C registers already sit per lane.
__device__ __forceinline__ bf16x8v trp_frag(const unsigned char* img, int kb, int nb, int lane) {
  const int gq = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int ch = (nb >> 3) + (p >> 1);
  const unsigned char* a0 = img + ks_off256(kb + 4 * gq + q, ch) + 8 * (p & 1);
  const unsigned char* a1 = img + ks_off256(kb + 16 + 4 * gq + q, ch) + 8 * (p & 1);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8v, v);
}

// S^T tile: acc[mi][yb][j] = img[yb*16 + 4(lane>>4) + j] . X[xbase + 16 mi + (lane&15)]
// (the register rows' A fragments double as the B operand)
__device__ __forceinline__ void st_tile(f32x4 (&acc)[2][4], const bf16x8v (&qf)[2][4], const unsigned char* img,
                                        int lane) {
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int yb = 0; yb < 4; ++yb) acc[mi][yb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int yb = 0; yb < 4; ++yb) {
      const bf16x8v af = row_frag(img, yb * 16 + (lane & 15), s * 4 + (lane >> 4));
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
        acc[mi][yb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, qf[mi][s], acc[mi][yb], 0, 0, 0);
    }
}

template <bool FIXED>
__global__ __launch_bounds__(256, 2) void cl_fwd_k(ClArgs a) {
  __shared__ __attribute__((aligned(16))) ClTile sh;
  const int mb = blockIdx.y;
  const Geo g = geo(a, mb);
  const int r0 = blockIdx.x * CL_ROWS;
  if (r0 >= g.n) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, rg = 4 * (lane >> 4);
  bf16x8v qf[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
    reg_frags(qf[mi], lane, g.n, r0 + 32 * w + 16 * mi, [&](int r) { return out_row(a, g, r); });
  const float it = 1.f / a.tau;
  // this lane's rows: r = r0 + 32 w + 16 mi + col  (one per mi)
  float m[2], l[2], pv[2], dg[2];
  int cn[2], rk[2], rsq[2], rr[2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int r = r0 + 32 * w + 16 * mi + col;
    rr[mi] = r;
    m[mi] = FIXED ? it : -INFINITY;
    l[mi] = 0.f; pv[mi] = -INFINITY; cn[mi] = 0; rk[mi] = 0;
    dg[mi] = (r < g.n) ? a.diag[(int64_t)mb * a.n_max + r] : 0.f;
    rsq[mi] = (r < g.n) ? r / g.L : -2;
  }
  const int ntile = (g.n + 63) / 64;
  u32x4 pf[4];
  cl_fetch(pf, tid, g.n, [&](int i) { return in_row(a, g, i); });
  cl_store(sh.img[0], tid, pf);
  if (tid < 64) {
    sh.seq[0][tid] = tid < g.n ? tid / g.L : -1;
    sh.pad[0][tid] = tid < g.n ? (pad_of(a, g, tid) ? 1 : 0) : 1;
  }
  __syncthreads();
  for (int tI = 0; tI < ntile; ++tI) {
    const int cur = tI & 1, c0 = tI * 64;
    const bool more = tI + 1 < ntile;
    if (more) cl_fetch(pf, tid, g.n - c0 - 64, [&](int i) { return in_row(a, g, c0 + 64 + i); });
    f32x4 acc[2][4];
    st_tile(acc, qf, sh.img[cur], lane);
    int csq[4][4];
    bool cok[4][4];
#pragma unroll
    for (int yb = 0; yb < 4; ++yb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cl = yb * 16 + rg + j;
        csq[yb][j] = sh.seq[cur][cl];
        cok[yb][j] = !sh.pad[cur][cl];
      }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int r = rr[mi];
      if constexpr (!FIXED) {
        float bm = -INFINITY;
#pragma unroll
        for (int yb = 0; yb < 4; ++yb)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int c = c0 + yb * 16 + rg + j;
            if (cok[yb][j] && (csq[yb][j] != rsq[mi] || c == r)) bm = fmaxf(bm, acc[mi][yb][j] * it);
          }
        bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
        bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
        const float mn = fmaxf(m[mi], bm);
        if (mn != -INFINITY) {
          l[mi] *= (m[mi] == -INFINITY) ? 0.f : __expf(m[mi] - mn);
          m[mi] = mn;
        }
      }
#pragma unroll
      for (int yb = 0; yb < 4; ++yb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = c0 + yb * 16 + rg + j;
          const float v = acc[mi][yb][j] * it;
          if (c == r) pv[mi] = v;
          if (cok[yb][j] && (csq[yb][j] != rsq[mi] || c == r)) {
            l[mi] += __expf(v - m[mi]);
            cn[mi] += 1;
            rk[mi] += (c != r && v > dg[mi]) ? 1 : 0;
          }
        }
    }
    if (more) {
      cl_store(sh.img[cur ^ 1], tid, pf);
      if (tid < 64) {
        const int c = c0 + 64 + tid;
        sh.seq[cur ^ 1][tid] = c < g.n ? c / g.L : -1;
        sh.pad[cur ^ 1][tid] = c < g.n ? (pad_of(a, g, c) ? 1 : 0) : 1;
      }
    }
    __syncthreads();
  }
  // combine the 4 lane groups that share each row
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    float mm = m[mi], ll = l[mi], pp = pv[mi];
    int cc = cn[mi], kk = rk[mi];
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      if constexpr (FIXED) {
        ll += __shfl_xor(ll, o, 64);
      } else {
        const float m2 = __shfl_xor(mm, o, 64), l2 = __shfl_xor(ll, o, 64);
        const float mn = fmaxf(mm, m2);
        ll = (mm == -INFINITY ? 0.f : ll * __expf(mm - mn)) + (m2 == -INFINITY ? 0.f : l2 * __expf(m2 - mn));
        mm = mn;
      }
      pp = fmaxf(pp, __shfl_xor(pp, o, 64));
      cc += __shfl_xor(cc, o, 64);
      kk += __shfl_xor(kk, o, 64);
    }
    const int r = rr[mi];
    if (rg == 0 && r < g.n) {
      const int64_t o = (int64_t)mb * a.n_max + r;
      a.lse[o] = (cc > 0) ? mm + __logf(ll) : -INFINITY;
      a.pos[o] = pp;
      a.cnt[o] = cc;
      a.rank[o] = kk;
    }
  }
}

// ROWS = true : register rows are `out` rows r, image rows are `in` cols c  -> dOut
// ROWS = false: register rows are `in` cols c, image rows are `out` rows r  -> dIn
// The S^T tile leaves dS in the A-operand lanes of dS . img (k order matched by
// trp_frag), so no LDS round trip is needed between the two MFMAs.
template <bool ROWS>
__global__ __launch_bounds__(256, 2) void cl_bwd_k(ClArgs a) {
  __shared__ __attribute__((aligned(16))) ClTile sh;
  const int mb = blockIdx.y;
  const Geo g = geo(a, mb);
  const int x0 = blockIdx.x * CL_ROWS;
  if (x0 >= g.n) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, rg = 4 * (lane >> 4);
  const int64_t base = (int64_t)mb * a.n_max;
  const float it = 1.f / a.tau;
  bf16x8v qf[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    if (ROWS) reg_frags(qf[mi], lane, g.n, x0 + 32 * w + 16 * mi, [&](int r) { return out_row(a, g, r); });
    else reg_frags(qf[mi], lane, g.n, x0 + 32 * w + 16 * mi, [&](int c) { return in_row(a, g, c); });
  }
  // this lane's register row per mi (x = x0 + 32 w + 16 mi + col)
  float xl_[2], xw[2];
  bool xpad[2];
  int xsq[2], xx[2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int x = x0 + 32 * w + 16 * mi + col;
    const bool in = x < g.n;
    xx[mi] = x;
    xl_[mi] = (ROWS && in) ? a.lse[base + x] : 0.f;
    xw[mi] = (ROWS && in) ? a.w[base + x] : 0.f;
    xpad[mi] = in ? (ROWS ? false : pad_of(a, g, x)) : true;
    xsq[mi] = in ? x / g.L : -2;
  }
  f32x4 dacc[2][8];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int i = 0; i < 8; ++i) dacc[mi][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto img_row = [&](int i) { return ROWS ? in_row(a, g, i) : out_row(a, g, i); };
  auto meta = [&](int buf, int y) {
    const bool in = y < g.n;
    const int t = y & 63;
    sh.seq[buf][t] = in ? y / g.L : -1;
    sh.pad[buf][t] = in ? (pad_of(a, g, y) ? 1 : 0) : 1;
    sh.lse[buf][t] = (!ROWS && in) ? a.lse[base + y] : 0.f;
    sh.w[buf][t] = (!ROWS && in) ? a.w[base + y] : 0.f;
  };
  const int ntile = (g.n + 63) / 64;
  u32x4 pf[4];
  cl_fetch(pf, tid, g.n, img_row);
  cl_store(sh.img[0], tid, pf);
  if (tid < 64) meta(0, tid);
  __syncthreads();
  for (int tI = 0; tI < ntile; ++tI) {
    const int cur = tI & 1, y0 = tI * 64;
    const bool more = tI + 1 < ntile;
    if (more) cl_fetch(pf, tid, g.n - y0 - 64, [&](int i) { return img_row(y0 + 64 + i); });
    const unsigned char* img = sh.img[cur];
    f32x4 acc[2][4];
    st_tile(acc, qf, img, lane);
    // dS in place: acc[mi][yb][j] <- dS[x][y],  y = y0 + yb*16 + rg + j
#pragma unroll
    for (int yb = 0; yb < 4; ++yb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int yl = yb * 16 + rg + j, y = y0 + yl;
        const bool ypad = sh.pad[cur][yl];
        const int ysq = sh.seq[cur][yl];
        const float ylse = sh.lse[cur][yl], yw = sh.w[cur][yl];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          const int x = xx[mi];
          float ds = 0.f;
          if (ROWS) {
            const bool ok = !ypad && (ysq != xsq[mi] || x == y) && xw[mi] != 0.f;
            if (ok) ds = xw[mi] * (__expf(acc[mi][yb][j] * it - xl_[mi]) - (x == y ? 1.f : 0.f));
          } else {
            const bool ok = !xpad[mi] && (ysq != xsq[mi] || x == y) && yw != 0.f;
            if (ok) ds = yw * (__expf(acc[mi][yb][j] * it - ylse) - (x == y ? 1.f : 0.f));
          }
          acc[mi][yb][j] = ds;
        }
      }
    // dacc[32 x 128] += dS[32 x 64] . img[64 x 128]   (k = y, in trp_frag order)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8v af[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        s16x8 h;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          h[i] = (short)f2bf(acc[mi][2 * ks][i]);
          h[4 + i] = (short)f2bf(acc[mi][2 * ks + 1][i]);
        }
        af[mi] = __builtin_bit_cast(bf16x8v, h);
      }
#pragma unroll
      for (int nd = 0; nd < 8; ++nd) {
        const bf16x8v bfr = trp_frag(img, ks * 32, nd * 16, lane);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          dacc[mi][nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr, dacc[mi][nd], 0, 0, 0);
      }
    }
    if (more) {
      cl_store(sh.img[cur ^ 1], tid, pf);
      if (tid < 64) meta(cur ^ 1, y0 + 64 + tid);
    }
    __syncthreads();
  }
  // write: dacc[mi][nd][j] = d[x = x0 + 32 w + 16 mi + rg + j][e = nd*16 + col]
  const float gs = (a.gscale ? *a.gscale : 1.f) * it;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = x0 + 32 * w + 16 * mi + rg + j;
      if (x >= g.n) continue;
      const int b = x / g.L, t = x - (x / g.L) * g.L;
      float* dst = ROWS ? a.d_out + (((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head) * DE
                        : a.d_in + ((g.b0 + b) * a.T + t + g.off) * DE;
#pragma unroll
      for (int nd = 0; nd < 8; ++nd) {
        const float v = gs * dacc[mi][nd][j];
        if (ROWS) dst[nd * 16 + col] = v;
        else dst[nd * 16 + col] += v;
      }
    }
}

}  // namespace lthm

using namespace lthm;

static ClArgs cl_args(const lthm_contrastive_desc* d) {
  ClArgs a;
  a.out_n = (const bf16_t*)d->out_n; a.in_n = (const bf16_t*)d->in_n; a.mask = d->mask; a.mask_stride = d->mask_stride;
  a.B = d->B; a.T = d->T; a.NH = d->n_heads; a.head = d->head; a.mbs = d->mb_size; a.n_mb = d->n_mb; a.n_max = d->n_max;
  a.offsets = d->offsets; a.tau = d->tau;
  a.lse = d->lse; a.pos = d->pos; a.cnt = d->cnt; a.rank = d->rank; a.diag = d->diag; a.w = d->w;
  a.gscale = d->gscale;
  a.d_out = d->d_out; a.d_in = d->d_in;
  return a;
}

static int cl_check(const lthm_contrastive_desc* d) {
  if (!d || d->De != DE || d->B <= 0 || d->T <= 0 || d->mb_size <= 0 || d->n_mb <= 0) return 1;
  if ((int64_t)d->mb_size * d->T > d->n_max || d->n_max > 4096) return 1;
  if (d->head < 0 || d->head >= d->n_heads) return 1;
  return 0;
}

extern "C" int lthm_rownorm(const void* x, int32_t x_dtype, int64_t rows, int32_t D, void* out_bf16, float* norms,
                            void* stream) {
  LTHM_REQUIRE(rows >= 0 && D > 0 && D <= 256);
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(rows, 4, 256 * 8);
  if (x_dtype == LTHM_BF16)
    hipLaunchKernelGGL((rownorm_k<bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, rows, D, (bf16_t*)out_bf16, norms);
  else
    hipLaunchKernelGGL((rownorm_k<float>), dim3(grid), dim3(256), 0, s, (const float*)x, rows, D, (bf16_t*)out_bf16, norms);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_rownorm_bwd(const void* x, int32_t x_dtype, const float* norms, const float* g, int64_t rows,
                                int32_t D, void* dx_bf16, float* dx_f32, void* stream) {
  LTHM_REQUIRE(rows >= 0 && D > 0 && D <= 256);
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(rows, 4, 256 * 8);
  if (x_dtype == LTHM_BF16)
    hipLaunchKernelGGL((rownorm_bwd_k<bf16_t>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, norms, g, rows, D,
                       (bf16_t*)dx_bf16, dx_f32);
  else
    hipLaunchKernelGGL((rownorm_bwd_k<float>), dim3(grid), dim3(256), 0, s, (const float*)x, norms, g, rows, D,
                       (bf16_t*)dx_bf16, dx_f32);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_contrastive_fwd(const lthm_contrastive_desc* d, float* stats, int32_t nstat, const int32_t* ks,
                                    int32_t nk, float loss_scale, void* stream) {
  LTHM_REQUIRE(cl_check(d) == 0 && stats && d->lse && d->pos && d->cnt && d->rank && d->diag && d->w);
  LTHM_REQUIRE(nstat >= 7 + nk);
  ClArgs a = cl_args(d);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(cl_diag_k, dim3(64, d->n_mb), dim3(256), 0, s, a);
  LTHM_CHECK_LAUNCH();
  const dim3 grid((d->n_max + CL_ROWS - 1) / CL_ROWS, d->n_mb);
  if (2.f / d->tau <= 80.f) hipLaunchKernelGGL((cl_fwd_k<true>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((cl_fwd_k<false>), grid, dim3(256), 0, s, a);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL(cl_stats_k, dim3(d->n_mb), dim3(256), 0, s, a, stats, nstat, (const int*)ks, nk, loss_scale,
                     (float*)d->w);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_contrastive_bwd(const lthm_contrastive_desc* d, void* stream) {
  LTHM_REQUIRE(cl_check(d) == 0 && d->lse && d->w && d->d_out && d->d_in);
  ClArgs a = cl_args(d);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((d->n_max + CL_ROWS - 1) / CL_ROWS, d->n_mb);
  hipLaunchKernelGGL((cl_bwd_k<true>), grid, dim3(256), 0, s, a);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL((cl_bwd_k<false>), grid, dim3(256), 0, s, a);
  LTHM_CHECK_LAUNCH();
  return 0;
}
