// Fused in-batch contrastive loss of the LTHM wrapper
// (models/lthm/sequence/wrapper.py:114-245), forward + backward, for gfx950.
//
// Per mini-batch of <= 32 sequences and per lookahead head i with offset o
// (drawn per mini-batch, wrapper.py:147-153):
//   rows r = (b, t), t < L = T - o:   out_r = normalize(next_token_emb[b, t, i])
//   cols c = (b', t'):                in_c  = normalize(current_token_emb[b', t' + o])
//   logits = out . in^T / tau, -inf where same sequence & r != c, or col/row pad;
//   rows kept iff not pad and >= 1 finite negative; CE(logits, r) averaged.
// The [n, n] logits (n <= 32 T) are never written: 64 x 64 tiles are produced
// by bf16 MFMA (K = 128) from LDS-staged column tiles, reduced on the fly to
// per-row (max, sum-exp, finite count, rank of the positive).  The backward
// recomputes each tile from the saved LSE: the row kernel accumulates dOut in
// registers, the column kernel (roles swapped) dIn — no atomics, no T^2 buffer.
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

// ---------------------------------------------------------------- tile engine
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

// stage 64 rows (row(i) for i < cnt, zero beyond) of DE bf16 into a ks_off256 image
template <typename RowFn>
__device__ __forceinline__ void stage64(unsigned char* img, int tid, int cnt, RowFn rowp) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int idx = tid + 256 * k;  // 1024 chunks of 16 B
    const int row = idx >> 4, ch = idx & 15;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (row < cnt) v = *reinterpret_cast<const u32x4*>(rowp(row) + ch * 8);
    *reinterpret_cast<u32x4*>(img + ks_off256(row, ch)) = v;
  }
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

// S tile: acc[nsub][j] = sum_k regrow[16w + 4(lane>>4) + j][k] * img[nsub*16 + (lane&15)][k]
__device__ __forceinline__ void s_tile(f32x4 (&acc)[4], const bf16x8v (&qf)[4], const unsigned char* img, int lane) {
#pragma unroll
  for (int ns = 0; ns < 4; ++ns) acc[ns] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int ns = 0; ns < 4; ++ns)
      acc[ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[s], row_frag(img, ns * 16 + (lane & 15), s * 4 + (lane >> 4)),
                                                         acc[ns], 0, 0, 0);
}

// ---------------------------------------------------------------- forward
__global__ __launch_bounds__(256) void cl_fwd_k(ClArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char img[64 * 256];
  __shared__ uint8_t cpad[64];
  const int mb = blockIdx.y;
  const Geo g = geo(a, mb);
  const int r0 = blockIdx.x * 64;
  if (r0 >= g.n) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  bf16x8v qf[4];
  reg_frags(qf, lane, g.n, r0 + 16 * w, [&](int r) { return out_row(a, g, r); });
  float m[4], l[4], pv[4], dg[4];
  int cn[4], rk[4], rsq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = r0 + 16 * w + 4 * (lane >> 4) + j;
    m[j] = -INFINITY; l[j] = 0.f; pv[j] = -INFINITY; cn[j] = 0; rk[j] = 0;
    dg[j] = (r < g.n) ? a.diag[(int64_t)mb * a.n_max + r] : 0.f;
    rsq[j] = (r < g.n) ? r / g.L : -1;
  }
  for (int c0 = 0; c0 < g.n; c0 += 64) {
    __syncthreads();
    stage64(img, tid, g.n - c0, [&](int i) { return in_row(a, g, c0 + i); });
    if (tid < 64) cpad[tid] = (c0 + tid < g.n) ? (pad_of(a, g, c0 + tid) ? 1 : 0) : 1;
    __syncthreads();
    f32x4 acc[4];
    s_tile(acc, qf, img, lane);
#pragma unroll
    for (int ns = 0; ns < 4; ++ns) {
      const int cl = ns * 16 + (lane & 15);
      const int c = c0 + cl;
      const bool cvalid = !cpad[cl];
      const int csq = c / g.L;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = r0 + 16 * w + 4 * (lane >> 4) + j;
        const float v = acc[ns][j] / a.tau;
        if (c == r) pv[j] = v;
        const bool ok = cvalid && (csq != rsq[j] || c == r);
        if (ok) {
          if (v > m[j]) { l[j] = l[j] * __expf(m[j] - v) + 1.f; m[j] = v; }
          else l[j] += __expf(v - m[j]);
          cn[j] += 1;
          if (c != r && v > dg[j]) rk[j] += 1;
        }
      }
    }
  }
  // combine the 16 lanes that share each row
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float mm = m[j], ll = l[j], pp = pv[j];
    int cc = cn[j], kk = rk[j];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const float m2 = __shfl_xor(mm, o, 64), l2 = __shfl_xor(ll, o, 64);
      const float mn = fmaxf(mm, m2);
      ll = (mm == -INFINITY ? 0.f : ll * __expf(mm - mn)) + (m2 == -INFINITY ? 0.f : l2 * __expf(m2 - mn));
      mm = mn;
      pp = fmaxf(pp, __shfl_xor(pp, o, 64));
      cc += __shfl_xor(cc, o, 64);
      kk += __shfl_xor(kk, o, 64);
    }
    const int r = r0 + 16 * w + 4 * (lane >> 4) + j;
    if ((lane & 15) == 0 && r < g.n) {
      const int64_t o = (int64_t)mb * a.n_max + r;
      a.lse[o] = mm + __logf(ll);
      a.pos[o] = pp;
      a.cnt[o] = cc;
      a.rank[o] = kk;
    }
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

// ---------------------------------------------------------------- backward
// ROWS = true : register rows are `out` rows r, image rows are `in` cols c  -> dOut
// ROWS = false: register rows are `in` cols c, image rows are `out` rows r  -> dIn
template <bool ROWS>
__global__ __launch_bounds__(256) void cl_bwd_k(ClArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char img[64 * 256];
  __shared__ __attribute__((aligned(16))) unsigned char dsb[4][16 * 128];  // per-wave dS tile [16][64] bf16
  __shared__ float t_lse[64], t_w[64];
  __shared__ uint8_t t_pad[64];
  const int mb = blockIdx.y;
  const Geo g = geo(a, mb);
  const int x0 = blockIdx.x * 64;
  if (x0 >= g.n) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t base = (int64_t)mb * a.n_max;
  bf16x8v qf[4];
  if (ROWS) reg_frags(qf, lane, g.n, x0 + 16 * w, [&](int r) { return out_row(a, g, r); });
  else reg_frags(qf, lane, g.n, x0 + 16 * w, [&](int c) { return in_row(a, g, c); });
  // per-register-row constants
  float rl[4], rw[4];
  bool rpad[4];
  int rsq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int x = x0 + 16 * w + 4 * (lane >> 4) + j;
    const bool in = x < g.n;
    rl[j] = (ROWS && in) ? a.lse[base + x] : 0.f;
    rw[j] = (ROWS && in) ? a.w[base + x] : 0.f;
    rpad[j] = in ? (ROWS ? false : pad_of(a, g, x)) : true;
    rsq[j] = in ? x / g.L : -1;
  }
  f32x4 dacc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  unsigned char* myds = dsb[w];
  for (int y0 = 0; y0 < g.n; y0 += 64) {
    __syncthreads();
    if (ROWS) stage64(img, tid, g.n - y0, [&](int i) { return in_row(a, g, y0 + i); });
    else stage64(img, tid, g.n - y0, [&](int i) { return out_row(a, g, y0 + i); });
    if (tid < 64) {
      const int y = y0 + tid;
      const bool in = y < g.n;
      t_pad[tid] = in ? (pad_of(a, g, y) ? 1 : 0) : 1;
      t_lse[tid] = (!ROWS && in) ? a.lse[base + y] : 0.f;
      t_w[tid] = (!ROWS && in) ? a.w[base + y] : 0.f;
    }
    __syncthreads();
    f32x4 acc[4];
    s_tile(acc, qf, img, lane);
    // dS (bf16) into this wave's [16][64] tile, row-major 128-B rows, chunk-swizzled
#pragma unroll
    for (int ns = 0; ns < 4; ++ns) {
      const int yl = ns * 16 + (lane & 15);
      const int y = y0 + yl;
      const int ysq = y / g.L;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int xl = 4 * (lane >> 4) + j;
        const int x = x0 + 16 * w + xl;
        float ds = 0.f;
        if (ROWS) {
          // x = r (row), y = c (col)
          const bool ok = !t_pad[yl] && (ysq != rsq[j] || x == y) && rw[j] != 0.f;
          if (ok) {
            const float p = __expf(acc[ns][j] / a.tau - rl[j]);
            ds = rw[j] * (p - (x == y ? 1.f : 0.f));
          }
        } else {
          // x = c (col, register), y = r (row, image)
          const bool ok = !rpad[j] && (ysq != rsq[j] || x == y) && t_w[yl] != 0.f;
          if (ok) {
            const float p = __expf(acc[ns][j] / a.tau - t_lse[yl]);
            ds = t_w[yl] * (p - (x == y ? 1.f : 0.f));
          }
        }
        // element (xl, yl) of the [16][64] tile
        const int chunk = yl >> 3;
        const int off = xl * 128 + ((chunk ^ (xl & 7)) << 4) + (yl & 7) * 2;
        *reinterpret_cast<bf16_t*>(myds + off) = f2bf(ds);
      }
    }
    __builtin_amdgcn_wave_barrier();
    // dacc[16 x 128] += dS[16 x 64] . img[64 x 128]   (k = y)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int xl = lane & 15;
      const int chunk = s * 4 + (lane >> 4);
      const bf16x8v af = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(myds + xl * 128 + ((chunk ^ (xl & 7)) << 4)));
#pragma unroll
      for (int nd = 0; nd < 8; ++nd) dacc[nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, tr_frag(img, s * 32, nd * 16, lane), dacc[nd], 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
  }
  // write: ROWS -> d_out[row of out] = dacc / tau ; cols -> d_in[row of in] += dacc / tau
  const float gs = a.gscale ? *a.gscale : 1.f;
#pragma unroll
  for (int nd = 0; nd < 8; ++nd) {
    const int col = nd * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = x0 + 16 * w + 4 * (lane >> 4) + j;
      if (x >= g.n) continue;
      const float v = gs * (dacc[nd][j] / a.tau);
      const int b = x / g.L, t = x - (x / g.L) * g.L;
      if (ROWS) {
        a.d_out[(((g.b0 + b) * (a.T + 1) + t) * a.NH + a.head) * DE + col] = v;
      } else {
        a.d_in[((g.b0 + b) * a.T + t + g.off) * DE + col] += v;
      }
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
  hipLaunchKernelGGL(cl_fwd_k, dim3((d->n_max + 63) / 64, d->n_mb), dim3(256), 0, s, a);
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
  dim3 grid((d->n_max + 63) / 64, d->n_mb);
  hipLaunchKernelGGL((cl_bwd_k<true>), grid, dim3(256), 0, s, a);
  LTHM_CHECK_LAUNCH();
  hipLaunchKernelGGL((cl_bwd_k<false>), grid, dim3(256), 0, s, a);
  LTHM_CHECK_LAUNCH();
  return 0;
}
