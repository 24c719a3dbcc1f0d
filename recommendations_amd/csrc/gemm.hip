// bf16 MFMA GEMM with fused epilogues for gfx950 (v_mfma_f32_16x16x32_bf16).
//
//   C[b] = epi( alpha * A[b] . B[b] )      fp32 accumulation
//
// Each operand is either K-CONTIGUOUS (A[m][k], B[n][k]: the Linear forward
// Y = X W^T and dX = dY W^T layouts) or K-STRIDED (A[k][m], B[k][n]: the
// weight-gradient dW = dY^T X layout).  K-strided tiles are staged into LDS
// untransposed and fed to the MFMA with ds_read_b64_tr_b16 (gfx950 hardware
// transpose read), so no operand is ever transposed in HBM.
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 MFMA
// 16x16 tiles.  Register-staged double-buffered LDS (64 KiB), one barrier per
// K-tile; XOR-swizzled LDS images (128-B rows for K-contiguous, the 256-B row
// swizzle of cdna_hip_programming.md T10(b) for K-strided).
//
// Reference call sites served: every nn.Linear of commons/transformers/layers.py
// (MultiHeadAttention.c_attn/c_proj :240-241, _MLP.c_fc/c_proj :274-276),
// commons/layers.py:65-81 (MLP + QuickGELU), models/lthm/sequence/*.py Linears.
#include <algorithm>

#include "common.hpp"

namespace lthm {

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  int64_t M, N, K;
  int64_t lda, ldb, ldc;
  int64_t sA, sB, sC;  // batch strides (elements)
  int64_t k_per_split;
  float alpha;
  const float* bias;   // [N] f32 or null
  int act;             // LTHM_ACT_*
  const bf16_t* aux;   // pre-activation input for *_GRAD acts [M, ldaux]
  bf16_t* aux_out;     // pre-activation store for GELU/QGELU [M, ldaux]
  int64_t ldaux;
  const void* res1;
  const void* res2;
  int64_t ldr1, ldr2;
  int res1_dt, res2_dt;
  int out_dt;
  float* ws;           // split-K slabs [splits][M][N] f32 (when splits > 1)
  bool fast_ok;        // 16-B aligned operands and leading dims (interior-tile fast path)
  const float* sa;     // fp8 per-tensor scales (device scalars), or null
  const float* sb;
  unsigned* amax;      // atomic max of |C| as f32 bits (gemm_ps_k epilogues), or null
};

__device__ __forceinline__ float ld_any(const void* p, int dt, int64_t i) {
  return dt == LTHM_F32 ? reinterpret_cast<const float*>(p)[i] : bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
}

__device__ __forceinline__ float epilogue(const GemmArgs g, float v, int64_t row, int64_t col, int64_t b) {
  if (g.bias) v += g.bias[col];
  if (g.act == LTHM_ACT_GELU || g.act == LTHM_ACT_QGELU) {
    if (g.aux_out) g.aux_out[b * g.M * g.ldaux + row * g.ldaux + col] = f2bf(v);
    v = (g.act == LTHM_ACT_GELU) ? gelu_tanh(v) : qgelu(v);
  } else if (g.act == LTHM_ACT_GELU_GRAD) {
    v *= gelu_tanh_grad(bf2f(g.aux[b * g.M * g.ldaux + row * g.ldaux + col]));
  } else if (g.act == LTHM_ACT_QGELU_GRAD) {
    v *= qgelu_grad(bf2f(g.aux[b * g.M * g.ldaux + row * g.ldaux + col]));
  } else if (g.act == LTHM_ACT_GELU_D) {
    float dv;
    v = gelu_tanh_and_grad(v, dv);
    if (g.aux_out) g.aux_out[b * g.M * g.ldaux + row * g.ldaux + col] = f2bf(dv);
  } else if (g.act == LTHM_ACT_MUL_AUX) {
    v *= bf2f(g.aux[b * g.M * g.ldaux + row * g.ldaux + col]);
  }
  if (g.res1) v += ld_any(g.res1, g.res1_dt, b * g.M * g.ldr1 + row * g.ldr1 + col);
  if (g.res2) v += ld_any(g.res2, g.res2_dt, b * g.M * g.ldr2 + row * g.ldr2 + col);
  return v;
}

// ---- 8-wide epilogue helpers (vector path when the 8 columns are in range and 16-B aligned)
__device__ __forceinline__ void ld8(const void* p, int dt, int64_t idx, int nv, float (&out)[8]) {
  if (dt == LTHM_F32) {
    const float* q = reinterpret_cast<const float*>(p) + idx;
    if (nv == 8 && ((reinterpret_cast<uintptr_t>(q) & 15) == 0)) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(q), c = *reinterpret_cast<const f32x4*>(q + 4);
      out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w; out[4] = c.x; out[5] = c.y; out[6] = c.z; out[7] = c.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] = (e < nv) ? q[e] : 0.f;
    }
  } else {
    const bf16_t* q = reinterpret_cast<const bf16_t*>(p) + idx;
    if (nv == 8 && ((reinterpret_cast<uintptr_t>(q) & 15) == 0)) {
      load_vec<bf16_t, 16>(q, out);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] = (e < nv) ? bf2f(q[e]) : 0.f;
    }
  }
}
__device__ __forceinline__ void st8(void* p, int dt, int64_t idx, int nv, const float (&v)[8]) {
  if (dt == LTHM_F32) {
    float* q = reinterpret_cast<float*>(p) + idx;
    if (nv == 8 && ((reinterpret_cast<uintptr_t>(q) & 15) == 0)) {
      *reinterpret_cast<f32x4*>(q) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(q + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < nv) q[e] = v[e];
    }
  } else {
    bf16_t* q = reinterpret_cast<bf16_t*>(p) + idx;
    if (nv == 8 && ((reinterpret_cast<uintptr_t>(q) & 15) == 0)) {
      store_vec<bf16_t, 8>(q, v);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < nv) q[e] = f2bf(v[e]);
    }
  }
}

__device__ __forceinline__ void epilogue8(const GemmArgs& g, float (&v)[8], int64_t row, int64_t col0, int64_t b, int split) {
  const int nv = (int)min((int64_t)8, g.N - col0);
  if (g.ws) {  // split-K slab (raw alpha * acc); the combine kernel applies the epilogue
    st8(g.ws, LTHM_F32, ((int64_t)split * gridDim.y + b) * g.M * g.N + row * g.N + col0, nv, v);
    return;
  }
  float t[8];
  if (g.bias) {
    ld8(g.bias, LTHM_F32, col0, nv, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t[e];
  }
  const int64_t ai = b * g.M * g.ldaux + row * g.ldaux + col0;
  if (g.act == LTHM_ACT_GELU || g.act == LTHM_ACT_QGELU) {
    if (g.aux_out) st8(g.aux_out, LTHM_BF16, ai, nv, v);
    if (g.act == LTHM_ACT_GELU) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = qgelu(v[e]);
    }
  } else if (g.act == LTHM_ACT_GELU_GRAD || g.act == LTHM_ACT_QGELU_GRAD) {
    ld8(g.aux, LTHM_BF16, ai, nv, t);
    if (g.act == LTHM_ACT_GELU_GRAD) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= gelu_tanh_grad(t[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= qgelu_grad(t[e]);
    }
  } else if (g.act == LTHM_ACT_GELU_D) {
    float dv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_tanh_and_grad(v[e], dv[e]);
    if (g.aux_out) st8(g.aux_out, LTHM_BF16, ai, nv, dv);
  } else if (g.act == LTHM_ACT_MUL_AUX) {
    ld8(g.aux, LTHM_BF16, ai, nv, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= t[e];
  }
  if (g.res1) {
    ld8(g.res1, g.res1_dt, b * g.M * g.ldr1 + row * g.ldr1 + col0, nv, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t[e];
  }
  if (g.res2) {
    ld8(g.res2, g.res2_dt, b * g.M * g.ldr2 + row * g.ldr2 + col0, nv, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t[e];
  }
  st8(g.C, g.out_dt, b * g.sC + row * g.ldc + col0, nv, v);
}

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = 128 * 64 * 2;  // one operand tile, 16 KiB

// byte offset in a K-contiguous image [128 rows][64 k] (128-B rows)
__device__ __forceinline__ int kc_off(int r, int chunk) { return r * 128 + ((chunk ^ ((r >> 1) & 7)) << 4); }
// byte offset in a K-strided image [64 k-rows][128] (256-B rows), T10(b) swizzle
__device__ __forceinline__ int ks_off(int kr, int ch) {
  return kr * 256 + ((ch ^ (((kr & 3) << 2) | ((kr >> 2) & 3))) << 4);
}

template <bool KCONTIG>
__device__ __forceinline__ void load_tile(const bf16_t* __restrict__ P, int64_t ld, int64_t rows, int64_t r0,
                                          int64_t k, int64_t k1, int tid, u32x4 (&reg)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + 256 * i;
    int64_t gr, gk;
    if constexpr (KCONTIG) {
      gr = r0 + (idx >> 3);
      gk = k + (idx & 7) * 8;
    } else {
      gk = k + (idx >> 4);
      gr = r0 + (idx & 15) * 8;
    }
    // the chunk's 8 elements are contiguous in memory (along k, or along rows)
    const int64_t lim = KCONTIG ? (k1 - gk) : (rows - gr);
    if (gr < rows && gk < k1) {
      const bf16_t* src = KCONTIG ? (P + gr * ld + gk) : (P + gk * ld + gr);
      if (lim >= 8 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
        reg[i] = *reinterpret_cast<const u32x4*>(src);
      } else {  // ragged tail / unaligned row stride: element loads, zero fill (static indices only)
        uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t v = (e < lim) ? (uint32_t)src[e] : 0u;
          w[e >> 1] |= v << ((e & 1) * 16);
        }
        reg[i] = u32x4{w[0], w[1], w[2], w[3]};
      }
    } else {
      reg[i] = u32x4{0u, 0u, 0u, 0u};
    }
  }
}

// interior tiles (whole tile inside the operand, K % 64 == 0): per-thread chunk
// pointers are computed once per tile and advanced by one K-tile per step, no
// bounds tests
template <bool KCONTIG>
__device__ __forceinline__ void chunk_ptrs(const bf16_t* (&p)[4], const bf16_t* __restrict__ P, int64_t ld,
                                           int64_t r0, int64_t k0, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + 256 * i;
    if constexpr (KCONTIG) p[i] = P + (r0 + (idx >> 3)) * ld + k0 + (idx & 7) * 8;
    else p[i] = P + (k0 + (idx >> 4)) * ld + r0 + (idx & 15) * 8;
  }
}
__device__ __forceinline__ void load_fast(const bf16_t* const (&p)[4], int64_t off, u32x4 (&reg)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) reg[i] = *reinterpret_cast<const u32x4*>(p[i] + off);
}

template <bool KCONTIG>
__device__ __forceinline__ void store_tile(unsigned char* lds, int tid, const u32x4 (&reg)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + 256 * i;
    const int off = KCONTIG ? kc_off(idx >> 3, idx & 7) : ks_off(idx >> 4, idx & 15);
    *reinterpret_cast<u32x4*>(lds + off) = reg[i];
  }
}

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

template <bool KCONTIG>
__device__ __forceinline__ bf16x8v read_frag(const unsigned char* lds, int rbase, int s, int lane) {
  if constexpr (KCONTIG) {
    const int r = rbase + (lane & 15);
    const int chunk = s * 4 + (lane >> 4);
    u32x4 v = *reinterpret_cast<const u32x4*>(lds + kc_off(r, chunk));
    return __builtin_bit_cast(bf16x8v, v);
  } else {
    const int gq = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int kr = s * 32 + 8 * gq + q;
    const int ch = (rbase >> 3) + (p >> 1);
    const unsigned char* a0 = lds + ks_off(kr, ch) + 8 * (p & 1);
    const unsigned char* a1 = lds + ks_off(kr + 4, ch) + 8 * (p & 1);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a1));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8v, v);
  }
}

template <bool KA, bool KB>
__global__ __launch_bounds__(256, 2) void gemm_k(GemmArgs g, int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware order: the tiles_n column tiles of one row panel land on one XCD, so
  // the panel of A is fetched from HBM once and re-read from that XCD's L2
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t m0 = (int64_t)(tile / tiles_n) * BM;
  const int64_t n0 = (int64_t)(tile % tiles_n) * BN;
  const int64_t b = blockIdx.y;
  const int split = blockIdx.z;
  const bf16_t* A = g.A + b * g.sA;
  const bf16_t* B = g.B + b * g.sB;
  const int64_t k0 = (int64_t)split * g.k_per_split;
  const int64_t k1 = min(g.K, k0 + g.k_per_split);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[4], rb[4];
  // interior fast path: 16-B aligned chunks everywhere, no tails
  const bool fast = (m0 + BM <= g.M) && (n0 + BN <= g.N) && ((k1 - k0) % BK == 0) && g.fast_ok;
  const bf16_t* pa[4];
  const bf16_t* pb[4];
  if (fast) {
    chunk_ptrs<KA>(pa, A, g.lda, m0, k0, tid);
    chunk_ptrs<KB>(pb, B, g.ldb, n0, k0, tid);
  }
  const int64_t sta = KA ? BK : BK * g.lda, stb = KB ? BK : BK * g.ldb;  // elements per K-tile
  if (k0 < k1) {
    if (fast) {
      load_fast(pa, 0, ra);
      load_fast(pb, 0, rb);
    } else {
      load_tile<KA>(A, g.lda, g.M, m0, k0, k1, tid, ra);
      load_tile<KB>(B, g.ldb, g.N, n0, k0, k1, tid, rb);
    }
    store_tile<KA>(smem, tid, ra);
    store_tile<KB>(smem + TILE_BYTES, tid, rb);
  }
  __syncthreads();
  int cur = 0;
  int64_t oa = 0, ob = 0;
  for (int64_t kt = k0; kt < k1; kt += BK) {
    const bool has_next = kt + BK < k1;
    if (has_next) {
      if (fast) {
        oa += sta;
        ob += stb;
        load_fast(pa, oa, ra);
        load_fast(pb, ob, rb);
      } else {
        load_tile<KA>(A, g.lda, g.M, m0, kt + BK, k1, tid, ra);
        load_tile<KB>(B, g.ldb, g.N, n0, kt + BK, k1, tid, rb);
      }
    }
    const unsigned char* sa = smem + cur * 2 * TILE_BYTES;
    const unsigned char* sb = sa + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8v af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<KA>(sa, wm * 64 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<KB>(sb, wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (has_next) {
      unsigned char* nxt = smem + (cur ^ 1) * 2 * TILE_BYTES;
      store_tile<KA>(nxt, tid, ra);
      store_tile<KB>(nxt + TILE_BYTES, tid, rb);
    }
    __syncthreads();
    cur ^= 1;
  }

  // epilogue: restage the 128x128 f32 tile through LDS in two 64-row halves
  // (static accumulator indices only), then every thread finishes 8 contiguous
  // columns of a row with 16-B loads/stores.
  float* ct = reinterpret_cast<float*>(smem);  // [64][CT_LD]
  constexpr int CT_LD = 132;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (wm == half) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ct[(i * 16 + (lane >> 4) * 4 + r) * CT_LD + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
    for (int q = tid; q < 64 * 16; q += 256) {
      const int lr = q >> 4, c8 = (q & 15) * 8;
      const int64_t row = m0 + half * 64 + lr;
      const int64_t col0 = n0 + c8;
      if (row < g.M && col0 < g.N) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = g.alpha * ct[lr * CT_LD + c8 + e];
        epilogue8(g, v, row, col0, b, split);
      }
    }
    __syncthreads();
  }
}

// split-K combine, 4 adjacent columns per thread (N % 4 == 0): 16-B partial loads, eight
// splits' loads in flight ahead of the adds; each element still sums s = 0, 1, ... in order
// (bit-identical to splitk_reduce_k)
__global__ __launch_bounds__(256) void splitk_reduce4_k(GemmArgs g, int splits) {
  const int64_t MN = g.M * g.N, total4 = MN / 4;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total4; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t rc = t * 4;
    const int64_t row = rc / g.N, col = rc - row * g.N;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    const float* p = g.ws + rc;
#pragma unroll 8
    for (int s = 0; s < splits; ++s) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(p + (int64_t)s * MN);
      v[0] += w[0]; v[1] += w[1]; v[2] += w[2]; v[3] += w[3];
    }
    const int64_t o = row * g.ldc + col;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float r = epilogue(g, v[e], row, col + e, 0);
      if (g.out_dt == LTHM_F32) reinterpret_cast<float*>(g.C)[o + e] = r;
      else reinterpret_cast<bf16_t*>(g.C)[o + e] = f2bf(r);
    }
  }
}

// split-K combine: C = epi(sum_s ws[s])
__global__ __launch_bounds__(256) void splitk_reduce_k(GemmArgs g, int splits, int batch) {
  const int64_t MN = g.M * g.N;
  const int64_t total = MN * batch;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / MN;
    const int64_t rc = t - b * MN;
    const int64_t row = rc / g.N, col = rc - row * g.N;
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += g.ws[((int64_t)s * batch + b) * MN + rc];
    v = epilogue(g, v, row, col, b);
    const int64_t o = b * g.sC + row * g.ldc + col;
    if (g.out_dt == LTHM_F32) reinterpret_cast<float*>(g.C)[o] = v;
    else reinterpret_cast<bf16_t*>(g.C)[o] = f2bf(v);
  }
}

// ---------------------------------------------------------------- persistent ring GEMM
// The encoder's forward / dgrad GEMMs are tall and skinny (M = B*T' = 528k rows,
// N <= 1024, K 256..1024): HBM-bound on the A stream and the C writes, and with
// only K/64 = 4 K-tiles per output tile the one-tile-at-a-time kernel above spends
// most of a tile's life waiting on the load latency of its first K-tile and on its
// epilogue.  This kernel keeps the A stream in flight across tile boundaries:
//
//  * one workgroup per CU, persistent: 4 compute waves (2x2, 64x64 each) and 4
//    loader waves that only issue LDS-DMA (global_load_lds_dwordx4) into a 4-deep
//    ring of 64-k stages; a stage is retired by a counted `s_waitcnt vmcnt` in the
//    loaders + a raw s_barrier, so three stages stay in flight behind the MFMAs and
//    behind the previous tile's epilogue;
//  * each workgroup owns ONE 128-column tile of C for the whole launch and walks
//    row panels: with K <= 256 its B slab (128 x K, <= 64 KiB) is loaded into LDS
//    once (BRES), otherwise B k-tiles ride the ring with A;
//  * XCD-aware: workgroup w runs on XCD w % 8; the tiles_n column owners of one
//    XCD walk the same row panels (p = xcd + 8 (r + R i)) in step, so each A panel
//    is fetched from HBM once and re-read from that XCD's L2;
//  * the epilogue is per wave (no block barrier) and compiled per form (EPI): the
//    bias is held in registers for the whole launch, the residual / pre-activation
//    loads of a 16-row slice are issued one slice ahead, so the in-order vmcnt
//    never waits on this wave's own earlier C stores; slices of the wave's 64x64
//    accumulator are restaged through a wave-private LDS strip and finished 8
//    columns per lane with 16-B loads / stores.
// Requires: A K-contiguous, K % 64 == 0, batch 1, no split-K, 16-B aligned
// operands, leading dims % 8 == 0, N % 8 == 0.
constexpr int PS_NST = 4;
constexpr int PS_LD = 68;  // staging row pitch (floats): conflict-free C-layout writes
constexpr int PS_NLW = 4;  // loader waves
constexpr int PS_THREADS = 64 * (4 + PS_NLW);
// epilogue forms
constexpr int EPI_PLAIN = 0;  // (+ bias)
constexpr int EPI_ACT = 1;    // (+ bias), GELU / QuickGELU, optional pre-activation (or GELU') store
constexpr int EPI_GRAD = 2;   // * act'(aux), or * aux
constexpr int EPI_RES1 = 3;   // (+ bias) + res1 (f32)
constexpr int EPI_RES2 = 4;   // (+ bias) + res1 + res2 (f32)
__device__ __attribute__((aligned(16))) unsigned char gemm_zero16[16];

template <bool BRES>
struct PsSmem {
  unsigned char ring[PS_NST][BRES ? TILE_BYTES : 2 * TILE_BYTES];
  unsigned char bslab[BRES ? 4 : 1][BRES ? TILE_BYTES : 16];
  float stg[4][16 * PS_LD];
};

// DMA pieces [d0, d0 + ND) (1 KiB each) of a 128 x 64 k-tile of a K-contiguous operand
template <int ND>
__device__ __forceinline__ void ps_dma_kc(unsigned char* img, const bf16_t* P, int64_t ld, int64_t rows, int64_t r0,
                                          int64_t k, int lane, int d0) {
#pragma unroll
  for (int d = d0; d < d0 + ND; ++d) {
    const int row = 8 * d + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);  // lane-linear slot -> kc_off swizzle
    const int64_t gr = r0 + row;
    const void* src = gr < rows ? (const void*)(P + gr * ld + k + ch * 8) : (const void*)gemm_zero16;
    glds16(src, img + d * 1024);
  }
}
// ... of a K-strided operand [64 k][128 cols] (256-B rows, ks_off swizzle)
template <int ND>
__device__ __forceinline__ void ps_dma_ks(unsigned char* img, const bf16_t* P, int64_t ld, int64_t cols, int64_t c0,
                                          int64_t k, int lane, int d0) {
#pragma unroll
  for (int d = d0; d < d0 + ND; ++d) {
    const int kr = 4 * d + (lane >> 4);
    const int ch = (lane & 15) ^ (((kr & 3) << 2) | ((kr >> 2) & 3));
    const int64_t gc = c0 + ch * 8;
    const void* src = gc < cols ? (const void*)(P + (k + kr) * ld + gc) : (const void*)gemm_zero16;
    glds16(src, img + d * 1024);
  }
}

// epilogue inputs of one 16-row slice (the lane's 2 chunks of 8 columns)
template <int EPI>
struct PsIn {
  float x[EPI == EPI_RES1 || EPI == EPI_RES2 ? 2 : 1][8];
  float y[EPI == EPI_RES2 ? 2 : 1][8];
  u32x4 xb[EPI == EPI_GRAD ? 2 : 1];  // GRAD: the aux chunks kept as packed bf16 until used
};
// element e of the GRAD aux chunk u
template <int EPI>
__device__ __forceinline__ float ps_aux(const PsIn<EPI>& q, int u, int e) {
  const uint32_t w = q.xb[u][e >> 1];
  return __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
}
template <int EPI>
__device__ __forceinline__ void ps_epi_load(const GemmArgs& g, PsIn<EPI>& in, int64_t r0, int64_t col0) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int64_t row = min(r0 + 8 * u, g.M - 1);  // clamped: the store is predicated
    if constexpr (EPI == EPI_GRAD) in.xb[u] = *reinterpret_cast<const u32x4*>(g.aux + row * g.ldaux + col0);
    if constexpr (EPI == EPI_RES1 || EPI == EPI_RES2) {
      const float* p = reinterpret_cast<const float*>(g.res1) + row * g.ldr1 + col0;
      load_vec<float, 16>(p, in.x[u]);
      load_vec<float, 16>(p + 4, in.x[u] + 4);
    }
    if constexpr (EPI == EPI_RES2) {
      const float* p = reinterpret_cast<const float*>(g.res2) + row * g.ldr2 + col0;
      load_vec<float, 16>(p, in.y[u]);
      load_vec<float, 16>(p + 4, in.y[u] + 4);
    }
  }
}

// running max of |C| over one lane's 8 stored values (rounded as stored)
__device__ __forceinline__ float ps_amax8(float m, const float* v, int dt) {
#pragma unroll
  for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(dt == LTHM_F32 ? v[e] : bf2f(f2bf(v[e]))));
  return m;
}

typedef int i32x8v __attribute__((ext_vector_type(8)));
// fp8 A/B fragment of v_mfma_scale_f32_16x16x128_f8f6f4: lane l holds row rbase + (l & 15),
// k bytes 32 (l >> 4) .. + 31 = the two 16-B chunks 2 (l >> 4), 2 (l >> 4) + 1 of a 128-B row
__device__ __forceinline__ i32x8v read_frag8(const unsigned char* lds, int rbase, int lane) {
  const int r = rbase + (lane & 15), c = 2 * (lane >> 4);
  const u32x4 lo = *reinterpret_cast<const u32x4*>(lds + kc_off(r, c));
  const u32x4 hi = *reinterpret_cast<const u32x4*>(lds + kc_off(r, c + 1));
  return i32x8v{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

// F8: A and B are e4m3 bytes; the host passes K and the leading dims in 2-byte units so
// that the 16-KiB stage / B-slab / DMA geometry is byte-identical to the bf16 kernel (a
// stage holds 128 k of fp8 instead of 64 k of bf16) and one 16x16x128 MFMA (unit block
// scales) replaces the two 16x16x32 steps; the per-tensor scales fold into alpha.
template <bool KB, bool BRES, int EPI, bool F8 = false>
__global__ __launch_bounds__(PS_THREADS, 1) void gemm_ps_k(GemmArgs g, int tiles_m, int tiles_n, int R) {
  __shared__ __attribute__((aligned(16))) PsSmem<BRES> sh;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int xcd = blockIdx.x & 7, jj = blockIdx.x >> 3;
  const int nt = jj % tiles_n, r = jj / tiles_n;
  const int64_t n0 = (int64_t)nt * BN;
  const int NK = (int)(g.K / BK);
  const int first = xcd + 8 * r;
  const int ntile = first < tiles_m ? (tiles_m - 1 - first) / (8 * R) + 1 : 0;
  const int S = ntile * NK;
  if (S == 0) return;  // uniform over the workgroup
  const bool loader = wave >= 4;

  if constexpr (BRES) {  // the workgroup's B slab, once
    if (!loader) {
      u32x4 rb[4];
      for (int kk = 0; kk < NK; ++kk) {
        load_tile<KB>(g.B, g.ldb, g.N, n0, (int64_t)kk * BK, g.K, tid, rb);
        store_tile<KB>(sh.bslab[kk], tid, rb);
      }
    }
    __syncthreads();
  }

  if (loader) {
    // loader waves: each stages a quarter of A's (and B's, BRES off) 16 1-KiB pieces
    constexpr int ND = 16 / PS_NLW;
    constexpr int DPS = (BRES ? 1 : 2) * ND;  // DMAs per stage and loader wave
    const int d0 = (wave - 4) * ND;
    auto issue = [&](int s) {
      const int i = s / NK, kk = s - i * NK;
      const int64_t m0 = (int64_t)(first + 8 * R * i) * BM;
      unsigned char* st = sh.ring[s % PS_NST];
      ps_dma_kc<ND>(st, g.A, g.lda, g.M, m0, (int64_t)kk * BK, lane, d0);
      if constexpr (!BRES) {
        if constexpr (KB) ps_dma_kc<ND>(st + TILE_BYTES, g.B, g.ldb, g.N, n0, (int64_t)kk * BK, lane, d0);
        else ps_dma_ks<ND>(st + TILE_BYTES, g.B, g.ldb, g.N, n0, (int64_t)kk * BK, lane, d0);
      }
    };
    retire_loads();
    for (int s = 0; s < PS_NST && s < S; ++s) issue(s);
    for (int s = 0; s < S; ++s) {
      // stages issued so far: 0 .. min(S-1, s == 0 ? NST-1 : s+NST-2); step s must have landed
      const int behind = min(S - 1, s == 0 ? PS_NST - 1 : s + PS_NST - 2) - s;
      if (behind >= 3) wait_vm<3 * DPS>();
      else if (behind == 2) wait_vm<2 * DPS>();
      else if (behind == 1) wait_vm<DPS>();
      else wait_vm<0>();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s >= 1 && s + PS_NST - 1 < S) issue(s + PS_NST - 1);  // into the stage step s-1 freed
    }
    return;
  }

  // ---------------- compute waves
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t col0 = n0 + wn * 64 + (lane & 7) * 8;  // this lane's 8 epilogue columns (fixed)
  const int64_t colc = col0 < g.N ? col0 : 0;           // clamped for loads
  float bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias[e] = 0.f;
  if (g.bias && EPI != EPI_GRAD) load_vec<float, 16>(g.bias + colc, bias), load_vec<float, 16>(g.bias + colc + 4, bias + 4);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float* stg = sh.stg[wave];
  const float alpha = F8 ? g.alpha * *g.sa * *g.sb : g.alpha;
  float amx = 0.f;  // max |C| of this lane's stores (g.amax)

  // Forward forms (K-contiguous B) defer their epilogue; the dgrad forms and the
  // two-residual epilogue keep the in-line one (the deferred accumulator spills them).
  constexpr bool DEFER = KB && EPI != EPI_RES2 && !F8;
  if constexpr (DEFER) {
  // Deferred epilogue: a finished tile's accumulator moves to eacc and its four 16-row
  // slices are finished one per K-stage of the next tile (after that stage's MFMAs are
  // issued), so the epilogue's VALU / LDS / stores overlap this wave's own MFMAs instead
  // of following them.  Slices still pending when a tile ends are finished first.
  f32x4 eacc[4][4];
  int64_t erb = 0;  // row base of the deferred tile
  PsIn<EPI> ein, enx;
  // slice i of the deferred tile (i a compile-time constant: eacc stays in registers)
  auto epi_slice = [&](auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    if (i + 1 < 4) ps_epi_load<EPI>(g, enx, erb + 16 * (i + 1), colc);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) stg[((lane >> 4) * 4 + rr) * PS_LD + j * 16 + (lane & 15)] = eacc[i][j][rr];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int lr = (lane >> 3) + 8 * u;
      const int64_t row = erb + 16 * i + 8 * u;
      float v[8];
      const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + lr * PS_LD + (lane & 7) * 8);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + lr * PS_LD + (lane & 7) * 8 + 4);
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      const PsIn<EPI>& q = ein;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = alpha * v[e] + bias[e];
      const bool ok = row < g.M && col0 < g.N;
      if constexpr (EPI == EPI_ACT) {
        if (g.act == LTHM_ACT_GELU_D) {
          float dv[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_tanh_and_grad(v[e], dv[e]);
          if (g.aux_out && ok) store_vec<bf16_t, 8>(g.aux_out + row * g.ldaux + col0, dv);
        } else {
          if (g.aux_out && ok) store_vec<bf16_t, 8>(g.aux_out + row * g.ldaux + col0, v);
          if (g.act == LTHM_ACT_GELU) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = qgelu(v[e]);
          }
        }
      }
      if constexpr (EPI == EPI_GRAD) {
        if (g.act == LTHM_ACT_MUL_AUX) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= ps_aux(q, u, e);
        } else if (g.act == LTHM_ACT_GELU_GRAD) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= gelu_tanh_grad(ps_aux(q, u, e));
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= qgelu_grad(ps_aux(q, u, e));
        }
      }
      if constexpr (EPI == EPI_RES1 || EPI == EPI_RES2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += q.x[u][e];
      }
      if constexpr (EPI == EPI_RES2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += q.y[u][e];
      }
      if (g.amax && ok) amx = ps_amax8(amx, v, g.out_dt);
      if (ok) {
        if (g.out_dt == LTHM_F32) {
          float* o = reinterpret_cast<float*>(g.C) + row * g.ldc + col0;
          *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
          *reinterpret_cast<f32x4*>(o + 4) = f32x4{v[4], v[5], v[6], v[7]};
        } else {
          store_vec<bf16_t, 8>(reinterpret_cast<bf16_t*>(g.C) + row * g.ldc + col0, v);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    ein = enx;
  };
  auto epi_all = [&]() __attribute__((always_inline)) {
    epi_slice(std::integral_constant<int, 0>{});
    epi_slice(std::integral_constant<int, 1>{});
    epi_slice(std::integral_constant<int, 2>{});
    epi_slice(std::integral_constant<int, 3>{});
  };
  int s = 0;  // ring stage counter (one per K-step, across tiles)
  auto kstep = [&](int kk) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of the stage the loaders refill next are done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const unsigned char* sa = sh.ring[s % PS_NST];
    const unsigned char* sb = BRES ? sh.bslab[kk] : sa + TILE_BYTES;
    ++s;
    if constexpr (F8) {
      i32x8v af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag8(sa, wm * 64 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag8(sb, wn * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, 127, 0, 127);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8v af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = read_frag<true>(sa, wm * 64 + i * 16, s2, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = read_frag<KB>(sb, wn * 64 + j * 16, s2, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  for (int ti = 0; ti < ntile; ++ti) {
    if (NK >= 4 && ti > 0) {
      // the previous tile's four slices beside the first four K-steps' MFMAs
      kstep(0);
      epi_slice(std::integral_constant<int, 0>{});
      kstep(1);
      epi_slice(std::integral_constant<int, 1>{});
      kstep(2);
      epi_slice(std::integral_constant<int, 2>{});
      kstep(3);
      epi_slice(std::integral_constant<int, 3>{});
      for (int kk = 4; kk < NK; ++kk) kstep(kk);
    } else {
      if (ti > 0) epi_all();
      for (int kk = 0; kk < NK; ++kk) kstep(kk);
    }
    // ---- tile done: defer its epilogue
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        eacc[i][j] = acc[i][j];
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    erb = (int64_t)(first + 8 * R * ti) * BM + wm * 64 + (lane >> 3);  // + 16 i + 8 u
    ps_epi_load<EPI>(g, ein, erb, colc);
  }
  if (ntile > 0) epi_all();
  } else {
  int kk = 0, ti = 0;
  for (int s = 0; s < S; ++s) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of the stage the loaders refill next are done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const unsigned char* sa = sh.ring[s % PS_NST];
    const unsigned char* sb = BRES ? sh.bslab[kk] : sa + TILE_BYTES;
    if constexpr (F8) {
      i32x8v af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag8(sa, wm * 64 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag8(sb, wn * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, 127, 0, 127);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8v af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = read_frag<true>(sa, wm * 64 + i * 16, s2, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = read_frag<KB>(sb, wn * 64 + j * 16, s2, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (++kk < NK) continue;
    // ---- tile done: per-wave epilogue, 16 rows at a time through the wave's strip
    kk = 0;
    const int64_t rbase = (int64_t)(first + 8 * R * ti) * BM + wm * 64 + (lane >> 3);  // + 16 i + 8 u
    ++ti;
    PsIn<EPI> in[2];
    ps_epi_load<EPI>(g, in[0], rbase, colc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i + 1 < 4) ps_epi_load<EPI>(g, in[(i + 1) & 1], rbase + 16 * (i + 1), colc);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) stg[((lane >> 4) * 4 + rr) * PS_LD + j * 16 + (lane & 15)] = acc[i][j][rr];
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int lr = (lane >> 3) + 8 * u;
        const int64_t row = rbase + 16 * i + 8 * u;
        float v[8];
        const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + lr * PS_LD + (lane & 7) * 8);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + lr * PS_LD + (lane & 7) * 8 + 4);
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        const PsIn<EPI>& q = in[i & 1];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = alpha * v[e] + bias[e];
        const bool ok = row < g.M && col0 < g.N;
        if constexpr (EPI == EPI_ACT) {
          if (g.act == LTHM_ACT_GELU_D) {
            float dv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = gelu_tanh_and_grad(v[e], dv[e]);
            if (g.aux_out && ok) store_vec<bf16_t, 8>(g.aux_out + row * g.ldaux + col0, dv);
          } else {
            if (g.aux_out && ok) store_vec<bf16_t, 8>(g.aux_out + row * g.ldaux + col0, v);
            if (g.act == LTHM_ACT_GELU) {
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = qgelu(v[e]);
            }
          }
        }
        if constexpr (EPI == EPI_GRAD) {
          if (g.act == LTHM_ACT_MUL_AUX) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= ps_aux(q, u, e);
          } else if (g.act == LTHM_ACT_GELU_GRAD) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= gelu_tanh_grad(ps_aux(q, u, e));
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= qgelu_grad(ps_aux(q, u, e));
          }
        }
        if constexpr (EPI == EPI_RES1 || EPI == EPI_RES2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += q.x[u][e];
        }
        if constexpr (EPI == EPI_RES2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += q.y[u][e];
        }
        if (g.amax && ok) amx = ps_amax8(amx, v, g.out_dt);
        if (ok) {
          if (g.out_dt == LTHM_F32) {
            float* o = reinterpret_cast<float*>(g.C) + row * g.ldc + col0;
            *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
            *reinterpret_cast<f32x4*>(o + 4) = f32x4{v[4], v[5], v[6], v[7]};
          } else {
            store_vec<bf16_t, 8>(reinterpret_cast<bf16_t*>(g.C) + row * g.ldc + col0, v);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
  }
  if (g.amax) {
    amx = wave_max(amx);
    if (lane == 0) atomicMax(g.amax, __float_as_uint(amx));
  }
}

// ---------------------------------------------------------------- weight-gradient GEMM
// dW = dY^T X over M = B*T' = 528k token rows (both operands K-strided), N_out x
// N_in <= 1024 x 1024.  The one-tile kernel re-reads each operand slice from L2
// once per 128-wide output tile; this kernel gives a workgroup a 256 x 256 output
// tile (8 compute waves as 4 x 2, 64 x 128 each: 128 accumulator registers per
// lane) and a split of the M range, halving the LDS fill traffic per flop.  The
// waves themselves stream 32-k stages (A 256 + B 256 columns, 2 x 16 KiB) into a
// 4-deep LDS ring by LDS-DMA, retired by counted vmcnt waits + s_barrier; nothing
// else in the loop touches vmcnt.  XCD-aware: the logical order split-major /
// tile-minor keeps the output tiles of one split on one XCD, so each k-slice of
// the operands is fetched from HBM once and re-read from that XCD's L2.  Each
// workgroup writes its raw f32 partial tile to the split-K slab; splitk_reduce_k
// applies alpha's epilogue (accumulate / output dtype).
// Requires: A and B K-strided, batch 1, 16-B aligned operands and leading dims % 8 == 0; any
// K (k rows past the end read a zero chunk).  A 64-k-stage, two-buffer form of this kernel
// (the gemm_pp_k schedule) measured 5-10 % slower on every wgrad shape (profiles/r04ac/).
constexpr int WG_NST = 4;
constexpr int WG_BK = 32;
constexpr int WG_SUB = 32 * 256;  // one [32 k][128 cols] sub-image (8 KiB)
struct WgSmem {
  unsigned char ring[WG_NST][4][WG_SUB];  // per stage: A cols 0-127, A 128-255, B 0-127, B 128-255
};

__global__ __launch_bounds__(512, 1) void gemm_wg_k(GemmArgs g, int tiles_m, int tiles_n, int splits, int64_t kps) {
  __shared__ __attribute__((aligned(16))) WgSmem sh;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nblk = tiles_m * tiles_n * splits;
  const int lid = xcd_remap(blockIdx.x, nblk);
  const int split = lid / (tiles_m * tiles_n), tile = lid - split * (tiles_m * tiles_n);
  const int64_t m0 = (int64_t)(tile / tiles_n) * 256, n0 = (int64_t)(tile % tiles_n) * 256;
  const int64_t kb = (int64_t)split * kps, ke = min(g.K, kb + kps);
  const int S = ke > kb ? (int)((ke - kb + WG_BK - 1) / WG_BK) : 0;
  // stage s: pieces 0..31 (1 KiB each, 4 k-rows x 256 B of one sub-image); wave w issues w, w+8, w+16, w+24
  auto issue = [&](int st) {
    const int64_t k = kb + (int64_t)st * WG_BK;
    unsigned char* base = sh.ring[st % WG_NST][0];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int piece = wave + 8 * u;  // u = sub-image: 0,1 -> A halves, 2,3 -> B halves
      const int sub = piece >> 3, d = piece & 7;
      const bool isA = sub < 2;
      const bf16_t* P = isA ? g.A : g.B;
      const int64_t ld = isA ? g.lda : g.ldb, cols = isA ? g.M : g.N;
      const int64_t c0 = (isA ? m0 : n0) + (sub & 1) * 128;
      const int kr = 4 * d + (lane >> 4);
      const int ch = (lane & 15) ^ (((kr & 3) << 2) | ((kr >> 2) & 3));
      const int64_t gc = c0 + ch * 8;
      const void* src = (gc < cols && k + kr < ke) ? (const void*)(P + (k + kr) * ld + gc) : (const void*)gemm_zero16;
      glds16(src, base + sub * WG_SUB + d * 1024);
    }
  };
  const int wm = wave >> 1, wn = wave & 1;  // rows wm*64.., cols wn*128..
  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  retire_loads();
  for (int st = 0; st < WG_NST - 1 && st < S; ++st) issue(st);
  for (int s = 0; s < S; ++s) {
    // issued: 0 .. min(S-1, s+NST-2); step s must have landed (4 DMAs per wave and stage)
    const int behind = min(S - 1, s + WG_NST - 2) - s;
    if (behind >= 2) wait_vm<8>();
    else if (behind == 1) wait_vm<4>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the stage being freed are done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + WG_NST - 1 < S) issue(s + WG_NST - 1);  // into the stage step s-1 freed
    const unsigned char* sa = sh.ring[s % WG_NST][wm >> 1];  // A rows wm*64: sub-image wm/2, cols (wm&1)*64
    const unsigned char* sb = sh.ring[s % WG_NST][2 + wn];  // B cols wn*128..: sub-image 2 + wn
    bf16x8v af[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = read_frag<false>(sa, (wm & 1) * 64 + i * 16, 0, lane);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bf16x8v bfr = read_frag<false>(sb, j * 16, 0, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
    }
  }
  // raw alpha * partial tile -> split-K slab [split][M][N] (16 lanes = 64 contiguous bytes)
  float* ws = g.ws + (int64_t)split * g.M * g.N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const int64_t col = n0 + wn * 128 + j * 16 + (lane & 15);
        if (row < g.M && col < g.N) ws[row * g.N + col] = g.alpha * acc[i][j][r];
      }
}

// ---------------------------------------------------------------- 256 x 256 forward / dgrad GEMM
// Both operands K-contiguous (Y = X W^T, dX = dY W^T on a W^T copy) at K > 256, where the
// persistent kernel's resident B slab no longer fits and its 128 x 128 tile re-reads the
// LDS per flop at one compute wave per SIMD: the ranker MLPs (K = 2,176 / 1,024 / 512,
// M = 65,536) and the C5 encoder forms (K 512 / 2,048).  A workgroup of 8 waves owns one
// 256 x 256 tile of C (4 x 2 waves, 64 x 128 each: 128 accumulator registers per lane);
// all 8 waves stream 32-k stages of A and B (256 rows x 64 B each, 16 KiB) into a 4-deep
// LDS ring by LDS-DMA, retired by counted vmcnt waits + one barrier per stage.  Image rows
// are 64 B with the 16-B chunk c of row r at slot c ^ (3 (r >> 2) & 3): conflict-free for
// the 16x16x32 operand reads (ds_read_b128 lane groups).  The epilogue restages each
// wave's 16-row slices through the (drained) ring and runs the generic 8-wide epilogue
// (bias, activations / their gradients, aux, residuals).  Grid order: XCD-contiguous tiles,
// the tiles of one row panel adjacent (each A panel fetched once per XCD).
constexpr int BT_NST = 4, BT_BK = 32;
constexpr int BT_SUB = 256 * 64;  // one operand stage (256 rows x 32 k), 16 KiB
struct BtSmem {
  unsigned char ring[BT_NST][2][BT_SUB];  // 128 KiB: [stage][A, B]
};

__device__ __forceinline__ int bt_off(int r, int c) { return r * 64 + ((c ^ ((3 * (r >> 2)) & 3)) << 4); }

// F8: A and B are e4m3 bytes with K and the leading dims in 2-byte units (the geometry of the
// bf16 kernel: a stage is 64 k of fp8); one v_mfma_scale_f32_16x16x128_f8f6f4 (unit block
// scales) consumes TWO stages: lane group kg takes 16 B of stage s and 16 B of stage s + 1
// (the same k permutation for A and B, so the dot products are unchanged); the per-tensor
// scales fold into alpha.
template <bool F8>
__global__ __launch_bounds__(512, 1) void gemm_bt_k(GemmArgs g, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) BtSmem sh;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nblk = tiles_m * tiles_n;
  const int lid = xcd_remap(blockIdx.x, nblk);
  const int64_t m0 = (int64_t)(lid / tiles_n) * 256, n0 = (int64_t)(lid % tiles_n) * 256;
  const int S = (int)(g.K / BT_BK);
  // stage st: A pieces 0..15, B pieces 0..15 (1 KiB = 16 rows x 64 B each); wave w issues
  // A w, w + 8 and B w, w + 8.  Lane l lands at row 16 d + l / 4, slot l % 4 and so loads
  // chunk slot ^ f(row) (the swizzle is an involution in the chunk index).
  auto issue = [&](int st) {
    const int64_t k = (int64_t)st * BT_BK;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool isA = u < 2;
      const int d = wave + 8 * (u & 1);
      const int row = 16 * d + (lane >> 2);
      const int ch = (lane & 3) ^ ((3 * (row >> 2)) & 3);
      const bf16_t* P = isA ? g.A : g.B;
      const int64_t ld = isA ? g.lda : g.ldb, rows = isA ? g.M : g.N;
      const int64_t gr = (isA ? m0 : n0) + row;
      const void* src = gr < rows ? (const void*)(P + gr * ld + k + ch * 8) : (const void*)gemm_zero16;
      glds16(src, sh.ring[st % BT_NST][isA ? 0 : 1] + d * 1024);
    }
  };
  const int wm = wave >> 1, wn = wave & 1;  // rows wm * 64 .., cols wn * 128 ..
  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  retire_loads();
  const int r16 = lane & 15, c4 = lane >> 4;
  if constexpr (F8) {
    // stage pairs (p = 2 stages) double-buffered in the 4-stage ring
    for (int st = 0; st < 2 && st < S; ++st) issue(st);
    for (int s = 0; s < S; s += 2) {
      // this pair landed: stages s, s + 1 (issued: 0 .. min(S - 1, s + 1)); 4 DMAs per wave and stage
      wait_vm<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s + 2 < S) issue(s + 2);
      if (s + 3 < S) issue(s + 3);
      const unsigned char* sa0 = sh.ring[s % BT_NST][0];
      const unsigned char* sb0 = sh.ring[s % BT_NST][1];
      const unsigned char* sa1 = sh.ring[(s + 1) % BT_NST][0];
      const unsigned char* sb1 = sh.ring[(s + 1) % BT_NST][1];
      i32x8v af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + r16;
        const u32x4 lo = *reinterpret_cast<const u32x4*>(sa0 + bt_off(r, c4));
        const u32x4 hi = *reinterpret_cast<const u32x4*>(sa1 + bt_off(r, c4));
        af[i] = i32x8v{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = wn * 128 + j * 16 + r16;
        const u32x4 lo = *reinterpret_cast<const u32x4*>(sb0 + bt_off(r, c4));
        const u32x4 hi = *reinterpret_cast<const u32x4*>(sb1 + bt_off(r, c4));
        const i32x8v bfr = {(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr, acc[i][j], 0, 0, 0, 127, 0, 127);
      }
    }
  } else {
  for (int st = 0; st < BT_NST - 1 && st < S; ++st) issue(st);
  for (int s = 0; s < S; ++s) {
    // issued: 0 .. min(S-1, s+NST-2); step s must have landed (4 DMAs per wave and stage)
    const int behind = min(S - 1, s + BT_NST - 2) - s;
    if (behind >= 2) wait_vm<8>();
    else if (behind == 1) wait_vm<4>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the stage being freed are done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + BT_NST - 1 < S) issue(s + BT_NST - 1);  // into the stage step s-1 freed
    const unsigned char* sa = sh.ring[s % BT_NST][0];
    const unsigned char* sb = sh.ring[s % BT_NST][1];
    bf16x8v af[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      af[i] = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(sa + bt_off(wm * 64 + i * 16 + r16, c4)));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bf16x8v bfr =
          __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(sb + bt_off(wn * 128 + j * 16 + r16, c4)));
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
    }
  }
  }
  const float alpha = F8 ? g.alpha * *g.sa * *g.sb : g.alpha;
  // epilogue: every wave's ring reads are done before the ring becomes the staging area
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  constexpr int LDP = 132;  // staging row pitch (floats)
  float* stg = reinterpret_cast<float*>(&sh.ring[0][0][0]) + wave * 16 * LDP;
  const int cq = (lane & 15) * 8;  // this lane's 8 columns of the wave's 128
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) stg[((lane >> 4) * 4 + r) * LDP + j * 16 + (lane & 15)] = acc[i][j][r];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int lr = (lane >> 4) + 4 * u;
      const int64_t row = m0 + wm * 64 + i * 16 + lr;
      const int64_t col0 = n0 + wn * 128 + cq;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + lr * LDP + cq);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + lr * LDP + cq + 4);
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= alpha;
      if (row < g.M && col0 < g.N) epilogue8(g, v, row, col0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

// ---------------------------------------------------------------------------
// 256 x 256 tiles for K-contiguous A and B at K >= 512 (the MFMA-bound forms: the ranker MLPs,
// the C5 encoder's K = 512 / 2,048 GEMMs, the K = 1,024 dgrad of C2's MLP).  8 waves as
// 2 (M) x 4 (N), each wave a 128 x 64 block of C = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16
// (128 accumulator registers).  K-tiles of 64 ride two LDS buffers of four 16-KiB halves
// (A rows 0-127 / 128-255, B rows 0-127 / 128-255), each half 16 LDS-DMA pieces of 8 rows
// x 128 B, the 16-B chunk c of row r at slot c ^ ((r >> 1) & 7): conflict-free for the
// 16-row ds_read_b128 fragment reads.  One barrier per K-tile: behind it every wave issues the
// next K-tile's DMA into the other buffer (read by all waves before they reached the barrier)
// and computes this K-tile in four quadrant phases (64 x 32 of the wave's block, 16 MFMAs
// each; A and B fragments re-read per phase, B of quadrant columns 0 kept across phases 1 and
// 4).  Epilogue: 16-row slices restaged through the drained buffers, the generic 8-wide epilogue.
constexpr int PP_BK = 64;
constexpr int PP_HALF = 128 * 128;  // bytes of one half image (128 rows x 64 k bf16)

// LayerNorm epilogues of the N = 256 GEMMs (round 5): a 256 x 256 tile holds whole rows of a
// d = 256 LayerNorm, so the block finishes the LayerNorm itself instead of writing the GEMM
// output for a separate pass to re-read.
//  * PP_LNB (lthm_dgrad_layernorm_bwd): dh = dy W stays f32 on chip, then layernorm.hip
//    ln_bwd_v4_k's arithmetic: dx (+ residuals), its bf16 copy, per-tile dw / db partials;
//  * PP_LNF (lthm_linear_layernorm_fwd): x1 = res1 + o W^T + bias is written (f32) and
//    ln_fwd_v4_k's arithmetic (two-pass statistics, the same lane layout) gives the bf16
//    LayerNorm output and the row statistics.
constexpr int PP_PLAIN = 0, PP_LNB = 1, PP_LNF = 2;
// rows per wave whose LayerNorm-epilogue loads (x / residuals) are in flight together: the
// epilogue is a chain of HBM round trips, 16 rows per wave and half in 16 / PP_EPR of them
// (round 6: 8, was 4: dgrad_ln 0.574 / 0.568 -> 0.565 ms per C2 call, profiles/r06c/; -DLTHM_PP_EPR=4
// rebuilds the old form)
#ifndef LTHM_PP_EPR
#define LTHM_PP_EPR 8
#endif
constexpr int PP_EPR = LTHM_PP_EPR;
struct LnbArgs {
  const float* x;      // LNB: LayerNorm input [M, 256] f32
  const float* w;      // LayerNorm weight [256]
  const float* mean;   // LNB: [M] (read)
  const float* rstd;   // LNB: [M] (read)
  const float* res1;   // [M, 256] f32 or null (LNF: the residual added before the LayerNorm)
  const float* res2;   // LNB: [M, 256] f32 or null
  float* dx;           // LNB: [M, 256] f32;  LNF: x1 [M, 256] f32
  bf16_t* dxb;         // LNB: [M, 256] bf16 copy or null;  LNF: the LayerNorm output [M, 256] bf16
  float* dw_part;      // LNB: [tiles, 256] per-tile weight-gradient partials
  float* db_part;      // LNB: [tiles, 256]
  int res1_twice;      // LNB: the f32 dx carries res1 once more than the bf16 copy
  const float* b;      // LNF: LayerNorm bias [256] or null
  const float* bias;   // LNF: the linear layer's bias [256] or null
  float* mean_out;     // LNF: [M]
  float* rstd_out;     // LNF: [M]
};


// F8: A and B are e4m3 bytes with K and the leading dims in 2-byte units (a K-tile row is 128 k
// of fp8): one v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales) per fragment pair and
// K-tile, lane group c4 taking chunks 2 c4 and 2 c4 + 1 of the row; the per-tensor scales fold
// into alpha.
// SPREAD: the next K-tile's four half images are issued one per quadrant phase (2 DMAs each)
// instead of all eight DMAs behind the barrier (bf16: C4 forms 4-6 % faster; the fp8 form ran
// 3x slower so, and raising the MFMA phases' wave priority lost 5-7 %, profiles/r04ab/)
template <bool F8, bool SPREAD = false, int EPX = PP_PLAIN>
__global__ __launch_bounds__(512, 1) void gemm_pp_k(GemmArgs g, int tiles_m, int tiles_n, LnbArgs L = LnbArgs{}) {
  __shared__ __attribute__((aligned(16))) unsigned char sh[2 * 4 * PP_HALF];  // [buf][A0, A1, B0, B1]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nblk = tiles_m * tiles_n;
  const int lid = xcd_remap(blockIdx.x, nblk);
  const int64_t m0 = (int64_t)(lid / tiles_n) * 256, n0 = (int64_t)(lid % tiles_n) * 256;
  const int nk = (int)(g.K / PP_BK);
  const int wr = wave >> 2, wc = wave & 3;
  // this lane's DMA rows: piece d = wave + 8 u of a half, row 8 d + lane / 8, slot lane % 8
  const int prow0 = 8 * wave + (lane >> 3), slot = lane & 7;
  auto issue_half = [&](int kt, int buf, int hf) {
    const int64_t k = (int64_t)kt * PP_BK;
    const bool isA = hf < 2;
    const bf16_t* P = isA ? g.A : g.B;
    const int64_t ld = isA ? g.lda : g.ldb, rows = isA ? g.M : g.N;
    const int64_t r0 = (isA ? m0 : n0) + 128 * (hf & 1);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = prow0 + 64 * u;
      const int c = slot ^ ((row >> 1) & 7);
      const int64_t gr = r0 + row;
      const void* src = gr < rows ? (const void*)(P + gr * ld + k + c * 8) : (const void*)gemm_zero16;
      glds16(src, sh + (buf * 4 + hf) * PP_HALF + (wave + 8 * u) * 1024);
    }
  };
  auto issue = [&](int kt, int buf) {
#pragma unroll
    for (int hf = 0; hf < 4; ++hf) issue_half(kt, buf, hf);
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  retire_loads();
  issue(0, 0);
  const int r16 = lane & 15, c4 = lane >> 4;
  // lane-constant fragment offsets: rows 16 i + r16 share the swizzle of r16
  const int fa = r16 * 128, sw = (r16 >> 1) & 7;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool more = kt + 1 < nk;
    if (!SPREAD && more) issue(kt + 1, buf ^ 1);
    const unsigned char* Ah = sh + (buf * 4 + wr) * PP_HALF;
    const unsigned char* Bh = sh + (buf * 4 + 2 + (wc >> 1)) * PP_HALF + (wc & 1) * 64 * 128;
    if constexpr (F8) {
      i32x8v b0[2], b1[2];  // [j within the quadrant]
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        if (SPREAD && more) issue_half(kt + 1, buf ^ 1, ph);
        const int mi = ph >> 1;
        const int nj = (ph == 1 || ph == 2) ? 1 : 0;
        i32x8v af[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const unsigned char* ra = Ah + (64 * mi + 16 * i) * 128 + fa;
          const u32x4 lo = *reinterpret_cast<const u32x4*>(ra + (((2 * c4) ^ sw) << 4));
          const u32x4 hi = *reinterpret_cast<const u32x4*>(ra + (((2 * c4 + 1) ^ sw) << 4));
          af[i] = i32x8v{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
        }
        if (ph == 0 || ph == 1) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const unsigned char* rb = Bh + (32 * nj + 16 * j) * 128 + fa;
            const u32x4 lo = *reinterpret_cast<const u32x4*>(rb + (((2 * c4) ^ sw) << 4));
            const u32x4 hi = *reinterpret_cast<const u32x4*>(rb + (((2 * c4 + 1) ^ sw) << 4));
            const i32x8v v = {(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
            if (ph == 0) b0[j] = v;
            else b1[j] = v;
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[4 * mi + i][2 * nj + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                af[i], nj ? b1[j] : b0[j], acc[4 * mi + i][2 * nj + j], 0, 0, 0, 127, 0, 127);
      }
      continue;
    }
    bf16x8v b0[2][2], b1[2][2];  // [j within the quadrant][k-step]
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      if (SPREAD && more) issue_half(kt + 1, buf ^ 1, ph);
      const int mi = ph >> 1;            // quadrant rows 64 mi ..
      const int nj = (ph == 1 || ph == 2) ? 1 : 0;  // columns 32 nj .. (order 0, 1, 1, 0)
      bf16x8v af[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          af[i][s2] = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(
                                                      Ah + (64 * mi + 16 * i) * 128 + fa + (((4 * s2 + c4) ^ sw) << 4)));
      if (ph == 0 || ph == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const bf16x8v v = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u32x4*>(
                                                    Bh + (32 * nj + 16 * j) * 128 + fa + (((4 * s2 + c4) ^ sw) << 4)));
            if (ph == 0) b0[j][s2] = v;
            else b1[j][s2] = v;
          }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[4 * mi + i][2 * nj + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                af[i][s2], nj ? b1[j][s2] : b0[j][s2], acc[4 * mi + i][2 * nj + j], 0, 0, 0);
    }
  }
  // epilogue: the buffers are free once every wave's last fragment reads are done
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if constexpr (EPX != PP_PLAIN) {
    // 128 rows x 256 f32 per half (rows 64 hb .. of both row waves), column c of row t at
    // c ^ (((t >> 2) & 3) << 4): the accumulator stores (16 consecutive columns x 4 row groups
    // per instruction) hit 64 distinct banks, the row reads stay 16-B contiguous
    float* T = reinterpret_cast<float*>(sh);
    const int c = lane * 4;
    float wg[4], dwa[4] = {0.f, 0.f, 0.f, 0.f}, dba[4] = {0.f, 0.f, 0.f, 0.f};
    load_vec<float, 16>(L.w + c, wg);
    const float alpha = g.alpha;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int t = wr * 64 + 16 * i + 4 * c4 + r, col = wc * 64 + 16 * j + r16;
            T[t * 256 + (col ^ (((t >> 2) & 3) << 4))] = acc[4 * hb + i][j][r] * alpha;
          }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if constexpr (EPX == PP_LNF) {
        float lb[4] = {0.f, 0.f, 0.f, 0.f}, bb[4] = {0.f, 0.f, 0.f, 0.f};
        if (L.b) load_vec<float, 16>(L.b + c, lb);
        if (L.bias) load_vec<float, 16>(L.bias + c, bb);
#pragma unroll 1
        for (int q0 = 0; q0 < 16; q0 += PP_EPR) {
          float r1[PP_EPR][4];
          int64_t grow[PP_EPR];
#pragma unroll
          for (int u = 0; u < PP_EPR; ++u) {
            const int t = wave * 16 + q0 + u;
            grow[u] = m0 + (t >> 6) * 128 + hb * 64 + (t & 63);
            const int64_t gr = grow[u] < g.M ? grow[u] : 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) r1[u][e] = 0.f;
            if (L.res1) load_vec<float, 16>(L.res1 + gr * 256 + c, r1[u]);
          }
#pragma unroll
          for (int u = 0; u < PP_EPR; ++u) {
            const int t = wave * 16 + q0 + u;
            const f32x4 a4 = *reinterpret_cast<const f32x4*>(T + t * 256 + (c ^ (((t >> 2) & 3) << 4)));
            float v[4] = {a4.x + bb[0], a4.y + bb[1], a4.z + bb[2], a4.w + bb[3]};
            float sm = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] += r1[u][e];
              sm += v[e];
            }
            sm = wave_sum(sm);
            const float mu = sm / 256.f;
            float qq = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float dd = v[e] - mu;
              qq += dd * dd;
            }
            qq = wave_sum(qq);
            const float rs = 1.f / sqrtf(qq / 256.f + 1e-5f);
            if (grow[u] < g.M) {
              store_vec<float, 4>(L.dx + grow[u] * 256 + c, v);
              float o[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) o[e] = (v[e] - mu) * rs * wg[e] + lb[e];
              store_vec<bf16_t, 4>(L.dxb + grow[u] * 256 + c, o);
              if (lane == 0) {
                L.mean_out[grow[u]] = mu;
                L.rstd_out[grow[u]] = rs;
              }
            }
          }
        }
      } else {
        // wave w: staged rows 16 w .. 16 w + 15, PP_EPR rows' loads in flight at a time
  #pragma unroll 1
        for (int q0 = 0; q0 < 16; q0 += PP_EPR) {
          float xv[PP_EPR][4], r1[PP_EPR][4], r2[PP_EPR][4], mu[PP_EPR], rs[PP_EPR];
          int64_t grow[PP_EPR];
  #pragma unroll
          for (int u = 0; u < PP_EPR; ++u) {
            const int t = wave * 16 + q0 + u;
            grow[u] = m0 + (t >> 6) * 128 + hb * 64 + (t & 63);
            const bool ok = grow[u] < g.M;
            const int64_t gr = ok ? grow[u] : 0;
  #pragma unroll
            for (int e = 0; e < 4; ++e) { r1[u][e] = 0.f; r2[u][e] = 0.f; }
            load_vec<float, 16>(L.x + gr * 256 + c, xv[u]);
            if (L.res1) load_vec<float, 16>(L.res1 + gr * 256 + c, r1[u]);
            if (L.res2) load_vec<float, 16>(L.res2 + gr * 256 + c, r2[u]);
            mu[u] = L.mean[gr];
            rs[u] = L.rstd[gr];
          }
  #pragma unroll
          for (int u = 0; u < PP_EPR; ++u) {
            const int t = wave * 16 + q0 + u;
            const f32x4 d4 = *reinterpret_cast<const f32x4*>(T + t * 256 + (c ^ (((t >> 2) & 3) << 4)));
            const float d[4] = {d4.x, d4.y, d4.z, d4.w};
            float gg[4], xh[4], s1 = 0.f, s2 = 0.f;
  #pragma unroll
            for (int e = 0; e < 4; ++e) {
              xh[e] = (xv[u][e] - mu[u]) * rs[u];
              gg[e] = d[e] * wg[e];
              s1 += gg[e];
              s2 += gg[e] * xh[e];
            }
            s1 = wave_sum(s1) / 256.f;
            s2 = wave_sum(s2) / 256.f;
            if (grow[u] < g.M) {
              float o[4];
  #pragma unroll
              for (int e = 0; e < 4; ++e) {
                dwa[e] += d[e] * xh[e];
                dba[e] += d[e];
                o[e] = rs[u] * (gg[e] - s1 - xh[e] * s2) + r1[u][e] + r2[u][e];
              }
              if (L.dxb) store_vec<bf16_t, 4>(L.dxb + grow[u] * 256 + c, o);
              if (L.res1_twice) {
  #pragma unroll
                for (int e = 0; e < 4; ++e) o[e] += r1[u][e];
              }
              store_vec<float, 4>(L.dx + grow[u] * 256 + c, o);
            }
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if constexpr (EPX == PP_LNF) return;
    // per-tile weight-gradient partials: the 8 waves' column sums in a fixed order
    const int tile = lid / tiles_n;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const float* src = pass ? dba : dwa;
      *reinterpret_cast<f32x4*>(T + wave * 256 + c) = f32x4{src[0], src[1], src[2], src[3]};
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (tid < 256) {
        float sacc = 0.f;
#pragma unroll
        for (int v = 0; v < 8; ++v) sacc += T[v * 256 + tid];
        (pass ? L.db_part : L.dw_part)[(int64_t)tile * 256 + tid] = sacc;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    return;
  }
  // each wave's 128 x 64 block in two 64-row halves through its 16-KiB slice of the buffers
  // (column groups of 16 XOR-rotated by row / 4: conflict-free stores), then a row loop with the
  // generic epilogue (one copy of its code: the accumulator indices stay static)
  float* stg = reinterpret_cast<float*>(sh) + wave * 64 * 64;
  const int cq = (lane & 7) * 8;  // this lane's 8 columns of the wave's 64
  const float alpha = F8 ? g.alpha * *g.sa * *g.sb : g.alpha;
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * c4 + r, col = 16 * j + r16;
          stg[row * 64 + (col ^ (((row >> 2) & 3) << 4))] = acc[4 * hb + i][j][r];
        }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    for (int lr = lane >> 3; lr < 64; lr += 8) {
      const int64_t row = m0 + wr * 128 + hb * 64 + lr;
      const int64_t col0 = n0 + wc * 64 + cq;
      const float* sp = stg + lr * 64 + (cq ^ (((lr >> 2) & 3) << 4));
      const f32x4 lo = *reinterpret_cast<const f32x4*>(sp);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(sp + 4);
      float v[8] = {lo.x * alpha, lo.y * alpha, lo.z * alpha, lo.w * alpha,
                    hi.x * alpha, hi.y * alpha, hi.z * alpha, hi.w * alpha};
      if (row < g.M && col0 < g.N) epilogue8(g, v, row, col0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

}  // namespace lthm

using namespace lthm;

static int lthm_cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

// 0: never, 1: when eligible (default), set by LTHM_GEMM_PS
static int lthm_gemm_ps_mode() {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("LTHM_GEMM_PS");
    mode = (e && e[0] == '0') ? 0 : 1;
  }
  return mode;
}

// 256 x 256 big-K kernel: off by default (LTHM_GEMM_BT=1 selects it where eligible).  Measured
// against the default kernels (profiles/r04d_*): C4 12.66 -> 12.18 M samples/s, C5 5,424 -> 4,664
// samples/s (C5 forward GEMMs 1.28 -> 2.04 ms bf16, 0.98 -> 1.51 ms fp8 per call)
static int lthm_gemm_bt_mode() {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("LTHM_GEMM_BT");
    mode = (e && e[0] == '1') ? 1 : 0;
  }
  return mode;
}

// 256 x 256 kernel (gemm_pp_k) for K-contiguous operands at K >= 512: LTHM_GEMM_PP=0 turns it off,
// 2 issues the next K-tile's DMA all behind the barrier instead of per phase (A/B)
static int lthm_gemm_pp_mode() {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("LTHM_GEMM_PP");
    mode = e ? atoi(e) : 1;
  }
  return mode;
}

// the fp8 form of gemm_pp_k (K >= 1,024): LTHM_GEMM_PP_F8=0 turns it off
static int lthm_gemm_pp_f8() {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("LTHM_GEMM_PP_F8");
    mode = (e && e[0] == '0') ? 0 : 1;
  }
  return mode;
}

extern "C" int lthm_dgrad_layernorm_bwd_tiles(int64_t M) { return (int)((M + 255) / 256); }

extern "C" int lthm_dgrad_layernorm_bwd(const void* dy, const void* wt, int64_t M, int32_t D, int64_t K,
                                        const float* x, const float* w, const float* mean, const float* rstd,
                                        const float* res1, const float* res2, float* dx, void* dx_bf16,
                                        float* partials, int32_t flags, void* stream) {
  LTHM_REQUIRE(D == 256 && M >= 0 && K > 0 && K % PP_BK == 0 && (flags & ~1) == 0);
  LTHM_REQUIRE(dy && wt && x && w && mean && rstd && dx && partials && (!(flags & 1) || res1));
  auto al16 = [](const void* p) { return ((uintptr_t)p % 16) == 0; };
  LTHM_REQUIRE(al16(dy) && al16(wt) && al16(x) && al16(w) && al16(dx) && al16(partials) && (!res1 || al16(res1)) &&
               (!res2 || al16(res2)) && ((uintptr_t)dx_bf16 % 8) == 0);
  if (M == 0) return 0;
  GemmArgs g{};
  g.A = (const bf16_t*)dy; g.B = (const bf16_t*)wt; g.C = nullptr;
  g.M = M; g.N = 256; g.K = K;
  g.lda = K; g.ldb = K; g.ldc = 256;
  g.alpha = 1.f;
  g.act = LTHM_ACT_NONE;
  g.fast_ok = true;
  const int tm = lthm_dgrad_layernorm_bwd_tiles(M);
  LnbArgs L{x, w, mean, rstd, res1, res2, dx, (bf16_t*)dx_bf16, partials, partials + (int64_t)tm * 256, flags & 1};
  hipLaunchKernelGGL((gemm_pp_k<false, false, PP_LNB>), dim3(tm), dim3(512), 0, (hipStream_t)stream, g, tm, 1, L);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_linear_layernorm_fwd(const void* x, const void* w, const float* bias, const float* res1, int64_t M,
                                         int32_t D, int64_t K, const float* ln_w, const float* ln_b, float* x1,
                                         void* h, float* mean, float* rstd, void* stream) {
  LTHM_REQUIRE(D == 256 && M >= 0 && K > 0 && K % PP_BK == 0);
  LTHM_REQUIRE(x && w && ln_w && x1 && h && mean && rstd);
  auto al16 = [](const void* p) { return ((uintptr_t)p % 16) == 0; };
  LTHM_REQUIRE(al16(x) && al16(w) && al16(ln_w) && al16(x1) && ((uintptr_t)h % 8) == 0 && (!bias || al16(bias)) &&
               (!ln_b || al16(ln_b)) && (!res1 || al16(res1)));
  if (M == 0) return 0;
  GemmArgs g{};
  g.A = (const bf16_t*)x; g.B = (const bf16_t*)w; g.C = nullptr;
  g.M = M; g.N = 256; g.K = K;
  g.lda = K; g.ldb = K; g.ldc = 256;
  g.alpha = 1.f;
  g.act = LTHM_ACT_NONE;
  g.fast_ok = true;
  const int tm = (int)((M + 255) / 256);
  LnbArgs L{};
  L.w = ln_w; L.b = ln_b; L.bias = bias; L.res1 = res1;
  L.dx = x1; L.dxb = (bf16_t*)h; L.mean_out = mean; L.rstd_out = rstd;
  hipLaunchKernelGGL((gemm_pp_k<false, false, PP_LNF>), dim3(tm), dim3(512), 0, (hipStream_t)stream, g, tm, 1, L);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_gemm(const lthm_gemm_desc* d, void* stream) {
  LTHM_REQUIRE(d != nullptr);
  LTHM_REQUIRE(d->M >= 0 && d->N >= 0 && d->K >= 0 && d->batch >= 1);
  LTHM_REQUIRE(d->out_dtype == LTHM_F32 || d->out_dtype == LTHM_BF16);
  if (d->M == 0 || d->N == 0) return 0;
  const bool ka = d->a_kcontig != 0, kb = d->b_kcontig != 0;
  // any shape / stride: aligned full chunks take 16-B loads, ragged tails element loads
  LTHM_REQUIRE(((uintptr_t)d->A % 2) == 0 && ((uintptr_t)d->B % 2) == 0);
  LTHM_REQUIRE(d->lda >= (ka ? d->K : d->M) && d->ldb >= (kb ? d->K : d->N));
  LTHM_REQUIRE(d->act >= 0 && d->act <= LTHM_ACT_MUL_AUX);
  LTHM_REQUIRE(!(d->act == LTHM_ACT_GELU_GRAD || d->act == LTHM_ACT_QGELU_GRAD || d->act == LTHM_ACT_MUL_AUX) ||
               d->aux != nullptr);
  int splits = d->splits < 1 ? 1 : d->splits;
  LTHM_REQUIRE(splits == 1 || d->workspace != nullptr);
  GemmArgs g;
  g.A = (const bf16_t*)d->A; g.B = (const bf16_t*)d->B; g.C = d->C;
  g.M = d->M; g.N = d->N; g.K = d->K;
  g.lda = d->lda; g.ldb = d->ldb; g.ldc = d->ldc;
  g.sA = d->sA; g.sB = d->sB; g.sC = d->sC;
  int64_t kps = (d->K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  if (kps < BK) kps = BK;
  splits = (int)((d->K + kps - 1) / kps);
  if (splits < 1) splits = 1;
  g.k_per_split = (splits == 1) ? (d->K > 0 ? d->K : 1) : kps;
  g.alpha = d->alpha;
  g.bias = d->bias; g.act = d->act; g.aux = (const bf16_t*)d->aux; g.aux_out = (bf16_t*)d->aux_out;
  g.ldaux = d->ldaux > 0 ? d->ldaux : d->N;
  g.res1 = d->res1; g.res2 = d->res2; g.ldr1 = d->ldr1 > 0 ? d->ldr1 : d->N; g.ldr2 = d->ldr2 > 0 ? d->ldr2 : d->N;
  g.res1_dt = d->res1_dtype; g.res2_dt = d->res2_dtype; g.out_dt = d->out_dtype;
  g.ws = (splits > 1) ? d->workspace : nullptr;
  g.sa = nullptr;
  g.sb = nullptr;
  g.amax = reinterpret_cast<unsigned*>(d->amax_out);
  // the kernels other than gemm_ps_k leave amax_out to a pass over C afterwards
  LTHM_REQUIRE(!d->amax_out || (d->batch == 1 && d->ldc == d->N && (d->M * d->N) % 8 == 0 &&
                                ((uintptr_t)d->C % 16) == 0));
  auto amax_after = [&]() -> int {
    return d->amax_out ? lthm_amax(d->C, d->out_dtype, d->M * d->N, d->amax_out, stream) : 0;
  };
  g.fast_ok = ((uintptr_t)d->A % 16) == 0 && ((uintptr_t)d->B % 16) == 0 && d->lda % 8 == 0 && d->ldb % 8 == 0 &&
              d->sA % 8 == 0 && d->sB % 8 == 0;
  if (splits > 1) {
    LTHM_REQUIRE(d->workspace_bytes >= (size_t)splits * d->batch * d->M * d->N * 4);
  }
  const int tiles_m = (int)((d->M + BM - 1) / BM), tiles_n = (int)((d->N + BN - 1) / BN);
  hipStream_t s = (hipStream_t)stream;
  // weight gradients: 256 x 256 split-K tiles (splits bounded by the caller's workspace)
  // (any K: the packed rows of a shared pad prefix have no alignment; k rows past K read zeros)
  static const bool wg_ragged = !(getenv("LTHM_WG_RAGGED") && getenv("LTHM_WG_RAGGED")[0] == '0');  // A/B
  if (lthm_gemm_ps_mode() && !ka && !kb && d->batch == 1 && d->workspace && g.fast_ok && d->M % 8 == 0 &&
      d->N % 8 == 0 && d->act == LTHM_ACT_NONE && !d->bias && d->M * d->N > 0 && (wg_ragged || d->K % WG_BK == 0)) {
    const int tm = (int)((d->M + 255) / 256), tn = (int)((d->N + 255) / 256);
    const int64_t cap = (int64_t)(d->workspace_bytes / ((size_t)d->M * d->N * 4));
    int64_t sp = std::min<int64_t>(std::max(1, lthm_cu_count() / (tm * tn)), cap);
    sp = std::min<int64_t>(sp, d->K / (WG_BK * 8));  // >= 8 stages per split
    if (sp >= 2 && tm * tn <= lthm_cu_count()) {
      int64_t kpw = (d->K + sp - 1) / sp;
      kpw = (kpw + WG_BK - 1) / WG_BK * WG_BK;
      const int spl = (int)((d->K + kpw - 1) / kpw);
      GemmArgs gw = g;
      gw.ws = d->workspace;
      gw.res1 = nullptr; gw.res2 = nullptr;
      hipLaunchKernelGGL(gemm_wg_k, dim3(tm * tn * spl), dim3(512), 0, s, gw, tm, tn, spl, kpw);
      LTHM_CHECK_LAUNCH();
      GemmArgs gr = g;
      gr.ws = d->workspace;
      gr.alpha = 1.f;  // alpha already applied to the partials
      const int64_t total = d->M * d->N;
      if (d->N % 4 == 0 && ((uintptr_t)d->workspace % 16) == 0)
        hipLaunchKernelGGL(splitk_reduce4_k, dim3(grid_for(total / 4, 256, 256 * 8)), dim3(256), 0, s, gr, spl);
      else
        hipLaunchKernelGGL(splitk_reduce_k, dim3(grid_for(total, 256, 256 * 8)), dim3(256), 0, s, gr, spl, 1);
      LTHM_CHECK_LAUNCH();
      return amax_after();
    }
  }
  const int per_xcd = lthm_cu_count() / 8;
  int epi = -1;
  {
    const bool a16 = ((uintptr_t)d->C % 16) == 0 && d->ldc % 8 == 0 && ((uintptr_t)d->bias % 16) == 0;
    const bool r1 = d->res1 && d->res1_dtype == LTHM_F32 && ((uintptr_t)d->res1 % 16) == 0 && g.ldr1 % 8 == 0;
    const bool r2 = d->res2 && d->res2_dtype == LTHM_F32 && ((uintptr_t)d->res2 % 16) == 0 && g.ldr2 % 8 == 0;
    const bool ax = ((uintptr_t)d->aux % 16) == 0 && ((uintptr_t)d->aux_out % 16) == 0 && g.ldaux % 8 == 0;
    const int act = d->act;
    if (!a16 || !ax) epi = -1;
    else if (act == LTHM_ACT_NONE && !d->res1 && !d->res2) epi = EPI_PLAIN;
    else if ((act == LTHM_ACT_GELU || act == LTHM_ACT_QGELU || act == LTHM_ACT_GELU_D) && !d->res1 && !d->res2)
      epi = EPI_ACT;
    else if ((act == LTHM_ACT_GELU_GRAD || act == LTHM_ACT_QGELU_GRAD || act == LTHM_ACT_MUL_AUX) && !d->bias &&
             !d->res1 && !d->res2)
      epi = EPI_GRAD;
    else if (act == LTHM_ACT_NONE && r1 && !d->res2) epi = EPI_RES1;
    else if (act == LTHM_ACT_NONE && r1 && r2) epi = EPI_RES2;
  }
  if (d->ab_dtype == LTHM_FP8_E4M3) {
    // fp8 encoder GEMMs: persistent kernel only, geometry in 2-byte units
    LTHM_REQUIRE(epi >= 0 && ka && kb && splits == 1 && d->batch == 1 && d->K % 128 == 0 && d->K > 0);
    LTHM_REQUIRE(d->a_scale && d->b_scale && d->lda % 16 == 0 && d->ldb % 16 == 0 && d->N % 8 == 0);
    LTHM_REQUIRE(((uintptr_t)d->A % 16) == 0 && ((uintptr_t)d->B % 16) == 0 && tiles_n <= per_xcd);
    GemmArgs g8 = g;
    g8.K = d->K / 2; g8.lda = d->lda / 2; g8.ldb = d->ldb / 2;
    g8.sa = d->a_scale; g8.sb = d->b_scale;
    if (lthm_gemm_pp_mode() && lthm_gemm_pp_f8() && d->K >= 1024 && d->K % (2 * PP_BK) == 0 && d->M >= 256 &&
        d->N >= 256 && !d->amax_out) {
      // 256 x 256 tiles (the bf16 kernel's geometry in 2-byte units).  From K = 1,024 on (8 K-tiles):
      // C5 fc2 (K = 2,048) 0.767 -> 0.660 ms, 4096^3 0.091 -> 0.065 ms (2.1 PF); the K = 512 forms
      // ran 17-24 % slower here than on the persistent kernel (profiles/r04ab/)
      const int tm = (int)((d->M + 255) / 256), tn = (int)((d->N + 255) / 256);
      g8.ws = nullptr;
      g8.amax = nullptr;
      hipLaunchKernelGGL((gemm_pp_k<true, false>), dim3(tm * tn), dim3(512), 0, s, g8, tm, tn);
      LTHM_CHECK_LAUNCH();
      return 0;
    }
    if (lthm_gemm_bt_mode() && d->K > 256 && d->K % 128 == 0 && d->M >= 4096 && d->N >= 512 && !d->amax_out) {
      // 256 x 256 tiles (the persistent kernel's 128 x 128 tile re-reads the LDS per flop at K >= 512)
      const int tm = (int)((d->M + 255) / 256), tn = (int)((d->N + 255) / 256);
      g8.ws = nullptr;
      g8.amax = nullptr;
      hipLaunchKernelGGL(gemm_bt_k<true>, dim3(tm * tn), dim3(512), 0, s, g8, tm, tn);
      LTHM_CHECK_LAUNCH();
      return 0;
    }
    const int R = per_xcd / tiles_n;
    dim3 grid(8 * R * tiles_n);
    const bool bres = g8.K <= 4 * BK;
#define LTHM_PS8(BRES_, EPI_) \
  hipLaunchKernelGGL((gemm_ps_k<true, BRES_, EPI_, true>), grid, dim3(PS_THREADS), 0, s, g8, tiles_m, tiles_n, R)
#define LTHM_PS8_EPI(BRES_)                              \
  switch (epi) {                                         \
    case EPI_PLAIN: LTHM_PS8(BRES_, EPI_PLAIN); break;   \
    case EPI_ACT: LTHM_PS8(BRES_, EPI_ACT); break;       \
    case EPI_GRAD: LTHM_PS8(BRES_, EPI_GRAD); break;     \
    case EPI_RES1: LTHM_PS8(BRES_, EPI_RES1); break;     \
    default: LTHM_PS8(BRES_, EPI_RES2); break;           \
  }
    if (bres) { LTHM_PS8_EPI(true) }
    else { LTHM_PS8_EPI(false) }
#undef LTHM_PS8_EPI
#undef LTHM_PS8
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  if (lthm_gemm_pp_mode() && d->ab_dtype != LTHM_FP8_E4M3 && ka && kb && splits == 1 && d->batch == 1 &&
      g.fast_ok && d->K >= 512 && d->K % PP_BK == 0 && d->M >= 256 && d->N >= 256) {
    // (K = 256 forms stay on the persistent kernel: the C2 qkv / proj / fc forwards ran 5-26 %
    // slower here, profiles/r04z_gemm_*; from K = 512 on this kernel wins: C4 fc1 forward 0.456 ->
    // 0.349 ms, its dgrad 0.701 -> 0.376, C5 fc2 forward 1.456 -> 1.133, 4096^3 767 -> 1,179 TF)
    const int tm = (int)((d->M + 255) / 256), tn = (int)((d->N + 255) / 256);
    GemmArgs gp = g;
    gp.ws = nullptr;
    // per-phase DMA issue where there are several column tiles (C4: 4-6 % faster); a single
    // 256-column tile (C2's N = 256 dgrads) runs ~2 % faster with the DMA behind the barrier
    // (profiles/r04am_ab.log)
    if (lthm_gemm_pp_mode() == 2 || d->N <= 256)
      hipLaunchKernelGGL((gemm_pp_k<false, false>), dim3(tm * tn), dim3(512), 0, s, gp, tm, tn);
    else hipLaunchKernelGGL((gemm_pp_k<false, true>), dim3(tm * tn), dim3(512), 0, s, gp, tm, tn);
    LTHM_CHECK_LAUNCH();
    return amax_after();
  }
  if (lthm_gemm_bt_mode() && d->ab_dtype != LTHM_FP8_E4M3 && ka && kb && splits == 1 && d->batch == 1 &&
      g.fast_ok && d->K > 4 * BK &&
      d->K % BT_BK == 0 && d->M >= 4096 && d->N >= 512) {
    // (N = 256 stays on the persistent kernel: C2 dX / qkv-dgrad forms ran 0.45 ms here against
    // its ~0.4, HBM-bound either way)
    const int tm = (int)((d->M + 255) / 256), tn = (int)((d->N + 255) / 256);
    GemmArgs gb = g;
    gb.ws = nullptr;
    hipLaunchKernelGGL(gemm_bt_k<false>, dim3(tm * tn), dim3(512), 0, s, gb, tm, tn);
    LTHM_CHECK_LAUNCH();
    return amax_after();
  }
  if (lthm_gemm_ps_mode() && epi >= 0 && ka && splits == 1 && d->batch == 1 && g.fast_ok && d->K % BK == 0 &&
      d->K > 0 && d->N % 8 == 0 && tiles_n <= per_xcd && (int64_t)tiles_m * tiles_n >= 4 * 8 * per_xcd) {
    const int R = per_xcd / tiles_n;  // row-panel walkers per column tile and XCD
    dim3 grid(8 * R * tiles_n);
    const bool bres = d->K <= 4 * BK;
#define LTHM_PS(KB_, BRES_, EPI_) \
  hipLaunchKernelGGL((gemm_ps_k<KB_, BRES_, EPI_>), grid, dim3(PS_THREADS), 0, s, g, tiles_m, tiles_n, R)
#define LTHM_PS_EPI(KB_, BRES_)                        \
  switch (epi) {                                       \
    case EPI_PLAIN: LTHM_PS(KB_, BRES_, EPI_PLAIN); break; \
    case EPI_ACT: LTHM_PS(KB_, BRES_, EPI_ACT); break;     \
    case EPI_GRAD: LTHM_PS(KB_, BRES_, EPI_GRAD); break;   \
    case EPI_RES1: LTHM_PS(KB_, BRES_, EPI_RES1); break;   \
    default: LTHM_PS(KB_, BRES_, EPI_RES2); break;         \
  }
    if (bres && kb) { LTHM_PS_EPI(true, true) }
    else if (bres) { LTHM_PS_EPI(false, true) }
    else if (kb) { LTHM_PS_EPI(true, false) }
    else { LTHM_PS_EPI(false, false) }
#undef LTHM_PS_EPI
#undef LTHM_PS
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid(tiles_m * tiles_n, d->batch, splits);
  const size_t shmem = 4 * TILE_BYTES;
  if (ka && kb) hipLaunchKernelGGL((gemm_k<true, true>), grid, dim3(256), shmem, s, g, tiles_n);
  else if (ka && !kb) hipLaunchKernelGGL((gemm_k<true, false>), grid, dim3(256), shmem, s, g, tiles_n);
  else if (!ka && kb) hipLaunchKernelGGL((gemm_k<false, true>), grid, dim3(256), shmem, s, g, tiles_n);
  else hipLaunchKernelGGL((gemm_k<false, false>), grid, dim3(256), shmem, s, g, tiles_n);
  LTHM_CHECK_LAUNCH();
  if (splits > 1) {
    const int64_t total = d->M * d->N * d->batch;
    if (d->batch == 1 && d->N % 4 == 0 && ((uintptr_t)d->workspace % 16) == 0)
      hipLaunchKernelGGL(splitk_reduce4_k, dim3(grid_for(total / 4, 256, 256 * 8)), dim3(256), 0, s, g, splits);
    else
      hipLaunchKernelGGL(splitk_reduce_k, dim3(grid_for(total, 256, 256 * 8)), dim3(256), 0, s, g, splits, d->batch);
    LTHM_CHECK_LAUNCH();
  }
  return amax_after();
}
