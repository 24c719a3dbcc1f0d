// Fused encoder MLP for gfx950: _MLP (commons/transformers/layers.py:279-284)
//
//   out = res1 [+ res2] + c_proj( GELU( c_fc(x) ) )      x = ln_2 output, bf16
//
// with the [M, 4d] hidden never written to HBM.  The forward keeps it in
// registers; the backward recomputes it (two kernels, below).  All three kernels
// share one structure:
//
//  * v_mfma_f32_32x32x16_bf16 throughout; a wave owns 32 token rows (dX-style
//    kernels) or 32 hidden units (the weight-gradient kernel);
//  * the hidden dimension is walked in chunks of 32 units.  A chunk's first
//    product is computed TRANSPOSED (pre^T = W1_j . x^T: hidden on the
//    accumulator's registers, token rows on its lanes), so the accumulator,
//    packed to bf16, is directly the A operand of the second product, which sums
//    over the hidden index (cdna_hip_programming.md §3, accumulator as operand):
//    no LDS round trip, no transpose;
//  * the weights stream through LDS in [32 x d] chunk images (c_fc.weight rows
//    and c_proj.weight^T rows, both contiguous 32 x d blocks), double-buffered
//    by LDS-DMA (global_load_lds_dwordx4), one barrier per chunk.  The same
//    image serves row reads (ds_read_b128: the chunk as an A operand over d) and
//    transposed reads (ds_read_b64_tr_b16: the chunk as a B operand over the
//    permuted hidden index of the packed accumulator); the XOR swizzle
//    ch ^ ((r & 3) << 2 | (r >> 2) & 3) makes both conflict-free.
//
// Per token row and layer the forward moves x (2d B), res1 (4d B) and out (4d B)
// instead of the unfused chain's 4d-wide bf16 hidden + GELU' aux writes and their
// re-reads (2 x 2 x 4d B written, read twice more in the backward).
#include <algorithm>

#include "common.hpp"

namespace lthm {

struct MlpArgs {
  const bf16_t* X;    // [M, D] ln_2 output (bf16)
  const bf16_t* W1;   // [HID, D] c_fc.weight (bf16)
  const bf16_t* W2T;  // [HID, D] c_proj.weight^T (bf16)
  const float* b1;    // [HID] or null
  const float* b2;    // [D] or null
  const float* res1;  // [M, D] f32 or null
  const float* res2;  // [M, D] f32 or null
  float* out;         // [M, D] f32
  int64_t M;
  int HID;
  int ntiles;
  // ln_2 fused in the prologue (ln_w non-null): X is unused, the input rows are LN(x32)
  const float* x32;   // [M, D] f32 (the block's x1; usually also res1)
  const float* ln_w;  // [D]
  const float* ln_b;  // [D] or null
  bf16_t* h_out;      // [M, D] bf16: the LN output, saved for the backward (or null)
  float* mean;        // [M] (or null)
  float* rstd;        // [M] (or null)
};

struct MlpBwdArgs {
  const bf16_t* X;    // [M, D] ln_2 output (bf16)
  const bf16_t* dY;   // [M, D] gradient of the MLP output (bf16)
  const bf16_t* W1;   // [HID, D] c_fc.weight (bf16)
  const bf16_t* W2T;  // [HID, D] c_proj.weight^T (bf16)
  const float* b1;    // [HID] or null
  bf16_t* G;          // [M, HID] GELU(pre) (bf16)
  bf16_t* dP;         // [M, HID] d pre (bf16)
  float* dXf;         // [M, D] dX (f32), or
  bf16_t* dXb;        // [M, D] dX (bf16)
  int dx_f32;
  int64_t M;
  int HID;
};

// The weight-gradient kernel (mlp_wgrad_k): per (token slice, hidden group) partial slabs
struct MlpWgArgs {
  const bf16_t* X;    // [M, D] ln_2 output (bf16)
  const bf16_t* dY;   // [M, D] gradient of the MLP output (bf16)
  const bf16_t* W1;   // [HID, D] c_fc.weight (bf16)
  const bf16_t* W2T;  // [HID, D] c_proj.weight^T (bf16)
  const float* b1;    // [HID] or null
  float* dW1p;        // [nslice][HID][D] partial dW1 = dpre^T x
  float* dW2Tp;       // [nslice][HID][D] partial dW2^T = g^T dy
  float* db1p;        // [nslice][HID] partial colsum dpre (or null)
  int64_t M;
  int HID;
  int nslice;         // token slices
  int ngroup;         // hidden groups (HID / (32 NW))
};

typedef __bf16 bf16x8m __attribute__((ext_vector_type(8)));
typedef short s16x4m __attribute__((ext_vector_type(4)));
typedef short s16x8m __attribute__((ext_vector_type(8)));

// [rows][D] bf16 images as 8-row x 32-column subtiles of 512 B (cdna_hip_programming.md T10,
// layout (a)): byte offset of 16-B chunk c (8 columns) of row r.  Every offset is a per-lane
// base plus a multiple of 512 in the chunk's high bits, so an unrolled loop over k-steps or
// output tiles needs two base registers, not one per read.  Conflict-free for the 32x32x16
// row reads (ds_read_b128) and the transposed reads (ds_read_b64_tr_b16) alike.
template <int D>
__device__ __forceinline__ int mlp_off(int r, int c) {
  return (16 * D) * (r >> 3) + 512 * (c >> 2) + 64 * (r & 7) + 16 * ((c & 3) ^ ((r >> 2) & 3));
}

// LDS-DMA of a [32 x D] bf16 block (rows contiguous, row stride D) into a mlp_off image:
// the DMA writes 16-B slot base + lane of each wave-instruction, so the layout is applied
// to the source address (slot -> row, chunk by inverting mlp_off).
template <int D, int NTH>
__device__ __forceinline__ void mlp_dma32(unsigned char* img, const bf16_t* P, int tid) {
  constexpr int SLOTS = 32 * D / 8;
  static_assert(SLOTS % NTH == 0, "image slots must divide over the workgroup");
  const int wbase = tid & ~63;
#pragma unroll
  for (int m = 0; m < SLOTS / NTH; ++m) {
    const int o = (m * NTH + tid) * 16;
    const int r1 = o % (16 * D);
    const int r = 8 * (o / (16 * D)) + (r1 % 512) / 64;
    const int c = 4 * (r1 / 512) + (((r1 % 64) / 16) ^ ((r >> 2) & 3));
    glds16(P + (int64_t)r * D + c * 8, img + (m * NTH + wbase) * 16);
  }
}

// mlp_dma32 of the rows row0 .. row0 + 31 of a [M, D] tensor, rows past nvalid read as row
// row0 + nvalid - 1 (in bounds; the kernel zeroes their contributions)
template <int D, int NTH>
__device__ __forceinline__ void mlp_dma32c(unsigned char* img, const bf16_t* P, int64_t row0, int nvalid, int tid) {
  constexpr int SLOTS = 32 * D / 8;
  static_assert(SLOTS % NTH == 0, "image slots must divide over the workgroup");
  const int wbase = tid & ~63;
#pragma unroll
  for (int m = 0; m < SLOTS / NTH; ++m) {
    const int o = (m * NTH + tid) * 16;
    const int r1 = o % (16 * D);
    const int r = 8 * (o / (16 * D)) + (r1 % 512) / 64;
    const int c = 4 * (r1 / 512) + (((r1 % 64) / 16) ^ ((r >> 2) & 3));
    glds16(P + (row0 + min(r, nvalid - 1)) * D + c * 8, img + (m * NTH + wbase) * 16);
  }
}

// mlp_dma32 with the per-thread source offsets precomputed (MlpDmaPlan) and the destination given
// as an LDS byte address: per piece one 64-bit add and the DMA
template <int D, int NTH>
struct MlpDmaPlan {
  static constexpr int PIECES = 32 * D / 8 / NTH;
  int off[PIECES];  // element offset of piece m's 16 source bytes within a [32 x D] block
  __device__ __forceinline__ void init(int tid) {
#pragma unroll
    for (int m = 0; m < PIECES; ++m) {
      const int o = (m * NTH + tid) * 16;
      const int r1 = o % (16 * D);
      const int r = 8 * (o / (16 * D)) + (r1 % 512) / 64;
      const int c = 4 * (r1 / 512) + (((r1 % 64) / 16) ^ ((r >> 2) & 3));
      off[m] = r * D + c * 8;
    }
  }
  // block P (32 rows of D, row stride D) into the image at LDS byte address lds (wave-uniform base
  // of the image + the wave's 1-KiB slice: lds_img + (tid & ~63) * 16)
  __device__ __forceinline__ void issue(const bf16_t* P, uint32_t lds_wave) const {
#pragma unroll
    for (int m = 0; m < PIECES; ++m) glds16_m0(P + off[m], lds_wave + m * NTH * 16);
  }
};

// A operand of 32x32x16 from a [32][D] image: lane (r = l & 31, h = l >> 5) row r, k 16 ks + 8 h ..
template <int D>
__device__ __forceinline__ bf16x8m mlp_row_frag(const unsigned char* img, int lane, int ks) {
  return *reinterpret_cast<const bf16x8m*>(img + mlp_off<D>(lane & 31, 2 * ks + (lane >> 5)));
}

// B operand of 32x32x16 over the PERMUTED k order of a packed accumulator (k-step s2 of a
// 32-row block of the image, output columns 32 t ..): element e of lane half h is image row
// 16 s2 + 8 (e >> 2) + 4 h + (e & 3), column 32 t + (lane & 31) -- two transposed reads.
template <int D>
__device__ __forceinline__ bf16x8m mlp_tr_frag(const unsigned char* img, int lane, int s2, int t) {
  const int h = lane >> 5, q = (lane >> 2) & 3, p = lane & 3, g1 = (lane >> 4) & 1;
  const int c = 4 * t + 2 * g1 + (p >> 1);
  const int r0 = 16 * s2 + 4 * h + q;
  typedef __attribute__((address_space(3))) s16x4m lds_s16x4;
  const s16x4m lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mlp_off<D>(r0, c) + 8 * (p & 1)));
  const s16x4m hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mlp_off<D>(r0 + 8, c) + 8 * (p & 1)));
  const s16x8m v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8m, v);
}

// registers 8 s .. 8 s + 7 of a 32x32 accumulator, packed to bf16: the k-step s fragment
__device__ __forceinline__ bf16x8m mlp_pack(const float* v) {
  u32x4 w;
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = pack_bf16x2(v[2 * i], v[2 * i + 1]);
  return __builtin_bit_cast(bf16x8m, w);
}

__device__ __forceinline__ f32x16 mfma32(bf16x8m a, bf16x8m b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- forward
// Workgroup = NW waves, persistent over a contiguous range of token rows, in tiles of 32 NW
// rows (a wave owns 32).  The hidden chunks of consecutive tiles form ONE stream c = 0, 1, ...
// (chunk c % NC of the WG's tile c / NC); step c of the software pipeline is
//   S'  = W1_{c+1} . x^T            phase 1 of the NEXT chunk (A: W1 image rows; B: x in registers)
//   Hp  = bf16(GELU(S + b1_c))      issued between those MFMAs (independent VALU)
//   Y  += Hp . W2T_c                phase 2 of this chunk (B: W2T image, transposed reads)
// W1 and W2T images ride separate 2-slot rings: step c consumes W2T_c and W1_{c+1} and its
// LDS-DMAs fetch W2T_{c+1} and W1_{c+2} into the slots step c - 1 released; one barrier per
// step.  The residual (+ b2) is loaded INTO the accumulator when a tile starts, so the
// epilogue only stores (LDS-restaged 16-B rows, no load after a store on the in-order vmcnt);
// the next tile's x rows are loaded one step before the tile's last phase 1 needs them.
// out[row, :] = acc + b2 + res1 [+ res2] for the wave's rows rb .. min(rb + 32, lim): each
// 32-column tile t of the accumulator goes through the wave's 4-KiB LDS strip (C layout in,
// 128-B rows out), then every lane finishes four 16-B pieces with vector loads / stores; the
// residual pieces of tile t are loaded before the tile is restaged.
template <int D, int NT, int NRES>
__device__ __forceinline__ void mlp_fwd_epi(const MlpArgs& a, const f32x16 (&acc)[NT], const float* b2s,
                                            float* stg, int64_t rb, int64_t lim, int lane) {
  const int r32 = lane & 31, h = lane >> 5;
  const int pr = lane >> 3, pc = 4 * (lane & 7);  // piece m: row pr + 8 m, columns pc .. pc + 3
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    f32x4 rv[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {  // in flight while the tile is restaged
      const int64_t o = min(rb + pr + 8 * m, lim - 1) * D + 32 * t + pc;
      rv[m] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (NRES >= 1) rv[m] = *reinterpret_cast<const f32x4*>(a.res1 + o);
      if constexpr (NRES >= 2) rv[m] += *reinterpret_cast<const f32x4*>(a.res2 + o);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) stg[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r32] = acc[t][i];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const f32x4 bias = *reinterpret_cast<const f32x4*>(b2s + 32 * t + pc);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t row = rb + pr + 8 * m;
      f32x4 v = *reinterpret_cast<const f32x4*>(stg + (pr + 8 * m) * 32 + pc);
      v += bias + rv[m];
      if (row < lim) *reinterpret_cast<f32x4*>(a.out + row * D + 32 * t + pc) = v;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

template <int D, int KS>
__device__ __forceinline__ void mlp_load_x(const bf16_t* X, int64_t row, bool ok, int h, bf16x8m (&xf)[KS]) {
  const bf16_t* p = X + (ok ? row : 0) * D + 8 * h;
#pragma unroll
  for (int s = 0; s < KS; ++s)
    xf[s] = __builtin_bit_cast(bf16x8m, ok ? *reinterpret_cast<const u32x4*>(p + 16 * s) : u32x4{0u, 0u, 0u, 0u});
}

// ln_2 in the prologue: lane (row r, half h) holds columns 16 s + 8 h .. + 7 of its row (the B
// operand layout); the row's statistics combine the two halves through one lane exchange.
// Same two-pass arithmetic as ln_fwd_v4_k (mean, then the mean squared deviation, eps 1e-5).
template <int D, int KS>
__device__ __forceinline__ void mlp_ld8f(const float* p, bool ok, float (&v)[8]) {
  const f32x4 lo = ok ? *reinterpret_cast<const f32x4*>(p) : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 hi = ok ? *reinterpret_cast<const f32x4*>(p + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
  v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
}
// ln_2 in the prologue: lane (row r, half h) holds columns 16 s + 8 h .. + 7 of its row (the B
// operand layout); the row's statistics combine the two halves through one lane exchange.
// Same two-pass arithmetic as ln_fwd_v4_k (mean, then the mean squared deviation, eps 1e-5);
// the lane's half-row is streamed three times (sum, deviations, normalise: L1 / L2 hits after
// the first) instead of held in 128 registers.
template <int D, int KS>
__device__ __forceinline__ void mlp_load_ln(const MlpArgs& a, const float* lw, const float* lb, int64_t row, bool ok,
                                            int h, bf16x8m (&xf)[KS]) {
  const float* p = a.x32 + (ok ? row : 0) * D + 8 * h;
  float s = 0.f;
#pragma unroll 4
  for (int k = 0; k < KS; ++k) {
    float v[8];
    mlp_ld8f<D, KS>(p + 16 * k, ok, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[e];
  }
  s += __shfl_xor(s, 32, 64);
  const float mu = s / (float)D;
  float q = 0.f;
#pragma unroll 4
  for (int k = 0; k < KS; ++k) {
    float v[8];
    mlp_ld8f<D, KS>(p + 16 * k, ok, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float dd = v[e] - mu;
      q += dd * dd;
    }
  }
  q += __shfl_xor(q, 32, 64);
  const float rs = 1.f / sqrtf(q / (float)D + 1e-5f);
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    float v[8], y[8];
    mlp_ld8f<D, KS>(p + 16 * k, ok, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = 16 * k + 8 * h + e;
      y[e] = (v[e] - mu) * rs * lw[c] + (lb ? lb[c] : 0.f);
    }
    u32x4 w4;
#pragma unroll
    for (int i = 0; i < 4; ++i) w4[i] = pack_bf16x2(y[2 * i], y[2 * i + 1]);
    xf[k] = __builtin_bit_cast(bf16x8m, w4);
    if (ok && a.h_out) *reinterpret_cast<u32x4*>(a.h_out + row * D + 16 * k + 8 * h) = w4;
  }
  if (ok && h == 0) {
    if (a.mean) a.mean[row] = mu;
    if (a.rstd) a.rstd[row] = rs;
  }
}

// Weight chunks ride a 3-slot LDS-DMA ring.  STAG (two waves per SIMD): waves NW/2 .. NW - 1
// share their SIMDs with waves 0 .. NW/2 - 1 and would run in lockstep with them (one barrier per
// chunk), so both would issue the S chain, then both the GELU, then both the output products.
// The upper half instead lags half a chunk: at step j it finishes chunk j - 1 (GELU, then
// Y += H W2T_{j-1}) and then forms S of chunk j, carried across the barrier; its VALU runs
// beside the partner's S MFMAs and its output MFMAs beside the partner's GELU
// (MI355X_MICROARCH.md, two waves per SIMD, item 9).  The ring then prefetches one chunk ahead
// (chunk j - 1 stays readable during step j); without STAG it prefetches two.
// cost-ladder builds of mlp_fwd_k (tools/build_variant.sh ... -DLTHM_MLPF_X=n; timing only, wrong
// results): 1 no DMA waits, 2 no GELU (the bias add only), 3 no per-chunk barrier, 4 no S MFMAs
#ifndef LTHM_MLPF_X
#define LTHM_MLPF_X 0
#endif
// LTHM_MLPF_STAMP=1 (diagnostic build, tools/build_variant.sh): mlp_fwd_k sums per wave the
// s_memtime cycles of each phase of the chunk loop (wait + barrier, DMA issue + S issue, S
// completion, GELU + Y issue) and of the tile epilogues into g_mlpf_stamps, read back with
// lthm_debug_mlpf_stamps.  Timing only (the stamps' lgkmcnt waits perturb the LDS prefetch).
#ifndef LTHM_MLPF_STAMP
#define LTHM_MLPF_STAMP 0
#endif
// LTHM_MLPF_TRPF=2: W2T fragments read before the GELU and two output tiles ahead (A/B build)
#ifndef LTHM_MLPF_TRPF
#define LTHM_MLPF_TRPF 0
#endif
#if LTHM_MLPF_STAMP
__device__ unsigned long long g_mlpf_stamps[2048 * 8 * 8];
#define MLPF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#else
#define MLPF_T(v)
#endif
template <int D, int NW, bool STAG>
__global__ __launch_bounds__(64 * NW, 1) void mlp_fwd_k(MlpArgs a) {
  constexpr int NS = 3, DIST = STAG ? 1 : 2;
  constexpr int NTH = 64 * NW, IMG = 32 * D * 2, KS = D / 16, NT = D / 32, TR = 32 * NW;
  constexpr int DPC = 2 * (32 * D / 8) / NTH;  // DMAs per thread and chunk (both images)
  __shared__ __attribute__((aligned(16))) unsigned char img[NS][2][IMG];  // [slot][W1_j, W2T_j]
  __shared__ __attribute__((aligned(16))) float stg_all[NW][32 * 32];    // per-wave epilogue strips
  extern __shared__ float b1s[];                                         // [HID] b1, [D] b2, [D] ln w, [D] ln b
  float* b2s = b1s + a.HID;
  float* lws = b2s + D;
  float* lbs = lws + D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const bool lag = STAG && wave >= NW / 2;  // wave-uniform
  const int NC = a.HID / 32;
  const int64_t rs = a.M * blockIdx.x / gridDim.x, re = a.M * (blockIdx.x + 1) / gridDim.x;
  if (rs >= re) return;  // uniform
  for (int i = tid; i < a.HID; i += NTH) b1s[i] = a.b1 ? a.b1[i] : 0.f;
  for (int i = tid; i < D; i += NTH) b2s[i] = a.b2 ? a.b2[i] : 0.f;
  if (a.ln_w)
    for (int i = tid; i < D; i += NTH) {
      lws[i] = a.ln_w[i];
      lbs[i] = a.ln_b ? a.ln_b[i] : 0.f;
    }
  float* stg = stg_all[wave];
  retire_loads();
#if LTHM_MLPF_STAMP
  MLPF_T(tk0);
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  const int64_t ntile_wg = (re - rs + TR - 1) / TR;
  // chunks 0 .. DIST - 1 of the stream (chunk c: index c % NC of tile c / NC)
#pragma unroll
  for (int c = 0; c < DIST; ++c)
    if (c / NC < ntile_wg) {
      mlp_dma32<D, NTH>(img[c][0], a.W1 + (int64_t)(c % NC) * 32 * D, tid);
      mlp_dma32<D, NTH>(img[c][1], a.W2T + (int64_t)(c % NC) * 32 * D, tid);
    }
  __syncthreads();  // b1s / b2s / ln
  // S^T = W1_j . x^T (hidden units of chunk j on the registers, the token on the lane)
  auto s_phase = [&](const unsigned char* w1, const bf16x8m(&xf)[KS]) {
    // LDS reads one step ahead of their MFMA; the compiler fences keep the unrolled loops
    // from hoisting every read (register pressure: 2 waves per SIMD)
    f32x16 S = f32x16{};
    if (LTHM_MLPF_X == 4) {
      S[0] = (float)mlp_row_frag<D>(w1, lane, 0)[0];
      return S;
    }
    bf16x8m fa = mlp_row_frag<D>(w1, lane, 0);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const bf16x8m fn = mlp_row_frag<D>(w1, lane, k + 1 < KS ? k + 1 : k);
      S = mfma32(fa, xf[k], S);
      fa = fn;
      asm volatile("" ::: "memory");
    }
    return S;
  };
  // H = bf16(GELU(S + b1_j)), Y += H . W2T_j
  auto gelu_out = [&](const f32x16& S, int j, const unsigned char* w2, f32x16(&acc)[NT]) {
    if (LTHM_MLPF_TRPF >= 2) {
      // the first two output tiles' W2T fragments are read BEFORE the GELU (they land while its
      // VALU runs), then two tiles ahead of their MFMAs: the phase-stamp build measured the
      // GELU + Y block at 53 % of a chunk step with the reads one tile ahead (tools/mlp_stamp.py)
      bf16x8m b0 = mlp_tr_frag<D>(w2, lane, 0, 0), b1 = mlp_tr_frag<D>(w2, lane, 1, 0);
      bf16x8m c0 = mlp_tr_frag<D>(w2, lane, 0, 1), c1 = mlp_tr_frag<D>(w2, lane, 1, 1);
      u32x4 hw0, hw1;  // H packed as it is formed (no 16-float staging)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b1s + 32 * j + 8 * m + 4 * h);
        float hv4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) hv4[e] = LTHM_MLPF_X == 2 ? S[4 * m + e] + bb[e] : gelu_tanh(S[4 * m + e] + bb[e]);
        const uint32_t p0 = pack_bf16x2(hv4[0], hv4[1]), p1 = pack_bf16x2(hv4[2], hv4[3]);
        if (m < 2) { hw0[2 * m] = p0; hw0[2 * m + 1] = p1; }
        else { hw1[2 * (m - 2)] = p0; hw1[2 * (m - 2) + 1] = p1; }
      }
      const bf16x8m hf0 = __builtin_bit_cast(bf16x8m, hw0), hf1 = __builtin_bit_cast(bf16x8m, hw1);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int tn = t + 2 < NT ? t + 2 : NT - 1;
        const bf16x8m n0 = mlp_tr_frag<D>(w2, lane, 0, tn), n1 = mlp_tr_frag<D>(w2, lane, 1, tn);
        acc[t] = mfma32(hf0, b0, acc[t]);
        acc[t] = mfma32(hf1, b1, acc[t]);
        b0 = c0;
        b1 = c1;
        c0 = n0;
        c1 = n1;
        asm volatile("" ::: "memory");
      }
      return;
    }
    float hv[16];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b1s + 32 * j + 8 * m + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) hv[4 * m + e] = LTHM_MLPF_X == 2 ? S[4 * m + e] + bb[e] : gelu_tanh(S[4 * m + e] + bb[e]);
    }
    const bf16x8m hf0 = mlp_pack(hv), hf1 = mlp_pack(hv + 8);
    bf16x8m b0 = mlp_tr_frag<D>(w2, lane, 0, 0), b1 = mlp_tr_frag<D>(w2, lane, 1, 0);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int tn = t + 1 < NT ? t + 1 : t;
      const bf16x8m n0 = mlp_tr_frag<D>(w2, lane, 0, tn), n1 = mlp_tr_frag<D>(w2, lane, 1, tn);
      acc[t] = mfma32(hf0, b0, acc[t]);
      acc[t] = mfma32(hf1, b1, acc[t]);
      b0 = n0;
      b1 = n1;
      asm volatile("" ::: "memory");
    }
  };
  int g = 0;
  int64_t tix = 0;
  for (int64_t t0 = rs; t0 < re; t0 += TR, ++tix) {
    const int64_t lim = min(t0 + TR, re), rb = t0 + 32 * wave;
    const bool active = rb < lim;  // wave-uniform: a wave past the tile's rows only streams weights
    bf16x8m xf[KS];
    if (a.ln_w) mlp_load_ln<D, KS>(a, lws, a.ln_b ? lbs : nullptr, rb + r32, rb + r32 < lim, h, xf);
    else mlp_load_x<D, KS>(a.X, rb + r32, rb + r32 < lim, h, xf);
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
    f32x16 S = f32x16{};  // lagging waves: chunk j - 1's S across the barrier
    for (int j = 0; j < NC; ++j, ++g) {
      MLPF_T(ts0);
      // retire chunk g; at prefetch distance 2 chunk g + 1 stays in flight (a tile's first step
      // drains: the x / residual / output accesses were issued behind the DMAs)
      if (LTHM_MLPF_X != 1) {
        if (DIST == 1 || j == 0) wait_vm<0>();
        else wait_vm<DPC>();
      }
      if (LTHM_MLPF_X != 3) __syncthreads();  // chunk g landed everywhere; every wave is done with chunk g + DIST - NS
      asm volatile("" ::: "memory");
      {
        // chunk g + DIST: of this tile, or the next tile's (same weights, chunk index wraps)
        const int64_t cg = (int64_t)j + DIST;
        if (tix + cg / NC < ntile_wg) {
          const int jn = (int)(cg % NC);
          unsigned char* dst = img[(g + DIST) % NS][0];
          mlp_dma32<D, NTH>(dst, a.W1 + (int64_t)jn * 32 * D, tid);
          mlp_dma32<D, NTH>(dst + IMG, a.W2T + (int64_t)jn * 32 * D, tid);
        }
      }
      if (!active) continue;
      if (lag) {
        if (j > 0) gelu_out(S, j - 1, img[(g + NS - 1) % NS][1], acc);
        S = s_phase(img[g % NS][0], xf);
      } else {
#if LTHM_MLPF_STAMP
        MLPF_T(ts1);
        const f32x16 Sj = s_phase(img[g % NS][0], xf);
        MLPF_T(ts2);
        {
          float dep = Sj[15] + Sj[0];  // in-order issue: the stamp below waits for the S chain
          asm volatile("" : "+v"(dep));
          asm volatile("" ::"v"(dep));
        }
        MLPF_T(ts3);
        gelu_out(Sj, j, img[g % NS][1], acc);
        MLPF_T(ts4);
        if (tix > 0) {
          st_acc[0] += ts1 - ts0;  // wait + barrier + DMA issue
          st_acc[1] += ts2 - ts1;  // S issue (LDS row reads)
          st_acc[2] += ts3 - ts2;  // S completion
          st_acc[3] += ts4 - ts3;  // GELU + Y issue
          st_acc[4] += 1;
        }
#else
        const f32x16 Sj = s_phase(img[g % NS][0], xf);
        gelu_out(Sj, j, img[g % NS][1], acc);
#endif
        S = f32x16{};  // nothing carried: keeps the loop-carried S out of this path's live range
      }
    }
#if LTHM_MLPF_STAMP
    MLPF_T(te0);
#endif
    if (active) {
      if (lag) gelu_out(S, NC - 1, img[(g + NS - 1) % NS][1], acc);  // chunk g - 1: slot kept until step g + 1
      if (a.res1 && a.res2) mlp_fwd_epi<D, NT, 2>(a, acc, b2s, stg, rb, lim, lane);
      else if (a.res1) mlp_fwd_epi<D, NT, 1>(a, acc, b2s, stg, rb, lim, lane);
      else mlp_fwd_epi<D, NT, 0>(a, acc, b2s, stg, rb, lim, lane);
    }
#if LTHM_MLPF_STAMP
    MLPF_T(te1);
    if (tix > 0) {
      st_acc[5] += te1 - te0;  // tile epilogue issue
      st_acc[6] += 1;
    }
#endif
  }
#if LTHM_MLPF_STAMP
  MLPF_T(tk);
  st_acc[7] = tk - tk0;
  if (lane == 0 && blockIdx.x < 2048)
    for (int k = 0; k < 8; ++k) g_mlpf_stamps[(blockIdx.x * 8 + wave) * 8 + k] = st_acc[k];
#endif
}

// ---------------------------------------------------------------- forward, two workgroups per CU
// mlp_fwd_k's chunk loop at 4 waves (128-row tiles) with everything that kept a second workgroup
// off the CU removed, so that two independent workgroups share each CU and one's tile edges (the
// x / residual loads, the output stores, the first chunk's drain) run beside the other's MFMAs:
//  * the accumulator starts as b2 + res1 (+ res2), loaded straight into the C layout when the tile
//    starts (register i of tile t: row 4 h + (i & 3) + 8 (i >> 2), column 32 t + r32; each
//    half-wave reads one 128-B row piece), and leaves from the C layout the same way, so the tile
//    end is stores only, no LDS strip and no load after a store;
//  * W1 / W2T chunks on a 2-slot ring (prefetch distance 1): 64 KiB of images + 5 KiB of biases.
// Two workgroups of 4 waves are 2 waves per SIMD (256 registers each, as the 8-wave form).
#ifndef LTHM_MLPF2_PF
#define LTHM_MLPF2_PF 1
#endif
template <int D, int NRES>
__global__ __launch_bounds__(256, 2) void mlp_fwd2_k(MlpArgs a) {
  constexpr int NW = 4, NTH = 64 * NW, IMG = 32 * D * 2, KS = D / 16, NT = D / 32, TR = 32 * NW;
  __shared__ __attribute__((aligned(16))) unsigned char img[2][2][IMG];  // [slot][W1_j, W2T_j]
  extern __shared__ float b1s[];                                         // [HID] b1, [D] b2
  float* b2s = b1s + a.HID;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int NC = a.HID / 32;
  const int64_t rs = a.M * blockIdx.x / gridDim.x, re = a.M * (blockIdx.x + 1) / gridDim.x;
  if (rs >= re) return;  // uniform
  for (int i = tid; i < a.HID; i += NTH) b1s[i] = a.b1 ? a.b1[i] : 0.f;
  for (int i = tid; i < D; i += NTH) b2s[i] = a.b2 ? a.b2[i] : 0.f;
  retire_loads();
  const int64_t ntile_wg = (re - rs + TR - 1) / TR;
  mlp_dma32<D, NTH>(img[0][0], a.W1, tid);
  mlp_dma32<D, NTH>(img[0][1], a.W2T, tid);
  __syncthreads();  // b1s / b2s
  int g = 0;
  int64_t tix = 0;
  for (int64_t t0 = rs; t0 < re; t0 += TR, ++tix) {
    const int64_t lim = min(t0 + TR, re), rb = t0 + 32 * wave;
    const bool active = rb < lim;  // wave-uniform: a wave past the tile's rows only streams weights
    bf16x8m xf[KS];
    mlp_load_x<D, KS>(a.X, rb + r32, rb + r32 < lim, h, xf);
    f32x16 acc[NT];
    // register i of tile t holds wave row (i & 3) + 8 (i >> 2) + 4 h; rows past `last` (the wave's
    // last row in range) read row `last` and are never stored
    const int last = active ? (int)min((int64_t)32, lim - rb) - 1 : 0;
    if (active) {  // acc = b2 + res1 (res2 joins in the epilogue, where the registers are free)
      const float* r1 = a.res1 + rb * D;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float bb = b2s[32 * t + r32];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int o = min((i & 3) + 8 * (i >> 2) + 4 * h, last) * D + 32 * t + r32;
          float v = bb;
          if constexpr (NRES >= 1) v += r1[o];
          acc[t][i] = v;
        }
      }
    }
    for (int j = 0; j < NC; ++j, ++g) {
      wait_vm<0>();     // chunk g landed (a tile's first step also drains its x / residual loads)
      __syncthreads();  // ... everywhere; every wave is done with chunk g - 1's slot
      asm volatile("" ::: "memory");
      if (j + 1 < NC || tix + 1 < ntile_wg) {
        const int jn = j + 1 < NC ? j + 1 : 0;
        mlp_dma32<D, NTH>(img[(g + 1) & 1][0], a.W1 + (int64_t)jn * 32 * D, tid);
        mlp_dma32<D, NTH>(img[(g + 1) & 1][1], a.W2T + (int64_t)jn * 32 * D, tid);
      }
      if (!active) continue;
      const unsigned char* w1 = img[g & 1][0];
      const unsigned char* w2 = img[g & 1][1];
      // S^T = W1_j . x^T (LDS row reads LTHM_MLPF2_PF steps ahead of their MFMA)
      f32x16 S = f32x16{};
      if (LTHM_MLPF2_PF >= 2) {
        bf16x8m fa = mlp_row_frag<D>(w1, lane, 0), fb = mlp_row_frag<D>(w1, lane, 1);
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          const bf16x8m fn = mlp_row_frag<D>(w1, lane, k + 2 < KS ? k + 2 : KS - 1);
          S = mfma32(fa, xf[k], S);
          fa = fb;
          fb = fn;
          asm volatile("" ::: "memory");
        }
      } else {
        bf16x8m fa = mlp_row_frag<D>(w1, lane, 0);
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          const bf16x8m fn = mlp_row_frag<D>(w1, lane, k + 1 < KS ? k + 1 : k);
          S = mfma32(fa, xf[k], S);
          fa = fn;
          asm volatile("" ::: "memory");
        }
      }
      // H = bf16(GELU(S + b1_j)), Y += H . W2T_j
      float hv[16];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b1s + 32 * j + 8 * m + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) hv[4 * m + e] = gelu_tanh(S[4 * m + e] + bb[e]);
      }
      const bf16x8m hf0 = mlp_pack(hv), hf1 = mlp_pack(hv + 8);
      bf16x8m b0 = mlp_tr_frag<D>(w2, lane, 0, 0), b1 = mlp_tr_frag<D>(w2, lane, 1, 0);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int tn = t + 1 < NT ? t + 1 : t;
        const bf16x8m n0 = mlp_tr_frag<D>(w2, lane, 0, tn), n1 = mlp_tr_frag<D>(w2, lane, 1, tn);
        acc[t] = mfma32(hf0, b0, acc[t]);
        acc[t] = mfma32(hf1, b1, acc[t]);
        b0 = n0;
        b1 = n1;
        asm volatile("" ::: "memory");
      }
    }
    if (active) {
      float* o = a.out + rb * D;
      if constexpr (NRES >= 2) {  // + res2, two column tiles' loads in flight at a time
        const float* r2 = a.res2 + rb * D;
#pragma unroll
        for (int t = 0; t < NT; t += 2) {
          float rv[2][16];
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int i = 0; i < 16; ++i)
              rv[u][i] = r2[min((i & 3) + 8 * (i >> 2) + 4 * h, last) * D + 32 * (t + u) + r32];
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[t + u][i] += rv[u][i];
          asm volatile("" ::: "memory");
        }
      }
      if (last == 31) {  // wave-uniform: a full 32-row wave tile
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[((i & 3) + 8 * (i >> 2) + 4 * h) * D + 32 * t + r32] = acc[t][i];
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int rr = (i & 3) + 8 * (i >> 2) + 4 * h;
            if (rr <= last) o[rr * D + 32 * t + r32] = acc[t][i];
          }
      }
    }
  }
}

// ---------------------------------------------------------------- forward, software-pipelined
// One wave per SIMD (4 waves, 512 registers each), the chunk stream software-pipelined inside
// the wave so that the MFMAs and the GELU VALU of different chunks issue side by side: phase k
// of a tile runs
//   S_k   = W1_k . x^T                        (16 MFMAs, one accumulation chain)
//   H_k-1 = bf16(GELU(S_k-1 + b1))            (VALU, between those MFMAs)
//   Y    += H_k-2 . W2T_k-2                   (16 MFMAs on the 8 output tiles)
// for k = 0 .. NC + 1 (the terms whose chunk exists).  Per steady phase 32 MFMAs (1,024 cycles
// of the matrix pipe) carry ~620 cycles of GELU in their issue gaps.  W1 and W2T chunks ride
// separate 2-slot LDS-DMA rings, one barrier per phase.  The accumulator starts as the residual
// (+ b2), loaded straight into the C layout (each half-wave reads a 128-B row piece), and is
// stored from the C layout the same way: no LDS restaging.
// one phase of mlp_fwd_pipe_k: DS: S_k = W1_k . x^T into Sp (after its GELU is taken); DG: H =
// GELU(Sp + b1) into ho (after its products are issued); DO: Y += ho . W2T.  Step i pairs S
// MFMA i with output MFMA i (tile i / 2, k-step i % 2) and GELU element i; the LDS fragments
// are read one step ahead (compiler fences keep the unrolled steps from hoisting every read).
// LTHM_MLPP_PF: LDS fragment reads this many steps ahead of their MFMA (1 or 2; one wave per
// SIMD, so an LDS read the MFMA waits on idles the matrix pipe)
#ifndef LTHM_MLPP_PF
#define LTHM_MLPP_PF 2
#endif
template <int D, bool DS, bool DG, bool DO>
__device__ __forceinline__ void mlp_pipe_phase(const unsigned char* w1, const unsigned char* w2, const float* bj,
                                               const bf16x8m (&xf)[D / 16], f32x16 (&acc)[D / 32], f32x16& Sp,
                                               bf16x8m& ho0, bf16x8m& ho1, int lane) {
  constexpr int KS = D / 16;
  static_assert(16 % KS == 0, "GELU elements per step");
  f32x16 Sn = f32x16{};
  float hv[16];
  bf16x8m fa[LTHM_MLPP_PF], fb[LTHM_MLPP_PF];
#pragma unroll
  for (int q = 0; q < LTHM_MLPP_PF; ++q) {
    fa[q] = fb[q] = bf16x8m{};
    if (DS) fa[q] = mlp_row_frag<D>(w1, lane, q < KS ? q : KS - 1);
    if (DO) fb[q] = mlp_tr_frag<D>(w2, lane, (q < KS ? q : KS - 1) & 1, (q < KS ? q : KS - 1) >> 1);
  }
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    const int in = i + LTHM_MLPP_PF < KS ? i + LTHM_MLPP_PF : KS - 1;
    bf16x8m na = fa[0], nb = fb[0];
    if (DS) na = mlp_row_frag<D>(w1, lane, in);
    if (DO) nb = mlp_tr_frag<D>(w2, lane, in & 1, in >> 1);
    if (DS) Sn = mfma32(fa[0], xf[i], Sn);
    if (DO) acc[i >> 1] = mfma32((i & 1) ? ho1 : ho0, fb[0], acc[i >> 1]);
    // 16 / KS GELU elements per step (element e: unit 8 (e >> 2) + 4 h + (e & 3) of the chunk)
    if (DG) {
#pragma unroll
      for (int ee = 0; ee < 16 / KS; ++ee) {
        const int e = i * (16 / KS) + ee;
        hv[e] = gelu_tanh(Sp[e] + bj[8 * (e >> 2) + (e & 3)]);
      }
    }
#pragma unroll
    for (int q = 0; q + 1 < LTHM_MLPP_PF; ++q) {
      fa[q] = fa[q + 1];
      fb[q] = fb[q + 1];
    }
    fa[LTHM_MLPP_PF - 1] = na;
    fb[LTHM_MLPP_PF - 1] = nb;
    asm volatile("" ::: "memory");
  }
  if (DG) {
    ho0 = mlp_pack(hv);
    ho1 = mlp_pack(hv + 8);
  }
  if (DS) Sp = Sn;
}

template <int D, int NRES>
__global__ __launch_bounds__(256, 1) void mlp_fwd_pipe_k(MlpArgs a) {
  constexpr int NW = 4, NTH = 64 * NW, IMG = 32 * D * 2, KS = D / 16, NT = D / 32, TR = 32 * NW;
  static_assert(KS == 2 * NT, "one S MFMA and one output MFMA per step");
  __shared__ __attribute__((aligned(16))) unsigned char im1[2][IMG];  // W1 chunk ring
  __shared__ __attribute__((aligned(16))) unsigned char im2[2][IMG];  // W2T chunk ring
  extern __shared__ float b1s[];                                      // [HID] b1, [D] b2
  float* b2s = b1s + a.HID;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int NC = a.HID / 32;
  const int64_t rs = a.M * blockIdx.x / gridDim.x, re = a.M * (blockIdx.x + 1) / gridDim.x;
  if (rs >= re) return;  // uniform
  for (int i = tid; i < a.HID; i += NTH) b1s[i] = a.b1 ? a.b1[i] : 0.f;
  for (int i = tid; i < D; i += NTH) b2s[i] = a.b2 ? a.b2[i] : 0.f;
  retire_loads();
  const int64_t ntile_wg = (re - rs + TR - 1) / TR;
  mlp_dma32<D, NTH>(im1[0], a.W1, tid);
  mlp_dma32<D, NTH>(im2[0], a.W2T, tid);
  __syncthreads();  // b1s / b2s
  // W1 / W2T chunk reads so far (ring slot: count & 1), and the chunk / tile of the next read
  int w1c = 0, w2c = 0, n1c = NC > 1 ? 1 : 0, n1t = NC > 1 ? 0 : 1, n2c = n1c, n2t = n1t;
  for (int64_t t0 = rs; t0 < re; t0 += TR) {
    const int64_t lim = min(t0 + TR, re), rb = t0 + 32 * wave;
    const bool active = rb < lim;  // wave-uniform
    bf16x8m xf[KS];
    mlp_load_x<D, KS>(a.X, rb + r32, rb + r32 < lim, h, xf);
    f32x16 acc[NT];
    // acc = b2 + res1 (+ res2) in the C layout: register i of tile t is row rb + 4 h + (i & 3) +
    // 8 (i >> 2), column 32 t + r32.  One 32-bit offset per register row (rows past the range
    // clamped to its last row: their values are never stored), the tile in the immediate.
    const int nrow = (int)min((int64_t)32, lim - rb) - 4 * h;  // live register rows: (i & 3) + 8 (i >> 2) < nrow
    uint32_t ro[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ro[i] = (uint32_t)(min(rb + 4 * h + (i & 3) + 8 * (i >> 2), lim - 1) * D + r32);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float bb = b2s[32 * t + r32];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float v = bb;
        if constexpr (NRES >= 1) v += a.res1[ro[i] + 32 * t];
        if constexpr (NRES >= 2) v += a.res2[ro[i] + 32 * t];
        acc[t][i] = v;
      }
    }
    f32x16 Sp = f32x16{};       // S of the previous phase's chunk
    bf16x8m ho0 = {}, ho1 = {};  // H of the chunk two phases back
    for (int k = 0; k < NC + 2; ++k) {
      const bool rd1 = k < NC, rd2 = k >= 2;
      wait_vm<0>();
      __syncthreads();  // this phase's chunks landed; the slots the DMAs below refill are free
      asm volatile("" ::: "memory");
      if (rd1 && n1t < ntile_wg) mlp_dma32<D, NTH>(im1[(w1c + 1) & 1], a.W1 + n1c * 32 * D, tid);
      if (rd2 && n2t < ntile_wg) mlp_dma32<D, NTH>(im2[(w2c + 1) & 1], a.W2T + n2c * 32 * D, tid);
      if (active) {
        // every phase runs all three streams (one code path keeps the register allocation within
        // the 512 of one wave per SIMD); the edge phases' extra terms are inert: H starts as zero
        // (the products of phases 0 and 1 add exact zeros, their W2T slot holds finite weights),
        // the S chains of phases NC and NC + 1 read finite stale or next-tile W1 data and feed
        // only a GELU whose H is discarded when the tile ends
        const int jg = min(max(k - 1, 0), NC - 1);  // chunk of the GELU
        mlp_pipe_phase<D, true, true, true>(im1[w1c & 1], im2[w2c & 1], b1s + 32 * jg + 4 * h, xf, acc, Sp, ho0, ho1,
                                            lane);
        if (k == 0) ho0 = ho1 = bf16x8m{};
      }
      if (rd1) {
        ++w1c;
        if (++n1c == NC) n1c = 0, ++n1t;
      }
      if (rd2) {
        ++w2c;
        if (++n2c == NC) n2c = 0, ++n2t;
      }
    }
    if (active) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((i & 3) + 8 * (i >> 2) < nrow) a.out[ro[i] + 32 * t] = acc[t][i];
    }
  }
}

// ---------------------------------------------------------------- backward (recompute)
// The training backward of the fused MLP: the hidden is recomputed, never read from HBM.
// Per token row x (ln_2 output, bf16) and upstream gradient dy (bf16):
//   pre  = x W1^T + b1        g = GELU(pre)          (hidden unit i: c_fc row i)
//   dH   = dy W2              dpre = dH * GELU'(pre)
//   dX   = dpre W1                                    (-> the ln_2 backward)
// and the two [M, HID] operands of the weight gradients, g (for dW2 = dy^T g) and dpre
// (for dW1 = dpre^T x, db1 = colsum dpre), are written once (bf16).  Same structure as
// the forward: a wave owns 32 token rows with x and dy held in registers as B operands,
// the hidden is walked in 32-unit chunks whose W1 / W2T images ride a 2-slot LDS-DMA
// ring; per chunk
//   S^T  = W1_j . x^T,  dH^T = W2T_j . dy^T        (hidden on registers, tokens on lanes)
//   dp   = dH * GELU'(S + b1), g = GELU(S + b1)     (one v_exp + v_rcp per element)
//   dX  += dp . W1_j                                (dp packed to bf16 IS the A operand; B:
//                                                    transposed reads of the same W1_j image)
// g and dp leave through the wave's LDS strip as 64-B row pieces.  One wave per SIMD (the
// x / dy fragments and the dX accumulator are 256 registers).
template <int D, int NW, bool GH>
__global__ __launch_bounds__(64 * NW, 1) void mlp_bwd_k(MlpBwdArgs a) {
  constexpr int NTH = 64 * NW, IMG = 32 * D * 2, KS = D / 16, NT = D / 32, TR = 32 * NW;
  __shared__ __attribute__((aligned(16))) unsigned char img[2][2][IMG];  // [stage][W1_j, W2T_j]
  __shared__ __attribute__((aligned(16))) float stg_all[NW][32 * 32];    // per-wave strips
  __shared__ float b1s[8192];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int NC = a.HID / 32;
  const int64_t rs = a.M * blockIdx.x / gridDim.x, re = a.M * (blockIdx.x + 1) / gridDim.x;
  if (rs >= re) return;  // uniform
  for (int i = tid; i < a.HID; i += NTH) b1s[i] = a.b1 ? a.b1[i] : 0.f;
  float* stg = stg_all[wave];
  bf16_t* stb = reinterpret_cast<bf16_t*>(stg);  // bf16 view: [32 rows][32 units] g, then dp
  retire_loads();
  mlp_dma32<D, NTH>(img[0][0], a.W1, tid);
  mlp_dma32<D, NTH>(img[0][1], a.W2T, tid);
  __syncthreads();  // b1s
  int g = 0;
  for (int64_t t0 = rs; t0 < re; t0 += TR) {
    const int64_t lim = min(t0 + TR, re), rb = t0 + 32 * wave;
    const bool active = rb < lim;  // wave-uniform
    bf16x8m xf[KS], df[KS];
    mlp_load_x<D, KS>(a.X, rb + r32, rb + r32 < lim, h, xf);
    mlp_load_x<D, KS>(a.dY, rb + r32, rb + r32 < lim, h, df);
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
    const bool more_tiles = t0 + TR < re;
    for (int j = 0; j < NC; ++j, ++g) {
      wait_vm<0>();
      __syncthreads();  // chunk j landed everywhere; every wave is done with chunk j - 1's stage
      asm volatile("" ::: "memory");
      if (j + 1 < NC || more_tiles) {
        const int jn = j + 1 < NC ? j + 1 : 0;
        mlp_dma32<D, NTH>(img[(g + 1) & 1][0], a.W1 + (int64_t)jn * 32 * D, tid);
        mlp_dma32<D, NTH>(img[(g + 1) & 1][1], a.W2T + (int64_t)jn * 32 * D, tid);
      }
      if (!active) continue;
      const unsigned char* w1 = img[g & 1][0];
      const unsigned char* w2 = img[g & 1][1];
      f32x16 S = f32x16{}, dH = f32x16{};
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        S = mfma32(mlp_row_frag<D>(w1, lane, k), xf[k], S);
        dH = mfma32(mlp_row_frag<D>(w2, lane, k), df[k], dH);
        __builtin_amdgcn_sched_barrier(0);
      }
      // g straight into the strip (8-B writes of 4 consecutive units), dp kept for the MFMA
      float dp[16];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b1s + 32 * j + 8 * m + 4 * h);
        float gv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float gd;
          gv[e] = gelu_tanh_and_grad(S[4 * m + e] + bb[e], gd);
          dp[4 * m + e] = dH[4 * m + e] * gd;
        }
        if constexpr (GH)
          *reinterpret_cast<uint2*>(stb + r32 * 32 + 8 * (m ^ ((r32 >> 2) & 3)) + 4 * h) =
              uint2{pack_bf16x2(gv[0], gv[1]), pack_bf16x2(gv[2], gv[3])};
      }
      const bf16x8m d0 = mlp_pack(dp), d1 = mlp_pack(dp + 8);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t] = mfma32(d0, mlp_tr_frag<D>(w1, lane, 0, t), acc[t]);
        acc[t] = mfma32(d1, mlp_tr_frag<D>(w1, lane, 1, t), acc[t]);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (!GH) continue;  // dX only (the weight gradients come from mlp_wgrad_k)
      // g and dp of the chunk: [32 tokens][32 units] bf16 through the strip (8-B writes of
      // 4 consecutive units), then 16-B row pieces: lane -> row l / 4 (+ 16), piece l % 4
#pragma unroll
      for (int m = 0; m < 4; ++m)
        *reinterpret_cast<uint2*>(stb + 1024 + r32 * 32 + 8 * (m ^ ((r32 >> 2) & 3)) + 4 * h) =
            uint2{pack_bf16x2(dp[4 * m], dp[4 * m + 1]), pack_bf16x2(dp[4 * m + 2], dp[4 * m + 3])};
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int rl = (lane >> 2) + 16 * q, pc = 8 * (lane & 3);
        const int64_t row = rb + rl;
        const u32x4 vg = *reinterpret_cast<const u32x4*>(stb + rl * 32 + (pc ^ (8 * ((rl >> 2) & 3))));
        const u32x4 vd = *reinterpret_cast<const u32x4*>(stb + 1024 + rl * 32 + (pc ^ (8 * ((rl >> 2) & 3))));
        if (row < lim) {
          *reinterpret_cast<u32x4*>(a.G + row * a.HID + 32 * j + pc) = vg;
          *reinterpret_cast<u32x4*>(a.dP + row * a.HID + 32 * j + pc) = vd;
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
    if (!active) continue;
    // dX [32 tokens][D]: each 32-column tile through the strip, 16-B pieces out
    const int pr = lane >> 3, pc = 4 * (lane & 7);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) stg[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r32] = acc[t][i];
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int64_t row = rb + pr + 8 * m;
        const f32x4 v = *reinterpret_cast<const f32x4*>(stg + (pr + 8 * m) * 32 + pc);
        if (row < lim) {
          if (a.dx_f32) {
            *reinterpret_cast<f32x4*>(a.dXf + row * D + 32 * t + pc) = v;
          } else {
            *reinterpret_cast<uint2*>(a.dXb + row * D + 32 * t + pc) =
                uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
}

// dX alone, software-pipelined (round 5; the weight gradients come from mlp_wgrad_k, so neither
// G nor dP is written).  One wave per SIMD, a wave owns 32 token rows (x and dy in registers as B
// operands, the dX sum in the accumulator registers); the hidden chunks' W1_j / W2T_j images ride
// a 4-slot LDS-DMA ring.  Step j of a tile is ONE interleaved loop of KS iterations; iteration k
// issues
//   S'^T += W1_{j+1} . x^T, dH'^T += W2T_{j+1} . dy^T   k-step k (2 MFMAs; row reads one step ahead)
//   dX   += dp_{j-1} . W1_{j-1}                          output tile k / 2, k-half k % 2 (1 MFMA)
//   GELU' element(s) of chunk j from its S^T / dH^T      (the VALU in those MFMAs' issue gaps)
// so the vector work of a chunk spreads over all 48 of its MFMAs.  The chunk stream runs on across
// tiles (chunk index wraps); a tile's first step adds dp = 0 (exact zeros), its last step's S' / dH'
// (of the next tile's first chunk image, with this tile's x / dy) are discarded.
template <int D, int NW>
__global__ __launch_bounds__(64 * NW, 1) void mlp_bwdx_k(MlpBwdArgs a) {
  constexpr int NTH = 64 * NW, IMG = 32 * D * 2, KS = D / 16, NT = D / 32, TR = 32 * NW, NS = 4;
  static_assert(KS == 2 * NT, "one dX MFMA per k-step");
  constexpr int EPK = 16 / KS;  // GELU' elements per iteration
  __shared__ __attribute__((aligned(16))) unsigned char img[NS][2][IMG];  // [slot][W1_j, W2T_j]
  __shared__ __attribute__((aligned(16))) float stg_all[NW][32 * 32];    // per-wave epilogue strips
  __shared__ __attribute__((aligned(16))) float b1s[4096];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int NC = a.HID / 32;
  const int64_t rs = a.M * blockIdx.x / gridDim.x, re = a.M * (blockIdx.x + 1) / gridDim.x;
  if (rs >= re) return;  // uniform
  for (int i = tid; i < a.HID; i += NTH) b1s[i] = a.b1 ? a.b1[i] : 0.f;
  float* stg = stg_all[wave];
  retire_loads();
  const int64_t ntile = (re - rs + TR - 1) / TR;
  const int nchunk = (int)(ntile * NC);  // the workgroup's chunk stream
  MlpDmaPlan<D, NTH> plan;
  plan.init(tid);
  const uint32_t lds0 = lds_addr(img[0][0]) + (uint32_t)(tid & ~63) * 16u;  // this wave's slice of slot 0
  int sjn = 0;  // hidden chunk index of the next chunk to stage (the stream's index mod NC)
  auto stage = [&](int c) {  // chunk c of the stream, hidden chunk sjn
    const uint32_t d = lds0 + (uint32_t)(c & (NS - 1)) * (2u * IMG);
    plan.issue(a.W1 + (int64_t)sjn * 32 * D, d);
    plan.issue(a.W2T + (int64_t)sjn * 32 * D, d + IMG);
    if (++sjn == NC) sjn = 0;
  };
  stage(0);
  if (nchunk > 1) stage(1);
  int g = 0;  // chunk index of the current step in the workgroup's stream
  for (int64_t t0 = rs; t0 < re; t0 += TR) {
    // every wave computes (a wave past the tile's rows reads the clamped first row and stores
    // nothing): no wave-dependent branch around the accumulator updates
    const int64_t lim = min(t0 + TR, re), rb = t0 + 32 * wave;
    const bool active = rb < lim;  // wave-uniform
    bf16x8m xf[KS], df[KS];
    mlp_load_x<D, KS>(a.X, rb + r32, rb + r32 < lim, h, xf);
    mlp_load_x<D, KS>(a.dY, rb + r32, rb + r32 < lim, h, df);
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
    // chunk g (the tile's first) landed everywhere (also: the x / dy loads above)
    wait_vm<0>();
    __syncthreads();
    f32x16 S = f32x16{}, H = f32x16{};
    {
      const unsigned char* w1 = img[g & (NS - 1)][0];
      const unsigned char* w2 = img[g & (NS - 1)][1];
      bf16x8m fa = mlp_row_frag<D>(w1, lane, 0), fb = mlp_row_frag<D>(w2, lane, 0);
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int kn = k + 1 < KS ? k + 1 : k;
        const bf16x8m na = mlp_row_frag<D>(w1, lane, kn), nb = mlp_row_frag<D>(w2, lane, kn);
        S = mfma32(fa, xf[k], S);
        H = mfma32(fb, df[k], H);
        fa = na;
        fb = nb;
        asm volatile("" ::: "memory");
      }
    }
    u32x4 dp0 = {0u, 0u, 0u, 0u}, dp1 = dp0;  // packed dp of the previous chunk (zero before the first)
    for (int j = 0; j < NC; ++j, ++g) {
      if (j > 0) {
        // every wave is done with step j - 1 (the slot of chunk g - 2 is free); chunk g + 1 landed
        wait_vm<0>();
        __syncthreads();
        asm volatile("" ::: "memory");
      }
      // chunk g + 2 into the slot of chunk g - 2 (last read by step g - 1: every wave passed this
      // step's barrier, or the tile's opening one at j = 0)
      if (g + 2 < nchunk) stage(g + 2);
      const unsigned char* w1p = img[(j > 0 ? g - 1 : g) & (NS - 1)][0];  // dX: chunk g - 1's W1 (or dp = 0)
      const unsigned char* w1n = img[(g + 1) & (NS - 1)][0];              // S' / dH' of chunk g + 1
      const unsigned char* w2n = img[(g + 1) & (NS - 1)][1];
      const bf16x8m d0 = __builtin_bit_cast(bf16x8m, dp0), d1 = __builtin_bit_cast(bf16x8m, dp1);
      f32x16 Sn = f32x16{}, Hn = f32x16{};
      float dl = 0.f;
      f32x4 bb = *reinterpret_cast<const f32x4*>(b1s + 32 * j + 4 * h);
      // LDS fragments two iterations ahead (one iteration is 3 MFMAs, ~100 cycles: less than an LDS
      // read's latency under load)
      bf16x8m fa = mlp_row_frag<D>(w1n, lane, 0), fb = mlp_row_frag<D>(w2n, lane, 0);
      bf16x8m bt = mlp_tr_frag<D>(w1p, lane, 0, 0);
      bf16x8m fa1 = mlp_row_frag<D>(w1n, lane, 1), fb1 = mlp_row_frag<D>(w2n, lane, 1);
      bf16x8m bt1 = mlp_tr_frag<D>(w1p, lane, 1, 0);
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int kn = k + 2 < KS ? k + 2 : KS - 1;
        const bf16x8m na = mlp_row_frag<D>(w1n, lane, kn), nb = mlp_row_frag<D>(w2n, lane, kn);
        const bf16x8m nt_ = mlp_tr_frag<D>(w1p, lane, kn & 1, kn >> 1);
        Sn = mfma32(fa, xf[k], Sn);
        acc[k >> 1] = mfma32((k & 1) ? d1 : d0, bt, acc[k >> 1]);
        Hn = mfma32(fb, df[k], Hn);
#pragma unroll
        for (int ee = 0; ee < EPK; ++ee) {
          const int e = k * EPK + ee;  // register e: unit 8 (e >> 2) + 4 h + (e & 3) of chunk j
          if ((e & 3) == 0 && e > 0) bb = *reinterpret_cast<const f32x4*>(b1s + 32 * j + 8 * (e >> 2) + 4 * h);
          const float dk = H[e] * gelu_tanh_grad(S[e] + bb[e & 3]);
          if (e & 1) {
            uint32_t dw = pack_bf16x2(dl, dk);
            asm volatile("" : "+v"(dw)::"memory");  // element e's VALU stays beside these MFMAs
            if (e < 8) dp0[(e >> 1) & 3] = dw;
            else dp1[(e >> 1) & 3] = dw;
          } else {
            dl = dk;
            asm volatile("" : "+v"(dl)::"memory");
          }
        }
        fa = fa1;
        fb = fb1;
        bt = bt1;
        fa1 = na;
        fb1 = nb;
        bt1 = nt_;
      }
      S = Sn;
      H = Hn;
    }
    {  // dX of the tile's last chunk (g - 1)
      const unsigned char* w1p = img[(g - 1) & (NS - 1)][0];
      const bf16x8m d0 = __builtin_bit_cast(bf16x8m, dp0), d1 = __builtin_bit_cast(bf16x8m, dp1);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t] = mfma32(d0, mlp_tr_frag<D>(w1p, lane, 0, t), acc[t]);
        acc[t] = mfma32(d1, mlp_tr_frag<D>(w1p, lane, 1, t), acc[t]);
      }
    }
    // dX [32 tokens][D]: each 32-column tile through the strip, 16-B pieces out
    const int pr = lane >> 3, pc = 4 * (lane & 7);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) stg[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r32] = acc[t][i];
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int64_t row = rb + pr + 8 * m;
        const f32x4 v = *reinterpret_cast<const f32x4*>(stg + (pr + 8 * m) * 32 + pc);
        if (active && row < lim) {
          if (a.dx_f32) {
            *reinterpret_cast<f32x4*>(a.dXf + row * D + 32 * t + pc) = v;
          } else {
            *reinterpret_cast<uint2*>(a.dXb + row * D + 32 * t + pc) =
                uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
}

// The split backward: the same recompute without the dX accumulator (dX = dP W1 then runs on
// the GEMM), so the x / dy fragments (128 registers) leave room for two waves per SIMD.
template <int D, int NW>
__global__ __launch_bounds__(64 * NW, 1) void mlp_bwdp_k(MlpBwdArgs a) {
  constexpr int NTH = 64 * NW, IMG = 32 * D * 2, KS = D / 16, TR = 32 * NW;
  __shared__ __attribute__((aligned(16))) unsigned char img[2][2][IMG];  // [stage][W1_j, W2T_j]
  // per-wave g / dp strips: 32 rows x four 16-B chunks, chunk c of row r at c ^ ((r >> 2) & 3) (the
  // C-layout b64 writes 2-way instead of 8-way bank-conflicted, the 16-B row reads conflict-free)
  __shared__ __attribute__((aligned(16))) bf16_t stb_all[NW][2 * 32 * 32];
  __shared__ float b1s[4096];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int NC = a.HID / 32;
  const int64_t rs = a.M * blockIdx.x / gridDim.x, re = a.M * (blockIdx.x + 1) / gridDim.x;
  if (rs >= re) return;  // uniform
  for (int i = tid; i < a.HID; i += NTH) b1s[i] = a.b1 ? a.b1[i] : 0.f;
  bf16_t* stb = stb_all[wave];
  retire_loads();
  mlp_dma32<D, NTH>(img[0][0], a.W1, tid);
  mlp_dma32<D, NTH>(img[0][1], a.W2T, tid);
  __syncthreads();  // b1s
  int g = 0;
  // the previous step issued its 4 G / dP stores AFTER the DMA of this step's chunk: a full-tile
  // wave retires the DMA with vmcnt 4, leaving its stores in flight (vmcnt retires in order)
  bool st4 = false;
#if LTHM_MLPF_STAMP
  MLPF_T(tk0);
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t tix = 0;
#endif
  for (int64_t t0 = rs; t0 < re; t0 += TR) {
    const int64_t lim = min(t0 + TR, re), rb = t0 + 32 * wave;
    const bool active = rb < lim;  // wave-uniform
    const bool full = rb + 32 <= lim;
    bf16x8m xf[KS], df[KS];
    mlp_load_x<D, KS>(a.X, rb + r32, rb + r32 < lim, h, xf);
    mlp_load_x<D, KS>(a.dY, rb + r32, rb + r32 < lim, h, df);
    const bool more_tiles = t0 + TR < re;
    for (int j = 0; j < NC; ++j, ++g) {
      MLPF_T(ts0);
      if (st4) wait_vm<4>();
      else wait_vm<0>();
      st4 = false;
      __syncthreads();  // chunk j landed everywhere; every wave is done with chunk j - 1's stage
      asm volatile("" ::: "memory");
      if (j + 1 < NC || more_tiles) {
        const int jn = j + 1 < NC ? j + 1 : 0;
        mlp_dma32<D, NTH>(img[(g + 1) & 1][0], a.W1 + (int64_t)jn * 32 * D, tid);
        mlp_dma32<D, NTH>(img[(g + 1) & 1][1], a.W2T + (int64_t)jn * 32 * D, tid);
      }
      if (!active) continue;
      MLPF_T(ts1);
      const unsigned char* w1 = img[g & 1][0];
      const unsigned char* w2 = img[g & 1][1];
      f32x16 S = f32x16{}, dH = f32x16{};
      bf16x8m fa = mlp_row_frag<D>(w1, lane, 0), fb = mlp_row_frag<D>(w2, lane, 0);
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int kn = k + 1 < KS ? k + 1 : k;
        const bf16x8m na = mlp_row_frag<D>(w1, lane, kn), nb = mlp_row_frag<D>(w2, lane, kn);
        S = mfma32(fa, xf[k], S);
        dH = mfma32(fb, df[k], dH);
        fa = na;
        fb = nb;
        asm volatile("" ::: "memory");
      }
#if LTHM_MLPF_STAMP
      MLPF_T(ts2);
      {
        float dep = S[15] + dH[15];  // in-order issue: the stamp below waits for both chains
        asm volatile("" : "+v"(dep));
        asm volatile("" ::"v"(dep));
      }
      MLPF_T(ts3);
#endif
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b1s + 32 * j + 8 * m + 4 * h);
        float gv[4], dv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float gd;
          gv[e] = gelu_tanh_and_grad(S[4 * m + e] + bb[e], gd);
          dv[e] = dH[4 * m + e] * gd;
        }
        *reinterpret_cast<uint2*>(stb + r32 * 32 + 8 * (m ^ ((r32 >> 2) & 3)) + 4 * h) = uint2{pack_bf16x2(gv[0], gv[1]), pack_bf16x2(gv[2], gv[3])};
        *reinterpret_cast<uint2*>(stb + 1024 + r32 * 32 + 8 * (m ^ ((r32 >> 2) & 3)) + 4 * h) =
            uint2{pack_bf16x2(dv[0], dv[1]), pack_bf16x2(dv[2], dv[3])};
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#if LTHM_MLPF_STAMP
      MLPF_T(ts4);
#endif
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int rl = (lane >> 2) + 16 * q, pc = 8 * (lane & 3);
        const int64_t row = rb + rl;
        const u32x4 vg = *reinterpret_cast<const u32x4*>(stb + rl * 32 + (pc ^ (8 * ((rl >> 2) & 3))));
        const u32x4 vd = *reinterpret_cast<const u32x4*>(stb + 1024 + rl * 32 + (pc ^ (8 * ((rl >> 2) & 3))));
        if (row < lim) {
          *reinterpret_cast<u32x4*>(a.G + row * a.HID + 32 * j + pc) = vg;
          *reinterpret_cast<u32x4*>(a.dP + row * a.HID + 32 * j + pc) = vd;
        }
      }
      st4 = full;  // every lane stored: exactly 4 store instructions issued
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#if LTHM_MLPF_STAMP
      MLPF_T(ts5);
      if (tix > 0) {
        st_acc[0] += ts1 - ts0;  // wait + barrier + DMA issue
        st_acc[1] += ts2 - ts1;  // S / dH issue
        st_acc[2] += ts3 - ts2;  // S / dH completion
        st_acc[3] += ts4 - ts3;  // GELU' + strip writes
        st_acc[4] += 1;
        st_acc[5] += ts5 - ts4;  // strip reads + G / dP store issue
      }
#endif
    }
#if LTHM_MLPF_STAMP
    ++tix;
#endif
  }
#if LTHM_MLPF_STAMP
  MLPF_T(tk);
  st_acc[7] = tk - tk0;
  if (lane == 0 && blockIdx.x < 2048)
    for (int k = 0; k < 8; ++k) g_mlpf_stamps[(blockIdx.x * 8 + wave) * 8 + k] = st_acc[k];
#endif
}

// mlp_bwdp_k at 4 waves with two workgroups per CU (round 6, as mlp_fwd2_k): 2-slot W1 / W2T ring
// (64 KiB), one 2-KiB strip per wave that g and then dp pass through, b1 in dynamic LDS: 76 KiB
// per workgroup, so a second workgroup's chunk loop runs beside one's tile edges and store bursts.
template <int D>
__global__ __launch_bounds__(256, 2) void mlp_bwdp2_k(MlpBwdArgs a) {
  constexpr int NW = 4, NTH = 64 * NW, IMG = 32 * D * 2, KS = D / 16, TR = 32 * NW;
  __shared__ __attribute__((aligned(16))) unsigned char img[2][2][IMG];  // [stage][W1_j, W2T_j]
  __shared__ __attribute__((aligned(16))) bf16_t stb_all[NW][32 * 32];   // g, then dp, of the chunk
  extern __shared__ float b1s[];                                          // [HID]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int NC = a.HID / 32;
  const int64_t rs = a.M * blockIdx.x / gridDim.x, re = a.M * (blockIdx.x + 1) / gridDim.x;
  if (rs >= re) return;  // uniform
  for (int i = tid; i < a.HID; i += NTH) b1s[i] = a.b1 ? a.b1[i] : 0.f;
  bf16_t* stb = stb_all[wave];
  retire_loads();
  mlp_dma32<D, NTH>(img[0][0], a.W1, tid);
  mlp_dma32<D, NTH>(img[0][1], a.W2T, tid);
  __syncthreads();  // b1s
  int g = 0;
  for (int64_t t0 = rs; t0 < re; t0 += TR) {
    const int64_t lim = min(t0 + TR, re), rb = t0 + 32 * wave;
    const bool active = rb < lim;  // wave-uniform
    bf16x8m xf[KS], df[KS];
    mlp_load_x<D, KS>(a.X, rb + r32, rb + r32 < lim, h, xf);
    mlp_load_x<D, KS>(a.dY, rb + r32, rb + r32 < lim, h, df);
    const bool more_tiles = t0 + TR < re;
    for (int j = 0; j < NC; ++j, ++g) {
      wait_vm<0>();
      __syncthreads();  // chunk j landed everywhere; every wave is done with chunk j - 1's stage
      asm volatile("" ::: "memory");
      if (j + 1 < NC || more_tiles) {
        const int jn = j + 1 < NC ? j + 1 : 0;
        mlp_dma32<D, NTH>(img[(g + 1) & 1][0], a.W1 + (int64_t)jn * 32 * D, tid);
        mlp_dma32<D, NTH>(img[(g + 1) & 1][1], a.W2T + (int64_t)jn * 32 * D, tid);
      }
      if (!active) continue;
      const unsigned char* w1 = img[g & 1][0];
      const unsigned char* w2 = img[g & 1][1];
      f32x16 S = f32x16{}, dH = f32x16{};
      bf16x8m fa = mlp_row_frag<D>(w1, lane, 0), fb = mlp_row_frag<D>(w2, lane, 0);
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int kn = k + 1 < KS ? k + 1 : k;
        const bf16x8m na = mlp_row_frag<D>(w1, lane, kn), nb = mlp_row_frag<D>(w2, lane, kn);
        S = mfma32(fa, xf[k], S);
        dH = mfma32(fb, df[k], dH);
        fa = na;
        fb = nb;
        asm volatile("" ::: "memory");
      }
      uint2 dpk[4];  // dp of the chunk, packed, until g has left the strip
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b1s + 32 * j + 8 * m + 4 * h);
        float gv[4], dv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float gd;
          gv[e] = gelu_tanh_and_grad(S[4 * m + e] + bb[e], gd);
          dv[e] = dH[4 * m + e] * gd;
        }
        *reinterpret_cast<uint2*>(stb + r32 * 32 + 8 * (m ^ ((r32 >> 2) & 3)) + 4 * h) =
            uint2{pack_bf16x2(gv[0], gv[1]), pack_bf16x2(gv[2], gv[3])};
        dpk[m] = uint2{pack_bf16x2(dv[0], dv[1]), pack_bf16x2(dv[2], dv[3])};
      }
      // [32 tokens][32 units] bf16 out of the strip as 16-B row pieces: lane -> row l / 4 (+ 16), piece l % 4
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        bf16_t* dst = pass == 0 ? a.G : a.dP;
        u32x4 v[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int rl = (lane >> 2) + 16 * q, pc = 8 * (lane & 3);
          v[q] = *reinterpret_cast<const u32x4*>(stb + rl * 32 + (pc ^ (8 * ((rl >> 2) & 3))));
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        if (pass == 0) {
#pragma unroll
          for (int m = 0; m < 4; ++m) *reinterpret_cast<uint2*>(stb + r32 * 32 + 8 * (m ^ ((r32 >> 2) & 3)) + 4 * h) = dpk[m];
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int rl = (lane >> 2) + 16 * q, pc = 8 * (lane & 3);
          const int64_t row = rb + rl;
          if (row < lim) *reinterpret_cast<u32x4*>(dst + row * a.HID + 32 * j + pc) = v[q];
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
}

// ---------------------------------------------------------------- weight gradients (recompute)
// dW1 = dpre^T x, dW2^T = g^T dy, db1 = colsum dpre with g / dpre recomputed per token tile and
// never written: the loop order is the transpose of the kernels above.  A wave OWNS 32 hidden
// units j (its W1_j / W2T_j rows live in registers as B operands) and its dW1_j / dW2^T_j
// [32 x D] sums live in the accumulator registers for the whole kernel; the workgroup (NW
// waves, NW * 32 hidden units = one hidden group) walks the token tiles of its slice, each
// [32 x D] x and dy tile staged once into LDS by LDS-DMA (3-slot ring) and read by every wave:
//   S  = x . W1_j^T,  dH = dy . W2T_j^T      (tokens on the accumulator registers, hidden units
//                                             on the lanes: 2 x D / 16 MFMAs)
//   g  = GELU(S + b1), dp = dH GELU'(S + b1)  (one v_exp + one v_rcp per element)
//   dW1_j   += dp^T . x,  dW2^T_j += g^T . dy (the packed accumulators ARE the A operands over
//                                             the permuted token order; B = transposed reads of
//                                             the staged tiles: 2 x D / 16 MFMAs)
// so per token tile and wave 4 D / 16 MFMAs, no HBM traffic beyond x and dy (read once per
// hidden group; the groups of one slice run on one XCD, so the repeats are L2 hits).  The slabs
// [nslice][HID][D] are folded in slice order by mlp_wgrad_fold_k (no atomics, deterministic).
template <int D, int NW, bool FULL>
__global__ __launch_bounds__(64 * NW, 1) void mlp_wgrad_k(MlpWgArgs a) {
  constexpr int NTH = 64 * NW, IMG = 32 * D * 2, KS = D / 16, NT = D / 32, NS = 3;
  constexpr int DPT = 2 * (32 * D / 8) / NTH;  // DMAs per thread and tile (both images)
  // 3-slot ring of (x, dy) tiles + each wave's W2T_j image: 160 KiB at D = 256.  The dW sums take
  // the 256 accumulator registers and W1_j's B operands 64 of the 256 others, so W2T_j's B
  // operands are read from LDS (a second ds_read_b128 in the dH MFMA gaps)
  __shared__ __attribute__((aligned(16))) unsigned char img[NS][2][IMG];  // [slot][x, dy]
  __shared__ __attribute__((aligned(16))) unsigned char wimg[NW][IMG];    // W2T_j per wave
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  // XCD-contiguous logical order: the hidden groups of one slice share an XCD's L2
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int slice = lid / a.ngroup, grp = lid - slice * a.ngroup;
  const int64_t ntile_all = (a.M + 31) / 32;
  const int64_t t_lo = ntile_all * slice / a.nslice, t_hi = ntile_all * (slice + 1) / a.nslice;
  const int j0 = (grp * NW + wave) * 32;  // this wave's hidden units j0 .. j0 + 31
  // B operands over d of the wave's W1 rows: lane -> unit j0 + r32, k 16 k + 8 h ..
  bf16x8m w1f[KS];
  {
    const bf16_t* p1 = a.W1 + (int64_t)(j0 + r32) * D + 8 * h;
#pragma unroll
    for (int k = 0; k < KS; ++k) w1f[k] = __builtin_bit_cast(bf16x8m, *reinterpret_cast<const u32x4*>(p1 + 16 * k));
  }
  unsigned char* w2i = wimg[wave];
  const float bj = a.b1 ? a.b1[j0 + r32] : 0.f;
  f32x16 acc1[NT], acc2[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc1[t] = acc2[t] = f32x16{};
  float dbs = 0.f;
  retire_loads();
  const int nt = (int)(t_hi - t_lo);
  MlpDmaPlan<D, NTH> plan;
  plan.init(tid);
  const uint32_t lds0 = lds_addr(img[0][0]) + (uint32_t)(tid & ~63) * 16u;  // this wave's slice of slot 0
  auto stage = [&](int64_t ti, int slot) {
    const int64_t r0 = ti * 32;
    if (FULL) {  // every tile whole: the precomputed plan
      const uint32_t d = lds0 + (uint32_t)slot * (2u * IMG);
      plan.issue(a.X + r0 * D, d);
      plan.issue(a.dY + r0 * D, d + IMG);
    } else {
      const int nv = (int)min((int64_t)32, a.M - r0);
      mlp_dma32c<D, NTH>(img[slot][0], a.X, r0, nv, tid);
      mlp_dma32c<D, NTH>(img[slot][1], a.dY, r0, nv, tid);
    }
  };
  // Software pipeline, one wave per SIMD (the dW sums hold the 256 accumulator registers): step i
  // runs
  //   phase B: dW += of tile i - 1 (32 MFMAs; transposed tile reads one pair ahead)  ||  GELU of
  //            tile i from its S / dH registers (the VALU in the MFMA issue gaps), packed to bf16
  //   barrier; LDS-DMA of tile i + 2 into the slot of tile i - 1 (free now)
  //   phase A: S / dH of tile i + 1 (32 MFMAs)
  // so only one S / dH pair and two packed operand sets are live.  Tile i + 1 was staged during
  // step i - 1 (after its barrier); tile i is not read by step i at all.
  mlp_dma32<D, 64>(w2i, a.W2T + (int64_t)j0 * D, lane);  // the wave's own image (retired with tile 0)
  if (nt > 0) stage(t_lo, 0);
  if (nt > 1) stage(t_lo + 1, 1);
  f32x16 S = f32x16{}, H = f32x16{};
  auto phase_a = [&](const unsigned char* xn, const unsigned char* yn) {
    bf16x8m fa = mlp_row_frag<D>(xn, lane, 0), fb = mlp_row_frag<D>(yn, lane, 0), fw = mlp_row_frag<D>(w2i, lane, 0);
    S = f32x16{};
    H = f32x16{};
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int kn = k + 1 < KS ? k + 1 : k;
      const bf16x8m na = mlp_row_frag<D>(xn, lane, kn), nb = mlp_row_frag<D>(yn, lane, kn);
      const bf16x8m nw = mlp_row_frag<D>(w2i, lane, kn);
      S = mfma32(fa, w1f[k], S);
      H = mfma32(fb, fw, H);
      fa = na;
      fb = nb;
      fw = nw;
      asm volatile("" ::: "memory");
    }
  };
  if (nt > 0) {
    if (nt > 1) wait_vm<DPT>();
    else wait_vm<0>();
    __syncthreads();
    phase_a(img[0][0], img[0][1]);
  }
  // packed operands of the previous tile (zero before tile 0: phase B of step 0 adds exact zeros
  // from tile 0's finite rows)
  u32x4 gp0 = {0u, 0u, 0u, 0u}, gp1 = gp0, dp0 = gp0, dp1 = gp0;
  for (int i = 0; i < nt; ++i) {
    // ---- phase B: dW of tile i - 1 || GELU of tile i
    {
      const int ip = i > 0 ? i - 1 : 0;
      const unsigned char* xi = img[ip % NS][0];
      const unsigned char* yi = img[ip % NS][1];
      const int nv = (int)min((int64_t)32, a.M - (t_lo + i) * 32);  // valid token rows of tile i
      const bf16x8m d0 = __builtin_bit_cast(bf16x8m, dp0), d1 = __builtin_bit_cast(bf16x8m, dp1);
      const bf16x8m g0 = __builtin_bit_cast(bf16x8m, gp0), g1 = __builtin_bit_cast(bf16x8m, gp1);
      float gl = 0.f, dl = 0.f;
      bf16x8m b0 = mlp_tr_frag<D>(xi, lane, 0, 0), b1 = mlp_tr_frag<D>(xi, lane, 1, 0);
#pragma unroll
      for (int k = 0; k < 2 * NT; ++k) {  // step k: output tile t = k / 2, half u = k % 2 (dW1, dW2^T)
        const int t = k >> 1, u = k & 1, tn = t + 1 < NT ? t + 1 : t;
        const unsigned char* nimg = u == 0 ? yi : xi;
        const int nt_ = u == 0 ? t : tn;
        const bf16x8m n0 = mlp_tr_frag<D>(nimg, lane, 0, nt_), n1 = mlp_tr_frag<D>(nimg, lane, 1, nt_);
        if (u == 0) {
          acc1[t] = mfma32(d0, b0, acc1[t]);
          acc1[t] = mfma32(d1, b1, acc1[t]);
        } else {
          acc2[t] = mfma32(g0, b0, acc2[t]);
          acc2[t] = mfma32(g1, b1, acc2[t]);
        }
        // GELU elements of tile i beside this step's MFMAs: 16 / (2 NT) per step (register e: token
        // row 8 (e >> 2) + 4 h + (e & 3))
        constexpr int EPS = 16 / (2 * NT);
#pragma unroll
        for (int ee = 0; ee < EPS; ++ee) {
          const int e = k * EPS + ee;
          float gd;
          const float gg = gelu_tanh_and_grad(S[e] + bj, gd);
          const bool ok = FULL || 8 * (e >> 2) + 4 * h + (e & 3) < nv;  // token rows past M
          const float gk = ok ? gg : 0.f, dk = ok ? H[e] * gd : 0.f;
          dbs += dk;
          if (e & 1) {
            uint32_t gw = pack_bf16x2(gl, gk), dw = pack_bf16x2(dl, dk);
            // pins element e's VALU into this step's scheduling region, beside its MFMAs
            asm volatile("" : "+v"(gw), "+v"(dw), "+v"(dbs)::"memory");
            const int q = (e >> 1) & 3;
            if (e < 8) {
              gp0[q] = gw;
              dp0[q] = dw;
            } else {
              gp1[q] = gw;
              dp1[q] = dw;
            }
          } else {
            gl = gk;
            dl = dk;
            asm volatile("" : "+v"(gl), "+v"(dl), "+v"(dbs)::"memory");
          }
        }
        b0 = n0;
        b1 = n1;
      }
    }
    // ---- every wave is done with tile i - 1's slot; tile i + 1 landed everywhere
    wait_vm<0>();
    __syncthreads();
    asm volatile("" ::: "memory");
    if (i + 2 < nt) stage(t_lo + i + 2, (int)((i + 2) % NS));
    // ---- phase A: S / dH of tile i + 1 (past the last tile: a stale slot, results unused)
    phase_a(img[(i + 1) % NS][0], img[(i + 1) % NS][1]);
  }
  if (nt > 0) {  // phase B of the last tile
    const unsigned char* xi = img[(nt - 1) % NS][0];
    const unsigned char* yi = img[(nt - 1) % NS][1];
    const bf16x8m d0 = __builtin_bit_cast(bf16x8m, dp0), d1 = __builtin_bit_cast(bf16x8m, dp1);
    const bf16x8m g0 = __builtin_bit_cast(bf16x8m, gp0), g1 = __builtin_bit_cast(bf16x8m, gp1);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      acc1[t] = mfma32(d0, mlp_tr_frag<D>(xi, lane, 0, t), acc1[t]);
      acc1[t] = mfma32(d1, mlp_tr_frag<D>(xi, lane, 1, t), acc1[t]);
      acc2[t] = mfma32(g0, mlp_tr_frag<D>(yi, lane, 0, t), acc2[t]);
      acc2[t] = mfma32(g1, mlp_tr_frag<D>(yi, lane, 1, t), acc2[t]);
    }
  }
  // partial slabs: register v of tile t is unit j0 + 8 (v >> 2) + 4 h + (v & 3), column 32 t + r32
  float* p1 = a.dW1p + ((int64_t)slice * a.HID + j0) * D;
  float* p2 = a.dW2Tp + ((int64_t)slice * a.HID + j0) * D;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int64_t o = (int64_t)(8 * (v >> 2) + 4 * h + (v & 3)) * D + 32 * t + r32;
      p1[o] = acc1[t][v];
      p2[o] = acc2[t][v];
    }
  dbs += __shfl_xor(dbs, 32, 64);
  if (a.db1p && h == 0) a.db1p[(int64_t)slice * a.HID + j0 + r32] = dbs;
}

// dW1 [HID][D] = sum over slices of dW1p; dW2 [D][HID] = (sum of dW2Tp)^T; db1 = sum of db1p --
// the slices in order 0, 1, ... (deterministic).  One block per 32 x 32 (unit, column) tile;
// the transposed dW2 goes out through an LDS tile.
__global__ __launch_bounds__(256) void mlp_wgrad_fold_k(const float* __restrict__ dW1p, const float* __restrict__ dW2Tp,
                                                        const float* __restrict__ db1p, int nslice, int HID, int D,
                                                        float* __restrict__ dW1, float* __restrict__ dW2,
                                                        float* __restrict__ db1) {
  __shared__ float tl[32][33];
  const int u0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows of 32 per pass
  const int64_t sl = (int64_t)HID * D;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int u = u0 + ty + 8 * q;
    const int64_t o = (int64_t)u * D + c0 + tx;
    float s1 = 0.f, s2 = 0.f;
    for (int s = 0; s < nslice; ++s) {
      s1 += dW1p[s * sl + o];
      s2 += dW2Tp[s * sl + o];
    }
    dW1[o] = s1;
    tl[ty + 8 * q][tx] = s2;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = c0 + ty + 8 * q;
    dW2[(int64_t)c * HID + u0 + tx] = tl[tx][ty + 8 * q];
  }
  if (db1 && blockIdx.x == 0 && threadIdx.x < 32) {
    float s = 0.f;
    for (int sidx = 0; sidx < nslice; ++sidx) s += db1p[(int64_t)sidx * HID + u0 + threadIdx.x];
    db1[u0 + threadIdx.x] = s;
  }
}

}  // namespace lthm

using namespace lthm;

static int mlp_cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

// waves per forward workgroup: 8 (one workgroup per CU, 256-row tiles) or 4 (two per CU);
// LTHM_MLP_NW overrides (measurement)
static int mlp_fwd_waves() {
  static int nw = 0;
  if (nw == 0) {
    const char* e = getenv("LTHM_MLP_NW");
    nw = (e && e[0] == '4') ? 4 : 8;
  }
  return nw;
}

#if LTHM_MLPF_STAMP
extern "C" int lthm_debug_mlpf_stamps(unsigned long long* host, int64_t n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mlpf_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif

extern "C" int lthm_mlp_supported(int32_t D, int32_t HID) {
  return (D == 128 || D == 256) && HID >= 32 && HID % 32 == 0 && HID <= 8192;
}

static int mlp_fwd_launch(MlpArgs a, int D, void* stream);

extern "C" int lthm_mlp_fwd_ln(const float* x, const float* ln_w, const float* ln_b, int64_t M, int32_t D,
                               int32_t HID, const void* W1, const float* b1, const void* W2T, const float* b2,
                               const float* res1, const float* res2, float* out, void* h_out, float* mean,
                               float* rstd, void* stream) {
  LTHM_REQUIRE(lthm_mlp_supported(D, HID) && M >= 0);
  LTHM_REQUIRE(x && ln_w && W1 && W2T && out);
  LTHM_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)W1 % 16) == 0 && ((uintptr_t)W2T % 16) == 0 &&
               ((uintptr_t)b1 % 16) == 0 && ((uintptr_t)h_out % 16) == 0);
  if (M == 0) return 0;
  MlpArgs a{};
  a.X = nullptr; a.W1 = (const bf16_t*)W1; a.W2T = (const bf16_t*)W2T;
  a.b1 = b1; a.b2 = b2; a.res1 = res1; a.res2 = res2; a.out = out;
  a.M = M; a.HID = HID;
  a.x32 = x; a.ln_w = ln_w; a.ln_b = ln_b; a.h_out = (bf16_t*)h_out; a.mean = mean; a.rstd = rstd;
  return mlp_fwd_launch(a, D, stream);
}

extern "C" int lthm_mlp_fwd(const void* X, int64_t M, int32_t D, int32_t HID, const void* W1, const float* b1,
                            const void* W2T, const float* b2, const float* res1, const float* res2, float* out,
                            void* stream) {
  LTHM_REQUIRE(lthm_mlp_supported(D, HID) && M >= 0);
  LTHM_REQUIRE(X && W1 && W2T && out);
  LTHM_REQUIRE(((uintptr_t)X % 16) == 0 && ((uintptr_t)W1 % 16) == 0 && ((uintptr_t)W2T % 16) == 0 &&
               ((uintptr_t)b1 % 16) == 0);
  if (M == 0) return 0;
  MlpArgs a{};
  a.X = (const bf16_t*)X; a.W1 = (const bf16_t*)W1; a.W2T = (const bf16_t*)W2T;
  a.b1 = b1; a.b2 = b2; a.res1 = res1; a.res2 = res2; a.out = out;
  a.M = M; a.HID = HID;
  return mlp_fwd_launch(a, D, stream);
}

static int mlp_fwd_launch(MlpArgs a, int D, void* stream) {
  const int64_t M = a.M;
  const int HID = a.HID;
  hipStream_t s = (hipStream_t)stream;
  const size_t dyn = (size_t)(HID + 3 * D) * 4;
  const int nw = mlp_fwd_waves();
  a.ntiles = (int)((M + 32 * nw - 1) / (32 * nw));
  const int per_cu = 1;
  int grid = std::min<int64_t>(a.ntiles, (int64_t)mlp_cu_count() * per_cu);
  // LTHM_MLP_PIPE=1: the software-pipelined one-wave-per-SIMD form (no ln_2 prologue)
  static const bool pipe = getenv("LTHM_MLP_PIPE") && getenv("LTHM_MLP_PIPE")[0] == '1';
  if (pipe && !a.ln_w && M * D < ((int64_t)1 << 29)) {
    a.ntiles = (int)((M + 127) / 128);
    const int gp = std::min<int64_t>(a.ntiles, (int64_t)mlp_cu_count());
    const size_t dynp = (size_t)(HID + D) * 4;
    if (!a.res1 && a.res2) std::swap(a.res1, a.res2);
    const int nres = a.res2 ? 2 : a.res1 ? 1 : 0;
#define LTHM_MLPP(D_)                                                                                      \
    if (nres == 2) hipLaunchKernelGGL((mlp_fwd_pipe_k<D_, 2>), dim3(gp), dim3(256), dynp, s, a);           \
    else if (nres == 1) hipLaunchKernelGGL((mlp_fwd_pipe_k<D_, 1>), dim3(gp), dim3(256), dynp, s, a);      \
    else hipLaunchKernelGGL((mlp_fwd_pipe_k<D_, 0>), dim3(gp), dim3(256), dynp, s, a);
    if (D == 256) { LTHM_MLPP(256) } else { LTHM_MLPP(128) }
#undef LTHM_MLPP
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  // two 4-wave workgroups per CU (mlp_fwd2_k; LTHM_MLP_FWD2=1: on), no ln_2 prologue
  static const bool fwd2 = getenv("LTHM_MLP_FWD2") && getenv("LTHM_MLP_FWD2")[0] == '1';
  if (fwd2 && !a.ln_w) {
    a.ntiles = (int)((M + 127) / 128);
    const int g2 = std::min<int64_t>(a.ntiles, (int64_t)mlp_cu_count() * 2);
    const size_t dyn2 = (size_t)(HID + D) * 4;
    if (!a.res1 && a.res2) std::swap(a.res1, a.res2);
    const int nres = a.res2 ? 2 : a.res1 ? 1 : 0;
#define LTHM_MLPF2(D_)                                                                                     \
    if (nres == 2) hipLaunchKernelGGL((mlp_fwd2_k<D_, 2>), dim3(g2), dim3(256), dyn2, s, a);               \
    else if (nres == 1) hipLaunchKernelGGL((mlp_fwd2_k<D_, 1>), dim3(g2), dim3(256), dyn2, s, a);          \
    else hipLaunchKernelGGL((mlp_fwd2_k<D_, 0>), dim3(g2), dim3(256), dyn2, s, a);
    if (D == 256) { LTHM_MLPF2(256) } else { LTHM_MLPF2(128) }
#undef LTHM_MLPF2
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  // LTHM_MLP_STAG=1: the 8-wave form with the half-chunk lag of waves 4-7 (A/B)
  static const bool stag = getenv("LTHM_MLP_STAG") && getenv("LTHM_MLP_STAG")[0] == '1';
#define LTHM_MLPF(D_, NW_)                                                                                 \
  do {                                                                                                     \
    if (stag && NW_ == 8) hipLaunchKernelGGL((mlp_fwd_k<D_, NW_, true>), dim3(grid), dim3(64 * NW_), dyn, s, a); \
    else hipLaunchKernelGGL((mlp_fwd_k<D_, NW_, false>), dim3(grid), dim3(64 * NW_), dyn, s, a);          \
  } while (0)
  if (D == 256) { if (nw == 8) LTHM_MLPF(256, 8); else LTHM_MLPF(256, 4); }
  else { if (nw == 8) LTHM_MLPF(128, 8); else LTHM_MLPF(128, 4); }
#undef LTHM_MLPF
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_mlp_bwd(const void* X, const void* dY, int64_t M, int32_t D, int32_t HID, const void* W1,
                            const float* b1, const void* W2T, void* dX, int32_t dx_dtype, void* G, void* dP,
                            void* stream) {
  LTHM_REQUIRE(lthm_mlp_supported(D, HID) && M >= 0);
  LTHM_REQUIRE(X && dY && W1 && W2T && dX && G && dP && (dx_dtype == LTHM_F32 || dx_dtype == LTHM_BF16));
  LTHM_REQUIRE(((uintptr_t)X % 16) == 0 && ((uintptr_t)dY % 16) == 0 && ((uintptr_t)W1 % 16) == 0 &&
               ((uintptr_t)W2T % 16) == 0 && ((uintptr_t)b1 % 16) == 0 && ((uintptr_t)dX % 16) == 0 &&
               ((uintptr_t)G % 16) == 0 && ((uintptr_t)dP % 16) == 0);
  if (M == 0) return 0;
  MlpBwdArgs a;
  a.X = (const bf16_t*)X; a.dY = (const bf16_t*)dY; a.W1 = (const bf16_t*)W1; a.W2T = (const bf16_t*)W2T;
  a.b1 = b1; a.G = (bf16_t*)G; a.dP = (bf16_t*)dP;
  a.dx_f32 = dx_dtype == LTHM_F32;
  a.dXf = (float*)dX; a.dXb = (bf16_t*)dX;
  a.M = M; a.HID = HID;
  hipStream_t s = (hipStream_t)stream;
  constexpr int NW = 4;
  const int64_t ntiles = (M + 32 * NW - 1) / (32 * NW);
  const int grid = (int)std::min<int64_t>(ntiles, (int64_t)mlp_cu_count());
  if (D == 256) hipLaunchKernelGGL((mlp_bwd_k<256, NW, true>), dim3(grid), dim3(64 * NW), 0, s, a);
  else hipLaunchKernelGGL((mlp_bwd_k<128, NW, true>), dim3(grid), dim3(64 * NW), 0, s, a);
  LTHM_CHECK_LAUNCH();
  return 0;
}

// waves per weight-gradient workgroup (one per SIMD: the two [32 x D] sums are 2 D / 2 registers)
constexpr int MLP_WG_NW = 4;

static void mlp_wgrad_geometry(int64_t M, int D, int HID, int* nslice, int* ngroup) {
  *ngroup = HID / (32 * MLP_WG_NW);
  const int64_t ntile = (M + 31) / 32;
  // one workgroup per CU: slices x groups ~ the CU count, at least one token tile per slice
  int ns = std::max(1, mlp_cu_count() / std::max(1, *ngroup));
  *nslice = (int)std::max<int64_t>(1, std::min<int64_t>(ns, ntile));
  (void)D;
}

extern "C" int64_t lthm_mlp_wgrad_ws_bytes(int64_t M, int32_t D, int32_t HID) {
  if (!lthm_mlp_supported(D, HID) || HID % (32 * MLP_WG_NW) || M < 0) return -1;
  int ns, ng;
  mlp_wgrad_geometry(M, D, HID, &ns, &ng);
  return (int64_t)ns * HID * (2 * (int64_t)D + 1) * 4;
}

extern "C" int lthm_mlp_wgrad(const void* X, const void* dY, int64_t M, int32_t D, int32_t HID, const void* W1,
                              const float* b1, const void* W2T, float* dW1, float* dW2, float* db1, void* workspace,
                              int64_t ws_bytes, void* stream) {
  LTHM_REQUIRE(lthm_mlp_supported(D, HID) && HID % (32 * MLP_WG_NW) == 0 && M >= 0);
  LTHM_REQUIRE(X && dY && W1 && W2T && dW1 && dW2 && workspace);
  LTHM_REQUIRE(((uintptr_t)X % 16) == 0 && ((uintptr_t)dY % 16) == 0 && ((uintptr_t)W1 % 16) == 0 &&
               ((uintptr_t)W2T % 16) == 0 && ((uintptr_t)workspace % 16) == 0);
  LTHM_REQUIRE(ws_bytes >= lthm_mlp_wgrad_ws_bytes(M, D, HID));
  hipStream_t s = (hipStream_t)stream;
  int ns, ng;
  mlp_wgrad_geometry(M, D, HID, &ns, &ng);
  MlpWgArgs a{};
  a.X = (const bf16_t*)X; a.dY = (const bf16_t*)dY; a.W1 = (const bf16_t*)W1; a.W2T = (const bf16_t*)W2T;
  a.b1 = b1;
  a.dW1p = (float*)workspace;
  a.dW2Tp = a.dW1p + (int64_t)ns * HID * D;
  a.db1p = db1 ? a.dW2Tp + (int64_t)ns * HID * D : nullptr;
  a.M = M; a.HID = HID; a.nslice = ns; a.ngroup = ng;
  if (M > 0) {
    // every token tile full (M % 32 == 0, C2's 528,384 rows): no per-element row mask
    const bool full = M % 32 == 0;
    if (D == 256) {
      if (full) hipLaunchKernelGGL((mlp_wgrad_k<256, MLP_WG_NW, true>), dim3(ns * ng), dim3(64 * MLP_WG_NW), 0, s, a);
      else hipLaunchKernelGGL((mlp_wgrad_k<256, MLP_WG_NW, false>), dim3(ns * ng), dim3(64 * MLP_WG_NW), 0, s, a);
    } else {
      if (full) hipLaunchKernelGGL((mlp_wgrad_k<128, MLP_WG_NW, true>), dim3(ns * ng), dim3(64 * MLP_WG_NW), 0, s, a);
      else hipLaunchKernelGGL((mlp_wgrad_k<128, MLP_WG_NW, false>), dim3(ns * ng), dim3(64 * MLP_WG_NW), 0, s, a);
    }
    LTHM_CHECK_LAUNCH();
  } else {
    LTHM_REQUIRE(hipMemsetAsync(workspace, 0, (size_t)lthm_mlp_wgrad_ws_bytes(M, D, HID), s) == hipSuccess);
  }
  hipLaunchKernelGGL(mlp_wgrad_fold_k, dim3(D / 32, HID / 32), dim3(256), 0, s, (const float*)a.dW1p,
                     (const float*)a.dW2Tp, (const float*)a.db1p, ns, HID, D, dW1, dW2, db1);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_mlp_bwd_dx(const void* X, const void* dY, int64_t M, int32_t D, int32_t HID, const void* W1,
                               const float* b1, const void* W2T, void* dX, int32_t dx_dtype, void* stream) {
  LTHM_REQUIRE(lthm_mlp_supported(D, HID) && M >= 0);
  LTHM_REQUIRE(X && dY && W1 && W2T && dX && (dx_dtype == LTHM_F32 || dx_dtype == LTHM_BF16));
  LTHM_REQUIRE(((uintptr_t)X % 16) == 0 && ((uintptr_t)dY % 16) == 0 && ((uintptr_t)W1 % 16) == 0 &&
               ((uintptr_t)W2T % 16) == 0 && ((uintptr_t)b1 % 16) == 0 && ((uintptr_t)dX % 16) == 0);
  if (M == 0) return 0;
  MlpBwdArgs a{};
  a.X = (const bf16_t*)X; a.dY = (const bf16_t*)dY; a.W1 = (const bf16_t*)W1; a.W2T = (const bf16_t*)W2T;
  a.b1 = b1;
  a.dx_f32 = dx_dtype == LTHM_F32;
  a.dXf = (float*)dX; a.dXb = (bf16_t*)dX;
  a.M = M; a.HID = HID;
  hipStream_t s = (hipStream_t)stream;
  constexpr int NW = 4;
  const int64_t ntiles = (M + 32 * NW - 1) / (32 * NW);
  const int grid = (int)std::min<int64_t>(ntiles, (int64_t)mlp_cu_count());
  LTHM_REQUIRE(HID <= 4096);
  if (D == 256) hipLaunchKernelGGL((mlp_bwdx_k<256, NW>), dim3(grid), dim3(64 * NW), 0, s, a);
  else hipLaunchKernelGGL((mlp_bwdx_k<128, NW>), dim3(grid), dim3(64 * NW), 0, s, a);
  LTHM_CHECK_LAUNCH();
  return 0;
}

extern "C" int lthm_mlp_bwd_hidden(const void* X, const void* dY, int64_t M, int32_t D, int32_t HID, const void* W1,
                                   const float* b1, const void* W2T, void* G, void* dP, void* stream) {
  LTHM_REQUIRE(lthm_mlp_supported(D, HID) && HID <= 4096 && M >= 0);
  LTHM_REQUIRE(X && dY && W1 && W2T && G && dP);
  LTHM_REQUIRE(((uintptr_t)X % 16) == 0 && ((uintptr_t)dY % 16) == 0 && ((uintptr_t)W1 % 16) == 0 &&
               ((uintptr_t)W2T % 16) == 0 && ((uintptr_t)b1 % 16) == 0 && ((uintptr_t)G % 16) == 0 &&
               ((uintptr_t)dP % 16) == 0);
  if (M == 0) return 0;
  MlpBwdArgs a{};
  a.X = (const bf16_t*)X; a.dY = (const bf16_t*)dY; a.W1 = (const bf16_t*)W1; a.W2T = (const bf16_t*)W2T;
  a.b1 = b1; a.G = (bf16_t*)G; a.dP = (bf16_t*)dP;
  a.M = M; a.HID = HID;
  hipStream_t s = (hipStream_t)stream;
  // two 4-wave workgroups per CU (mlp_bwdp2_k; LTHM_MLP_BWDP2=1: on)
  static const bool p2 = getenv("LTHM_MLP_BWDP2") && getenv("LTHM_MLP_BWDP2")[0] == '1';
  if (p2) {
    const int64_t nt2 = (M + 127) / 128;
    const int g2 = (int)std::min<int64_t>(nt2, (int64_t)mlp_cu_count() * 2);
    if (D == 256) hipLaunchKernelGGL((mlp_bwdp2_k<256>), dim3(g2), dim3(256), (size_t)HID * 4, s, a);
    else hipLaunchKernelGGL((mlp_bwdp2_k<128>), dim3(g2), dim3(256), (size_t)HID * 4, s, a);
    LTHM_CHECK_LAUNCH();
    return 0;
  }
  constexpr int NW = 8;
  const int64_t ntiles = (M + 32 * NW - 1) / (32 * NW);
  const int grid = (int)std::min<int64_t>(ntiles, (int64_t)mlp_cu_count());
  if (D == 256) hipLaunchKernelGGL((mlp_bwdp_k<256, NW>), dim3(grid), dim3(64 * NW), 0, s, a);
  else hipLaunchKernelGGL((mlp_bwdp_k<128, NW>), dim3(grid), dim3(64 * NW), 0, s, a);
  LTHM_CHECK_LAUNCH();
  return 0;
}
