// Shared device helpers for the LTHM gfx950 kernels.
//
// Everything here is written for CDNA4 (wave64, MFMA, 160 KiB LDS); there is no
// dual-platform path.  bf16 values travel as raw uint16_t so that every load and
// store is an explicit, vectorisable integer access (cdna_hip_programming.md G13).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lthm.h"

#define LTHM_WAVE 64

namespace lthm {

typedef uint16_t bf16_t;

// ---- XCD-aware block order ----
// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup
// dispatch): remap the linear block id so that each XCD walks a contiguous range
// of logical ids (neighbouring tiles share its L2).  Bijective for any nwg; a
// speed choice only, never needed for correctness.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// ---- bf16 <-> f32 (round-to-nearest-even, NaN stays NaN; identical to torch) ----
// f32 -> bf16 is gfx950's v_cvt_pk_bf16_f32 (RNE, two values per instruction).
typedef __bf16 bf16x2_hw __attribute__((ext_vector_type(2)));
typedef float f32x2_hw __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_hw{lo, hi}, bf16x2_hw));
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  return (bf16_t)(pack_bf16x2(f, 0.f) & 0xffffu);
}

// generic element load/store as f32
template <typename T> struct Elem;
template <> struct Elem<float> {
  __device__ __forceinline__ static float ld(const float* p) { return *p; }
  __device__ __forceinline__ static void st(float* p, float v) { *p = v; }
};
template <> struct Elem<bf16_t> {
  __device__ __forceinline__ static float ld(const bf16_t* p) { return bf2f(*p); }
  __device__ __forceinline__ static void st(bf16_t* p, float v) { *p = f2bf(v); }
};

// 16-byte vector of T (4 x f32 or 8 x bf16)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Load VB bytes (4/8/16) starting at p as f32 values into out[0..VB/sizeof(T))
template <typename T, int VB>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, float* out) {
  constexpr int N = VB / (int)sizeof(T);
  if constexpr (sizeof(T) == 4) {
    if constexpr (VB == 16) {
      f32x4 v = *reinterpret_cast<const f32x4*>(p);
      out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
    } else if constexpr (VB == 8) {
      float2 v = *reinterpret_cast<const float2*>(p);
      out[0] = v.x; out[1] = v.y;
    } else {
      out[0] = *reinterpret_cast<const float*>(p);
    }
  } else {
    if constexpr (VB == 16) {
      u32x4 v = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        out[2 * i] = __uint_as_float(v[i] << 16);
        out[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
      }
    } else if constexpr (VB == 8) {
      u32x2 v = *reinterpret_cast<const u32x2*>(p);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        out[2 * i] = __uint_as_float(v[i] << 16);
        out[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
      }
    } else {
      uint32_t v = *reinterpret_cast<const uint32_t*>(p);
      out[0] = __uint_as_float(v << 16);
      out[1] = __uint_as_float(v & 0xffff0000u);
    }
  }
  (void)N;
}

template <typename T, int N>
__device__ __forceinline__ void store_vec(T* __restrict__ p, const float* v) {
  if constexpr (sizeof(T) == 4) {
    if constexpr (N == 4) {
      *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    } else if constexpr (N == 2) {
      *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) p[i] = v[i];
    }
  } else {
    if constexpr (N == 8) {
      u32x4 w;
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = pack_bf16x2(v[2 * i], v[2 * i + 1]);
      *reinterpret_cast<u32x4*>(p) = w;
    } else if constexpr (N == 4) {
      u32x2 w;
#pragma unroll
      for (int i = 0; i < 2; ++i) w[i] = pack_bf16x2(v[2 * i], v[2 * i + 1]);
      *reinterpret_cast<u32x2*>(p) = w;
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) p[i] = f2bf(v[i]);
    }
  }
}

// ---- activations (GEMM epilogues, fused MLP) ----
// tanh-GELU through r = 1 / (e^(2u) + 1), u = sqrt(2/pi) (x + 0.044715 x^3):
// tanh(u) = 1 - 2r, so gelu(x) = 0.5 x (1 + tanh u) = x (1 - r) and
// gelu'(x) = (1 - r) (1 + 2 sqrt(2/pi) x r (1 + 3 * 0.044715 x^2)).
// One v_exp + one v_rcp per element (|error| ~ 1e-7 absolute); saturates
// correctly for large |x| (exp2 -> inf gives r = 0, exp2 -> 0 gives r = 1).
__device__ __forceinline__ float gelu_r(float x) {
  constexpr float kb2 = 2.f * 1.4426950408889634f * 0.7978845608028654f;   // 2 log2(e) sqrt(2/pi)
  constexpr float kk2 = kb2 * 0.044715f;
  return __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x * __builtin_fmaf(kk2, x * x, kb2)) + 1.f);
}
__device__ __forceinline__ float gelu_tanh(float x) { return __builtin_fmaf(-x, gelu_r(x), x); }
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  constexpr float kb = 0.7978845608028654f, k3 = 3.f * 0.044715f;
  const float r = gelu_r(x);
  return (1.f - r) * __builtin_fmaf(2.f * kb * x * r, __builtin_fmaf(k3, x * x, 1.f), 1.f);
}
// gelu(x) and gelu'(x) from one v_exp + one v_rcp (the forward that saves the
// derivative for the backward's plain multiply, LTHM_ACT_GELU_D)
__device__ __forceinline__ float gelu_tanh_and_grad(float x, float& dg) {
  constexpr float kb = 0.7978845608028654f, k3 = 3.f * 0.044715f;
  const float r = gelu_r(x), q = 1.f - r;
  dg = q * __builtin_fmaf(2.f * kb * x * r, __builtin_fmaf(k3, x * x, 1.f), 1.f);
  return x * q;
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float qgelu(float x) { return x * sigmoidf_(1.702f * x); }
__device__ __forceinline__ float qgelu_grad(float x) {
  const float s = sigmoidf_(1.702f * x);
  return s + 1.702f * x * s * (1.f - s);
}

// ---- wave reductions (64 lanes) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reduce inside aligned groups of G lanes (G power of two <= 64)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- KShift row index, bit-identical to commons/layers.py:174-185 ----
// c == 0: x mod P ; c >= 1: ((x << c) | (x >> (64 - c))) mod P with a wrapping
// left shift, an ARITHMETIC right shift on signed int64 and Python-style
// (non-negative) remainder (torch.remainder).
__device__ __host__ __forceinline__ int64_t kshift_row(int64_t x, int c, int64_t P) {
  int64_t y = x;
  if (c != 0) {
    uint64_t ux = (uint64_t)x;
    uint64_t hi = ux << c;
    uint64_t lo = (uint64_t)(x >> (64 - c));  // arithmetic shift: sign fill
    y = (int64_t)(hi | lo);
  }
  int64_t r = y % P;
  if (r < 0) r += P;
  return r;
}

// Python-style floor division + remainder for int64 (PatternFromTimelocal, QR)
__device__ __host__ __forceinline__ int64_t floordiv64(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}
__device__ __host__ __forceinline__ int64_t pymod64(int64_t a, int64_t b) {
  int64_t r = a % b;
  if (r != 0 && ((r < 0) != (b < 0))) r += b;
  return r;
}

// ---- LDS-DMA (global_load_lds_dwordx4) ----
typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

// LDS-DMA issued as asm: the compiler neither counts these loads nor guards LDS
// reads against them (the builtin makes it drain vmcnt(0) before unrelated LDS
// reads); the kernels retire them with explicit counted waits + a barrier.
// Ordinary loads stay correct: in-order vmcnt only makes their waits stricter.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lvoid_t*)p);
}
__device__ __forceinline__ void glds16(const void* src, void* lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds_addr(lds)) : "memory");
}
__device__ __forceinline__ void glds4(const void* src, void* lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds_addr(lds)) : "memory");
}
// glds16 with the LDS byte address already in hand (wave-uniform, e.g. a base read once by
// lds_addr plus constants): no per-call address-space cast or readfirstlane
__device__ __forceinline__ void glds16_m0(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// retire every ordinary load issued so far, visibly to the compiler's own wait
// bookkeeping (vmcnt(0), expcnt / lgkmcnt untouched): issued before the DMA
// prologue, so no first use inside the tile loop drains the DMA ring
__device__ __forceinline__ void retire_loads() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__host__ __forceinline__ int grid_for(int64_t work, int per_block, int cap = 256 * 16) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace lthm

#define LTHM_CHECK_LAUNCH() \
  do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)
#define LTHM_REQUIRE(cond) \
  do { if (!(cond)) return (int)hipErrorInvalidValue; } while (0)
