// XXH32 / XXH64 (the published xxHash algorithms, v0.8 "classic" variants) as
// host+device functions, for the id ingest of commons/feature_utils.py:36-46:
//   hash_feature_name_to_int(name)      = xxh32(lower(name), seed 0)
//   hash_string_to_long(v, seed, lower) = xxh64(str(v), seed) - 2^63  (as int64)
// Reference dependency: python-xxhash 3.5.0 (uv.lock:902-903), whose xxh32 /
// xxh64 intdigest() are these functions; pinned by tests/golden/hashing.npz.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lthm {
namespace xxh {

constexpr uint32_t P32_1 = 0x9E3779B1u, P32_2 = 0x85EBCA77u, P32_3 = 0xC2B2AE3Du, P32_4 = 0x27D4EB2Fu,
                   P32_5 = 0x165667B1u;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full, P64_3 = 0x165667B19E3779F9ull,
                   P64_4 = 0x85EBCA77C2B2AE63ull, P64_5 = 0x27D4EB2F165667C5ull;

__host__ __device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__host__ __device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// little-endian unaligned reads (gfx950 and x86-64 are little-endian)
__host__ __device__ __forceinline__ uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__host__ __device__ __forceinline__ uint64_t rd64(const uint8_t* p) {
  return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32);
}

__host__ __device__ __forceinline__ uint32_t round32(uint32_t acc, uint32_t in) {
  acc += in * P32_2;
  acc = rotl32(acc, 13);
  return acc * P32_1;
}

__host__ __device__ inline uint32_t xxh32(const uint8_t* p, int64_t len, uint32_t seed) {
  const uint8_t* end = p + len;
  uint32_t h;
  if (len >= 16) {
    uint32_t v1 = seed + P32_1 + P32_2, v2 = seed + P32_2, v3 = seed, v4 = seed - P32_1;
    const uint8_t* lim = end - 16;
    do {
      v1 = round32(v1, rd32(p));
      v2 = round32(v2, rd32(p + 4));
      v3 = round32(v3, rd32(p + 8));
      v4 = round32(v4, rd32(p + 12));
      p += 16;
    } while (p <= lim);
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  } else {
    h = seed + P32_5;
  }
  h += (uint32_t)len;
  while (p + 4 <= end) {
    h += rd32(p) * P32_3;
    h = rotl32(h, 17) * P32_4;
    p += 4;
  }
  while (p < end) {
    h += (uint32_t)(*p) * P32_5;
    h = rotl32(h, 11) * P32_1;
    ++p;
  }
  h ^= h >> 15;
  h *= P32_2;
  h ^= h >> 13;
  h *= P32_3;
  h ^= h >> 16;
  return h;
}

__host__ __device__ __forceinline__ uint64_t round64(uint64_t acc, uint64_t in) {
  acc += in * P64_2;
  acc = rotl64(acc, 31);
  return acc * P64_1;
}
__host__ __device__ __forceinline__ uint64_t merge64(uint64_t acc, uint64_t v) {
  acc ^= round64(0, v);
  return acc * P64_1 + P64_4;
}

__host__ __device__ inline uint64_t xxh64(const uint8_t* p, int64_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed, v4 = seed - P64_1;
    const uint8_t* lim = end - 32;
    do {
      v1 = round64(v1, rd64(p));
      v2 = round64(v2, rd64(p + 8));
      v3 = round64(v3, rd64(p + 16));
      v4 = round64(v4, rd64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = merge64(h, v1);
    h = merge64(h, v2);
    h = merge64(h, v3);
    h = merge64(h, v4);
  } else {
    h = seed + P64_5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= round64(0, rd64(p));
    h = rotl64(h, 27) * P64_1 + P64_4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32(p) * P64_1;
    h = rotl64(h, 23) * P64_2 + P64_3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * P64_5;
    h = rotl64(h, 11) * P64_1;
    ++p;
  }
  h ^= h >> 33;
  h *= P64_2;
  h ^= h >> 29;
  h *= P64_3;
  h ^= h >> 32;
  return h;
}

// Python str(int) of an int64: decimal digits with a leading '-'; returns the length
__host__ __device__ inline int format_int64(int64_t v, uint8_t* buf /* >= 20 */) {
  uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1u : (uint64_t)v;
  uint8_t tmp[20];
  int n = 0;
  do {
    tmp[n++] = (uint8_t)('0' + (u % 10u));
    u /= 10u;
  } while (u);
  int k = 0;
  if (v < 0) buf[k++] = '-';
  while (n) buf[k++] = tmp[--n];
  return k;
}

// xxh64 - 2^63 as the int64 torch ids (feature_utils.py:46)
__host__ __device__ __forceinline__ int64_t to_id(uint64_t h) { return (int64_t)(h ^ 0x8000000000000000ull); }

}  // namespace xxh
}  // namespace lthm
