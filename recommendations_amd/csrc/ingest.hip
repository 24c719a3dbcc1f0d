// Id ingest (commons/feature_utils.py:21-46, 136-183): xxHash feature seeds and
// id hashes, the categorical-history hash / drop-label / cap / pad pass, and a
// device kernel hashing numeric ids (their Python str()) straight into the
// int64 [B, T] batch the hot path consumes.  Host entry points run on the CPU
// cores of the data path (the reference does this in pandas .apply loops);
// they own no state and are thread-safe.
#include <string.h>

#include "common.hpp"
#include "xxhash.hpp"

namespace lthm {

__global__ void hash_int64_str_k(const int64_t* __restrict__ vals, int64_t n, uint64_t seed, int64_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint8_t buf[20];
    const int len = xxh::format_int64(vals[i], buf);
    out[i] = xxh::to_id(xxh::xxh64(buf, len, seed));
  }
}

static inline bool ascii_lower(const uint8_t* s, int64_t len, uint8_t* dst) {
  for (int64_t i = 0; i < len; ++i) {
    const uint8_t c = s[i];
    if (c >= 0x80) return false;  // non-ASCII: Unicode lowering is left to the caller
    dst[i] = (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c;
  }
  return true;
}

}  // namespace lthm

using namespace lthm;

extern "C" {

uint32_t lthm_xxh32(const void* data, int64_t len, uint32_t seed) {
  return xxh::xxh32(reinterpret_cast<const uint8_t*>(data), len, seed);
}

uint64_t lthm_xxh64(const void* data, int64_t len, uint64_t seed) {
  return xxh::xxh64(reinterpret_cast<const uint8_t*>(data), len, seed);
}

int64_t lthm_hash_strings(const uint8_t* bytes, const int64_t* offsets, int64_t n, uint64_t seed, int32_t to_lower,
                          int64_t* out, uint8_t* needs_unicode_lower) {
  if (n < 0 || (n > 0 && (!bytes || !offsets || !out))) return -1;
  int64_t flagged = 0;
  uint8_t small[256];
  for (int64_t i = 0; i < n; ++i) {
    const int64_t a = offsets[i], len = offsets[i + 1] - offsets[i];
    if (len < 0) return -1;
    const uint8_t* s = bytes + a;
    if (needs_unicode_lower) needs_unicode_lower[i] = 0;
    if (to_lower) {
      uint8_t* tmp = len <= (int64_t)sizeof(small) ? small : (uint8_t*)malloc((size_t)len);
      if (!tmp) return -1;
      const bool ok = ascii_lower(s, len, tmp);
      if (ok) out[i] = xxh::to_id(xxh::xxh64(tmp, len, seed));
      if (tmp != small) free(tmp);
      if (!ok) {
        if (needs_unicode_lower) needs_unicode_lower[i] = 1;
        ++flagged;
      }
    } else {
      out[i] = xxh::to_id(xxh::xxh64(s, len, seed));
    }
  }
  return flagged;
}

int lthm_hash_int64_str(const int64_t* vals, int64_t n, uint64_t seed, int64_t* out) {
  if (n < 0 || (n > 0 && (!vals || !out))) return 1;
  uint8_t buf[20];
  for (int64_t i = 0; i < n; ++i) {
    const int len = xxh::format_int64(vals[i], buf);
    out[i] = xxh::to_id(xxh::xxh64(buf, len, seed));
  }
  return 0;
}

int lthm_hash_int64_str_dev(const int64_t* vals, int64_t n, uint64_t seed, int64_t* out, void* stream) {
  LTHM_REQUIRE(n >= 0);
  if (n == 0) return 0;
  hipLaunchKernelGGL(hash_int64_str_k, dim3(grid_for(n, 256, 256 * 32)), dim3(256), 0, (hipStream_t)stream, vals, n,
                     seed, out);
  LTHM_CHECK_LAUNCH();
  return 0;
}

int lthm_history_pad(const int64_t* items, const int64_t* row_offsets, int64_t n_rows, const int64_t* history_id,
                     int32_t remove_history_id, int32_t length, int64_t pad, int64_t* out) {
  if (n_rows < 0 || length < 0 || (remove_history_id && !history_id)) return 1;
  for (int64_t r = 0; r < n_rows; ++r) {
    int64_t* o = out + r * length;
    int found = 0;
    for (int64_t i = row_offsets[r]; i < row_offsets[r + 1] && found < length; ++i) {
      const int64_t h = items[i];
      if (remove_history_id && h == history_id[r]) continue;
      o[found++] = h;
    }
    for (int k = found; k < length; ++k) o[k] = pad;
  }
  return 0;
}

}  // extern "C"
