// Vocabulary hash table layout shared by the host loader (loader.cpp, g++) and the device
// bucketing kernels (bucketize.hip): the same 64-bit key hash and the same slot image, so a table
// built on the host is probed on the GPU unchanged (rk_vocab_export -> device copy).
#ifndef RANKOPS_VOCAB_HASH_H
#define RANKOPS_VOCAB_HASH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RK_HD __host__ __device__ __forceinline__
#else
#define RK_HD inline
#endif

namespace rk {

// One open-addressing slot (linear probing, power-of-two capacity): key bytes live at
// arena[off, off + len); idx < 0 marks an empty slot.  24 bytes, 8-byte aligned.
struct VocabSlot {
  uint64_t h;
  int64_t idx;
  uint32_t off, len;
};

// Little-endian load of n <= 8 bytes (zero-extended).
RK_HD uint64_t load_le(const char* p, uint32_t n) {
  uint64_t w = 0;
  for (uint32_t i = 0; i < n; ++i) w |= (uint64_t)(unsigned char)p[i] << (8 * i);
  return w;
}

RK_HD uint64_t vocab_hash(const char* p, uint32_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)n * 0xFF51AFD7ED558CCDull);
  while (n >= 8) {
    h = (h ^ load_le(p, 8)) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    p += 8;
    n -= 8;
  }
  h = (h ^ load_le(p, n) ^ ((uint64_t)n << 56)) * 0xBF58476D1CE4E5B9ull;
  h ^= h >> 31;
  h *= 0x94D049BB133111EBull;
  h ^= h >> 29;
  return h;
}

RK_HD bool bytes_equal(const char* a, const char* b, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// Row of key k (0 when absent: hazard H1).
RK_HD int64_t vocab_find(const VocabSlot* slots, uint64_t mask, const char* arena, const char* k, uint32_t n) {
  const uint64_t h = vocab_hash(k, n);
  for (uint64_t s = h & mask;; s = (s + 1) & mask) {
    const VocabSlot e = slots[s];
    if (e.idx < 0) return 0;
    if (e.h == h && e.len == n && bytes_equal(arena + e.off, k, n)) return e.idx;
  }
}

}  // namespace rk

#endif  // RANKOPS_VOCAB_HASH_H
