// Shared pieces of the training kernels: the counter-hash dropout mask (train_bn.hip header
// comment) used by the BatchNorm units, the DIN fcn and the BST blocks.
#pragma once

#include "common.h"

namespace rk {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// keep(i) for element i of a mask drawn with (seed, stream): drop with probability threshold / 2^32
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t stream, uint64_t i, uint32_t threshold) {
  const uint64_t h = mix64(seed ^ mix64(stream * 0x9E3779B97F4A7C15ull + i));
  return (uint32_t)(h >> 32) >= threshold;
}

static inline uint32_t dropout_threshold(double p) {
  if (!(p > 0.0)) return 0;
  const double t = p * 4294967296.0;
  return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

}  // namespace rk
