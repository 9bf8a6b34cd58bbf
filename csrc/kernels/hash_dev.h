// Device copy of the raw-wire feature hash of csrc/host/hashing.h (murmur3_32 of a
// categorical token's 4 little-endian bytes, one seed per field → field-aware signed slot).
// tests/test_rawwire.py pins GPU == CPU slot for every field.
#pragma once
#include <stdint.h>

namespace omldm {

constexpr uint32_t kHashSeedBase = 0x9747b28cu;
constexpr uint32_t kAbsentToken = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t rotl32d(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// murmur3_32 of exactly 4 bytes (one block, no tail)
__device__ __forceinline__ uint32_t murmur3_u32(uint32_t k1, uint32_t seed) {
  k1 *= 0xcc9e2d51u;
  k1 = rotl32d(k1, 15);
  k1 *= 0x1b873593u;
  uint32_t h1 = seed ^ k1;
  h1 = rotl32d(h1, 13);
  h1 = h1 * 5u + 0xe6546b64u;
  h1 ^= 4u;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  h1 ^= h1 >> 16;
  return h1;
}

// token of field f → slot | sign << 31 (−1 when absent), field-aware (hashing.h:
// hash_token): slot = dn + f·span + (h & 0x7fffffff) mod span, span = (dim − dn − 1) / dc.
__device__ __forceinline__ int hash_token_dev(uint32_t tok, int field, int dn, uint32_t span) {
  if (tok == kAbsentToken) return -1;
  const uint32_t h = murmur3_u32(tok, kHashSeedBase + (uint32_t)field);
  const uint32_t slot = (uint32_t)dn + (uint32_t)field * span + (h & 0x7fffffffu) % span;
  return (int)(slot | (h & 0x80000000u));
}

}  // namespace omldm
