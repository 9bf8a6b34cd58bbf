// Feature hashing shared by the host data plane (JSON parser, raw binary wire, CPU
// learners). The device copy lives in csrc/kernels/hash_dev.h; tests pin that both give
// identical slots (tests/test_rawwire.py).
//
// Reference: DataPointParser turns categorical strings into a feature vector
// (omldm/utils/parsers/dataStream/DataPointParser.scala:21-36); here every categorical
// value is hashed (murmur3_32, one seed per field) into a signed slot of the 2^k model.
#pragma once
#include <cstdint>
#include <cstring>

namespace omldm_hash {

inline uint32_t rotl32(uint32_t x, int8_t r) { return (x << r) | (x >> (32 - r)); }

inline uint32_t murmur3_32(const uint8_t* data, size_t len, uint32_t seed) {
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  uint32_t h1 = seed;
  const size_t nblocks = len / 4;
  for (size_t i = 0; i < nblocks; ++i) {
    uint32_t k1;
    std::memcpy(&k1, data + i * 4, 4);
    k1 *= c1;
    k1 = rotl32(k1, 15);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    h1 = h1 * 5 + 0xe6546b64u;
  }
  const uint8_t* tail = data + nblocks * 4;
  uint32_t k1 = 0;
  switch (len & 3) {
    case 3: k1 ^= uint32_t(tail[2]) << 16; [[fallthrough]];
    case 2: k1 ^= uint32_t(tail[1]) << 8; [[fallthrough]];
    case 1:
      k1 ^= tail[0];
      k1 *= c1;
      k1 = rotl32(k1, 15);
      k1 *= c2;
      h1 ^= k1;
  }
  h1 ^= uint32_t(len);
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  h1 ^= h1 >> 16;
  return h1;
}

constexpr uint32_t kSeedBase = 0x9747b28cu;

// Categorical token → signed slot in [dn, dim − 1) (slot dim − 1 is the intercept), sign
// in bit 31. Field j has its own seed, so one token in two fields lands in two slots.
inline int32_t hash_cat(const uint8_t* s, size_t n, int field, int dn, int64_t dim) {
  const uint32_t h = murmur3_32(s, n, kSeedBase + uint32_t(field));
  const int64_t span = dim - dn - 1;
  const int32_t slot = int32_t(dn + int64_t(h & 0x7fffffffu) % span);
  return (h & 0x80000000u) ? int32_t(uint32_t(slot) | 0x80000000u) : slot;
}

// Raw binary wire: a categorical value is a 32-bit token id (0xFFFFFFFF = absent),
// murmur3-hashed as its 4 little-endian bytes with the field's seed, FIELD-AWARE: field f
// owns the slot range [dn + f·span, dn + (f+1)·span), span = (dim − dn − 1) / dc (at
// 2^20 dims and 26 fields: 40,329 slots per field, 99.999 % of the model used). Equal
// slots therefore always come from the same field — what lets the GPU round group a
// chunk's shared values field by field without atomics (csrc/kernels/linear_seq.hip).
constexpr uint32_t kAbsentToken = 0xFFFFFFFFu;

inline int64_t field_span(int dn, int dc, int64_t dim) {
  return dc > 0 ? (dim - dn - 1) / dc : 0;
}

inline int32_t hash_token(uint32_t tok, int field, int dn, int dc, int64_t dim) {
  uint8_t b[4];
  std::memcpy(b, &tok, 4);
  const uint32_t h = murmur3_32(b, 4, kSeedBase + uint32_t(field));
  const int64_t span = field_span(dn, dc, dim);
  const int32_t slot = int32_t(dn + int64_t(field) * span + int64_t(h & 0x7fffffffu) % span);
  return (h & 0x80000000u) ? int32_t(uint32_t(slot) | 0x80000000u) : slot;
}

}  // namespace omldm_hash
