// CRC-32C (Castagnoli) for Kafka RecordBatch v2 checksums (slicing-by-8, no intrinsics
// so the host library stays portable across the build and GPU hosts).
#include <cstddef>
#include <cstdint>

#define OMLDM_HOST_API extern "C" __attribute__((visibility("default")))

namespace {
struct Table {
  uint32_t t[8][256];
  Table() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};
const Table kT;
}  // namespace

OMLDM_HOST_API uint32_t omldm_crc32c(const uint8_t* p, int64_t n, uint32_t crc) {
  crc = ~crc;
  while (n >= 8) {
    uint32_t lo = (uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 |
                   uint32_t(p[3]) << 24) ^ crc;
    uint32_t hi = uint32_t(p[4]) | uint32_t(p[5]) << 8 | uint32_t(p[6]) << 16 |
                  uint32_t(p[7]) << 24;
    crc = kT.t[7][lo & 0xFF] ^ kT.t[6][(lo >> 8) & 0xFF] ^ kT.t[5][(lo >> 16) & 0xFF] ^
          kT.t[4][lo >> 24] ^ kT.t[3][hi & 0xFF] ^ kT.t[2][(hi >> 8) & 0xFF] ^
          kT.t[1][(hi >> 16) & 0xFF] ^ kT.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n-- > 0) crc = kT.t[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return ~crc;
}
