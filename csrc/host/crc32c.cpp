// CRC-32C (Castagnoli) for Kafka RecordBatch v2 checksums: the SSE4.2 crc32 instruction
// when the CPU has it (checked at run time: ≈ 8 B/cycle vs 1.3 GB/s for the table form),
// slicing-by-8 tables otherwise.
#include <cstddef>
#include <cstdint>
#include <cstring>

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

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint64_t crc_run(uint64_t c, const uint8_t* p, int64_t n) {
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = uint32_t(c);
  while (n-- > 0) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}

// Three independent crc32 chains over consecutive kLane-byte stripes hide the instruction's
// 3-cycle latency; the chains are joined with the linear map "advance the register over
// kLane zero bytes" (4 × 256-entry tables per power, built once from its 32 basis images).
constexpr int64_t kLane = 4096;
struct Shift {
  uint32_t t[4][256];
  void build(int64_t zeros) {
    static const uint8_t z[kLane] = {};
    uint32_t basis[32];
    for (int b = 0; b < 32; ++b) {
      uint64_t c = uint32_t(1u << b);
      for (int64_t left = zeros; left > 0; left -= kLane) c = crc_run(c, z, left < kLane ? left : kLane);
      basis[b] = uint32_t(c);
    }
    for (int k = 0; k < 4; ++k)
      for (int v = 0; v < 256; ++v) {
        uint32_t r = 0;
        for (int b = 0; b < 8; ++b)
          if (v >> b & 1) r ^= basis[8 * k + b];
        t[k][v] = r;
      }
  }
  uint32_t operator()(uint32_t x) const {
    return t[0][x & 255] ^ t[1][(x >> 8) & 255] ^ t[2][(x >> 16) & 255] ^ t[3][x >> 24];
  }
};

struct HwCrc {
  bool ok = false;
  Shift s1, s2;
  HwCrc() {
    __builtin_cpu_init();  // static initialisers may run before libgcc's CPU model is set up
    ok = __builtin_cpu_supports("sse4.2");
    if (ok) {
      s1.build(kLane);
      s2.build(2 * kLane);
    }
  }
};
const HwCrc kHw;

__attribute__((target("sse4.2"))) uint32_t crc32c_hw(const uint8_t* p, int64_t n, uint32_t crc) {
  uint64_t c = uint32_t(~crc);
  while (n >= 3 * kLane) {
    uint64_t a = c, b = 0, d = 0;
    const uint8_t* q = p;
    for (int64_t i = 0; i < kLane; i += 8, q += 8) {
      uint64_t va, vb, vd;
      std::memcpy(&va, q, 8);
      std::memcpy(&vb, q + kLane, 8);
      std::memcpy(&vd, q + 2 * kLane, 8);
      a = __builtin_ia32_crc32di(a, va);
      b = __builtin_ia32_crc32di(b, vb);
      d = __builtin_ia32_crc32di(d, vd);
    }
    c = kHw.s2(uint32_t(a)) ^ kHw.s1(uint32_t(b)) ^ uint32_t(d);
    p += 3 * kLane;
    n -= 3 * kLane;
  }
  return ~uint32_t(crc_run(c, p, n));
}
#endif
}  // namespace

OMLDM_HOST_API uint32_t omldm_crc32c(const uint8_t* p, int64_t n, uint32_t crc) {
#if defined(__x86_64__)
  if (kHw.ok) return crc32c_hw(p, n, crc);
#endif
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
