// DIB: the binary DataInstance record of the topic logs. Decoded by csrc/host/ingest.cpp
// (parse_dib), rendered back to JSON by csrc/host/egress.cpp (forecast echoes), parsed on
// the GPU by csrc/kernels/json_ingest.hip; written by omldm_json_to_dib (ingest.cpp) and
// omldm_amd/io/dib.py.
//
// A DataInstance in binary ("DIB1"), newline-safe so it shares the topic logs' line
// framing with JSON records: byte 0xB1, then the payload SLIP-stuffed (0x0A → DB DC,
// 0xDB → DB DD), then the log's '\n'. Payload, little-endian:
//   u8 op (0 training, 1 forecasting, else invalid) | u8 flags (bit 0 target present,
//   bit 1 features present) | u8 nn | u8 nd | u8 nc | [f32 target] | f32 num[nn] |
//   f32 disc[nd] | u32 cat[nc]
// cat[j] = murmur3_32(category string j, kSeedBase + j): the hash the JSON parser takes of
// the string, so a DIB record and its JSON text hash to the same slots in every feature
// space. 13 numerical + 26 categorical features: 161 B + stuffing (≈ 1.3 B) vs ≈ 507 B of
// JSON text.
#pragma once
#include <cstdint>
#include <cstring>

namespace omldm_dib {

constexpr uint8_t kMagic = 0xB1;

struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  uint8_t get() {
    if (p >= e) return ok = false, 0;
    uint8_t c = *p++;
    if (c == 0xDB) {
      if (p >= e) return ok = false, 0;
      const uint8_t d = *p++;
      if (d == 0xDC) c = 0x0A;
      else if (d == 0xDD) c = 0xDB;
      else return ok = false, 0;
    }
    return c;
  }
  uint32_t get32() {
    uint32_t v = get();
    v |= uint32_t(get()) << 8;
    v |= uint32_t(get()) << 16;
    v |= uint32_t(get()) << 24;
    return v;
  }
  float getf() {
    const uint32_t u = get32();
    float f;
    std::memcpy(&f, &u, 4);
    return f;
  }
};

}  // namespace omldm_dib
