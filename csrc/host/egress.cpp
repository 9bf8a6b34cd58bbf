// Prediction egress: one call renders a whole forecast batch as Prediction JSON lines.
//
// Reference: every forecast becomes a `Prediction` object sunk to the predictions topic
// with toString (omldm/network/FlinkNetwork.scala:243-257, omldm/Job.scala:99-105); the
// prediction echoes the forecasting DataInstance kept on purpose by the parser
// (omldm/utils/parsers/dataStream/DataPointParser.scala:38-40,45-46). Here the echo is
// the record's raw bytes, copied straight from the tick's staging block, and the
// number is printed with the shortest round-trip representation (std::to_chars, the
// same digits as Python's repr / json.dumps).
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "dib.h"

#define OMLDM_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

inline bool is_ws(uint8_t c) { return c == ' ' || c == '\n' || c == '\r' || c == '\t'; }

// JSON number as Python's json.dumps prints a float: shortest round trip, ".0" added to
// integral values, NaN / Infinity / -Infinity for the non-finite ones.
int format_number(double v, char* p) {
  if (std::isnan(v)) { std::memcpy(p, "NaN", 3); return 3; }
  if (std::isinf(v)) {
    if (v < 0) { std::memcpy(p, "-Infinity", 9); return 9; }
    std::memcpy(p, "Infinity", 8);
    return 8;
  }
  auto r = std::to_chars(p, p + 40, v);
  int n = int(r.ptr - p);
  bool has_dot = false;
  for (int i = 0; i < n; ++i)
    if (p[i] == '.' || p[i] == 'e' || p[i] == 'E') has_dot = true;
  if (!has_dot) { p[n++] = '.'; p[n++] = '0'; }
  return n;
}

// A DIB record's echo as DataInstance JSON: its features (the categorical ones as the
// 32-bit hashes the record carries, "#%08x"), target and operation. Returns bytes written.
int render_dib(const uint8_t* a, const uint8_t* b, char* out) {
  omldm_dib::Reader r{a + 1, b};
  const uint8_t op = r.get(), flags = r.get(), nn = r.get(), nd = r.get(), nc = r.get();
  const float y = (flags & 1) ? r.getf() : 0.f;
  int pos = 0;
  auto put = [&](const char* t) {
    const size_t n = std::strlen(t);
    std::memcpy(out + pos, t, n);
    pos += int(n);
  };
  for (int arr = 0; arr < 2; ++arr) {
    put(arr == 0 ? "{\"numericalFeatures\": [" : "], \"discreteFeatures\": [");
    const int cnt = arr == 0 ? nn : nd;
    for (int j = 0; j < cnt; ++j) {
      if (j) put(", ");
      pos += format_number(double(r.getf()), out + pos);
    }
  }
  put("], \"categoricalFeatures\": [");
  static const char hx[] = "0123456789abcdef";
  for (int j = 0; j < nc; ++j) {
    const uint32_t h = r.get32();
    put(j ? ", \"#" : "\"#");
    for (int k = 7; k >= 0; --k) out[pos++] = hx[(h >> (4 * k)) & 15];
    out[pos++] = '"';
  }
  put("]");
  if (flags & 1) {
    put(", \"target\": ");
    pos += format_number(double(y), out + pos);
  }
  put(op == 0 ? ", \"operation\": \"training\"}" : ", \"operation\": \"forecasting\"}");
  return pos;
}

// JSON: surrounding whitespace; DIB: only the log's '\n' (payload bytes may be 0x20 …)
inline void trim(const uint8_t* buf, int64_t& a, int64_t& b) {
  while (a < b && is_ws(buf[a])) ++a;
  if (a < b && buf[a] == omldm_dib::kMagic) {
    if (buf[b - 1] == '\n') --b;
    return;
  }
  while (b > a && is_ws(buf[b - 1])) --b;
}

inline int64_t dib_bound(int64_t bytes) { return bytes * 10 + 160; }

}  // namespace

// Renders record i as {"mlpId": id, "dataPoint": <buf[starts[i], ends[i]) trimmed>,
// "prediction": preds[i]}\n into out. out_offs[0..n] receive the line boundaries.
// Returns the bytes written, or -(bytes needed) when cap is too small (nothing usable
// is written then; call again with a bigger buffer).
OMLDM_HOST_API int64_t omldm_format_predictions(const uint8_t* buf, const int64_t* starts,
                                                const int64_t* ends, int64_t n, int mlp_id,
                                                const float* preds, uint8_t* out, int64_t cap,
                                                int64_t* out_offs) {
  static const char k0[] = "{\"mlpId\": ";
  static const char k1[] = ", \"dataPoint\": ";
  static const char k2[] = ", \"prediction\": ";
  char idbuf[16];
  const int idn = int(std::to_chars(idbuf, idbuf + 16, mlp_id).ptr - idbuf);
  int64_t need = 0;
  for (int64_t i = 0; i < n; ++i) {
    int64_t a = starts[i], b = ends[i];
    trim(buf, a, b);
    const int64_t body = b - a > 0 ? (buf[a] == omldm_dib::kMagic ? dib_bound(b - a) : b - a) : 4;
    need += (sizeof(k0) - 1) + idn + (sizeof(k1) - 1) + body + (sizeof(k2) - 1) + 40 + 2;
  }
  if (need > cap) return -need;
  int64_t pos = 0;
  out_offs[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    int64_t a = starts[i], b = ends[i];
    trim(buf, a, b);
    std::memcpy(out + pos, k0, sizeof(k0) - 1);
    pos += sizeof(k0) - 1;
    std::memcpy(out + pos, idbuf, idn);
    pos += idn;
    std::memcpy(out + pos, k1, sizeof(k1) - 1);
    pos += sizeof(k1) - 1;
    if (b > a && buf[a] == omldm_dib::kMagic) {
      pos += render_dib(buf + a, buf + b, reinterpret_cast<char*>(out + pos));
    } else if (b > a) {
      std::memcpy(out + pos, buf + a, size_t(b - a));
      pos += b - a;
    } else {
      std::memcpy(out + pos, "null", 4);
      pos += 4;
    }
    std::memcpy(out + pos, k2, sizeof(k2) - 1);
    pos += sizeof(k2) - 1;
    pos += format_number(double(preds[i]), reinterpret_cast<char*>(out + pos));
    out[pos++] = '}';
    out[pos++] = '\n';
    out_offs[i + 1] = pos;
  }
  return pos;
}
