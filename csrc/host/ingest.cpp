// Host-side data plane: DataInstance JSON → hashed fixed-width batch, feature hashing,
// and a deterministic synthetic stream generator.
//
// Reference path being replaced: Kafka JSON → Jackson `DataInstance`
// (omldm/utils/parsers/DataInstanceParser.scala:12-22, which skips "EOS" and swallows
// malformed records) → DataPointParser building numerical ∥ discrete→double ∥
// categorical vectors (omldm/utils/parsers/dataStream/DataPointParser.scala:16-55).
//
// Batch layout (what the HIP learners consume, see csrc/kernels/linear_spoke.hip):
//   num [B, dn]  float   numerical features then discrete features (slot j == feature j)
//   cat [B, dc]  int32   hashed categorical slot in [dn, dim) | sign in bit 31, -1 = absent
//   y   [B]      float   target (NaN when absent, i.e. forecasting points)
//   op  [B]      int8    0 training, 1 forecasting, -1 invalid (dropped, counted)
// Records are parsed by a hand-written single-pass scanner on std::thread workers.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "dib.h"
#include "hashing.h"

#define OMLDM_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

using omldm_hash::hash_cat;
using omldm_hash::kSeedBase;
using omldm_hash::murmur3_32;

// Field-aware compact form: field f owns slots [dn + f·cspan, dn + (f+1)·cspan), the wire
// value is uint16 {sign:1, local:15} (0xFFFF = absent), cspan ≤ 32767.
inline uint16_t hash_cat16(const uint8_t* s, size_t n, int field, int cspan) {
  const uint32_t h = murmur3_32(s, n, kSeedBase + uint32_t(field));
  const uint32_t local = (h & 0x7fffffffu) % uint32_t(cspan);
  return uint16_t(((h >> 31) << 15) | local);
}

inline uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
inline double u01(uint64_t& s) { return (splitmix64(s) >> 11) * (1.0 / 9007199254740992.0); }
inline double gauss(uint64_t& s) {
  double u1 = u01(s), u2 = u01(s);
  if (u1 < 1e-300) u1 = 1e-300;
  return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

// ---------------------------------------------------------------- JSON scanner
struct Cursor {
  const char* p;
  const char* e;
  bool ok = true;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool eat(char c) {
    ws();
    if (p < e && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
  bool peek(char c) {
    ws();
    return p < e && *p == c;
  }
  // Returns a view of the string contents (escapes kept raw; hashing is over raw bytes,
  // identical to the Python fallback which also hashes the raw JSON text of the token).
  bool str(const char*& s, size_t& n) {
    ws();
    if (p >= e || *p != '"') return ok = false;
    ++p;
    s = p;
    for (;;) {  // memchr (vectorised) to the next quote; re-scan only across escapes
      const char* q = static_cast<const char*>(std::memchr(p, '"', size_t(e - p)));
      if (!q) return ok = false;
      const char* bs = static_cast<const char*>(std::memchr(p, '\\', size_t(q - p)));
      if (!bs) {
        p = q;
        break;
      }
      p = bs + 2;  // skip the escaped character
      if (p > e) return ok = false;
    }
    n = size_t(p - s);
    ++p;
    return true;
  }
  // JSON number. Fast path (Clinger): ≤ 19 significant digits and a decimal exponent
  // within ±22 convert exactly from one integer and one power-of-ten table entry
  // (both exactly representable in double); anything else falls back to strtod.
  bool num(double& v) {
    ws();
    const char* q = p;
    bool neg = false;
    if (q < e && (*q == '-' || *q == '+')) neg = *q++ == '-';
    uint64_t m = 0;
    int nd = 0, exp10 = 0;
    const char* d0 = q;
    while (q < e && unsigned(*q - '0') < 10u) {
      if (nd < 19) {
        m = m * 10 + unsigned(*q - '0');
        if (m) ++nd;
      } else {
        ++exp10;
      }
      ++q;
    }
    bool any = q > d0;
    if (q < e && *q == '.') {
      ++q;
      const char* f0 = q;
      while (q < e && unsigned(*q - '0') < 10u) {
        if (nd < 19) {
          m = m * 10 + unsigned(*q - '0');
          if (m) ++nd;
          --exp10;
        }
        ++q;
      }
      any = any || q > f0;
    }
    if (!any) return ok = false;
    if (q < e && (*q == 'e' || *q == 'E')) {
      ++q;
      bool eneg = false;
      if (q < e && (*q == '-' || *q == '+')) eneg = *q++ == '-';
      int ev = 0;
      const char* e0 = q;
      while (q < e && unsigned(*q - '0') < 10u) {
        if (ev < 100000) ev = ev * 10 + int(*q - '0');
        ++q;
      }
      if (q == e0) return ok = false;
      exp10 += eneg ? -ev : ev;
    }
    static const double kPow10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                    1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                    1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    if (m < (1ull << 53) && exp10 >= -22 && exp10 <= 22) {
      const double dm = double(m);
      v = exp10 >= 0 ? dm * kPow10[exp10] : dm / kPow10[-exp10];
      if (neg) v = -v;
      p = q;
      return true;
    }
    char* end = nullptr;  // rare: long mantissas, huge exponents
    v = std::strtod(p, &end);
    if (end == p || end > e) return ok = false;
    p = end;
    return true;
  }
  bool lit(const char* w) {
    ws();
    size_t n = std::strlen(w);
    if (size_t(e - p) >= n && std::memcmp(p, w, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  bool skip_value() {
    ws();
    if (p >= e) return ok = false;
    if (*p == '"') {
      const char* s;
      size_t n;
      return str(s, n);
    }
    if (*p == '{' || *p == '[') {
      int depth = 0;
      bool in_str = false;
      while (p < e) {
        char c = *p++;
        if (in_str) {
          if (c == '\\') ++p;
          else if (c == '"') in_str = false;
        } else if (c == '"') in_str = true;
        else if (c == '{' || c == '[') ++depth;
        else if (c == '}' || c == ']') {
          if (--depth == 0) return true;
        }
      }
      return ok = false;
    }
    if (lit("null") || lit("true") || lit("false")) return true;
    double v;
    return num(v);
  }
};

inline bool key_is(const char* s, size_t n, const char* k) {
  return std::strlen(k) == n && std::memcmp(s, k, n) == 0;
}

// ---------------------------------------------------------------- DIB (binary records)
// Format: csrc/host/dib.h.
int parse_dib(const uint8_t* b, const uint8_t* e, int dnum, int ddisc, int dc, int64_t dim,
              float* num, int32_t* cat, uint16_t* cat16, int cspan, float* y) {
  omldm_dib::Reader r{b + 1, e};
  const int dn = dnum + ddisc;
  const uint8_t op = r.get(), flags = r.get(), nn = r.get(), nd = r.get(), nc = r.get();
  if (flags & 1) *y = r.getf();
  for (int j = 0; j < nn; ++j) {
    const float v = r.getf();
    if (j < dnum) num[j] = v;
  }
  for (int j = 0; j < nd; ++j) {
    const float v = r.getf();
    if (j < ddisc) num[dnum + j] = v;
  }
  for (int j = 0; j < nc; ++j) {
    const uint32_t h = r.get32();
    if (j >= dc) continue;
    if (cat16) {
      cat16[j] = uint16_t(((h >> 31) << 15) | ((h & 0x7fffffffu) % uint32_t(cspan)));
    } else {
      const int32_t slot = int32_t(dn + int64_t(h & 0x7fffffffu) % (dim - dn - 1));
      cat[j] = (h & 0x80000000u) ? int32_t(uint32_t(slot) | 0x80000000u) : slot;
    }
  }
  if (!r.ok || op > 1 || !(flags & 2)) return -1;
  if (op == 0 && std::isnan(*y)) return -1;
  return op;
}

// Raw capture of a JSON record for the DIB encoder: the category hashes before they are
// reduced to slots, their count, and whether any feature array was present.
struct RawCapture {
  uint32_t* h;
  int nc = 0;
  bool any = false;
};

// Parses one record. Returns op code (0/1) or -1.
int parse_one(const char* b, const char* e, int dnum, int ddisc, int dc, int64_t dim, float* num,
              void* catv, int cspan, float* y, RawCapture* raw = nullptr) {
  int32_t* cat = static_cast<int32_t*>(catv);
  uint16_t* cat16 = static_cast<uint16_t*>(catv);
  if (cspan > 0) {
    if (cat16)
      for (int j = 0; j < dc; ++j) cat16[j] = 0xFFFF;
    cat = nullptr;
  }
  const int dn = dnum + ddisc;
  for (int j = 0; j < dn; ++j) num[j] = 0.f;
  if (cat)
    for (int j = 0; j < dc; ++j) cat[j] = -1;
  *y = std::nanf("");
  if (b < e && uint8_t(*b) == omldm_dib::kMagic && !raw)
    return parse_dib(reinterpret_cast<const uint8_t*>(b), reinterpret_cast<const uint8_t*>(e),
                     dnum, ddisc, dc, dim, num, cat, cat ? nullptr : cat16, cspan, y);
  Cursor c{b, e};
  c.ws();
  if (size_t(c.e - c.p) >= 3 && std::memcmp(c.p, "EOS", 3) == 0) return -1;
  if (!c.eat('{')) return -1;
  int op = -1;
  bool any_features = false;
  if (c.eat('}')) return -1;
  while (c.ok) {
    const char* k;
    size_t kn;
    if (!c.str(k, kn)) return -1;
    if (!c.eat(':')) return -1;
    if (key_is(k, kn, "numericalFeatures") || key_is(k, kn, "discreteFeatures")) {
      const bool is_num = k[0] == 'n';
      if (c.lit("null")) {
      } else {
        if (!c.eat('[')) return -1;
        int j = 0;
        if (!c.eat(']')) {
          while (true) {
            double v;
            if (!c.num(v)) return -1;
            const int lim = is_num ? dnum : ddisc;
            if (j < lim) num[(is_num ? 0 : dnum) + j] = float(v);
            ++j;
            if (c.eat(',')) continue;
            if (c.eat(']')) break;
            return -1;
          }
        }
        any_features = true;
      }
    } else if (key_is(k, kn, "categoricalFeatures")) {
      if (c.lit("null")) {
      } else {
        if (!c.eat('[')) return -1;
        int j = 0;
        if (!c.eat(']')) {
          while (true) {
            const char* s;
            size_t n;
            if (!c.str(s, n)) return -1;
            if (j < dc) {
              const uint8_t* us = reinterpret_cast<const uint8_t*>(s);
              if (raw) {
                raw->h[j] = murmur3_32(us, n, kSeedBase + uint32_t(j));
                raw->nc = j + 1;
              } else if (cat) {
                cat[j] = hash_cat(us, n, j, dn, dim);
              } else {
                cat16[j] = hash_cat16(us, n, j, cspan);
              }
            }
            ++j;
            if (c.eat(',')) continue;
            if (c.eat(']')) break;
            return -1;
          }
        }
        any_features = true;
      }
    } else if (key_is(k, kn, "target")) {
      if (!c.lit("null")) {
        double v;
        if (!c.num(v)) return -1;
        *y = float(v);
      }
    } else if (key_is(k, kn, "operation")) {
      const char* s;
      size_t n;
      if (!c.str(s, n)) return -1;
      if (key_is(s, n, "training")) op = 0;
      else if (key_is(s, n, "forecasting")) op = 1;
      else return -1;
    } else {
      if (!c.skip_value()) return -1;
    }
    if (c.eat(',')) continue;
    if (c.eat('}')) break;
    return -1;
  }
  if (raw) raw->any = any_features;
  if (!c.ok || !any_features) return -1;
  if (op == 0 && std::isnan(*y)) return -1;  // a training point needs a target
  return op;
}

inline void dib_put(std::vector<uint8_t>& o, uint8_t c) {
  if (c == 0x0A) {
    o.push_back(0xDB);
    o.push_back(0xDC);
  } else if (c == 0xDB) {
    o.push_back(0xDB);
    o.push_back(0xDD);
  } else {
    o.push_back(c);
  }
}
inline void dib_put32(std::vector<uint8_t>& o, uint32_t v) {
  for (int k = 0; k < 4; ++k) dib_put(o, uint8_t(v >> (8 * k)));
}
inline void dib_putf(std::vector<uint8_t>& o, float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  dib_put32(o, u);
}

template <typename F>
void parallel_for(int n, int nthreads, F&& f) {
  if (nthreads <= 1 || n < 256) {
    f(0, n);
    return;
  }
  nthreads = std::min(nthreads, (n + 255) / 256);
  std::vector<std::thread> th;
  const int chunk = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    const int a = t * chunk, b = std::min(n, a + chunk);
    if (a >= b) break;
    th.emplace_back([&, a, b] { f(a, b); });
  }
  for (auto& x : th) x.join();
}

}  // namespace

OMLDM_HOST_API uint32_t omldm_murmur3_32(const char* s, int64_t n, uint32_t seed) {
  return murmur3_32(reinterpret_cast<const uint8_t*>(s), size_t(n), seed);
}

OMLDM_HOST_API int32_t omldm_hash_cat(const char* s, int64_t n, int field, int dn, int64_t dim) {
  return hash_cat(reinterpret_cast<const uint8_t*>(s), size_t(n), field, dn, dim);
}

OMLDM_HOST_API int32_t omldm_hash_cat16(const char* s, int64_t n, int field, int cspan) {
  return hash_cat16(reinterpret_cast<const uint8_t*>(s), size_t(n), field, cspan);
}

// Parses n newline-free records buf[off[i]:off[i+1]]. Returns the number of valid records.
OMLDM_HOST_API int64_t omldm_parse_instances(const char* buf, const int64_t* off, int n, int dnum,
                                             int ddisc, int dc, int64_t dim, int cspan,
                                             float* num, void* cat, float* y, int8_t* op,
                                             int nthreads) {
  const int esz = cspan > 0 ? 2 : 4;
  const int dn = dnum + ddisc;
  std::atomic<int64_t> valid{0};
  parallel_for(n, nthreads, [&](int a, int b) {
    int64_t v = 0;
    for (int i = a; i < b; ++i) {
      const int r = parse_one(buf + off[i], buf + off[i + 1], dnum, ddisc, dc, dim,
                              num + int64_t(i) * dn,
                              static_cast<char*>(cat) + int64_t(i) * dc * esz, cspan, y + i);
      op[i] = int8_t(r);
      v += r >= 0;
    }
    valid += v;
  });
  return valid.load();
}

// JSON DataInstance records buf[off[i], off[i+1]) → DIB records (each ending in '\n')
// written back to back into out (cap bytes); out_offs[i] = start of record i,
// out_offs[n] = bytes written. A record the JSON parser rejects becomes an invalid DIB
// record (op 0xFF), so both topics count the same invalid records. Returns the bytes
// written, or -1 if cap is too small.
OMLDM_HOST_API int64_t omldm_json_to_dib(const char* buf, const int64_t* off, int n, int dnum,
                                         int ddisc, int dc, uint8_t* out, int64_t cap,
                                         int64_t* out_offs, int nthreads) {
  if (n <= 0) {
    out_offs[0] = 0;
    return 0;
  }
  const int nt = std::max(1, std::min(nthreads, (n + 255) / 256));
  std::vector<std::vector<uint8_t>> part(nt);
  std::vector<std::vector<int64_t>> lens(nt);
  const int chunk = (n + nt - 1) / nt;
  auto work = [&](int t) {
    const int a = t * chunk, b = std::min(n, a + chunk);
    std::vector<float> num(size_t(dnum + ddisc) + 1);
    std::vector<uint32_t> h(size_t(dc) + 1);
    auto& o = part[t];
    o.reserve(size_t(b - a) * size_t(16 + 4 * (dnum + ddisc + dc)));
    for (int i = a; i < b; ++i) {
      const size_t start = o.size();
      RawCapture rc{h.data()};
      float y;
      const int op = parse_one(buf + off[i], buf + off[i + 1], dnum, ddisc, dc, int64_t(1) << 30,
                               num.data(), nullptr, 1, &y, &rc);
      o.push_back(omldm_dib::kMagic);
      const bool has_y = !std::isnan(y);
      dib_put(o, op < 0 ? uint8_t(0xFF) : uint8_t(op));
      dib_put(o, uint8_t((has_y ? 1 : 0) | (rc.any ? 2 : 0)));
      dib_put(o, uint8_t(dnum));
      dib_put(o, uint8_t(ddisc));
      dib_put(o, uint8_t(rc.nc));
      if (has_y) dib_putf(o, y);
      for (int j = 0; j < dnum + ddisc; ++j) dib_putf(o, num[j]);
      for (int j = 0; j < rc.nc; ++j) dib_put32(o, h[j]);
      o.push_back('\n');
      lens[t].push_back(int64_t(o.size() - start));
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  int64_t pos = 0;
  int i = 0;
  for (int t = 0; t < nt; ++t) {
    if (pos + int64_t(part[t].size()) > cap) return -1;
    std::memcpy(out + pos, part[t].data(), part[t].size());
    for (int64_t L : lens[t]) {
      out_offs[i++] = pos;
      pos += L;
    }
  }
  out_offs[n] = pos;
  return pos;
}

// Deterministic synthetic stream (Criteo-like shape): dn Gaussian numerical features,
// dc categorical fields with skewed vocabularies hashed into [dn, dim), labels from a
// hidden linear model defined by a hash of the slot (no dim-sized table needed).
//   task 0: binary ±1 labels; 1: regression target; 2: K-class labels in [0, K)
// Example i of the stream is a pure function of (seed, start + i), so any shard of the
// stream can be generated independently on any rank.
OMLDM_HOST_API void omldm_synth_batch(uint64_t seed, int64_t start, int B, int dn, int dc,
                                      int64_t dim, int task, int n_classes, float noise,
                                      int cspan, float* num, void* cat, float* y, int nthreads) {
  const int64_t span = dim - dn - 1;  // slot dim-1 is reserved for the intercept
  parallel_for(B, nthreads, [&](int a, int b) {
    for (int i = a; i < b; ++i) {
      uint64_t s = mix64(seed * 0x9e3779b97f4a7c15ull + uint64_t(start + i));
      float* xn = num + int64_t(i) * dn;
      int32_t* xc = cspan > 0 ? nullptr : static_cast<int32_t*>(cat) + int64_t(i) * dc;
      uint16_t* xc16 = cspan > 0 ? static_cast<uint16_t*>(cat) + int64_t(i) * dc : nullptr;
      double score[16] = {0};
      const int K = task == 2 ? std::max(2, std::min(16, n_classes)) : 1;
      for (int j = 0; j < dn; ++j) {
        const double v = gauss(s);
        xn[j] = float(v);
        for (int k = 0; k < K; ++k) {
          uint64_t hs = mix64((seed ^ 0x5bd1e995ull) + uint64_t(j) * 131 + uint64_t(k) * 7919);
          score[k] += v * (gauss(hs) * 0.5);
        }
      }
      for (int j = 0; j < dc; ++j) {
        // field j vocabulary 10^(1 + j % 6); rank skewed toward small values (u^3).
        int64_t vocab = 10;
        for (int q = 0; q < j % 6; ++q) vocab *= 10;
        const double u = u01(s);
        const int64_t rank = int64_t(double(vocab) * u * u * u);
        const uint64_t h = mix64(seed + uint64_t(j) * 0x100000001b3ull + uint64_t(rank) * 0x9e37ull);
        const bool neg = (h >> 63) & 1ull;
        int32_t slot;
        if (xc16) {
          const uint32_t local = uint32_t((h & 0x7fffffffull) % uint64_t(cspan));
          slot = int32_t(dn + int64_t(j) * cspan + local);
          xc16[j] = uint16_t((neg ? 0x8000u : 0u) | local);
        } else {
          slot = int32_t(dn + int64_t(h & 0x7fffffffull) % span);
          xc[j] = neg ? int32_t(uint32_t(slot) | 0x80000000u) : slot;
        }
        const double sv = neg ? -1.0 : 1.0;
        for (int k = 0; k < K; ++k) {
          uint64_t hs = mix64((seed ^ 0x27d4eb2dull) + uint64_t(slot) * 31 + uint64_t(k) * 104729);
          score[k] += sv * (gauss(hs) * 0.5);
        }
      }
      const double eps = noise * gauss(s);
      if (task == 0) {
        y[i] = (score[0] + eps) >= 0.0 ? 1.f : -1.f;
      } else if (task == 1) {
        y[i] = float(score[0] + eps);
      } else {
        int best = 0;
        for (int k = 1; k < K; ++k)
          if (score[k] > score[best]) best = k;
        y[i] = float(best);
      }
    }
  });
}
