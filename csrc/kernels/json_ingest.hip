// GPU DataInstance JSON parser + feature hashing ("device feature_hash"),
// and the decoder of the binary DIB records that may share a topic with JSON (dib.h).
//
// Reference: Jackson parses every record on a JVM thread (DataInstanceParser /
// DataPointParser, omldm/utils/parsers/DataInstanceParser.scala:12-22,
// dataStream/DataPointParser.scala:16-55), ~0.5 M records/s per core for our C++ port.
// Here the raw JSON block (records back to back, int64 offsets) is copied to HBM once,
// each wave stages its 64 records' bytes in LDS, and every lane parses one record: numerical ∥ discrete features, categorical tokens
// hashed with murmur3-32 (per-field seeds — bit-identical to csrc/host/ingest.cpp), target,
// operation. Semantics match the host scanner exactly (same validity rules: "EOS",
// malformed JSON, missing features / operation, training point without target → -1).
// Numbers: the exact Clinger fast path (≤ 19 significant digits, |exp10| ≤ 22) as on the
// host; beyond it the host falls back to strtod and the device to m·10^e in double —
// identical after rounding to fp32 except in rare rounding ties.
#include "common.h"

namespace omldm {

namespace {

constexpr uint32_t kSeedBaseDev = 0x9747b28cu;

struct JCur {
  const unsigned char* p;
  const unsigned char* e;
  bool ok;
};

__device__ __forceinline__ void jws(JCur& c) {
  while (c.p < c.e) {
    const unsigned char ch = *c.p;
    if (ch == ' ' || ch == '\n' || ch == '\r' || ch == '\t') ++c.p;
    else break;
  }
}

__device__ __forceinline__ bool jeat(JCur& c, unsigned char x) {
  jws(c);
  if (c.p < c.e && *c.p == x) {
    ++c.p;
    return true;
  }
  return false;
}

__device__ __forceinline__ bool jstr(JCur& c, const unsigned char*& s, int& n) {
  jws(c);
  if (c.p >= c.e || *c.p != '"') return c.ok = false;
  ++c.p;
  s = c.p;
  while (c.p < c.e && *c.p != '"') {
    if (*c.p == '\\') ++c.p;
    ++c.p;
  }
  if (c.p >= c.e) return c.ok = false;
  n = (int)(c.p - s);
  ++c.p;
  return true;
}

__device__ __forceinline__ bool jlit(JCur& c, const char* w, int n) {
  jws(c);
  if (c.e - c.p < n) return false;
  for (int i = 0; i < n; ++i)
    if (c.p[i] != (unsigned char)w[i]) return false;
  c.p += n;
  return true;
}

__device__ __forceinline__ bool jkey(const unsigned char* s, int n, const char* k, int kn) {
  if (n != kn) return false;
  for (int i = 0; i < n; ++i)
    if (s[i] != (unsigned char)k[i]) return false;
  return true;
}

__device__ __forceinline__ bool jnum(JCur& c, double& v) {
  jws(c);
  const unsigned char* q = c.p;
  bool neg = false;
  if (q < c.e && (*q == '-' || *q == '+')) neg = *q++ == '-';
  unsigned long long m = 0;
  int nd = 0, exp10 = 0;
  const unsigned char* d0 = q;
  while (q < c.e && (unsigned)(*q - '0') < 10u) {
    if (nd < 19) {
      m = m * 10 + (unsigned)(*q - '0');
      if (m) ++nd;
    } else {
      ++exp10;
    }
    ++q;
  }
  bool any = q > d0;
  if (q < c.e && *q == '.') {
    ++q;
    const unsigned char* f0 = q;
    while (q < c.e && (unsigned)(*q - '0') < 10u) {
      if (nd < 19) {
        m = m * 10 + (unsigned)(*q - '0');
        if (m) ++nd;
        --exp10;
      }
      ++q;
    }
    any = any || q > f0;
  }
  if (!any) return c.ok = false;
  if (q < c.e && (*q == 'e' || *q == 'E')) {
    ++q;
    bool eneg = false;
    if (q < c.e && (*q == '-' || *q == '+')) eneg = *q++ == '-';
    int ev = 0;
    const unsigned char* e0 = q;
    while (q < c.e && (unsigned)(*q - '0') < 10u) {
      if (ev < 100000) ev = ev * 10 + (int)(*q - '0');
      ++q;
    }
    if (q == e0) return c.ok = false;
    exp10 += eneg ? -ev : ev;
  }
  const double dm = (double)m;
  if (m < (1ull << 53) && exp10 >= -22 && exp10 <= 22) {
    double p10 = 1.0;  // exact: 10^k for k ≤ 22 is representable
    for (int k = 0; k < (exp10 >= 0 ? exp10 : -exp10); ++k) p10 *= 10.0;
    v = exp10 >= 0 ? dm * p10 : dm / p10;
  } else {
    v = dm * pow(10.0, (double)exp10);
  }
  if (neg) v = -v;
  c.p = q;
  return true;
}

__device__ __forceinline__ bool jskip(JCur& c) {
  jws(c);
  if (c.p >= c.e) return c.ok = false;
  if (*c.p == '"') {
    const unsigned char* s;
    int n;
    return jstr(c, s, n);
  }
  if (*c.p == '{' || *c.p == '[') {
    int depth = 0;
    bool in_str = false;
    while (c.p < c.e) {
      const unsigned char ch = *c.p++;
      if (in_str) {
        if (ch == '\\') ++c.p;
        else if (ch == '"') in_str = false;
      } else if (ch == '"') {
        in_str = true;
      } else if (ch == '{' || ch == '[') {
        ++depth;
      } else if (ch == '}' || ch == ']') {
        if (--depth == 0) return true;
      }
    }
    return c.ok = false;
  }
  if (jlit(c, "null", 4) || jlit(c, "true", 4) || jlit(c, "false", 5)) return true;
  double v;
  return jnum(c, v);
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

__device__ uint32_t murmur3_dev(const unsigned char* d, int len, uint32_t seed) {
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  uint32_t h1 = seed;
  const int nb = len >> 2;
  for (int i = 0; i < nb; ++i) {
    uint32_t k1 = (uint32_t)d[4 * i] | ((uint32_t)d[4 * i + 1] << 8) |
                  ((uint32_t)d[4 * i + 2] << 16) | ((uint32_t)d[4 * i + 3] << 24);
    k1 *= c1;
    k1 = rotl(k1, 15);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl(h1, 13);
    h1 = h1 * 5 + 0xe6546b64u;
  }
  const unsigned char* t = d + 4 * nb;
  uint32_t k1 = 0;
  switch (len & 3) {
    case 3: k1 ^= (uint32_t)t[2] << 16; [[fallthrough]];
    case 2: k1 ^= (uint32_t)t[1] << 8; [[fallthrough]];
    case 1:
      k1 ^= t[0];
      k1 *= c1;
      k1 = rotl(k1, 15);
      k1 *= c2;
      h1 ^= k1;
  }
  h1 ^= (uint32_t)len;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  h1 ^= h1 >> 16;
  return h1;
}

// A DIB record (binary DataInstance, csrc/host/dib.h): 0xB1, then the SLIP-stuffed
// payload op | flags | nn | nd | nc | [f32 target] | f32 num[nn] | f32 disc[nd] |
// u32 murmur3 hash[nc]. Same outputs and validity rules as the host's parse_dib.
struct DibRd {
  const unsigned char* p;
  const unsigned char* e;
  bool ok;
  __device__ __forceinline__ uint32_t get() {
    if (p >= e) return ok = false, 0u;
    uint32_t c = *p++;
    if (c == 0xDBu) {
      if (p >= e) return ok = false, 0u;
      const uint32_t d = *p++;
      c = d == 0xDCu ? 0x0Au : (d == 0xDDu ? 0xDBu : (ok = false, 0u));
    }
    return c;
  }
  __device__ __forceinline__ uint32_t get32() {
    uint32_t v = get();
    v |= get() << 8;
    v |= get() << 16;
    v |= get() << 24;
    return v;
  }
};

__device__ __forceinline__ int parse_dib_record(const unsigned char* b, const unsigned char* e,
                                                int dnum, int ddisc, int dc, long long dim,
                                                int cspan, float* num, int* cat32,
                                                unsigned short* cat16, float* y) {
  const int dn = dnum + ddisc;
  DibRd r{b + 1, e, true};
  const uint32_t op = r.get(), flags = r.get(), nn = r.get(), nd = r.get(), nc = r.get();
  if (flags & 1u) *y = __uint_as_float(r.get32());
  for (uint32_t j = 0; j < nn; ++j) {
    const float v = __uint_as_float(r.get32());
    if ((int)j < dnum) num[j] = v;
  }
  for (uint32_t j = 0; j < nd; ++j) {
    const float v = __uint_as_float(r.get32());
    if ((int)j < ddisc) num[dnum + j] = v;
  }
  for (uint32_t j = 0; j < nc; ++j) {
    const uint32_t h = r.get32();
    if ((int)j >= dc) continue;
    if (cspan > 0) {
      cat16[j] = (unsigned short)(((h >> 31) << 15) | ((h & 0x7fffffffu) % (uint32_t)cspan));
    } else {
      const int slot = (int)(dn + (long long)(h & 0x7fffffffu) % (dim - dn - 1));
      cat32[j] = (h & 0x80000000u) ? (int)((uint32_t)slot | 0x80000000u) : slot;
    }
  }
  if (!r.ok || op > 1u || !(flags & 2u)) return -1;
  if (op == 0u && __builtin_isnan(*y)) return -1;
  return (int)op;
}

// One record → outputs; returns op (0 training, 1 forecasting) or -1.
__device__ __forceinline__ int parse_record(const unsigned char* b, const unsigned char* e, int dnum, int ddisc,
                            int dc, long long dim, int cspan, float* num, int* cat32,
                            unsigned short* cat16, float* y) {
  const int dn = dnum + ddisc;
  for (int j = 0; j < dn; ++j) num[j] = 0.f;
  for (int j = 0; j < dc; ++j) {
    if (cspan > 0) cat16[j] = 0xFFFFu;
    else cat32[j] = -1;
  }
  *y = __builtin_nanf("");
  if (b < e && *b == 0xB1u)
    return parse_dib_record(b, e, dnum, ddisc, dc, dim, cspan, num, cat32, cat16, y);
  JCur c{b, e, true};
  jws(c);
  if (c.e - c.p >= 3 && c.p[0] == 'E' && c.p[1] == 'O' && c.p[2] == 'S') return -1;
  if (!jeat(c, '{')) return -1;
  int op = -1;
  bool any = false;
  if (jeat(c, '}')) return -1;
  while (c.ok) {
    const unsigned char* k;
    int kn;
    if (!jstr(c, k, kn)) return -1;
    if (!jeat(c, ':')) return -1;
    if (jkey(k, kn, "numericalFeatures", 17) || jkey(k, kn, "discreteFeatures", 16)) {
      const bool is_num = k[0] == 'n';
      if (!jlit(c, "null", 4)) {
        if (!jeat(c, '[')) return -1;
        int j = 0;
        if (!jeat(c, ']')) {
          while (true) {
            double v;
            if (!jnum(c, v)) return -1;
            const int lim = is_num ? dnum : ddisc;
            if (j < lim) num[(is_num ? 0 : dnum) + j] = (float)v;
            ++j;
            if (jeat(c, ',')) continue;
            if (jeat(c, ']')) break;
            return -1;
          }
        }
        any = true;
      }
    } else if (jkey(k, kn, "categoricalFeatures", 19)) {
      if (!jlit(c, "null", 4)) {
        if (!jeat(c, '[')) return -1;
        int j = 0;
        if (!jeat(c, ']')) {
          while (true) {
            const unsigned char* s;
            int n;
            if (!jstr(c, s, n)) return -1;
            if (j < dc) {
              const uint32_t h = murmur3_dev(s, n, kSeedBaseDev + (uint32_t)j);
              if (cspan > 0) {
                const uint32_t local = (h & 0x7fffffffu) % (uint32_t)cspan;
                cat16[j] = (unsigned short)(((h >> 31) << 15) | local);
              } else {
                const long long span = dim - dn - 1;
                const int slot = (int)(dn + (long long)(h & 0x7fffffffu) % span);
                cat32[j] = (h & 0x80000000u) ? (int)((uint32_t)slot | 0x80000000u) : slot;
              }
            }
            ++j;
            if (jeat(c, ',')) continue;
            if (jeat(c, ']')) break;
            return -1;
          }
        }
        any = true;
      }
    } else if (jkey(k, kn, "target", 6)) {
      if (!jlit(c, "null", 4)) {
        double v;
        if (!jnum(c, v)) return -1;
        *y = (float)v;
      }
    } else if (jkey(k, kn, "operation", 9)) {
      const unsigned char* s;
      int n;
      if (!jstr(c, s, n)) return -1;
      if (jkey(s, n, "training", 8)) op = 0;
      else if (jkey(s, n, "forecasting", 11)) op = 1;
      else return -1;
    } else {
      if (!jskip(c)) return -1;
    }
    if (jeat(c, ',')) continue;
    if (jeat(c, '}')) break;
    return -1;
  }
  if (!c.ok || !any) return -1;
  if (op == 0 && __builtin_isnan(*y)) return -1;
  return op;
}

}  // namespace

__global__ __launch_bounds__(256) void json_parse_kernel(
    const unsigned char* __restrict__ buf, const long long* __restrict__ offs, int n, int dnum,
    int ddisc, int dc, long long dim, int cspan, float* __restrict__ num, void* __restrict__ cat,
    float* __restrict__ y, signed char* __restrict__ op, int* __restrict__ counts) {
  const int dn = dnum + ddisc;
  int ntrain = 0, nfcst = 0, nbad = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int r = parse_record(buf + offs[i], buf + offs[i + 1], dnum, ddisc, dc, dim, cspan,
                               num + (size_t)i * dn, static_cast<int*>(cat) + (size_t)i * dc,
                               static_cast<unsigned short*>(cat) + (size_t)i * dc, y + i);
    op[i] = (signed char)r;
    ntrain += r == 0;
    nfcst += r == 1;
    nbad += r < 0;
  }
  // counts[0..2] += (training, forecasting, invalid): one atomic per wave and kind
  float a = (float)ntrain, b = (float)nfcst;
  wave_sum2(a, b);
  const float c = wave_sum((float)nbad);
  if ((threadIdx.x & 63) == 0 && counts) {
    if (a > 0.f) atomicAdd(counts, (int)a);
    if (b > 0.f) atomicAdd(counts + 1, (int)b);
    if (c > 0.f) atomicAdd(counts + 2, (int)c);
  }
}

// Wave-staged variant (the launch path): one wave = one block = 64 consecutive records.
// Their bytes are contiguous in the buffer, so the wave first copies the group's byte
// range into LDS with 16-byte loads (every lane issuing, fully coalesced) and each lane
// then parses its record out of LDS — the scanner's ~500 dependent byte reads per record
// become LDS latencies instead of global-memory ones. A group larger than the LDS stage
// (a record with a huge skipped field) is parsed from global memory as before.
constexpr int kJsonStage = 36 * 1024;  // bytes per wave: 4 waves per CU fit in LDS

__global__ __launch_bounds__(64) void json_parse_staged_kernel(
    const unsigned char* __restrict__ buf, const long long* __restrict__ offs, int n, int dnum,
    int ddisc, int dc, long long dim, int cspan, float* __restrict__ num, void* __restrict__ cat,
    float* __restrict__ y, signed char* __restrict__ op, int* __restrict__ counts) {
  __shared__ uint4 stage[kJsonStage / 16];
  const int lane = threadIdx.x;
  const int dn = dnum + ddisc;
  int ntrain = 0, nfcst = 0, nbad = 0;
  const int groups = (n + 63) >> 6;
  for (int gi = blockIdx.x; gi < groups; gi += gridDim.x) {
    const int i0 = gi << 6, iend = min(n, i0 + 64), i = i0 + lane;
    const long long b0 = offs[i0], b1 = offs[iend];
    const long long a0 = b0 & ~15ll;  // 16-byte aligned start (hipMalloc bases are aligned)
    const long long bytes = b1 - a0;
    const bool staged = bytes <= kJsonStage;
    if (staged) {
      const int nfull = (int)(bytes >> 4);  // whole vectors inside [a0, b1): no over-read
      const uint4* src = reinterpret_cast<const uint4*>(buf + a0);
      for (int v = lane; v < nfull; v += 64) stage[v] = src[v];
      const int tail = (int)(bytes & 15);
      unsigned char* sb = reinterpret_cast<unsigned char*>(stage);
      if (lane < tail) sb[(nfull << 4) + lane] = buf[a0 + (nfull << 4) + lane];
    }
    __syncthreads();
    if (i < iend) {
      const unsigned char* sb = reinterpret_cast<const unsigned char*>(stage);
      const long long o0 = offs[i], o1 = offs[i + 1];
      float* nr = num + (size_t)i * dn;
      int* c32 = static_cast<int*>(cat) + (size_t)i * dc;
      unsigned short* c16 = static_cast<unsigned short*>(cat) + (size_t)i * dc;
      // two inlined copies: in the staged one every scanner read is provably LDS (ds_read)
      const int r = staged ? parse_record(sb + (o0 - a0), sb + (o1 - a0), dnum, ddisc, dc, dim,
                                          cspan, nr, c32, c16, y + i)
                           : parse_record(buf + o0, buf + o1, dnum, ddisc, dc, dim, cspan, nr,
                                          c32, c16, y + i);
      op[i] = (signed char)r;
      ntrain += r == 0;
      nfcst += r == 1;
      nbad += r < 0;
    }
    __syncthreads();  // the next group overwrites the stage
  }
  float a = (float)ntrain, b = (float)nfcst;
  wave_sum2(a, b);
  const float c = wave_sum((float)nbad);
  if (lane == 0 && counts) {
    if (a > 0.f) atomicAdd(counts, (int)a);
    if (b > 0.f) atomicAdd(counts + 1, (int)b);
    if (c > 0.f) atomicAdd(counts + 2, (int)c);
  }
}

}  // namespace omldm

using namespace omldm;

// buf/offs/outputs are device pointers; offs has n+1 entries (record i = buf[offs[i],
// offs[i+1])). Layout of the outputs as omldm_parse_instances (host). counts (optional,
// 3 ints, accumulated): training, forecasting and invalid records.
OMLDM_API int omldm_json_parse(const void* buf, const long long* offs, int n, int dnum,
                               int ddisc, int dc, long long dim, int cspan, float* num,
                               void* cat, float* y, signed char* op, int* counts,
                               void* stream) {
  if (n <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(buf) & 15) {  // the staged kernel needs an aligned base
    int blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(json_parse_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const unsigned char*)buf, offs, n, dnum, ddisc, dc, dim, cspan, num, cat,
                       y, op, counts);
    return (int)hipGetLastError();
  }
  int groups = (n + 63) / 64;
  if (groups > 8192) groups = 8192;  // grid-stride beyond 32 waves per CU
  hipLaunchKernelGGL(json_parse_staged_kernel, dim3(groups), dim3(64), 0, (hipStream_t)stream,
                     (const unsigned char*)buf, offs, n, dnum, ddisc, dc, dim, cspan, num, cat, y,
                     op, counts);
  return (int)hipGetLastError();
}
