// Kafka RecordBatch v2 data plane: record-set decoding straight into a pinned staging
// slot, and the four Kafka compression codecs.
//
// Reference: every OMLDM input is a FlinkKafkaConsumer source (omldm/Job.scala:42-57,
// 127-142). Flink's Kafka client decodes RecordBatch v2 and inflates gzip / snappy / lz4 /
// zstd batches transparently, so topics written by any producer configuration are
// readable. Here the same happens natively, without a Python object per record:
//   * omldm_kafka_decode_into: walks a Fetch response's record set (magic 2; older
//     message sets and transactional control batches skipped; CRC-32C checked),
//     decompresses the records section when the batch is compressed, and copies every
//     record value with offset ≥ min_offset into dst[0:cap] plus an offsets array — the
//     layout the GPU JSON parser consumes (omldm_amd/engine/ingest.py);
//   * codecs (attributes bits 0-2): 1 gzip (zlib), 2 snappy (own implementation; raw
//     blocks or the xerial framing the Java client writes), 3 lz4 (LZ4 frame format) and
//     4 zstd (frame format), the last two through the system liblz4 / libzstd, loaded on
//     first use (only the runtime .so files exist on this image, so the few entry points
//     used are declared here from their stable C ABI).
#include <dlfcn.h>
#include <zlib.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#define OMLDM_HOST_API extern "C" __attribute__((visibility("default")))

extern "C" uint32_t omldm_crc32c(const uint8_t* p, int64_t n, uint32_t crc);

namespace {

enum Codec : int { kNone = 0, kGzip = 1, kSnappy = 2, kLz4 = 3, kZstd = 4 };
enum Err : int {
  kOk = 0, kBadCodec = -1, kCorrupt = -2, kNoLib = -3, kTooBig = -4, kCrc = -5, kOom = -6
};

// ------------------------------------------------------------------ gzip (zlib)
int gzip_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out) {
  z_stream zs{};
  if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) return kCorrupt;
  out.resize(n * 4 + 1024);
  zs.next_in = const_cast<Bytef*>(src);
  zs.avail_in = (uInt)n;
  int rc = Z_OK;
  size_t done = 0;
  while (rc != Z_STREAM_END) {
    if (done == out.size()) out.resize(out.size() * 2);
    zs.next_out = out.data() + done;
    zs.avail_out = (uInt)(out.size() - done);
    rc = inflate(&zs, Z_NO_FLUSH);
    done = out.size() - zs.avail_out;
    if (rc == Z_STREAM_END && zs.avail_in > 0) {  // concatenated gzip members
      if (inflateReset(&zs) != Z_OK) break;
      rc = Z_OK;
      continue;
    }
    if (rc != Z_OK && rc != Z_STREAM_END && !(rc == Z_BUF_ERROR && zs.avail_out == 0)) {
      inflateEnd(&zs);
      return kCorrupt;
    }
    if (rc == Z_OK && zs.avail_in == 0 && zs.avail_out > 0) break;  // truncated input
  }
  inflateEnd(&zs);
  if (rc != Z_STREAM_END) return kCorrupt;
  out.resize(done);
  return kOk;
}

int gzip_compress(const uint8_t* src, size_t n, int level, std::vector<uint8_t>& out) {
  z_stream zs{};
  if (deflateInit2(&zs, level < 0 ? Z_DEFAULT_COMPRESSION : level, Z_DEFLATED, 16 + MAX_WBITS, 8,
                   Z_DEFAULT_STRATEGY) != Z_OK)
    return kCorrupt;
  out.resize(deflateBound(&zs, (uLong)n) + 32);
  zs.next_in = const_cast<Bytef*>(src);
  zs.avail_in = (uInt)n;
  zs.next_out = out.data();
  zs.avail_out = (uInt)out.size();
  const int rc = deflate(&zs, Z_FINISH);
  out.resize(out.size() - zs.avail_out);
  deflateEnd(&zs);
  return rc == Z_STREAM_END ? kOk : kCorrupt;
}

// ------------------------------------------------------------------ snappy
// Raw format: varint uncompressed length, then elements whose tag's low 2 bits select a
// literal (00), a copy with an 11-bit offset (01), a 16-bit (10) or a 32-bit offset (11).
int snappy_raw_decompress(const uint8_t* p, size_t n, std::vector<uint8_t>& out) {
  size_t i = 0;
  uint64_t len = 0;
  for (int s = 0;; s += 7) {
    if (i >= n || s > 35) return kCorrupt;
    const uint8_t b = p[i++];
    len |= uint64_t(b & 0x7F) << s;
    if (!(b & 0x80)) break;
  }
  const size_t base = out.size();
  if (len > (size_t(1) << 32)) return kTooBig;
  out.resize(base + len);
  uint8_t* o = out.data() + base;
  size_t w = 0;
  while (i < n) {
    const uint8_t tag = p[i++];
    size_t ln, off;
    switch (tag & 3) {
      case 0: {
        ln = (tag >> 2) + 1;
        if (ln > 60) {
          const int nb = int(ln - 60);
          if (i + nb > n) return kCorrupt;
          ln = 0;
          for (int k = 0; k < nb; ++k) ln |= size_t(p[i + k]) << (8 * k);
          ln += 1;
          i += nb;
        }
        if (i + ln > n || w + ln > len) return kCorrupt;
        std::memcpy(o + w, p + i, ln);
        i += ln;
        w += ln;
        continue;
      }
      case 1:
        if (i + 1 > n) return kCorrupt;
        ln = 4 + ((tag >> 2) & 7);
        off = (size_t(tag >> 5) << 8) | p[i];
        i += 1;
        break;
      case 2:
        if (i + 2 > n) return kCorrupt;
        ln = (tag >> 2) + 1;
        off = size_t(p[i]) | size_t(p[i + 1]) << 8;
        i += 2;
        break;
      default:
        if (i + 4 > n) return kCorrupt;
        ln = (tag >> 2) + 1;
        off = size_t(p[i]) | size_t(p[i + 1]) << 8 | size_t(p[i + 2]) << 16 |
              size_t(p[i + 3]) << 24;
        i += 4;
    }
    if (off == 0 || off > w || w + ln > len) return kCorrupt;
    if (off >= ln) {
      std::memcpy(o + w, o + w - off, ln);
    } else {
      for (size_t k = 0; k < ln; ++k) o[w + k] = o[w + k - off];  // overlapping: repeats
    }
    w += ln;
  }
  return w == len ? kOk : kCorrupt;
}

const uint8_t kXerialMagic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};

uint32_t be32(const uint8_t* p) {
  return uint32_t(p[0]) << 24 | uint32_t(p[1]) << 16 | uint32_t(p[2]) << 8 | p[3];
}
void put_be32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back(uint8_t(x >> 24));
  v.push_back(uint8_t(x >> 16));
  v.push_back(uint8_t(x >> 8));
  v.push_back(uint8_t(x));
}

int snappy_decompress(const uint8_t* p, size_t n, std::vector<uint8_t>& out) {
  out.clear();
  if (n >= 16 && std::memcmp(p, kXerialMagic, 8) == 0) {  // xerial: header + [len][block]*
    size_t i = 16;
    while (i < n) {
      if (i + 4 > n) return kCorrupt;
      const size_t bl = be32(p + i);
      i += 4;
      if (i + bl > n) return kCorrupt;
      const int rc = snappy_raw_decompress(p + i, bl, out);
      if (rc) return rc;
      i += bl;
    }
    return kOk;
  }
  return snappy_raw_decompress(p, n, out);
}

void snappy_emit_literal(std::vector<uint8_t>& o, const uint8_t* s, size_t ln) {
  const size_t m = ln - 1;
  if (m < 60) {
    o.push_back(uint8_t(m << 2));
  } else {
    int nb = m < (1u << 8) ? 1 : m < (1u << 16) ? 2 : m < (1u << 24) ? 3 : 4;
    o.push_back(uint8_t((59 + nb) << 2));
    for (int k = 0; k < nb; ++k) o.push_back(uint8_t(m >> (8 * k)));
  }
  o.insert(o.end(), s, s + ln);
}

void snappy_emit_copy(std::vector<uint8_t>& o, size_t off, size_t ln) {
  while (ln > 0) {  // 16-bit-offset copies of ≤ 64 bytes (offset < 32 KiB within a block)
    const size_t c = ln > 64 ? 64 : ln;
    o.push_back(uint8_t(((c - 1) << 2) | 2));
    o.push_back(uint8_t(off));
    o.push_back(uint8_t(off >> 8));
    ln -= c;
  }
}

// Greedy LZ77 over one ≤ 32 KiB block with a 4-byte hash table.
void snappy_raw_compress(const uint8_t* s, size_t n, std::vector<uint8_t>& o) {
  for (size_t v = n;;) {  // varint length
    if (v < 0x80) {
      o.push_back(uint8_t(v));
      break;
    }
    o.push_back(uint8_t(v | 0x80));
    v >>= 7;
  }
  constexpr int kBits = 14;
  int32_t table[1 << kBits];
  std::memset(table, -1, sizeof(table));
  size_t i = 0, lit = 0;
  auto h4 = [&](size_t k) {
    uint32_t x;
    std::memcpy(&x, s + k, 4);
    return (x * 0x1E35A7BDu) >> (32 - kBits);
  };
  while (i + 4 <= n) {
    const uint32_t h = h4(i);
    const int32_t cand = table[h];
    table[h] = int32_t(i);
    if (cand >= 0 && std::memcmp(s + cand, s + i, 4) == 0) {
      size_t ln = 4;
      while (i + ln < n && s[cand + ln] == s[i + ln]) ++ln;
      if (i > lit) snappy_emit_literal(o, s + lit, i - lit);
      snappy_emit_copy(o, i - size_t(cand), ln);
      i += ln;
      lit = i;
    } else {
      ++i;
    }
  }
  if (n > lit) snappy_emit_literal(o, s + lit, n - lit);
}

int snappy_compress(const uint8_t* s, size_t n, std::vector<uint8_t>& o) {
  o.assign(kXerialMagic, kXerialMagic + 8);  // xerial framing, as the Java client writes
  put_be32(o, 1);
  put_be32(o, 1);
  constexpr size_t kBlock = 32 * 1024;
  std::vector<uint8_t> blk;
  for (size_t i = 0; i < n || (n == 0 && i == 0); i += kBlock) {
    blk.clear();
    snappy_raw_compress(s + i, (n - i) < kBlock ? (n - i) : kBlock, blk);
    put_be32(o, uint32_t(blk.size()));
    o.insert(o.end(), blk.begin(), blk.end());
    if (n == 0) break;
  }
  return kOk;
}

// ------------------------------------------------------------------ lz4 / zstd (dlopen)
struct Lz4Api {
  unsigned (*isError)(size_t);
  size_t (*createD)(void**, unsigned);
  size_t (*freeD)(void*);
  size_t (*decompress)(void*, void*, size_t*, const void*, size_t*, const void*);
  size_t (*bound)(size_t, const void*);
  size_t (*compress)(void*, size_t, const void*, size_t, const void*);
};
struct ZstdApi {
  unsigned (*isError)(size_t);
  void* (*createD)();
  size_t (*freeD)(void*);
  size_t (*initD)(void*);
  size_t (*decompressStream)(void*, void*, void*);
  size_t (*bound)(size_t);
  size_t (*compress)(void*, size_t, const void*, size_t, int);
};
struct ZIn {
  const void* src;
  size_t size, pos;
};
struct ZOut {
  void* dst;
  size_t size, pos;
};

std::once_flag g_once;
Lz4Api g_lz4{};
ZstdApi g_zstd{};
bool g_has_lz4 = false, g_has_zstd = false;

template <class F>
bool sym(void* h, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(h, name));
  return f != nullptr;
}

void load_libs() {
  std::call_once(g_once, [] {
    for (const char* name : {"liblz4.so.1", "liblz4.so"}) {
      if (void* h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) {
        g_has_lz4 = sym(h, "LZ4F_isError", g_lz4.isError) &&
                    sym(h, "LZ4F_createDecompressionContext", g_lz4.createD) &&
                    sym(h, "LZ4F_freeDecompressionContext", g_lz4.freeD) &&
                    sym(h, "LZ4F_decompress", g_lz4.decompress) &&
                    sym(h, "LZ4F_compressFrameBound", g_lz4.bound) &&
                    sym(h, "LZ4F_compressFrame", g_lz4.compress);
        break;
      }
    }
    for (const char* name : {"libzstd.so.1", "libzstd.so"}) {
      if (void* h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) {
        g_has_zstd = sym(h, "ZSTD_isError", g_zstd.isError) &&
                     sym(h, "ZSTD_createDStream", g_zstd.createD) &&
                     sym(h, "ZSTD_freeDStream", g_zstd.freeD) &&
                     sym(h, "ZSTD_initDStream", g_zstd.initD) &&
                     sym(h, "ZSTD_decompressStream", g_zstd.decompressStream) &&
                     sym(h, "ZSTD_compressBound", g_zstd.bound) &&
                     sym(h, "ZSTD_compress", g_zstd.compress);
        break;
      }
    }
  });
}

int lz4_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out) {
  load_libs();
  if (!g_has_lz4) return kNoLib;
  void* ctx = nullptr;
  if (g_lz4.isError(g_lz4.createD(&ctx, 100 /* LZ4F_VERSION */))) return kCorrupt;
  out.resize(n * 4 + 65536);
  size_t in = 0, done = 0, hint = 1;
  while (in < n && hint != 0) {
    if (out.size() - done < 65536) out.resize(out.size() * 2);
    size_t dst = out.size() - done, srcn = n - in;
    hint = g_lz4.decompress(ctx, out.data() + done, &dst, src + in, &srcn, nullptr);
    if (g_lz4.isError(hint)) {
      g_lz4.freeD(ctx);
      return kCorrupt;
    }
    in += srcn;
    done += dst;
    if (srcn == 0 && dst == 0 && out.size() - done >= 65536) break;  // no progress
  }
  while (hint != 0) {  // flush what the context still holds
    if (out.size() - done < 65536) out.resize(out.size() * 2);
    size_t dst = out.size() - done, srcn = 0;
    hint = g_lz4.decompress(ctx, out.data() + done, &dst, src + in, &srcn, nullptr);
    if (g_lz4.isError(hint) || dst == 0) break;
    done += dst;
  }
  g_lz4.freeD(ctx);
  if (hint != 0) return kCorrupt;  // truncated frame
  out.resize(done);
  return kOk;
}

int lz4_compress(const uint8_t* src, size_t n, std::vector<uint8_t>& out) {
  load_libs();
  if (!g_has_lz4) return kNoLib;
  out.resize(g_lz4.bound(n, nullptr));
  const size_t r = g_lz4.compress(out.data(), out.size(), src, n, nullptr);
  if (g_lz4.isError(r)) return kCorrupt;
  out.resize(r);
  return kOk;
}

int zstd_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out) {
  load_libs();
  if (!g_has_zstd) return kNoLib;
  void* ds = g_zstd.createD();
  if (!ds || g_zstd.isError(g_zstd.initD(ds))) return kCorrupt;
  out.resize(n * 4 + 65536);
  ZIn in{src, n, 0};
  size_t done = 0, r = 1;
  while (true) {
    if (out.size() - done < 65536) out.resize(out.size() * 2);
    ZOut o{out.data() + done, out.size() - done, 0};
    r = g_zstd.decompressStream(ds, &o, &in);
    if (g_zstd.isError(r)) {
      g_zstd.freeD(ds);
      return kCorrupt;
    }
    done += o.pos;
    if (in.pos == in.size && (r == 0 || o.pos < o.size)) break;
  }
  g_zstd.freeD(ds);
  if (r != 0) return kCorrupt;  // frame incomplete
  out.resize(done);
  return kOk;
}

int zstd_compress(const uint8_t* src, size_t n, int level, std::vector<uint8_t>& out) {
  load_libs();
  if (!g_has_zstd) return kNoLib;
  out.resize(g_zstd.bound(n));
  const size_t r = g_zstd.compress(out.data(), out.size(), src, n, level < 0 ? 3 : level);
  if (g_zstd.isError(r)) return kCorrupt;
  out.resize(r);
  return kOk;
}

int decompress(int codec, const uint8_t* src, size_t n, std::vector<uint8_t>& out) {
  switch (codec) {
    case kGzip: return gzip_decompress(src, n, out);
    case kSnappy: return snappy_decompress(src, n, out);
    case kLz4: return lz4_decompress(src, n, out);
    case kZstd: return zstd_decompress(src, n, out);
    default: return kBadCodec;
  }
}

int compress(int codec, const uint8_t* src, size_t n, int level, std::vector<uint8_t>& out) {
  switch (codec) {
    case kGzip: return gzip_compress(src, n, level, out);
    case kSnappy: return snappy_compress(src, n, out);
    case kLz4: return lz4_compress(src, n, out);
    case kZstd: return zstd_compress(src, n, level, out);
    default: return kBadCodec;
  }
}

int hand_out(std::vector<uint8_t>& v, uint8_t** out, int64_t* out_n) {
  uint8_t* p = static_cast<uint8_t*>(std::malloc(v.size() ? v.size() : 1));
  if (!p) return kOom;
  if (!v.empty()) std::memcpy(p, v.data(), v.size());
  *out = p;
  *out_n = int64_t(v.size());
  return kOk;
}

// zig-zag varint of a record field
bool rd_varint(const uint8_t* p, size_t n, size_t& i, int64_t& v) {
  uint64_t u = 0;
  for (int s = 0; s < 64; s += 7) {
    if (i >= n) return false;
    const uint8_t b = p[i++];
    u |= uint64_t(b & 0x7F) << s;
    if (!(b & 0x80)) {
      v = int64_t(u >> 1) ^ -int64_t(u & 1);
      return true;
    }
  }
  return false;
}

int64_t be64(const uint8_t* p) {
  return int64_t(uint64_t(be32(p)) << 32 | be32(p + 4));
}

}  // namespace

OMLDM_HOST_API int omldm_codec_available(int codec) {
  load_libs();
  switch (codec) {
    case kNone:
    case kGzip:
    case kSnappy: return 1;
    case kLz4: return g_has_lz4 ? 1 : 0;
    case kZstd: return g_has_zstd ? 1 : 0;
    default: return 0;
  }
}

// *out is malloc'ed (release with omldm_codec_free). Returns 0 or a negative error.
OMLDM_HOST_API int omldm_codec_decompress(int codec, const uint8_t* src, int64_t n, uint8_t** out,
                                          int64_t* out_n) {
  std::vector<uint8_t> v;
  const int rc = decompress(codec, src, size_t(n), v);
  return rc ? rc : hand_out(v, out, out_n);
}

OMLDM_HOST_API int omldm_codec_compress(int codec, const uint8_t* src, int64_t n, int level,
                                        uint8_t** out, int64_t* out_n) {
  std::vector<uint8_t> v;
  const int rc = compress(codec, src, size_t(n), level, v);
  return rc ? rc : hand_out(v, out, out_n);
}

OMLDM_HOST_API void omldm_codec_free(void* p) { std::free(p); }

// Decodes the record set data[0:n] of one Fetch partition response. Record values with
// offset ≥ min_offset are appended to dst (≤ cap bytes, ≤ max_records records):
// offs[k+1] − offs[k] is record k's length (offs[0] = 0). *next_offset = offset after the
// last appended record (min_offset if none). A record that does not fit stops the walk
// (it is returned by the next call). Returns the number of records appended, or a negative
// error (kCrc: CRC-32C mismatch, kCorrupt, kNoLib: codec library missing). Control
// batches and fully consumed batches advance *next_offset past their last offset.
OMLDM_HOST_API int64_t omldm_kafka_decode_into(const uint8_t* data, int64_t n, int64_t min_offset,
                                               int64_t max_records, uint8_t* dst, int64_t cap,
                                               int64_t* offs, int64_t* next_offset,
                                               int verify_crc) {
  int64_t cnt = 0, used = 0;
  offs[0] = 0;
  *next_offset = min_offset;
  std::vector<uint8_t> inflated;
  size_t p = 0;
  while (p + 17 <= size_t(n) && cnt < max_records) {
    const int64_t base = be64(data + p);
    const int32_t blen = int32_t(be32(data + p + 8));
    const size_t end = p + 12 + size_t(blen);
    if (blen < 0 || end > size_t(n)) break;  // partial batch at the end of a fetch
    const uint8_t magic = data[p + 16];
    if (magic != 2 || blen < 49) {
      p = end;
      continue;
    }
    const uint8_t* body = data + p + 21;  // attributes … records
    const size_t blen2 = end - (p + 21);
    if (verify_crc && omldm_crc32c(body, int64_t(blen2), 0) != be32(data + p + 17)) return kCrc;
    const int attrs = int(uint16_t(body[0]) << 8 | body[1]);
    const int32_t count = int32_t(be32(body + 36));
    const int64_t last = base + int32_t(be32(body + 2));  // base + last offset delta
    if ((attrs & 0x20) || last < min_offset) {  // control batch / already consumed
      if (last + 1 > *next_offset) *next_offset = last + 1;  // step over a control batch
      p = end;
      continue;
    }
    const uint8_t* rec = body + 40;
    size_t rn = blen2 - 40;
    if (attrs & 7) {
      const int rc = decompress(attrs & 7, rec, rn, inflated);
      if (rc) return rc;
      rec = inflated.data();
      rn = inflated.size();
    }
    size_t q = 0;
    for (int32_t r = 0; r < count; ++r) {
      int64_t ln, tsd, od, kl, vl;
      if (!rd_varint(rec, rn, q, ln) || ln < 0 || q + size_t(ln) > rn) return kCorrupt;
      const size_t rend = q + size_t(ln);
      q += 1;  // record attributes
      if (!rd_varint(rec, rend, q, tsd) || !rd_varint(rec, rend, q, od) ||
          !rd_varint(rec, rend, q, kl))
        return kCorrupt;
      if (kl > 0) q += size_t(kl);
      if (!rd_varint(rec, rend, q, vl) || (vl > 0 && q + size_t(vl) > rend)) return kCorrupt;
      const int64_t off = base + od;
      if (off >= min_offset) {
        const int64_t len = vl > 0 ? vl : 0;
        if (used + len > cap || cnt >= max_records) return cnt;
        if (len) std::memcpy(dst + used, rec + q, size_t(len));
        used += len;
        offs[++cnt] = used;
        *next_offset = off + 1;
      }
      q = rend;
    }
    if (last + 1 > *next_offset) *next_offset = last + 1;  // compacted gaps included
    p = end;
  }
  return cnt;
}

namespace {
void put_varint(std::vector<uint8_t>& o, int64_t v) {
  uint64_t u = (uint64_t(v) << 1) ^ uint64_t(v >> 63);  // zig-zag
  while (u >= 0x80) {
    o.push_back(uint8_t(u | 0x80));
    u >>= 7;
  }
  o.push_back(uint8_t(u));
}
void put_be(std::vector<uint8_t>& o, uint64_t v, int bytes) {
  for (int k = bytes - 1; k >= 0; --k) o.push_back(uint8_t(v >> (8 * k)));
}
}  // namespace

// One RecordBatch v2 holding records block[offs[i] : offs[i+1]] (i < n; a trailing '\n'
// dropped when strip_nl) — the egress side: a tick's Prediction / response lines become
// one batch per Produce request without a Python object per record. Same layout as
// omldm_amd.io.kafka.encode_batch (null keys, no headers, one timestamp). *out is
// malloc'ed (omldm_codec_free). Returns 0 or a negative error.
OMLDM_HOST_API int omldm_kafka_encode_lines(const uint8_t* block, const int64_t* offs, int64_t n,
                                            int strip_nl, int64_t base_offset, int64_t ts_ms,
                                            int codec, int level, uint8_t** out,
                                            int64_t* out_n) {
  if (n <= 0) return kCorrupt;
  std::vector<uint8_t> recs, body;
  recs.reserve(size_t(offs[n] - offs[0]) + size_t(n) * 8);
  auto vsize = [](int64_t v) {
    uint64_t u = (uint64_t(v) << 1) ^ uint64_t(v >> 63);
    int k = 1;
    while (u >= 0x80) {
      u >>= 7;
      ++k;
    }
    return k;
  };
  for (int64_t i = 0; i < n; ++i) {
    int64_t a = offs[i], b = offs[i + 1];
    if (strip_nl && b > a && block[b - 1] == '\n') --b;
    const int64_t vl = b - a;
    // attributes, ts delta 0, offset delta i, null key, value length, value, 0 headers
    put_varint(recs, 1 + 1 + vsize(i) + 1 + vsize(vl) + vl + 1);
    recs.push_back(0);
    put_varint(recs, 0);
    put_varint(recs, i);
    put_varint(recs, -1);
    put_varint(recs, vl);
    recs.insert(recs.end(), block + a, block + b);
    recs.push_back(0);
  }
  const int c = codec & 7;
  put_be(body, uint64_t(c), 2);                          // attributes
  put_be(body, uint64_t(n - 1), 4);                      // last offset delta
  put_be(body, uint64_t(ts_ms), 8);                      // first timestamp
  put_be(body, uint64_t(ts_ms), 8);                      // max timestamp
  put_be(body, uint64_t(int64_t(-1)), 8);                // producer id
  put_be(body, uint64_t(uint16_t(int16_t(-1))), 2);      // producer epoch
  put_be(body, uint64_t(uint32_t(int32_t(-1))), 4);      // base sequence
  put_be(body, uint64_t(n), 4);                          // record count
  if (c) {
    std::vector<uint8_t> z;
    const int rc = compress(c, recs.data(), recs.size(), level, z);
    if (rc) return rc;
    body.insert(body.end(), z.begin(), z.end());
  } else {
    body.insert(body.end(), recs.begin(), recs.end());
  }
  std::vector<uint8_t> o;
  o.reserve(body.size() + 21);
  put_be(o, uint64_t(base_offset), 8);
  put_be(o, uint64_t(4 + 1 + 4 + body.size()), 4);  // batch length (after this field)
  put_be(o, 0, 4);                                  // partition leader epoch
  o.push_back(2);                                   // magic
  put_be(o, omldm_crc32c(body.data(), int64_t(body.size()), 0), 4);
  o.insert(o.end(), body.begin(), body.end());
  return hand_out(o, out, out_n);
}
