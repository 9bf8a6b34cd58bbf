// Host data-plane self-test, built and run under sanitizers by tests/test_sanitizers.py
// (the reference had none and crashed with a native race in ND4J).
//
//   ASan+UBSan: g++ -fsanitize=address,undefined  (memory errors, UB in the parsers)
//   TSan:       g++ -fsanitize=thread             (the multi-threaded parse/synth/round
//                                                   paths share output buffers by row range)
// It drives every exported host entry point with adversarial inputs (truncated JSON,
// huge numbers, empty records, absent fields) and multi-threaded configurations, and
// checks a few invariants so the run also fails on wrong results, not only on reports.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
uint32_t omldm_murmur3_32(const char* s, int64_t n, uint32_t seed);
uint32_t omldm_crc32c(const uint8_t* p, int64_t n, uint32_t crc);
int32_t omldm_hash_cat(const char* s, int64_t n, int field, int dn, int64_t dim);
int32_t omldm_hash_cat16(const char* s, int64_t n, int field, int cspan);
int64_t omldm_parse_instances(const char* buf, const int64_t* off, int n, int dnum, int ddisc,
                              int dc, int64_t dim, int cspan, float* num, void* cat, float* y,
                              int8_t* op, int nthreads);
void omldm_synth_batch(uint64_t seed, int64_t start, int B, int dn, int dc, int64_t dim, int task,
                       int n_classes, float noise, int cspan, float* num, void* cat, float* y,
                       int nthreads);
int omldm_cpu_linear_round(const void* w, int w_bf16, const float* num, int dn, const void* cat,
                           int dc, const float* y, int B, int R, int S, float* dacc, int dim,
                           float* stats, int rule, int variant, float C, float eps, float lr,
                           float lam, float inv_p, int bias, int cspan, int nthreads);
void omldm_cpu_linear_apply(float* w32, uint16_t* w16, float* dacc, int dim);
void omldm_cpu_linear_predict(const float* w, long long wstride, int M, const float* num, int dn,
                              const void* cat, int dc, int B, int dim, int bias, int cspan,
                              const float* wscale, float* out);
int omldm_codec_available(int codec);
int omldm_codec_decompress(int codec, const uint8_t* src, int64_t n, uint8_t** out, int64_t* on);
int omldm_codec_compress(int codec, const uint8_t* src, int64_t n, int level, uint8_t** out,
                         int64_t* on);
void omldm_codec_free(void* p);
int64_t omldm_kafka_decode_into(const uint8_t* data, int64_t n, int64_t min_offset,
                                int64_t max_records, uint8_t* dst, int64_t cap, int64_t* offs,
                                int64_t* next_offset, int verify_crc);
int omldm_kafka_encode_lines(const uint8_t* block, const int64_t* offs, int64_t n, int strip_nl,
                             int64_t base_offset, int64_t ts_ms, int codec, int level,
                             uint8_t** out, int64_t* out_n);
}

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                  \
    }                                                              \
  } while (0)

static void test_hashes() {
  CHECK(omldm_crc32c(reinterpret_cast<const uint8_t*>("123456789"), 9, 0) == 0xE3069283u);
  CHECK(omldm_murmur3_32("", 0, 0) == 0u);
  for (int f = 0; f < 26; ++f) {
    const int32_t s = omldm_hash_cat("abc", 3, f, 13, 1 << 20);
    const int32_t v = s & 0x7fffffff;  // bit 31 = feature sign
    CHECK(v >= 0 && v < (1 << 20));
    (void)omldm_hash_cat16("abc", 3, f, 1000);
  }
}

static void test_parser() {
  const char* recs[] = {
      R"({"numericalFeatures":[1.5,-2,3e2],"categoricalFeatures":["a","b"],"target":1,"operation":"training"})",
      R"({"numericalFeatures":[1e400,-1e-400,0],"target":-1})",
      R"({"numericalFeatures":[1,2,)",  // truncated
      R"()",
      R"({"operation":"forecasting","categoricalFeatures":["x","y","z","w","v"]})",
      R"({"numericalFeatures":[1,2,3,4,5,6,7,8,9,10,11,12,13,14,15],"target":0.5})",
      R"({"discreteFeatures":[1,2],"target":"oops"})",
      R"(EOS)",
      R"({"numericalFeatures":[],"categoricalFeatures":[],"target":null,"operation":"training"})",
  };
  const int n0 = sizeof(recs) / sizeof(recs[0]);
  std::string buf;
  std::vector<int64_t> off{0};
  for (int rep = 0; rep < 200; ++rep)
    for (int i = 0; i < n0; ++i) {
      buf += recs[i];
      off.push_back((int64_t)buf.size());
    }
  const int n = (int)off.size() - 1;
  const int dnum = 3, ddisc = 2, dc = 4;
  for (int cspan : {0, 1000}) {
    for (int threads : {1, 4}) {
      std::vector<float> num((size_t)n * (dnum + ddisc), -7.f), y(n, -7.f);
      std::vector<int32_t> cat((size_t)n * dc, -7);
      std::vector<int8_t> op(n, -7);
      const int64_t valid = omldm_parse_instances(buf.data(), off.data(), n, dnum, ddisc, dc,
                                                  1 << 20, cspan, num.data(), cat.data(),
                                                  y.data(), op.data(), threads);
      CHECK(valid > 0 && valid < n);
      for (int i = 0; i < n; ++i) CHECK(op[i] >= -1 && op[i] <= 2);
    }
  }
}

static void test_linear_paths() {
  const int dn = 13, dc = 26, dim = 1 << 16, B = 4096, S = 64, R = B / S;
  std::vector<float> num((size_t)B * dn), y(B);
  std::vector<int32_t> cat((size_t)B * dc);
  omldm_synth_batch(7, 0, B, dn, dc, dim, 0, 2, 0.1f, 0, num.data(), cat.data(), y.data(), 8);
  std::vector<float> w(dim, 0.f), dacc(dim + 2, 0.f), stats((size_t)S * 6, 0.f);  // [S, 6]
  std::vector<uint16_t> w16(dim, 0);
  for (int round = 0; round < 3; ++round) {
    const int rc = omldm_cpu_linear_round(w.data(), 0, num.data(), dn, cat.data(), dc, y.data(),
                                          B, R, S, dacc.data(), dim, stats.data(), 0, 1, 1.f,
                                          0.1f, 0.01f, 0.f, 1.f / S, 1, 0, 8);
    CHECK(rc == 0);
    omldm_cpu_linear_apply(w.data(), w16.data(), dacc.data(), dim);
  }
  std::vector<float> out(B);
  omldm_cpu_linear_predict(w.data(), dim, 1, num.data(), dn, cat.data(), dc, B, dim, 1, 0, nullptr,
                           out.data());
  int correct = 0;
  for (int i = 0; i < B; ++i) correct += (out[i] >= 0.f) == (y[i] > 0.f);
  CHECK(correct > B * 6 / 10);
  for (float v : w) CHECK(std::isfinite(v));
}

static void test_concurrent_callers() {
  // Several host threads drive the (internally threaded) generator at once on disjoint
  // outputs — the pattern of the engine's prefetch pool.
  const int dn = 13, dc = 26, B = 2048;
  std::vector<std::thread> ts;
  std::vector<std::vector<float>> nums(4, std::vector<float>((size_t)B * dn));
  std::vector<std::vector<uint16_t>> cats(4, std::vector<uint16_t>((size_t)B * dc));
  std::vector<std::vector<float>> ys(4, std::vector<float>(B));
  for (int t = 0; t < 4; ++t)
    ts.emplace_back([&, t] {
      omldm_synth_batch(3, (int64_t)t * B, B, dn, dc, 1 << 20, 0, 2, 0.1f, 1000, nums[t].data(),
                        cats[t].data(), ys[t].data(), 2);
    });
  for (auto& t : ts) t.join();
  CHECK(std::memcmp(nums[0].data(), nums[1].data(), nums[0].size() * 4) != 0);
}

// Kafka codecs: round trips from several threads at once (the libraries are loaded on
// first use, under TSan here), then mutated streams into every decoder and the record-set
// decoder — they must fail cleanly, never read or write out of bounds (ASan/UBSan).
static void test_kafka_wire() {
  std::vector<uint8_t> src(200000);
  for (size_t i = 0; i < src.size(); ++i) src[i] = uint8_t((i * 7) % 251 ^ (i / 1000));
  std::vector<std::thread> ts;
  std::vector<int> ok(8, 0);
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&, t] {
      const int codec = 1 + t % 4;
      if (!omldm_codec_available(codec)) {
        ok[t] = 1;
        return;
      }
      uint8_t *z = nullptr, *d = nullptr;
      int64_t zn = 0, dn = 0;
      if (omldm_codec_compress(codec, src.data(), (int64_t)src.size(), -1, &z, &zn)) return;
      if (omldm_codec_decompress(codec, z, zn, &d, &dn) == 0 && dn == (int64_t)src.size() &&
          std::memcmp(d, src.data(), src.size()) == 0)
        ok[t] = 1;
      omldm_codec_free(z);
      omldm_codec_free(d);
    });
  for (auto& t : ts) t.join();
  for (int v : ok) CHECK(v == 1);
  uint32_t rng = 12345;
  for (int codec = 1; codec <= 4; ++codec) {
    if (!omldm_codec_available(codec)) continue;
    uint8_t* z = nullptr;
    int64_t zn = 0;
    CHECK(omldm_codec_compress(codec, src.data(), 5000, -1, &z, &zn) == 0);
    std::vector<uint8_t> m(z, z + zn);
    omldm_codec_free(z);
    for (int trial = 0; trial < 200; ++trial) {
      std::vector<uint8_t> b = m;
      for (int k = 0; k < 3; ++k) {
        rng = rng * 1664525u + 1013904223u;
        b[rng % b.size()] ^= uint8_t(rng >> 24);
      }
      rng = rng * 1664525u + 1013904223u;
      const size_t cut = trial % 2 ? b.size() : rng % (b.size() + 1);
      uint8_t* d = nullptr;
      int64_t dn = 0;
      if (omldm_codec_decompress(codec, b.data(), (int64_t)cut, &d, &dn) == 0) omldm_codec_free(d);
    }
  }
  {  // encode a block of lines with every codec, decode it back into a staging buffer
    std::string blk;
    std::vector<int64_t> lo{0};
    for (int i = 0; i < 300; ++i) {
      blk += "{\"i\": " + std::to_string(i) + "}\n";
      lo.push_back((int64_t)blk.size());
    }
    for (int codec = 0; codec <= 4; ++codec) {
      if (!omldm_codec_available(codec)) continue;
      uint8_t* rs = nullptr;
      int64_t rn = 0;
      CHECK(omldm_kafka_encode_lines(reinterpret_cast<const uint8_t*>(blk.data()), lo.data(), 300,
                                     1, 40, 1, codec, -1, &rs, &rn) == 0);
      std::vector<uint8_t> dst2(blk.size());
      std::vector<int64_t> o2(301);
      int64_t nxt = 0;
      CHECK(omldm_kafka_decode_into(rs, rn, 40, 300, dst2.data(), (int64_t)dst2.size(), o2.data(),
                                    &nxt, 1) == 300);
      CHECK(nxt == 340 && o2[300] == (int64_t)blk.size() - 300);
      omldm_codec_free(rs);
    }
  }
  std::vector<uint8_t> junk(4096), dst(1 << 16);
  std::vector<int64_t> offs(1025);
  for (int trial = 0; trial < 200; ++trial) {
    for (auto& c : junk) {
      rng = rng * 1664525u + 1013904223u;
      c = uint8_t(rng >> 24);
    }
    junk[16] = 2;  // magic 2 so the walk reaches the record parser
    junk[8] = 0;
    junk[9] = 0;
    junk[10] = uint8_t(trial * 13);
    int64_t nxt = 0;
    (void)omldm_kafka_decode_into(junk.data(), (int64_t)junk.size(), 0, 1024, dst.data(),
                                  (int64_t)dst.size(), offs.data(), &nxt, 0);
  }
}

int main() {
  test_hashes();
  test_kafka_wire();
  test_parser();
  test_linear_paths();
  test_concurrent_callers();
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("host selftest OK\n");
  return 0;
}
