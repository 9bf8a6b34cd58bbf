// ORR Gram timing (diagnostics, standalone): gram_update_poly2 on the config-4 shape
// (13 raw features, 91 degree-2 pairs) by batch size; built twice, the second time with
// OMLDM_GRAM_PROBE_NOFLUSH (the blocks skip their final atomics into G).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc/kernels \
//          [-DOMLDM_GRAM_PROBE_NOFLUSH] -o /tmp/grp csrc/tests/gram_probe.hip
#include "../kernels/dense_learners.hip"

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

int main() {
  const int d0 = 13;
  std::vector<int> pairs;
  for (int a = 0; a < d0; ++a)
    for (int b = a; b < d0; ++b) {
      pairs.push_back(a);
      pairs.push_back(b);
    }
  const int np = (int)pairs.size() / 2, ld = 128;
  const long long Bmax = 262144;
  std::mt19937 rng(5);
  std::normal_distribution<float> N(0.f, 1.f);
  std::vector<float> x(Bmax * d0), y(Bmax);
  for (auto& v : x) v = N(rng);
  for (auto& v : y) v = N(rng);
  float *dx, *dy, *G;
  int* dp;
  double* cnt;
  float* part;
  hipMalloc(&dx, x.size() * 4);
  hipMalloc(&dy, y.size() * 4);
  hipMalloc(&G, ld * ld * 4);
  hipMalloc(&dp, pairs.size() * 4);
  hipMalloc(&cnt, 8);
  hipMalloc(&part, (size_t)256 * 10240 * 4);
  hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dy, y.data(), y.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dp, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (long long B : {64LL, 16384LL, 65536LL, 131072LL, 262144LL}) {
    float best = 1e9f;
    for (int it = 0; it < 20; ++it) {
      hipEventRecord(a, 0);
      const int rc = omldm_gram_update_poly2(dx, dy, (int)B, d0, dp, np, G, ld, cnt,
                                             getenv("GRP_ATOMICS") ? nullptr : part, nullptr);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      if (rc) {
        fprintf(stderr, "rc=%d\n", rc);
        return 1;
      }
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
#ifdef OMLDM_GRAM_PROBE_NOFLUSH
    const char* tag = "no flush";
#else
    const char* tag = "full";
#endif
    printf("gram poly2 d0=%d B=%lld (%s): %.1f us (incl. mirror launch)\n", d0, B, tag, best * 1000.f);
  }
  return 0;
}
