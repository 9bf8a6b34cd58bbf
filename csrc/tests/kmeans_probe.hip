// K-means assign timing by batch size (diagnostics, standalone): separates the fixed
// per-launch cost (centroid staging, flush) from the per-row cost.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc/kernels \
//          -o /tmp/kmp csrc/tests/kmeans_probe.hip
#include "../kernels/dense_learners.hip"

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const int d = argc > 1 ? atoi(argv[1]) : 13;
  const int k = argc > 2 ? atoi(argv[2]) : 256;
  const long long Bmax = 131072;
  std::mt19937 rng(5);
  std::normal_distribution<float> N(0.f, 1.f);
  std::vector<float> x(Bmax * d), c(k * d), y(Bmax, 0.f);
  for (auto& v : x) v = N(rng);
  for (auto& v : c) v = N(rng);
  float *dx, *dy, *dc, *ds, *dn, *di, *dp;
  CK(hipMalloc(&dx, x.size() * 4));
  CK(hipMalloc(&dy, y.size() * 4));
  CK(hipMalloc(&dc, c.size() * 4));
  CK(hipMalloc(&ds, c.size() * 4));
  CK(hipMalloc(&dn, k * 4));
  CK(hipMalloc(&di, 4));
  CK(hipMalloc(&dp, (size_t)512 * (k * d + k + 1) * 4));
  CK(hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dy, y.data(), y.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, c.data(), c.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (long long B : {32LL, 8192LL, 32768LL, 65536LL, 131072LL}) {
    for (int ab : {0, 3, 4}) {  // 4: per-block atomics instead of the partials image
      setenv("OMLDM_KMEANS_ABLATE", ab == 3 ? "3" : "0", 1);
      float best = 1e9f;
      for (int it = 0; it < 20; ++it) {
        CK(hipEventRecord(a, 0));
        const int rc = omldm_kmeans_assign(dx, dy, (int)B, d, k, dc, ds, dn, nullptr, di,
                                             ab == 4 ? nullptr : dp, nullptr);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        if (rc) {
          fprintf(stderr, "rc=%d\n", rc);
          return 1;
        }
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        best = std::min(best, ms);
      }
      printf("d=%d k=%d B=%lld ablate=%d: %.1f us\n", d, k, B, ab, best * 1000.f);
    }
  }
  return 0;
}
