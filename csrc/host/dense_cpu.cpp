// Host (CPU) forms of the dense online learners' exact per-point updates — the oracles of
// the GPU kernels and the CPU engine's path.
//
// omldm_cpu_kmeans_seq: sequential (MacQueen) k-means, csrc/kernels/kmeans_seq.hip's
// semantics exactly: the first k training points seed the centroids (n = 1), then each
// point moves its nearest centroid (ties: lowest index) by c ← c + (x − c)/n.
#include <cmath>
#include <cstdint>

#define OMLDM_API extern "C" __attribute__((visibility("default")))

OMLDM_API int omldm_cpu_kmeans_seq(const float* x, int ldx, const float* y, int B, int d, int k,
                                   float* cent, float* cnt, double* cum) {
  if (d < 1 || k < 1 || ldx < d) return -1;
  int seeded = 0;
  while (seeded < k && cnt[seeded] > 0.f) ++seeded;
  double inertia = 0.0, fitted = 0.0;
  for (int r = 0; r < B; ++r) {
    if (y && std::isnan(y[r])) continue;
    const float* xs = x + (size_t)r * ldx;
    fitted += 1.0;
    if (seeded < k) {
      for (int i = 0; i < d; ++i) cent[(size_t)seeded * d + i] = xs[i];
      cnt[seeded] = 1.f;
      ++seeded;
      continue;
    }
    int best = 0;
    float bd = INFINITY;
    for (int j = 0; j < k; ++j) {
      float dist = 0.f;
      for (int i = 0; i < d; ++i) {
        const float t = xs[i] - cent[(size_t)j * d + i];
        dist = std::fma(t, t, dist);
      }
      if (dist < bd) {
        bd = dist;
        best = j;
      }
    }
    inertia += (double)bd;
    cnt[best] += 1.f;
    const float a = 1.f / cnt[best];
    for (int i = 0; i < d; ++i) {
      float& c = cent[(size_t)best * d + i];
      c = std::fma(a, xs[i] - c, c);
    }
  }
  if (cum) {
    cum[0] += inertia;
    cum[1] += fitted;
  }
  return 0;
}
