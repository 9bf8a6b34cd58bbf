// Phase times of the fused NN round kernel (diagnostics, standalone): builds mlp.hip with
// OMLDM_MLP_STAMPS, runs the learner-bench round (131072 rows, [13 → 64 → 64 → 1], binary
// logistic, 512 spokes × 256 rows) and prints, per spoke, the shader-clock cycles spent in
// each mini-batch phase summed over the spoke's mini-batches.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc/kernels \
//          -o /tmp/mlpp csrc/tests/mlp_stamp_probe.hip
#define OMLDM_MLP_STAMPS 1
#include "../kernels/mlp.hip"

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
  const int S = argc > 1 ? atoi(argv[1]) : 512;
  const int bf16 = argc > 2 ? atoi(argv[2]) : 1;
  if (argc > 3) omldm_mlp_form(atoi(argv[3]));  // 0 v1 (phase stamps), 1 / 2 v2 (4 / 8 waves)
  const long long B = 131072;
  const int R = (int)(B / S);
  const int widths[4] = {13, 64, 64, 1};
  const int L = 3;
  long long nparams = 0;
  for (int l = 0; l < L; ++l) nparams += (long long)widths[l + 1] * widths[l] + widths[l + 1];
  std::mt19937 rng(5);
  std::normal_distribution<float> N(0.f, 1.f);
  std::vector<float> x(B * widths[0]), y(B), w(nparams);
  for (auto& v : x) v = N(rng);
  for (auto& v : y) v = N(rng) > 0 ? 1.f : -1.f;
  for (auto& v : w) v = 0.1f * N(rng);
  float *dx, *dy, *dw, *dacc, *stats, *ws;
  unsigned long long* stamps;
  CK(hipMalloc(&dx, x.size() * 4));
  CK(hipMalloc(&dy, y.size() * 4));
  CK(hipMalloc(&dw, w.size() * 4));
  CK(hipMalloc(&dacc, w.size() * 4));
  CK(hipMalloc(&stats, 64));
  CK(hipMalloc(&ws, (size_t)S * nparams * 4));
  CK(hipMalloc(&stamps, (size_t)S * 8 * 8));
  CK(hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dy, y.data(), y.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(omldm::g_mlp_stamps), &stamps, sizeof(stamps)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e9f;
  for (int it = 0; it < 10; ++it) {
    CK(hipMemset(stamps, 0, (size_t)S * 64));
    CK(hipEventRecord(a, 0));
    const int rc = omldm_mlp_round(dw, dx, dy, B, R, S, L, widths, 1, bf16 ? 256 : 0, 0.1f, dacc,
                                   stats, nullptr, ws, nullptr);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    if (rc) {
      fprintf(stderr, "omldm_mlp_round rc=%d\n", rc);
      return 1;
    }
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, ms);
  }
  std::vector<unsigned long long> st((size_t)S * 8);
  CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
  printf("S=%d R=%d bf16=%d: round (+colsum) best %.1f us\n", S, R, bf16, best * 1000.f);
  const bool v2 = omldm_mlp_form(-1) > 0;
  const char* ph1[] = {"", "stage+barrier", "forward", "loss", "backward rest", "bwd dH+sync",
                       "bwd W update", "bwd bias+sync"};
  const char* ph2[] = {"", "stage+barrier+cnt", "hidden forward", "output+loss", "bwd phase 0",
                       "bwd phase 1", "bwd phase 2", "bwd phase 3+"};
  const char* const* ph = v2 ? ph2 : ph1;
  const int mbs = (R + 31) / 32;
  for (int k = 1; k <= 7; ++k) {
    std::vector<double> v;
    for (int s = 0; s < S; ++s) v.push_back((double)st[s * 8 + k] / mbs);
    std::sort(v.begin(), v.end());
    printf("  %-14s cycles per mini-batch: p50 %8.0f  p90 %8.0f\n", ph[k], v[S / 2], v[S * 9 / 10]);
  }
  return 0;
}
