// Phase timestamps of the register-dedup linear round kernel (diagnostics, standalone).
// Builds linear_spoke.hip with OMLDM_RD_STAMPS: each spoke wave records a wall-clock
// start and shader-clock stamps after its row loads, w0 gathers, sequential chain, bucket
// inserts and flush (each after a full memory wait). Synthetic headline-shaped round:
// 8192 spokes × 16 rows, 13 bf16 numerical + 26 field-aware uint16 categorical features,
// int8 labels, 2^20 slots, bf16 model.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc/kernels \
//          -o /tmp/rdp csrc/tests/rd_stamp_probe.hip
#define OMLDM_RD_STAMPS 1
#include "../kernels/linear_spoke.hip"

#include <algorithm>
#include <cmath>
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
  const int S = argc > 1 ? atoi(argv[1]) : 8192, R = argc > 2 ? atoi(argv[2]) : 16;
  const int log2cap = argc > 3 ? atoi(argv[3]) : 10;
  const int B = S * R, dn = 13, dc = 26, dim = 1 << 20, cspan = 32767;
  std::mt19937 rng(25);
  std::vector<unsigned short> num(B * dn), cat(B * dc);
  std::vector<signed char> y(B);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  for (int i = 0; i < B * dn; ++i) {
    const float v = std::log1p(20.f * U(rng));
    __hip_bfloat16 b = __float2bfloat16(v);
    num[i] = *reinterpret_cast<unsigned short*>(&b);
  }
  // the bench stream's categorical law (csrc/host/ingest.cpp omldm_synth_batch): field j
  // has a vocabulary of 10^(1 + j % 6) values, ranks skewed toward small ones (u^3), and
  // a value's slot is a hash of (field, rank), so popular values recur inside a spoke
  for (int i = 0; i < B; ++i)
    for (int j = 0; j < dc; ++j) {
      double vocab = 10;
      for (int q = 0; q < j % 6; ++q) vocab *= 10;
      const double u = U(rng);
      const unsigned long long rank = (unsigned long long)(vocab * u * u * u);
      unsigned long long h = (j + 1) * 0x100000001b3ull ^ (rank * 0x9e3779b97f4a7c15ull);
      h ^= h >> 31;
      h *= 0xbf58476d1ce4e5b9ull;
      h ^= h >> 29;
      const unsigned local = (unsigned)((h & 0x7fffffffull) % cspan);
      cat[(size_t)i * dc + j] = (unsigned short)(local | ((h >> 63) ? 0x8000 : 0));
    }
  for (int i = 0; i < B; ++i) y[i] = U(rng) < 0.5f ? -1 : 1;
  void *dnum, *dcat, *dy, *dw, *dtab;
  float *dacc, *ws;
  double* cum;
  unsigned long long* stamps;
  CK(hipMalloc(&dnum, num.size() * 2));
  CK(hipMalloc(&dcat, cat.size() * 2));
  CK(hipMalloc(&dy, B));
  CK(hipMalloc(&dw, (size_t)dim * 2));
  CK(hipMalloc(&dacc, (size_t)(dim + 2) * 4));
  CK(hipMalloc(&ws, (size_t)S * (8 + dn + 1) * 4));
  CK(hipMalloc(&dtab, (size_t)S * ((1 << log2cap) + 64) * 8));
  CK(hipMalloc(&cum, 8 * 8));
  CK(hipMalloc(&stamps, (size_t)S * 8 * 8));
  CK(hipMemcpy(dnum, num.data(), num.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcat, cat.data(), cat.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dy, y.data(), B, hipMemcpyHostToDevice));
  CK(hipMemset(dw, 0, (size_t)dim * 2));
  CK(hipMemset(dacc, 0, (size_t)(dim + 2) * 4));
  CK(hipMemset(cum, 0, 64));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(omldm::g_rd_stamps), &stamps, sizeof(stamps)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 20;
  float best = 1e9f;
  for (int it = 0; it < iters; ++it) {
    CK(hipEventRecord(a, 0));
    int rc = omldm_linear_round(dw, 1, dnum, 1, dn, dcat, dc, dy, 1, B, R, S, dacc, dim, ws, dtab, cum,
                                0, 1, 1.f, 0.f, 0.1f, 0.f, 1.f / S, 1, cspan, log2cap, 8, 0, 1,
                                nullptr);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    if (rc) {
      fprintf(stderr, "omldm_linear_round rc=%d\n", rc);
      return 1;
    }
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, ms);
  }
  std::vector<unsigned long long> st((size_t)S * 8);
  CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
  printf("S=%d R=%d log2cap=%d: round+reduce best %.1f us\n", S, R, log2cap, best * 1000.f);
  const char* ph[] = {"loads", "gathers", "chain", "inserts", "flush+ws"};
  for (int k = 0; k < 5; ++k) {
    std::vector<double> v;
    for (int s = 0; s < S; ++s) v.push_back((double)(st[s * 8 + k + 2] - st[s * 8 + k + 1]));
    std::sort(v.begin(), v.end());
    double m = 0;
    for (double x : v) m += x;
    printf("  %-9s cycles: mean %8.0f  p10 %8.0f  p50 %8.0f  p90 %8.0f\n", ph[k], m / S, v[S / 10],
           v[S / 2], v[S * 9 / 10]);
  }
  std::vector<double> life, start;
  for (int s = 0; s < S; ++s) {
    life.push_back((double)(st[s * 8 + 6] - st[s * 8 + 1]));
    start.push_back((double)st[s * 8 + 0]);
  }
  std::sort(life.begin(), life.end());
  const double t0 = *std::min_element(start.begin(), start.end());
  for (auto& x : start) x = (x - t0) / 100.0;  // wall clock 100 MHz → µs
  std::vector<double> ss = start;
  std::sort(ss.begin(), ss.end());
  printf("  wave lifetime cycles p50 %.0f p90 %.0f; start times (us from first): p10 %.1f p50 %.1f p90 %.1f max %.1f\n",
         life[S / 2], life[S * 9 / 10], ss[S / 10], ss[S / 2], ss[S * 9 / 10], ss[S - 1]);
  return 0;
}
