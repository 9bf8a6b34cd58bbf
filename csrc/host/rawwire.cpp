// Raw binary DataInstance wire + the exact sequential CPU learner on it.
//
// Wire (one micro-batch, columnar, what bench.py ships over PCIe and the engine's binary
// topic carries):
//   num [B, dn] float32   numerical then discrete features
//   tok [B, dc] uint32    raw categorical token id per field (0xFFFFFFFF = absent) —
//                         hashed field-aware on the GPU inside the training kernel
//                         (hashing.h: hash_token)
//   y   [B]     float32 or int8 (±1 classification labels), NaN = no target
//
// omldm_cpu_linear_seq_round is the reference semantics of one Synchronous round
// (omldm/operators/spoke/FlinkSpoke.scala:92-107: every spoke fits its shard strictly
// one example at a time on its own full model replica; SynchronousParameterServer
// averages the replicas). It is the golden oracle of the GPU
// Gram-scan kernel (csrc/kernels/linear_seq.hip) and the reference-class CPU baseline:
// dense per-thread delta arrays (no hash maps), tokens hashed inline.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "hashing.h"

#define OMLDM_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

using omldm_hash::hash_token;
using omldm_hash::kAbsentToken;

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
inline uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9e3779b97f4a7c15ull);
  return mix64(z);
}
inline double u01(uint64_t& s) { return (splitmix64(s) >> 11) * (1.0 / 9007199254740992.0); }
inline double gauss(uint64_t& s) {
  double u1 = u01(s), u2 = u01(s);
  if (u1 < 1e-300) u1 = 1e-300;
  return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

template <typename F>
void parallel_for(int n, int nthreads, F&& f) {
  if (nthreads <= 1 || n < 2) {
    f(0, n, 0);
    return;
  }
  nthreads = std::min(nthreads, n);
  std::vector<std::thread> th;
  const int chunk = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    const int a = t * chunk, b = std::min(n, a + chunk);
    if (a >= b) break;
    th.emplace_back([&, a, b, t] { f(a, b, t); });
  }
  for (auto& x : th) x.join();
}

struct Rule {
  int rule, variant;
  float C, eps, lr, lam;
};

// (loss, mistake, sq_err, c) of one example with margin m, label y, ‖x‖² n2 — the same
// closed forms as the GPU kernels (Crammer et al. 2006 PA family). T is
// float (the GPU's precision) or double (the reference's Breeze Double vectors,
// omldm/state/StateAccumulators.scala:5,26).
template <typename T>
inline T step(const Rule& r, T m, T y, T n2, T& loss, T& mist, T& sqe) {
  const T C = (T)r.C, zero = (T)0, one = (T)1;
  if (r.rule == 0) {  // hinge: PA / PA-I / PA-II
    const T ym = y * m;
    const T l = std::fmax(zero, one - ym);
    loss += l;
    mist += ym <= zero ? one : zero;
    if (l <= zero || n2 <= zero) return zero;
    const T tau = r.variant == 0 ? l / n2
                : r.variant == 1 ? std::fmin(C, l / n2)
                                 : l / (n2 + (T)0.5 / C);
    return tau * y;
  }
  if (r.rule == 1) {  // ε-insensitive regression
    const T err = y - m;
    const T l = std::fmax(zero, std::fabs(err) - (T)r.eps);
    loss += l;
    sqe += err * err;
    if (l <= zero || n2 <= zero) return zero;
    const T tau = r.variant == 0 ? l / n2
                : r.variant == 1 ? std::fmin(C, l / n2)
                                 : l / (n2 + (T)0.5 / C);
    return err >= zero ? tau : -tau;
  }
  // logistic SGD
  const T z = y * m;
  loss += z > zero ? std::log1p(std::exp(-z)) : (-z + std::log1p(std::exp(z)));
  mist += z <= zero ? one : zero;
  return (T)r.lr * y / (one + std::exp(z));
}

}  // namespace

// Deterministic Criteo-shaped raw stream: dn Gaussian numerical features, dc categorical
// fields with skewed vocabularies (field j: 10^(1 + j % 6) values, rank ∝ u³), each value
// a 32-bit token id. Labels come from a hidden model over (field, token) — not over hash
// slots, so hashing collisions are real modelling noise. Example i is a pure function of
// (seed, start + i): any shard can be generated independently on any rank.
//   task 0: ±1 labels; 1: regression target; 2: K-class labels in [0, K)
OMLDM_HOST_API void omldm_synth_raw(uint64_t seed, int64_t start, int B, int dn, int dc, int task,
                                    int n_classes, float noise, float missing, float* num,
                                    uint32_t* tok, float* y, int nthreads) {
  parallel_for(B, nthreads, [&](int a, int b, int) {
    for (int i = a; i < b; ++i) {
      uint64_t s = mix64(seed * 0x9e3779b97f4a7c15ull + uint64_t(start + i) + 0x5151ull);
      float* xn = num + int64_t(i) * dn;
      uint32_t* xt = tok + int64_t(i) * dc;
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
        int64_t vocab = 10;
        for (int q = 0; q < j % 6; ++q) vocab *= 10;
        const double u = u01(s);
        const double um = u01(s);
        if (missing > 0.f && um < missing) {
          xt[j] = kAbsentToken;
          continue;
        }
        const int64_t rank = int64_t(double(vocab) * u * u * u);
        uint32_t t = uint32_t(mix64(seed + uint64_t(j) * 0x100000001b3ull + uint64_t(rank) * 0x9e37ull));
        if (t == kAbsentToken) t = 0;
        xt[j] = t;
        const uint64_t hv = mix64((seed ^ 0x27d4eb2dull) + uint64_t(j) * 0x1f1f1f1full + uint64_t(t));
        // the value's effect as seen through its hashed feature (x = ±1 by the hash sign)
        const double sv = (hash_token(t, j, 0, 1, int64_t(1) << 30) < 0) ? -1.0 : 1.0;
        for (int k = 0; k < K; ++k) {
          uint64_t hs = mix64(hv + uint64_t(k) * 104729);
          score[k] += sv * (gauss(hs) * 0.5);
        }
      }
      const double e = noise * gauss(s);
      if (task == 0) {
        y[i] = (score[0] + e) >= 0.0 ? 1.f : -1.f;
      } else if (task == 1) {
        y[i] = float(score[0] + e);
      } else {
        int best = 0;
        for (int k = 1; k < K; ++k)
          if (score[k] > score[best]) best = k;
        y[i] = float(best);
      }
    }
  });
}

// Raw tokens → the wide hashed form (int32 signed slot, -1 = absent) every learner reads.
OMLDM_HOST_API void omldm_cpu_hash_raw(const uint32_t* tok, int64_t B, int dc, int dn, int64_t dim,
                                   int32_t* cat, int nthreads) {
  parallel_for(int(std::min<int64_t>(B, 1 << 30)), nthreads, [&](int a, int b, int) {
    for (int64_t i = a; i < b; ++i)
      for (int j = 0; j < dc; ++j) {
        const uint32_t t = tok[i * dc + j];
        cat[i * dc + j] = t == kAbsentToken ? -1 : hash_token(t, j, dn, dc, dim);
      }
  });
}

// One round of S spokes (spoke s: rows [s·R, (s+1)·R)), each an exact sequential learner
// on its replica w + Δ_s. Accumulates like omldm_cpu_linear_round: dacc[:dim] += Δ_s·inv_p,
// dacc[dim] += inv_p, dacc[dim + 1] += inv_p for every spoke with rows (so linear_apply
// yields w + Σ Δ_s / P_active — model averaging). stats [S, 6]: loss, n, mistakes,
// sq_err, 1, 0. The merge runs in spoke order: the result does not depend on nthreads.
// y8 != 0: labels are int8.
template <typename T>
static int cpu_linear_seq_round(const T* w, const float* num, int dn,
                                              const uint32_t* tok, int dc, const void* yv,
                                              int y8, int B, int R, int S, T* dacc, int dim,
                                              float* stats, int rule, int variant, float C,
                                              float eps, float lr, float inv_p, int bias,
                                              int nthreads) {
  const Rule r{rule, variant, C, eps, lr, 0.f};
  if (S <= 0 || R <= 0) return 0;
  std::vector<std::vector<std::pair<int, T>>> out(S);
  const int nth = std::max(1, std::min(nthreads, S));
  parallel_for(S, nth, [&](int s0, int s1, int) {
    std::vector<T> D(dim, (T)0);
    std::vector<int> touched;
    std::vector<int> idx(dn + dc + 1);
    std::vector<T> xv(dn + dc + 1);
    for (int s = s0; s < s1; ++s) {
      const int64_t a = std::min<int64_t>(int64_t(s) * R, B);
      const int64_t b = std::min<int64_t>(a + R, B);
      T loss = 0, nex = 0, mist = 0, sqe = 0;
      touched.clear();
      for (int64_t t = a; t < b; ++t) {
        const T yt = y8 ? T(static_cast<const int8_t*>(yv)[t])
                        : T(static_cast<const float*>(yv)[t]);
        if (std::isnan(yt)) continue;
        int F = 0;
        for (int j = 0; j < dn && j < dim; ++j) {
          idx[F] = j;
          xv[F++] = num[t * dn + j];
        }
        for (int j = 0; j < dc; ++j) {
          const uint32_t tk = tok[t * dc + j];
          if (tk == kAbsentToken) continue;
          const int32_t h = hash_token(tk, j, dn, dc, dim);
          idx[F] = h & 0x7fffffff;
          xv[F++] = h < 0 ? T(-1) : T(1);
        }
        if (bias) {
          idx[F] = dim - 1;
          xv[F++] = T(1);
        }
        T m = 0, n2 = 0;
        for (int f = 0; f < F; ++f) {
          m += xv[f] * (w[idx[f]] + D[idx[f]]);
          n2 += xv[f] * xv[f];
        }
        const T c = step<T>(r, m, yt, n2, loss, mist, sqe);
        nex += T(1);
        if (c != T(0))
          for (int f = 0; f < F; ++f) {
            T& d = D[idx[f]];
            if (d == T(0)) touched.push_back(idx[f]);
            d += c * xv[f];
          }
      }
      auto& o = out[s];
      o.clear();
      for (int j : touched) {
        if (D[j] != T(0)) o.emplace_back(j, D[j]);
        D[j] = T(0);
      }
      // a key whose delta returned to exactly 0 and was touched again appears twice:
      // the first entry was taken and zeroed, the second finds 0 and is skipped
      float* st = stats ? stats + size_t(s) * 6 : nullptr;
      if (st) {
        st[0] = (float)loss;
        st[1] = (float)nex;
        st[2] = (float)mist;
        st[3] = (float)sqe;
        st[4] = 1.f;
        st[5] = 0.f;
      }
    }
  });
  for (int s = 0; s < S; ++s) {
    if (int64_t(s) * R >= B) continue;
    for (auto& kv : out[s]) dacc[kv.first] += kv.second * (T)inv_p;
    dacc[dim] += (T)inv_p;
    dacc[dim + 1] += (T)inv_p;
  }
  return 0;
}

OMLDM_HOST_API int omldm_cpu_linear_seq_round(const float* w, const float* num, int dn,
                                              const uint32_t* tok, int dc, const void* yv,
                                              int y8, int B, int R, int S, float* dacc, int dim,
                                              float* stats, int rule, int variant, float C,
                                              float eps, float lr, float inv_p, int bias,
                                              int nthreads) {
  return cpu_linear_seq_round<float>(w, num, dn, tok, dc, yv, y8, B, R, S, dacc, dim, stats,
                                     rule, variant, C, eps, lr, inv_p, bias, nthreads);
}

// The same round in double precision (the reference's Breeze Double model): w, dacc fp64;
// the bench's parity row (the fp32 kernels' accuracy against the Double learner's).
OMLDM_HOST_API int omldm_cpu_linear_seq_round64(const double* w, const float* num, int dn,
                                                const uint32_t* tok, int dc, const void* yv,
                                                int y8, int B, int R, int S, double* dacc,
                                                int dim, float* stats, int rule, int variant,
                                                float C, float eps, float lr, float inv_p,
                                                int bias, int nthreads) {
  return cpu_linear_seq_round<double>(w, num, dn, tok, dc, yv, y8, B, R, S, dacc, dim, stats,
                                      rule, variant, C, eps, lr, inv_p, bias, nthreads);
}
