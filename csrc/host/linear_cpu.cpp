// CPU implementation of the virtual-spoke linear round — the exact semantics of
// csrc/kernels/linear_spoke.hip (same feature decoding, same τ rules, same σ-scaled
// private delta, same σ·Δ/P shipping), used as
//   * the golden oracle for the HIP kernel numerics tests, and
//   * the CPU fallback / "reference-class" baseline (sequential per-example online
//     learning per spoke, as the reference's FlinkSpoke does on the JVM:
//     omldm/operators/spoke/FlinkSpoke.scala:92-107).
// Spokes run on std::thread workers; within a spoke everything is sequential.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

#define OMLDM_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

struct P {
  int rule, variant;
  float C, eps, lr, lam, inv_p, tbase;
};

inline float pa_tau(float loss, float n2, const P& p) {
  if (loss <= 0.f || n2 <= 0.f) return 0.f;
  if (p.variant == 0) return loss / n2;
  if (p.variant == 1) return std::fmin(p.C, loss / n2);
  return loss / (n2 + 0.5f / p.C);
}

inline float bf16_to_f(uint16_t b) {
  uint32_t u = uint32_t(b) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// Decodes categorical field j of row t (int32 signed-slot form, or the compact uint16
// field-aware form when cspan > 0). Returns false when absent / out of range.
inline bool cat_at(const void* cat, int dc, long long t, int j, int dn, int dim, int cspan,
                   int& idx, float& v) {
  if (cspan > 0) {
    const unsigned c = static_cast<const uint16_t*>(cat)[t * dc + j];
    if (c == 0xFFFFu) return false;
    idx = dn + j * cspan + int(c & 0x7fffu);
    v = (c & 0x8000u) ? -1.f : 1.f;
  } else {
    const int c = static_cast<const int32_t*>(cat)[t * dc + j];
    if (c == -1) return false;
    idx = c & 0x7fffffff;
    v = c < 0 ? -1.f : 1.f;
  }
  return idx < dim;
}

}  // namespace

// w: fp32 [dim] or bf16 [dim] (w_bf16); num: fp32 [B, dn]. stats: per-spoke [S, 6]
// (loss, n, mistakes, sq_err, σ, -). dacc: [dim + 2] accumulates σ·Δ/P, plus Σσ/P at
// [dim] and Σ1/P at [dim + 1], exactly like the kernel.
OMLDM_HOST_API int omldm_cpu_linear_round(const void* w, int w_bf16, const float* num, int dn,
                                          const void* cat, int dc, const float* y, int B,
                                          int R, int S, float* dacc, int dim, float* stats,
                                          int rule, int variant, float C, float eps, float lr,
                                          float lam, float inv_p, int bias, int cspan,
                                          float tbase, int nthreads) {
  const P p{rule, variant, C, eps, lr, lam, inv_p, tbase};
  const float* w32 = static_cast<const float*>(w);
  const uint16_t* w16 = static_cast<const uint16_t*>(w);
  auto wget = [&](int i) { return w_bf16 ? bf16_to_f(w16[i]) : w32[i]; };
  std::vector<std::unordered_map<int, float>> deltas(S);
  std::vector<float> sigmas(S, 1.f);
  auto run = [&](int s0, int s1) {
    std::vector<int> idx(dn + dc + 1);
    std::vector<float> xv(dn + dc + 1);
    for (int s = s0; s < s1; ++s) {
      auto& delta = deltas[s];
      float sigma = 1.f, loss_sum = 0.f, nex = 0.f, mist = 0.f, sqe = 0.f;
      const long long a = std::min<long long>((long long)s * R, B);
      const long long b = std::min<long long>(a + R, B);
      for (long long t = a; t < b; ++t) {
        const float yt = y[t];
        if (std::isnan(yt)) continue;
        int F = 0;
        for (int j = 0; j < dn; ++j) {
          if (j < dim) {
            idx[F] = j;
            xv[F++] = num[t * dn + j];
          }
        }
        for (int j = 0; j < dc; ++j) {
          int id;
          float v;
          if (!cat_at(cat, dc, t, j, dn, dim, cspan, id, v)) continue;
          idx[F] = id;
          xv[F++] = v;
        }
        if (bias) {
          idx[F] = dim - 1;
          xv[F++] = 1.f;
        }
        float pm = 0.f, pn = 0.f;
        for (int f = 0; f < F; ++f) {
          auto it = delta.find(idx[f]);
          const float d = it == delta.end() ? 0.f : it->second;
          pm += xv[f] * (wget(idx[f]) + d);
          pn += xv[f] * xv[f];
        }
        const float m = sigma * pm;
        float c = 0.f, shrink = 1.f;
        if (p.rule == 3) {  // Pegasos: η = 1/(λT), w ← (1 − 1/T)·w + η·y·x·[y·w·x < 1]
          const float T = p.tbase + (float)(t - a);
          const float ym = yt * m;
          loss_sum += std::fmax(0.f, 1.f - ym);
          mist += ym <= 0.f ? 1.f : 0.f;
          c = ym < 1.f ? (1.f / (p.lam * T)) * yt : 0.f;
          shrink = (T - 1.f) / T;
        } else if (p.rule == 0) {
          const float ym = yt * m;
          const float loss = std::fmax(0.f, 1.f - ym);
          loss_sum += loss;
          mist += ym <= 0.f ? 1.f : 0.f;
          c = pa_tau(loss, pn, p) * yt;
          shrink = 1.f - p.lam;
        } else if (p.rule == 1) {
          const float err = yt - m;
          const float loss = std::fmax(0.f, std::fabs(err) - p.eps);
          loss_sum += loss;
          sqe += err * err;
          c = pa_tau(loss, pn, p) * (err >= 0.f ? 1.f : -1.f);
          shrink = 1.f - p.lam;
        } else {
          const float z = yt * m;
          const float loss = z > 0.f ? std::log1p(std::exp(-z)) : (-z + std::log1p(std::exp(z)));
          loss_sum += loss;
          mist += z <= 0.f ? 1.f : 0.f;
          c = p.lr * yt / (1.f + std::exp(z));
          shrink = 1.f - p.lr * p.lam;
        }
        nex += 1.f;
        sigma *= shrink;
        if (c != 0.f) {
          const float cv = c / sigma;
          for (int f = 0; f < F; ++f) delta[idx[f]] += cv * xv[f];
        }
      }
      sigmas[s] = sigma;
      float* st = stats + (size_t)s * 6;
      st[0] = loss_sum;
      st[1] = nex;
      st[2] = mist;
      st[3] = sqe;
      st[4] = sigma;
      st[5] = 0.f;
    }
  };
  if (nthreads <= 1 || S < 2) {
    run(0, S);
  } else {
    std::vector<std::thread> th;
    const int n = std::min(nthreads, S);
    const int chunk = (S + n - 1) / n;
    for (int i = 0; i < n; ++i) {
      const int a = i * chunk, b = std::min(S, a + chunk);
      if (a < b) th.emplace_back(run, a, b);
    }
    for (auto& t : th) t.join();
  }
  // Deterministic merge (spoke order) — the kernel's atomics are order-free.
  // Idle spokes (no rows this round) are not workers of the round.
  for (int s = 0; s < S; ++s) {
    if ((long long)s * R >= B) continue;
    const float scale = sigmas[s] * p.inv_p;
    for (auto& kv : deltas[s]) dacc[kv.first] += kv.second * scale;
    dacc[dim] += scale;
    dacc[dim + 1] += p.inv_p;
  }
  return 0;
}

// w = (a·w + D)/n with a = D[dim], n = D[dim+1] (n == 0: unchanged) — see linear_apply_kernel.
// MultiClassPA round (CPU mirror of csrc/kernels/multiclass_spoke.hip, int32 cat format).
// dacc [K][dim] accumulates Σ_s Δ_s; stats[0..5] += loss, n, mistakes, active, -, -.
OMLDM_HOST_API int omldm_cpu_multiclass_round(const float* W, const float* num, int dn,
                                              const int32_t* cat, int dc, const float* y, int B,
                                              int R, int S, int dim, int nclass, int variant,
                                              float C, int bias, float* dacc, float* stats) {
  std::vector<int> idx(dn + dc + 1);
  std::vector<float> xv(dn + dc + 1), sc(nclass);
  for (int s = 0; s < S; ++s) {
    const long long a = std::min<long long>((long long)s * R, B);
    const long long b = std::min<long long>(a + R, B);
    if (a >= b) continue;
    std::unordered_map<long long, float> delta;  // key = k*dim + idx
    for (long long t = a; t < b; ++t) {
      if (std::isnan(y[t])) continue;
      const int yc = int(y[t]);
      int F = 0;
      for (int j = 0; j < dn && j < dim; ++j) {
        idx[F] = j;
        xv[F++] = num[t * dn + j];
      }
      for (int j = 0; j < dc; ++j) {
        int id;
        float v;
        if (!cat_at(cat, dc, t, j, dn, dim, 0, id, v)) continue;
        idx[F] = id;
        xv[F++] = v;
      }
      if (bias) {
        idx[F] = dim - 1;
        xv[F++] = 1.f;
      }
      float n2 = 0.f;
      for (int k = 0; k < nclass; ++k) sc[k] = 0.f;
      for (int f = 0; f < F; ++f) {
        n2 += xv[f] * xv[f];
        for (int k = 0; k < nclass; ++k) {
          auto it = delta.find((long long)k * dim + idx[f]);
          const float d = it == delta.end() ? 0.f : it->second;
          sc[k] += xv[f] * (W[(size_t)k * dim + idx[f]] + d);
        }
      }
      int r = -1;
      float best = -INFINITY;
      for (int k = 0; k < nclass; ++k)
        if (k != yc && sc[k] > best) {
          best = sc[k];
          r = k;
        }
      const float sy = (yc >= 0 && yc < nclass) ? sc[yc] : 0.f;
      const float margin = sy - best;
      const float loss = std::fmax(0.f, 1.f - margin);
      stats[0] += loss;
      stats[1] += 1.f;
      stats[2] += margin <= 0.f ? 1.f : 0.f;
      float tau = 0.f;
      if (loss > 0.f && n2 > 0.f && r >= 0) {
        const float den = 2.f * n2;
        tau = variant == 0 ? loss / den
                           : (variant == 1 ? std::fmin(C, loss / den) : loss / (den + 0.5f / C));
      }
      if (tau != 0.f)
        for (int f = 0; f < F; ++f) {
          if (yc >= 0 && yc < nclass) delta[(long long)yc * dim + idx[f]] += tau * xv[f];
          delta[(long long)r * dim + idx[f]] -= tau * xv[f];
        }
    }
    stats[3] += 1.f;
    for (auto& kv : delta) dacc[kv.first] += kv.second;
  }
  return 0;
}

OMLDM_HOST_API void omldm_cpu_linear_apply(float* w32, uint16_t* w16, float* dacc, int dim) {
  const float n = dacc[dim + 1];
  const float a = n > 0.f ? dacc[dim] : 1.f;
  const float r = n > 0.f ? 1.f / n : 1.f;
  const bool keep = !(n < 0.f);  // n < 0: a round its kernel marked failed (discarded)
  for (int i = 0; i < dim; ++i) {
    const float v = (a * w32[i] + (keep ? dacc[i] : 0.f)) * r;
    w32[i] = v;
    dacc[i] = 0.f;
    if (w16) {
      uint32_t u;
      std::memcpy(&u, &v, 4);
      const uint32_t r = ((u >> 16) & 1u) + 0x7fffu;  // RNE (NaN not expected here)
      w16[i] = uint16_t((u + r) >> 16);
    }
  }
  dacc[dim] = 0.f;
  dacc[dim + 1] = 0.f;
}

OMLDM_HOST_API void omldm_cpu_linear_predict(const float* w, long long wstride, int M,
                                             const float* num, int dn, const void* cat, int dc,
                                             int B, int dim, int bias, int cspan,
                                             const float* wscale, float* out) {
  for (int t = 0; t < B; ++t)
    for (int m = 0; m < M; ++m) {
      const float* wm = w + (size_t)m * wstride;
      float acc = 0.f;
      for (int j = 0; j < dn && j < dim; ++j) acc += num[(size_t)t * dn + j] * wm[j];
      for (int j = 0; j < dc; ++j) {
        int id;
        float v;
        if (cat_at(cat, dc, t, j, dn, dim, cspan, id, v)) acc += v * wm[id];
      }
      if (bias) acc += wm[dim - 1];
      out[(size_t)t * M + m] = acc * (wscale ? wscale[m] : 1.f);
    }
}
