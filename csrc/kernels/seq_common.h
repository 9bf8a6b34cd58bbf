// Shared pieces of the exact sequential linear rounds (linear_seq.hip: one workgroup per
// spoke builds and scans each chunk; linear_scan3.hip: chunk Grams precomputed by the
// whole GPU, one scan workgroup per spoke): the update rules and the round parameters.
#pragma once
#include "common.h"

namespace omldm {

// kSeqPegasos: the v3 table scan only (linear_scan3.hip)
enum SeqRule : int { kSeqHinge = 0, kSeqEps = 1, kSeqLogistic = 2, kSeqPegasos = 3 };

struct SeqParams {
  int rule, variant;
  float cclip;  // τ clip: C for PA-I, +inf otherwise
  float kadd;   // τ denominator offset: 1/(2C) for PA-II
  float eps, lr, inv_p;
  int bias, y8;
  uint32_t span;  // slots per categorical field: (dim − dn − 1) / dc (field-aware hashing)
  // v3 only — the model shrinks every step (w = σ·v): 0 none, 1 σ ×= r per row (L2: r = 1 − λ,
  // logistic 1 − lr·λ), 2 Pegasos σ ×= (T − 1)/T with T = tbase + the row's index in the spoke
  int shr;
  float lam, tbase;
};

// c(m) of one example for the lane's own row (the value is used only at its step).
template <int RULE>
__device__ __forceinline__ float seq_candidate(float m, float y, float inv, const SeqParams& p) {
  if constexpr (RULE == kSeqHinge) {
    const float l = fmaxf(0.f, fmaf(-y, m, 1.f));
    return fminf(p.cclip, l * inv) * y;
  } else if constexpr (RULE == kSeqEps) {
    const float err = y - m;
    const float l = fmaxf(0.f, fabsf(err) - p.eps);
    const float tau = fminf(p.cclip, l * inv);
    return err >= 0.f ? tau : -tau;
  } else {
    const float z = y * m;
    return p.lr * y * __builtin_amdgcn_rcpf(1.f + __expf(z));
  }
}

template <int RULE>
__device__ __forceinline__ void seq_stats(float m, float y, const SeqParams& p, float& loss,
                                          float& mist, float& sqe) {
  if constexpr (RULE == kSeqHinge || RULE == kSeqPegasos) {
    const float ym = y * m;
    loss += fmaxf(0.f, 1.f - ym);
    mist += ym <= 0.f ? 1.f : 0.f;
  } else if constexpr (RULE == kSeqEps) {
    const float err = y - m;
    loss += fmaxf(0.f, fabsf(err) - p.eps);
    sqe = fmaf(err, err, sqe);
  } else {
    const float z = y * m;
    loss += fmaxf(-z, 0.f) + __logf(1.f + __expf(-fabsf(z)));
    mist += z <= 0.f ? 1.f : 0.f;
  }
}

__device__ __forceinline__ float load_y(const void* yv, int t, int y8) {
  return y8 ? (float)static_cast<const int8_t*>(yv)[t] : static_cast<const float*>(yv)[t];
}

}  // namespace omldm
