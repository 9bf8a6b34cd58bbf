// MultiClassPA on hashed features — K prototype vectors W[K][dim], virtual spokes.
//
// Reference learner name "MultiClassPA" (omldm/utils/parsers/requestStream/
// PipelineMap.scala:68); rule (Crammer et al. 2006):
//   r = argmax_{k≠y} w_k·x,  ℓ = max(0, 1 − (w_y − w_r)·x),
//   τ = ℓ/(2‖x‖²) (PA), min(C, ℓ/(2‖x‖²)) (PA-I), ℓ/(2‖x‖² + 1/(2C)) (PA-II),
//   w_y += τx,  w_r −= τx.
// Same structure as linear_spoke.hip: one wavefront per virtual spoke, lane = feature,
// K scores per example by K interleaved DPP wave reductions; the spoke's private deltas
// live in an LDS table keyed by feature with K floats per key; dense features keep
// their K deltas in registers; round end ships Δ/P with row-contiguous atomics.
#include "common.h"

namespace omldm {

template <int K>
__global__ __launch_bounds__(64) void multiclass_round_kernel(
    const float* __restrict__ W, const float* __restrict__ num, int dn,
    const int* __restrict__ cat, int dc, const float* __restrict__ yv, int B, int R, int dim,
    int nclass, int variant, float C, int bias, float* __restrict__ dacc,
    float* __restrict__ stats, int log2cap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int cap = 1 << log2cap;
  int* keys = reinterpret_cast<int*>(smem);
  float* vals = reinterpret_cast<float*>(smem + (size_t)cap * sizeof(int));  // [cap][K]
  const int lane = threadIdx.x;
  const int s = blockIdx.x;
  const long long t0ll = (long long)s * R;
  const int t0 = t0ll > B ? B : (int)t0ll;
  const int t1 = (t0ll + R) > B ? B : (int)(t0ll + R);
  if (t0 >= t1) return;
  for (int i = lane; i < cap; i += kWave) {
    keys[i] = kEmptyKey;
#pragma unroll
    for (int k = 0; k < K; ++k) vals[(size_t)i * K + k] = 0.f;
  }
  __syncthreads();
  const int F = dn + dc + (bias ? 1 : 0);
  float loss_sum = 0.f, nex = 0.f, mist = 0.f, ovf = 0.f;
  float dreg[K];
#pragma unroll
  for (int k = 0; k < K; ++k) dreg[k] = 0.f;
  const bool dense = lane < dn || (bias && lane == dn + dc);
  for (int t = t0; t < t1; ++t) {
    const float yf = yv[t];
    if (__builtin_isnan(yf)) continue;
    const int yc = (int)yf;
    int idx = -1;
    float xv = 0.f;
    if (lane < F) {
      if (bias && lane == dn + dc) {
        idx = dim - 1;
        xv = 1.f;
      } else if (lane < dn) {
        idx = lane;
        xv = num[(size_t)t * dn + lane];
      } else {
        const int c = cat[(size_t)t * dc + (lane - dn)];
        if (c != -1) {
          idx = c & 0x7fffffff;
          xv = c < 0 ? -1.f : 1.f;
        }
      }
      if ((unsigned)idx >= (unsigned)dim) {
        idx = -1;
        xv = 0.f;
      }
    }
    int slot = -1;
    if (!dense && idx >= 0) {
      slot = lds_find_or_insert(keys, idx, log2cap);
      if (slot < 0) ovf += 1.f;
    }
    float sc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float wv = 0.f, d = 0.f;
      if (idx >= 0 && k < nclass) {
        wv = W[(size_t)k * dim + idx];
        d = dense ? dreg[k] : (slot >= 0 ? vals[(size_t)slot * K + k] : 0.f);
      }
      sc[k] = xv * (wv + d);
    }
    float n2 = xv * xv;
    // K + 1 interleaved wave reductions
#pragma unroll
    for (int k = 0; k < K; ++k) sc[k] = wave_sum(sc[k]);
    n2 = wave_sum(n2);
    int r = -1;
    float best = -INFINITY;
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < nclass && k != yc && sc[k] > best) {
        best = sc[k];
        r = k;
      }
    float sy = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k == yc) sy = sc[k];
    const float margin = sy - best;
    const float loss = fmaxf(0.f, 1.f - margin);
    loss_sum += loss;
    nex += 1.f;
    mist += margin <= 0.f ? 1.f : 0.f;
    float tau = 0.f;
    if (loss > 0.f && n2 > 0.f && r >= 0) {
      const float den = 2.f * n2;
      tau = variant == 0 ? loss / den : (variant == 1 ? fminf(C, loss / den) : loss / (den + 0.5f / C));
    }
    if (tau != 0.f && idx >= 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float g = k == yc ? tau * xv : (k == r ? -tau * xv : 0.f);
        if (g != 0.f) {
          if (dense) dreg[k] += g;
          else if (slot >= 0) atomicAdd(&vals[(size_t)slot * K + k], g);
        }
      }
    }
  }
  __syncthreads();
  // Round end: Δ/P (inv count is applied by the caller's averaging) into dacc[K][dim].
  for (int i = lane; i < cap; i += kWave) {
    const int key = keys[i];
    if (key >= 0)
      for (int k = 0; k < nclass; ++k) {
        const float v = vals[(size_t)i * K + k];
        if (v != 0.f) atomicAdd(&dacc[(size_t)k * dim + key], v);
      }
  }
  if (dense && lane < F) {
    const int key = lane < dn ? lane : dim - 1;
    for (int k = 0; k < nclass; ++k)
      if (dreg[k] != 0.f) atomicAdd(&dacc[(size_t)k * dim + key], dreg[k]);
  }
  const float ovf_total = wave_sum(ovf);
  if (lane == 0) {
    atomicAdd(stats + 0, loss_sum);
    atomicAdd(stats + 1, nex);
    atomicAdd(stats + 2, mist);
    atomicAdd(stats + 3, 1.f);  // active workers this round
    atomicAdd(stats + 5, ovf_total);
  }
}

// W[k] += dacc[k] / n_active ; dacc = 0.
__global__ __launch_bounds__(256) void multiclass_apply_kernel(float* __restrict__ W,
                                                               float* __restrict__ dacc,
                                                               long long n,
                                                               const float* __restrict__ nact) {
  const float na = *nact;
  const float r = na > 0.f ? 1.f / na : 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    W[i] = fmaf(dacc[i], r, W[i]);
    dacc[i] = 0.f;
  }
}

}  // namespace omldm

using namespace omldm;

// stats: [8] device accumulators (loss, n, mistakes, active, -, overflow)
OMLDM_API int omldm_multiclass_round(const float* W, const float* num, int dn, const int* cat,
                                     int dc, const float* y, int B, int R, int S, int dim,
                                     int nclass, int variant, float C, int bias, float* dacc,
                                     float* stats, int log2cap, void* stream) {
  if (S <= 0 || B <= 0) return 0;
  if (dn + dc + (bias ? 1 : 0) > 64) return -2;
  if (nclass < 2 || nclass > 16) return -3;
  const int K = nclass <= 2 ? 2 : nclass <= 4 ? 4 : nclass <= 8 ? 8 : 16;
  const size_t lds = (size_t(1) << log2cap) * (4 + 4 * (size_t)K);
  if (lds > 160 * 1024) return -1;
  hipStream_t st = (hipStream_t)stream;
#define OMLDM_MC(KK)                                                                           \
  {                                                                                            \
    int e = check_dyn_lds((const void*)multiclass_round_kernel<KK>, lds);                      \
    if (e) return e;                                                                           \
    hipLaunchKernelGGL(multiclass_round_kernel<KK>, dim3(S), dim3(64), lds, st, W, num, dn, cat, \
                       dc, y, B, R, dim, nclass, variant, C, bias, dacc, stats, log2cap);      \
  }
  if (K == 2) OMLDM_MC(2) else if (K == 4) OMLDM_MC(4) else if (K == 8) OMLDM_MC(8) else OMLDM_MC(16)
#undef OMLDM_MC
  return (int)hipGetLastError();
}

OMLDM_API int omldm_multiclass_apply(float* W, float* dacc, long long n, const float* nact,
                                     void* stream) {
  int blocks = (int)((n + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(multiclass_apply_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, W,
                     dacc, n, nact);
  return (int)hipGetLastError();
}
