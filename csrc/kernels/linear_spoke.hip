// Virtual-spoke online linear learners (PA / PA-I / PA-II, linear SVM, RegressorPA,
// logistic SGD) on hashed sparse features — the training hot loop of the engine.
//
// Reference semantics: every Flink spoke keeps a full model replica per pipeline and
// fits its stream shard strictly sequentially, one example at a time
// (omldm/operators/spoke/FlinkSpoke.scala:92-107 → BufferingWrapper.receiveTuple →
// MLPipeline.pipePoint → learner.fit, hs_err_pid77107.log:111-113); at the end of a
// protocol round the parameter server averages the worker models
// (SynchronousParameterServer).
//
// MI355X design: one wavefront == one virtual spoke. A launch == one protocol round.
//  * The global model w0 (fp32, or a bf16 shadow that stays resident in the 4 MiB
//    per-XCD L2) is read-only for the whole round, so its gathers are issued for a
//    chunk of CH examples at once, long before they are consumed.
//  * The spoke's private delta Δ lives in an LDS open-addressing hash table keyed by
//    feature index (up to 160 KiB per workgroup on gfx950), so the spoke's model is
//    w_spoke = σ·(w0 + Δ) with σ the running L2-shrink scale.
//  * Lane l holds feature l of the example (FPL features per lane beyond 64), so the
//    sequential part per example is: ds_read Δ → fma → DPP wave reduction →
//    closed-form τ → ds_add_f32. Slot lookups/inserts for the whole chunk happen
//    before the sequential part (they do not depend on the updates).
//  * At round end each spoke scatters σ·Δ/P into the dense round accumulator with
//    no-return global f32 atomics, plus σ/P into accumulator[dim] (the w0 weight);
//    the accumulator is then all-reduced over xGMI by RCCL and folded into w by
//    linear_apply (below) — that is the Synchronous PS round.
#include "common.h"

namespace omldm {

enum LinRule : int { kHinge = 0, kEpsInsensitive = 1, kLogistic = 2 };
enum PAVariant : int { kPA = 0, kPA1 = 1, kPA2 = 2 };

struct LinParams {
  int rule;
  int variant;
  float C;
  float eps;
  float lr;
  float lam;
  float inv_p;
  int bias;
};


__device__ __forceinline__ float pa_tau(float loss, float n2, const LinParams& p) {
  if (loss <= 0.f || n2 <= 0.f) return 0.f;
  if (p.variant == kPA) return loss / n2;
  if (p.variant == kPA1) return fminf(p.C, loss / n2);
  return loss / (n2 + 0.5f / p.C);
}

// Loads feature f of example t for this lane. Numeric features occupy slots [0, dn);
// categorical features carry their hashed slot in the low 31 bits and the hash sign in
// bit 31; -1 marks an absent categorical feature.
// With bias != 0 the feature right after the categorical ones is the intercept: slot
// dim-1 (reserved by the hasher) with constant value 1 (reference VectorBias, U23).
template <typename NumT>
__device__ __forceinline__ void load_feature(const NumT* __restrict__ num, int dn,
                                             const int* __restrict__ cat, int dc, int t, int j,
                                             int dim, int bias, int& idx, float& v) {
  idx = -1;
  v = 0.f;
  if (j == dn + dc && bias) {
    idx = dim - 1;
    v = 1.f;
  } else if (j < dn) {
    idx = j;
    v = to_f(num[(size_t)t * dn + j]);
  } else if (j < dn + dc) {
    const int c = cat[(size_t)t * dc + (j - dn)];
    if (c != -1) {
      idx = c & 0x7fffffff;
      v = c < 0 ? -1.f : 1.f;
    }
  }
  if ((unsigned)idx >= (unsigned)dim) {  // never gather out of bounds
    idx = -1;
    v = 0.f;
  }
}

// Per-spoke workspace row: [loss, n, mistakes, sq_err, sigma, overflow, σ/P, 1/P,
//                           Δ(dense slot 0..dn-1)·σ/P, Δ(intercept)·σ/P]
constexpr int kWsStat = 8;

// Dense column of feature j: numerical slot j → j, intercept → dn; hashed features → -1.
// Dense features live in a register per lane for the whole round (every example has
// them), so they never touch the LDS table and never hit the same global address from
// every spoke: they are reduced by linear_round_finish instead of by atomics.
__device__ __forceinline__ int dense_col(int j, int dn, int dc, int bias) {
  if (j < dn) return j;
  if (bias && j == dn + dc) return dn;
  return -1;
}

// ablate (timing diagnostics only, never set in production): bit0 skip the categorical
// flush atomics, bit1 skip the sequential phase, bit2 skip the LDS slot resolution.
template <int FPL, int CH, typename NumT, typename WT>
__global__ __launch_bounds__(64) void linear_round_kernel(
    const WT* __restrict__ w, const NumT* __restrict__ num, int dn, const int* __restrict__ cat,
    int dc, const float* __restrict__ yv, int B, int R, float* __restrict__ dacc, int dim,
    float* __restrict__ ws, LinParams p, int log2cap, int ablate) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int cap = 1 << log2cap;
  int* keys = reinterpret_cast<int*>(smem);
  float* vals = reinterpret_cast<float*>(smem + (size_t)cap * sizeof(int));
  const int lane = threadIdx.x;
  const int s = blockIdx.x;
  const int wsw = kWsStat + dn + 1;
  float* wrow = ws + (size_t)s * wsw;
  const long long t0ll = (long long)s * R;
  const int t0 = t0ll > B ? B : (int)t0ll;
  const int t1 = (t0ll + R) > B ? B : (int)(t0ll + R);
  if (t0 >= t1) {  // idle spoke: not a worker of this round (does not dilute the average)
    for (int k = lane; k < wsw; k += kWave) wrow[k] = k == 4 ? 1.f : 0.f;
    return;
  }
  for (int i = lane; i < cap; i += kWave) {
    keys[i] = kEmptyKey;
    vals[i] = 0.f;
  }
  __syncthreads();

  int dcol[FPL];
  float dreg[FPL];
#pragma unroll
  for (int f = 0; f < FPL; ++f) {
    dcol[f] = dense_col(lane + kWave * f, dn, dc, p.bias);
    dreg[f] = 0.f;
  }
  float sigma = 1.f, loss_sum = 0.f, nex = 0.f, mist = 0.f, sqe = 0.f, ovf = 0.f;

  for (int tc = t0; tc < t1; tc += CH) {
    int slot[CH][FPL];
    float xv[CH][FPL];
    float wv[CH][FPL];
    float yy[CH];
    // Phase 1a: stream the chunk's features in (all loads independent).
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int t = tc + e;
      const bool ok = t < t1;
      yy[e] = ok ? yv[t] : __builtin_nanf("");
#pragma unroll
      for (int f = 0; f < FPL; ++f) {
        int idx = -1;
        float v = 0.f;
        if (ok) load_feature(num, dn, cat, dc, t, lane + kWave * f, dim, p.bias, idx, v);
        slot[e][f] = idx;
        xv[e][f] = v;
      }
    }
    // Phase 1b: gather w0 for the whole chunk (read-only during the round).
#pragma unroll
    for (int e = 0; e < CH; ++e)
#pragma unroll
      for (int f = 0; f < FPL; ++f) wv[e][f] = slot[e][f] >= 0 ? to_f(w[slot[e][f]]) : 0.f;
    // Phase 1c: resolve LDS slots of the private delta for hashed features.
    if (!(ablate & 4)) {
#pragma unroll
      for (int e = 0; e < CH; ++e)
#pragma unroll
        for (int f = 0; f < FPL; ++f)
          if (dcol[f] < 0 && slot[e][f] >= 0) {
            const int sl = lds_find_or_insert(keys, slot[e][f], log2cap);
            if (sl < 0) ovf += 1.f;
            slot[e][f] = sl;
          }
    } else {
#pragma unroll
      for (int e = 0; e < CH; ++e)
#pragma unroll
        for (int f = 0; f < FPL; ++f)
          if (slot[e][f] >= 0) slot[e][f] = (int)hslot((uint32_t)slot[e][f], log2cap);
    }
    if (ablate & 2) {
#pragma unroll
      for (int e = 0; e < CH; ++e)
#pragma unroll
        for (int f = 0; f < FPL; ++f) loss_sum += wv[e][f] + xv[e][f] + (float)slot[e][f];
      continue;
    }
    // Phase 2: exact sequential online updates.
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const float y = yy[e];
      if (__builtin_isnan(y)) continue;  // wave-uniform
      float pm = 0.f, pn = 0.f;
#pragma unroll
      for (int f = 0; f < FPL; ++f) {
        const float d = dcol[f] >= 0 ? dreg[f] : (slot[e][f] >= 0 ? vals[slot[e][f]] : 0.f);
        pm = fmaf(xv[e][f], wv[e][f] + d, pm);
        pn = fmaf(xv[e][f], xv[e][f], pn);
      }
      wave_sum2(pm, pn);
      const float m = sigma * pm;
      float c = 0.f;      // coefficient of x in w-space
      float shrink = 1.f;  // multiplicative L2 shrink of w this step
      if (p.rule == kHinge) {
        const float ym = y * m;
        const float loss = fmaxf(0.f, 1.f - ym);
        loss_sum += loss;
        mist += ym <= 0.f ? 1.f : 0.f;
        c = pa_tau(loss, pn, p) * y;
        shrink = 1.f - p.lam;
      } else if (p.rule == kEpsInsensitive) {
        const float err = y - m;
        const float loss = fmaxf(0.f, fabsf(err) - p.eps);
        loss_sum += loss;
        sqe += err * err;
        c = pa_tau(loss, pn, p) * (err >= 0.f ? 1.f : -1.f);
        shrink = 1.f - p.lam;
      } else {
        const float z = y * m;
        const float loss = z > 0.f ? log1pf(__expf(-z)) : (-z + log1pf(__expf(z)));
        loss_sum += loss;
        mist += z <= 0.f ? 1.f : 0.f;
        c = p.lr * y / (1.f + __expf(z));
        shrink = 1.f - p.lr * p.lam;
      }
      nex += 1.f;
      sigma *= shrink;
      if (c != 0.f) {
        const float cv = c / sigma;
#pragma unroll
        for (int f = 0; f < FPL; ++f) {
          if (dcol[f] >= 0) dreg[f] = fmaf(cv, xv[e][f], dreg[f]);
          else if (slot[e][f] >= 0) atomicAdd(&vals[slot[e][f]], cv * xv[e][f]);
        }
      }
    }
  }
  __syncthreads();
  // Round end: ship σ·Δ/P. Hashed features: sparse scatter with no-return f32 atomics
  // (distinct spokes rarely share a hashed slot); dense features: workspace row.
  const float scale = sigma * p.inv_p;
  if (!(ablate & 1)) {
    for (int i = lane; i < cap; i += kWave) {
      const int k = keys[i];
      if (k >= 0) {
        const float v = vals[i];
        if (v != 0.f) atomicAdd(&dacc[k], v * scale);
      }
    }
  }
#pragma unroll
  for (int f = 0; f < FPL; ++f)
    if (dcol[f] >= 0) wrow[kWsStat + dcol[f]] = dreg[f] * scale;
  const float ovf_total = wave_sum(ovf);
  if (lane == 0) {
    wrow[0] = loss_sum;
    wrow[1] = nex;
    wrow[2] = mist;
    wrow[3] = sqe;
    wrow[4] = sigma;
    wrow[5] = ovf_total;
    wrow[6] = scale;
    wrow[7] = p.inv_p;
    if (!p.bias) wrow[kWsStat + dn] = 0.f;  // intercept column unused
  }
}

// Column sums of the per-spoke workspace (one block per column) → accumulator slots
// that every spoke would otherwise hit with same-address atomics:
//   dense columns → dacc[0:dn], intercept → dacc[dim-1], Σσ/P → dacc[dim],
//   Σ1/P → dacc[dim+1], loss/n/mistakes/sq_err/overflow → cum (device running totals).
__global__ __launch_bounds__(256) void linear_round_finish_kernel(const float* __restrict__ ws,
                                                                  int S, int dn, int dim,
                                                                  float* __restrict__ dacc,
                                                                  float* __restrict__ cum) {
  __shared__ float part[4];
  const int c = blockIdx.x;
  const int wsw = kWsStat + dn + 1;
  float acc = 0.f;
  for (int s = threadIdx.x; s < S; s += 256) acc += ws[(size_t)s * wsw + c];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = (part[0] + part[1]) + (part[2] + part[3]);
    if (c < kWsStat) {
      if (c == 6) dacc[dim] += t;
      else if (c == 7) dacc[dim + 1] += t;
      else if (c != 4 && cum) cum[c] += t;
    } else {
      const int j = c - kWsStat;
      dacc[j < dn ? j : dim - 1] += t;
    }
  }
}

// One wavefront per example; M stacked models (w + m*wstride) → out[t*M + m].
template <int FPL, typename NumT, typename WT>
__global__ __launch_bounds__(256) void linear_predict_kernel(
    const WT* __restrict__ w, long long wstride, int M, const NumT* __restrict__ num, int dn,
    const int* __restrict__ cat, int dc, int B, int dim, int bias,
    const float* __restrict__ wscale, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int m = blockIdx.y;
  const WT* wm = w + (size_t)m * wstride;
  const float sc = wscale ? wscale[m] : 1.f;
  for (int t = wv; t < B; t += nwaves) {
    float acc = 0.f;
#pragma unroll
    for (int f = 0; f < FPL; ++f) {
      int idx;
      float v;
      load_feature(num, dn, cat, dc, t, lane + kWave * f, dim, bias, idx, v);
      if (idx >= 0) acc = fmaf(v, to_f(wm[idx]), acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) out[(size_t)t * M + m] = acc * sc;
  }
}

// Model average over the round's active workers:
//   w = (a·w + D) / n,  a = D[dim] = Σσ/P, n = D[dim+1] = Σ1/P  (n == 0: no change);
// D[0:dim] = 0 (D[dim:dim+2] cleared by a memset node after the kernel);
// optional bf16 shadow of w for the gathers of the next round.
__global__ __launch_bounds__(256) void linear_apply_kernel(float* __restrict__ w32,
                                                           __hip_bfloat16* __restrict__ w16,
                                                           float* __restrict__ dacc, int dim) {
  const float n = dacc[dim + 1];
  const float a = n > 0.f ? dacc[dim] : 1.f;
  const float r = n > 0.f ? 1.f / n : 1.f;
  const int n4 = dim >> 2;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int stride = gridDim.x * blockDim.x;
  float4* w4 = reinterpret_cast<float4*>(w32);
  float4* d4 = reinterpret_cast<float4*>(dacc);
  for (int i = tid; i < n4; i += stride) {
    float4 wv = w4[i];
    const float4 dv = d4[i];
    wv.x = fmaf(a, wv.x, dv.x) * r;
    wv.y = fmaf(a, wv.y, dv.y) * r;
    wv.z = fmaf(a, wv.z, dv.z) * r;
    wv.w = fmaf(a, wv.w, dv.w) * r;
    w4[i] = wv;
    d4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (w16) {
      __hip_bfloat16 b[4] = {__float2bfloat16(wv.x), __float2bfloat16(wv.y),
                             __float2bfloat16(wv.z), __float2bfloat16(wv.w)};
      *reinterpret_cast<uint2*>(w16 + 4 * (size_t)i) = *reinterpret_cast<uint2*>(b);
    }
  }
  for (int i = (n4 << 2) + tid; i < dim; i += stride) {
    const float v = fmaf(a, w32[i], dacc[i]) * r;
    w32[i] = v;
    dacc[i] = 0.f;
    if (w16) w16[i] = __float2bfloat16(v);
  }
}

template <int FPL, int CH, typename NumT, typename WT>
static int launch_round(const void* w, const void* num, int dn, const int* cat, int dc,
                        const float* y, int B, int R, int S, float* dacc, int dim, float* ws,
                        float* cum, const LinParams& p, int log2cap, int ablate, hipStream_t st) {
  auto fn = linear_round_kernel<FPL, CH, NumT, WT>;
  const size_t lds = (size_t(1) << log2cap) * 8;
  int e = check_dyn_lds((const void*)fn, lds);
  if (e) return e;
  hipLaunchKernelGGL(fn, dim3(S), dim3(64), lds, st, (const WT*)w, (const NumT*)num, dn, cat, dc,
                     y, B, R, dacc, dim, ws, p, log2cap, ablate);
  hipLaunchKernelGGL(linear_round_finish_kernel, dim3(kWsStat + dn + 1), dim3(256), 0, st, ws, S,
                     dn, dim, dacc, cum);
  return (int)hipGetLastError();
}

template <int FPL, int CH>
static int dispatch_round(const void* w, int w_bf16, const void* num, int num_bf16, int dn,
                          const int* cat, int dc, const float* y, int B, int R, int S, float* dacc,
                          int dim, float* ws, float* cum, const LinParams& p, int log2cap,
                          int ablate, hipStream_t st) {
  if (num_bf16) {
    if (w_bf16)
      return launch_round<FPL, CH, __hip_bfloat16, __hip_bfloat16>(w, num, dn, cat, dc, y, B, R, S,
                                                                   dacc, dim, ws, cum, p, log2cap, ablate, st);
    return launch_round<FPL, CH, __hip_bfloat16, float>(w, num, dn, cat, dc, y, B, R, S, dacc, dim,
                                                        ws, cum, p, log2cap, ablate, st);
  }
  if (w_bf16)
    return launch_round<FPL, CH, float, __hip_bfloat16>(w, num, dn, cat, dc, y, B, R, S, dacc, dim,
                                                        ws, cum, p, log2cap, ablate, st);
  return launch_round<FPL, CH, float, float>(w, num, dn, cat, dc, y, B, R, S, dacc, dim, ws,
                                             cum, p, log2cap, ablate, st);
}

template <int FPL, typename NumT, typename WT>
static int launch_predict(const void* w, long long wstride, int M, const void* num, int dn,
                          const int* cat, int dc, int B, int dim, int bias, const float* wscale,
                          float* out, hipStream_t st) {
  const int waves = B < 1 ? 1 : B;
  int blocks = (waves + 3) / 4;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL((linear_predict_kernel<FPL, NumT, WT>), dim3(blocks, M), dim3(256), 0, st,
                     (const WT*)w, wstride, M, (const NumT*)num, dn, cat, dc, B, dim, bias, wscale, out);
  return (int)hipGetLastError();
}

template <int FPL>
static int dispatch_predict(const void* w, int w_bf16, long long wstride, int M, const void* num,
                            int num_bf16, int dn, const int* cat, int dc, int B, int dim, int bias,
                            const float* wscale, float* out, hipStream_t st) {
  if (num_bf16) {
    if (w_bf16)
      return launch_predict<FPL, __hip_bfloat16, __hip_bfloat16>(w, wstride, M, num, dn, cat, dc,
                                                                 B, dim, bias, wscale, out, st);
    return launch_predict<FPL, __hip_bfloat16, float>(w, wstride, M, num, dn, cat, dc, B, dim, bias,
                                                      wscale, out, st);
  }
  if (w_bf16)
    return launch_predict<FPL, float, __hip_bfloat16>(w, wstride, M, num, dn, cat, dc, B, dim, bias,
                                                      wscale, out, st);
  return launch_predict<FPL, float, float>(w, wstride, M, num, dn, cat, dc, B, dim, bias, wscale,
                                           out, st);
}

}  // namespace omldm

using namespace omldm;

OMLDM_API int omldm_linear_round(const void* w, int w_bf16, const void* num, int num_bf16, int dn,
                                 const int* cat, int dc, const float* y, int B, int R, int S,
                                 float* dacc, int dim, float* ws, float* cum, int rule,
                                 int variant,
                                 float C, float eps, float lr, float lam, float inv_p, int bias,
                                 int log2cap, int ablate, void* stream) {
  if (S <= 0) return 0;
  if (log2cap < 4 || log2cap > 14) return -1;  // ≤ 128 KiB of LDS per spoke
  const LinParams p{rule, variant, C, eps, lr, lam, inv_p, bias};
  const int F = dn + dc + (bias ? 1 : 0);
  hipStream_t st = (hipStream_t)stream;
  if (F <= 64) return dispatch_round<1, 16>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc, dim, ws, cum, p, log2cap, ablate, st);
  if (F <= 128) return dispatch_round<2, 8>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc, dim, ws, cum, p, log2cap, ablate, st);
  if (F <= 256) return dispatch_round<4, 4>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc, dim, ws, cum, p, log2cap, ablate, st);
  return -2;
}

OMLDM_API int omldm_linear_predict(const void* w, int w_bf16, long long wstride, int M,
                                   const void* num, int num_bf16, int dn, const int* cat, int dc,
                                   int B, int dim, int bias, const float* wscale, float* out,
                                   void* stream) {
  if (B <= 0 || M <= 0) return 0;
  const int F = dn + dc + (bias ? 1 : 0);
  hipStream_t st = (hipStream_t)stream;
  if (F <= 64) return dispatch_predict<1>(w, w_bf16, wstride, M, num, num_bf16, dn, cat, dc, B, dim, bias, wscale, out, st);
  if (F <= 128) return dispatch_predict<2>(w, w_bf16, wstride, M, num, num_bf16, dn, cat, dc, B, dim, bias, wscale, out, st);
  if (F <= 256) return dispatch_predict<4>(w, w_bf16, wstride, M, num, num_bf16, dn, cat, dc, B, dim, bias, wscale, out, st);
  return -2;
}

OMLDM_API int omldm_linear_apply(float* w32, void* w16, float* dacc, int dim, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int blocks = (dim / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(linear_apply_kernel, dim3(blocks), dim3(256), 0, st, w32,
                     (__hip_bfloat16*)w16, dacc, dim);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return (int)hipMemsetAsync(dacc + dim, 0, 2 * sizeof(float), st);
}
