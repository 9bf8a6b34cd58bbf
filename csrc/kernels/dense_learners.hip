// Dense-feature learners: ORR sufficient statistics (MFMA SYRK) and online K-means.
//
// ORR (online ridge regression): A = λI + Σ xxᵀ, b = Σ y·x,
// w = A⁻¹b. The statistics are additive, so a round (and a sync between workers) is a
// SUM — exactly mergeable. One pass over the micro-batch computes the Gram matrix of
// the augmented row z = [x, 1, y]:  G = Σ zzᵀ = [[XᵀX, Xᵀ1, Xᵀy], [.., n, Σy], [.., .., Σy²]]
// on the fp32-input matrix cores (v_mfma_f32_32x32x2_f32: exact fp32, one rounding per
// product — the normal equations need it), split over row-chunks across workgroups and
// combined with row-contiguous f32 atomics (256-B rows: full-rate atomics).
//
// K-means (online / sequential k-means, single-learner mode): assignment by nearest
// centroid and per-cluster sums; the centroid move c ← c + (Σx − m·c)/(n + m) is the
// micro-batch form of the sequential update c ← c + (x − c)/n.
#include "common.h"

namespace omldm {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Element (k, c) of the augmented row-major batch: c < d → x[k][c]; c == d → 1;
// c == d+1 → y[k]; beyond → 0 (tile padding). Rows ≥ B → 0.
__device__ __forceinline__ float zval(const float* __restrict__ x, const float* __restrict__ y,
                                      int B, int d, long long k, int c) {
  if (k >= B) return 0.f;
  if (c < d) return x[k * d + c];
  if (c == d) return 1.f;
  if (c == d + 1) {
    const float v = y[k];
    return __builtin_isnan(v) ? 0.f : v;
  }
  return 0.f;
}

// grid: (tiles_i, tiles_j, ksplit); one wave per block computes a 32×32 tile of G over
// its row range with K=2 steps of v_mfma_f32_32x32x2_f32, then atomically adds it to G.
// Rows with NaN targets (forecast / skipped) are excluded via the mask.
__global__ __launch_bounds__(64) void gram_mfma_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ y, int B, int d,
                                                       int rows_per_split,
                                                       float* __restrict__ G, int ld,
                                                       double* __restrict__ cnt) {
  const int lane = threadIdx.x;
  const int i0 = blockIdx.x * 32, j0 = blockIdx.y * 32;
  const long long r0 = (long long)blockIdx.z * rows_per_split;
  const long long r1 = min((long long)B, r0 + rows_per_split);
  const int dz = d + 2;
  f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int ci = i0 + (lane & 31), cj = j0 + (lane & 31);
  const int kh = lane >> 5;
  for (long long k = r0; k < r1; k += 2) {
    const long long kk = k + kh;
    const bool ok = kk < r1 && !__builtin_isnan(y[kk < B ? kk : 0]);
    const float a = ok && ci < dz ? zval(x, y, B, d, kk, ci) : 0.f;
    const float b = ok && cj < dz ? zval(x, y, B, d, kk, cj) : 0.f;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  // C/D map (32x32): col = lane & 31, row = (reg & 3) + 8·(reg >> 2) + 4·(lane >> 5).
  const int col = j0 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = i0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row < dz && col < dz && acc[r] != 0.f) {
      atomicAdd(&G[(size_t)row * ld + col], acc[r]);
      // entry (d, d) = Σ 1·1 over the split's valid rows: the split's fitted-row count
      // (exact: < 2^24 per split), added to the learner's fp64 running total without extra
      // launches (an fp32 total would stop counting past ~2^30 rows)
      if (cnt && row == d && col == d) atomicAdd(cnt, (double)acc[r]);
    }
  }
}

// ---- K-means -------------------------------------------------------------------------
// One thread per row: nearest centroid (centroids staged in LDS), per-block LDS sums of
// rows and counts per cluster, one atomic per (cluster, feature) per block.
__global__ __launch_bounds__(256) void kmeans_assign_kernel(
    const float* __restrict__ x, const float* __restrict__ yv, int B, int d, int k,
    const float* __restrict__ cent, float* __restrict__ sums, float* __restrict__ counts,
    int* __restrict__ assign, float* __restrict__ inertia) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* c = reinterpret_cast<float*>(smem);  // [k][d]
  float* s = c + k * d;                       // [k][d]
  float* n = s + k * d;                       // [k]
  __shared__ float part[4];
  for (int i = threadIdx.x; i < k * d; i += 256) {
    c[i] = cent[i];
    s[i] = 0.f;
  }
  for (int i = threadIdx.x; i < k; i += 256) n[i] = 0.f;
  __syncthreads();
  float my_in = 0.f;
  for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < B;
       r += (long long)gridDim.x * 256) {
    const float* xr = x + r * d;
    int best = 0;
    float bd = INFINITY;
    for (int j = 0; j < k; ++j) {
      float dd = 0.f;
      for (int f = 0; f < d; ++f) {
        const float t = xr[f] - c[j * d + f];
        dd = fmaf(t, t, dd);
      }
      if (dd < bd) {
        bd = dd;
        best = j;
      }
    }
    if (assign) assign[r] = best;
    const bool train = yv == nullptr || !__builtin_isnan(yv[r]);
    if (train && sums) {
      for (int f = 0; f < d; ++f) atomicAdd(&s[best * d + f], xr[f]);
      atomicAdd(&n[best], 1.f);
      my_in += bd;
    }
  }
  __syncthreads();
  if (sums) {
    for (int i = threadIdx.x; i < k * d; i += 256)
      if (s[i] != 0.f) atomicAdd(&sums[i], s[i]);
    for (int i = threadIdx.x; i < k; i += 256)
      if (n[i] != 0.f) atomicAdd(&counts[i], n[i]);
    const float w = wave_sum(my_in);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0 && inertia) atomicAdd(inertia, (part[0] + part[1]) + (part[2] + part[3]));
  }
}

// Count-weighted centroid move of one micro-batch, fused with the bookkeeping the learner
// used to do in ~12 small elementwise launches:
//   tot = n + cnt; c ← (n·c + Σx)/tot where tot > 0; n ← tot; Σx, cnt ← 0;
//   cum[0] += inertia, cum[1] += Σ cnt (training rows); inertia ← 0.
__global__ __launch_bounds__(256) void kmeans_apply_kernel(float* __restrict__ cent,
                                                           float* __restrict__ n, int k, int d,
                                                           float* __restrict__ sums,
                                                           float* __restrict__ counts,
                                                           float* __restrict__ inertia,
                                                           double* __restrict__ cum) {
  for (int i = threadIdx.x; i < k * d; i += 256) {
    const int j = i / d;
    const float nj = n[j], tot = nj + counts[j];
    if (tot > 0.f) cent[i] = (cent[i] * nj + sums[i]) / tot;
    sums[i] = 0.f;
  }
  __syncthreads();  // every centroid read n and counts before they change
  float fitted = 0.f;
  for (int j = threadIdx.x; j < k; j += 256) {
    fitted += counts[j];
    n[j] += counts[j];
    counts[j] = 0.f;
  }
  fitted = wave_sum(fitted);
  __shared__ float part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = fitted;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (cum) {
      cum[0] += (double)*inertia;
      cum[1] += (double)((part[0] + part[1]) + (part[2] + part[3]));
    }
    *inertia = 0.f;
  }
}

}  // namespace omldm

using namespace omldm;

OMLDM_API int omldm_kmeans_apply(float* cent, float* n, int k, int d, float* sums, float* counts,
                                 float* inertia, double* cum, void* stream) {
  hipLaunchKernelGGL(kmeans_apply_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, cent, n, k,
                     d, sums, counts, inertia, cum);
  return (int)hipGetLastError();
}

// G[ld×ld] += [X 1 y]ᵀ[X 1 y] over rows with finite y (ld ≥ d + 2).
// cnt (may be null): += number of rows with finite y.
OMLDM_API int omldm_gram_update(const float* x, const float* y, int B, int d, float* G, int ld,
                                double* cnt, void* stream) {
  if (B <= 0) return 0;
  const int dz = d + 2;
  if (ld < dz) return -1;
  const int t = (dz + 31) / 32;
  int ksplit = (2048 + t * t - 1) / (t * t);  // ≥ ~2048 waves in flight
  const long long maxsplit = (B + 63) / 64;
  if (ksplit > maxsplit) ksplit = (int)maxsplit;
  if (ksplit < 1) ksplit = 1;
  int rows = (int)((B + ksplit - 1) / ksplit);
  rows = (rows + 1) & ~1;
  ksplit = (B + rows - 1) / rows;
  hipLaunchKernelGGL(gram_mfma_kernel, dim3(t, t, ksplit), dim3(64), 0, (hipStream_t)stream, x,
                     y, B, d, rows, G, ld, cnt);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_kmeans_assign(const float* x, const float* y, int B, int d, int k,
                                  const float* cent, float* sums, float* counts, int* assign,
                                  float* inertia, void* stream) {
  if (B <= 0) return 0;
  const size_t lds = (size_t)(2 * k * d + k) * 4;
  if (lds > 150 * 1024) return -1;
  int e = check_dyn_lds((const void*)kmeans_assign_kernel, lds);
  if (e) return e;
  int blocks = (B + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(kmeans_assign_kernel, dim3(blocks), dim3(256), lds, (hipStream_t)stream, x,
                     y, B, d, k, cent, sums, counts, assign, inertia);
  return (int)hipGetLastError();
}
