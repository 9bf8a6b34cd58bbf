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

// ---- ORR Gram, v2: LDS-staged rows, every wave on every tile, feature map fused ------
// gram_mfma_kernel above reads each operand straight from global memory with one scalar
// load per lane and one 32×32 tile per wave: ≈ 4 % of the fp32 matrix-core peak (917 µs
// for 262144 rows × 106 columns, profiles/orr_fgm_kernel_summary.txt). Here a workgroup
// owns a contiguous row range. 64-row chunks of the RAW rows [x (d0 values), valid, y·valid,
// 0] are staged in LDS (coalesced global reads, the next chunk's loads in flight while the
// current one computes), and each of the 4 waves takes a quarter of the chunk's row pairs
// for ALL upper-triangle tiles (I ≤ J) of the (NB·32)² Gram — T = NB(NB+1)/2
// accumulators, so the waves are balanced whatever T is.
// Column c of z is a product of two staged entries, z_c = s[pa_c]·s[pb_c], formed in the
// operand fetch: c < d0 → x_c·valid; then the degree-2 pairs x_a·x_b of a fused
// PolynomialFeatures(2) (pairs table; zeroed rows stay zero); then valid (the intercept
// column), then y·valid; beyond → 0. So ORR behind PolynomialFeatures reads the d0 raw
// features instead of the expanded d0 + d0(d0+1)/2 ones (13 → 104 floats per row) and the
// expansion never reaches HBM. At the end the four waves' tiles are summed through LDS and
// the block adds them to G with full-rate atomics (each accumulator register of a wave
// covers two 128-B row segments); a second tiny launch mirrors the upper triangle into
// the lower one. Exact fp32 products (v_mfma_f32_32x32x2_f32), like the v1 kernel (a pair
// feature is rounded once, as the separate expansion rounds it).
template <int NB, int EPT>
__global__ __launch_bounds__(256) void gram_map_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ y, int B, int d0,
                                                       const int* __restrict__ pairs, int npairs,
                                                       int rows_per_block, float* __restrict__ G,
                                                       int ld, double* __restrict__ cnt) {
  constexpr int T = NB * (NB + 1) / 2;
  constexpr int RC = 64;  // rows per staged chunk
  constexpr int MAXW = NB * 32 + 1;
  const int d = d0 + npairs;     // z = [mapped features (d), 1, y]
  const int W = d0 + 3;          // staged row: x (d0), valid, y·valid, 0
  const int LDW = W | 1;         // odd row stride: the half-waves' rows on different banks
  const int ONE = d0, YC = d0 + 1, ZERO = d0 + 2;
  constexpr int ZF = 2 * RC * MAXW;
  constexpr int RF = T * 1024;  // floats of the tile-sum image
  __shared__ float lds[ZF > RF ? ZF : RF];
  float* xs = lds;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long r_begin = (long long)blockIdx.x * rows_per_block;
  const long long r_end = min((long long)B, r_begin + rows_per_block);
  for (int i = tid; i < 2 * RC * LDW; i += 256) xs[i] = 0.f;  // the ZERO column stays 0
  // operand map of this lane's column in each 32-column block
  const int half = lane >> 5, col = lane & 31;
  int fa[NB], fb[NB];
#pragma unroll
  for (int I = 0; I < NB; ++I) {
    const int c = I * 32 + col;
    if (c < d0) {
      fa[I] = c;
      fb[I] = ONE;
    } else if (c < d) {
      fa[I] = pairs[2 * (c - d0)];
      fb[I] = pairs[2 * (c - d0) + 1];
    } else if (c == d) {
      fa[I] = ONE;  // valid · valid · valid = valid
      fb[I] = ONE;
    } else if (c == d + 1) {
      fa[I] = YC;
      fb[I] = ONE;
    } else {
      fa[I] = ZERO;
      fb[I] = ZERO;
    }
  }
  // staging: the chunk's x values are RC·d0 contiguous floats; element slot k of this
  // thread is e = tid + 256k, the same (row, col) in every chunk (EPT ≥ RC·d0 / 256)
  const int nel = RC * d0;
  int eoff[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = tid + 256 * k;
    const int r = e < nel ? e / d0 : 0;
    eoff[k] = e < nel ? r * LDW + (e - r * d0) : -1;
  }
  float xr[EPT];
  float yr = 0.f;
  auto load = [&](long long rc) {
    const long long rows = min((long long)RC, r_end - rc);
    const float* xp = x + rc * d0;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = tid + 256 * k;
      xr[k] = xp[e < rows * d0 ? e : 0];  // unconditional (a load in a branch waits inside it)
    }
    if (tid < RC) {
      yr = y[rc + (tid < rows ? tid : 0)];
      if (tid >= rows) yr = __builtin_nanf("");  // past the range: excluded
    }
  };
  // raw x values as they are; a row's `valid` entry (0 for a NaN target or past the
  // range) multiplies every operand of that row (z_c = s[pa]·s[pb]·valid)
  auto store = [&](int buf) {
    float* b = xs + (size_t)buf * RC * LDW;
#pragma unroll
    for (int k = 0; k < EPT; ++k)
      if (eoff[k] >= 0) b[eoff[k]] = xr[k];
    if (tid < RC) {
      const bool valid = !__builtin_isnan(yr);
      b[(size_t)tid * LDW + ONE] = valid ? 1.f : 0.f;
      b[(size_t)tid * LDW + YC] = valid ? yr : 0.f;
    }
  };
  f32x16 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  int buf = 0;
  __syncthreads();
  if (r_begin < r_end) {
    load(r_begin);
    store(0);
  }
  __syncthreads();
  for (long long rc = r_begin; rc < r_end; rc += RC) {
    const bool more = rc + RC < r_end;
    if (more) load(rc + RC);  // in flight while this chunk computes
    const float* xb = xs + (size_t)buf * RC * LDW;
#pragma unroll
    for (int kp = wave; kp < RC / 2; kp += 4) {
      const float* xrow = xb + (size_t)(2 * kp + half) * LDW;
      float a[NB];
#pragma unroll
      for (int I = 0; I < NB; ++I) a[I] = (xrow[fa[I]] * xrow[fb[I]]) * xrow[ONE];
      int t = 0;
#pragma unroll
      for (int I = 0; I < NB; ++I)
#pragma unroll
        for (int J = I; J < NB; ++J, ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[I], a[J], acc[t], 0, 0, 0);
    }
    if (more) store(buf ^ 1);  // buffer buf^1 was last read two chunks ago
    __syncthreads();
    buf ^= 1;
  }
  // sum the four waves' tiles through LDS (the staging buffers are free now)
  float* red = lds;
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float* p = red + t * 1024 + r * 64 + lane;
          *p = (w == 0 ? 0.f : *p) + acc[t][r];
        }
    }
    __syncthreads();
  }
  // element e of the image: tile t, register r, lane l → (row, col) of that tile
  for (int e = tid; e < RF; e += 256) {
    const int t = e >> 10, r = (e >> 6) & 15, l = e & 63;
    int I = 0, J = 0, k = t;
    while (k >= NB - I) {  // t-th upper-triangle tile in row-major order
      k -= NB - I;
      ++I;
    }
    J = I + k;
    const int row = I * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    const int cl = J * 32 + (l & 31);
    const float v = red[e];
    if (v != 0.f && row < ld && cl < ld) {
      atomicAdd(&G[(size_t)row * ld + cl], v);
      // entry (d, d) = Σ 1·1 over the block's valid rows (exact: < 2^24 per block)
      if (cnt && row == d && cl == d) atomicAdd(cnt, (double)v);
    }
  }
}

// G[i][j] = G[j][i] for j < i < n (gram_map_kernel accumulates the upper triangle).
__global__ __launch_bounds__(256) void gram_mirror_kernel(float* __restrict__ G, int ld, int n) {
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n * n; e += gridDim.x * 256) {
    const int i = e / n, j = e % n;
    if (i > j) G[(size_t)i * ld + j] = G[(size_t)j * ld + i];
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

// Nearest-centroid assignment on the matrix cores (k ≥ 32 centroids): distances as
// ‖c‖² − 2·c·x (the row's own ‖x‖² does not change its argmin) with C·Xᵀ tiles on
// v_mfma_f32_32x32x2_f32 (exact fp32 products). A wave takes 32-row tiles; A = a 32-centroid
// tile staged in LDS (odd row stride: the 32 lanes of an operand column on distinct banks),
// B = the tile's rows, each lane keeping its row's features in registers across all
// centroid tiles. Lane (j, h) ends a tile holding c_i·x_j for 16 centroids i of its half,
// so the argmin is an in-lane minimum plus one exchange with lane j ^ 32. Training rows then
// add x into the block's LDS cluster sums as the scalar kernel does.
template <int DMAX>
__global__ __launch_bounds__(256) void kmeans_assign_mfma_kernel(
    const float* __restrict__ x, const float* __restrict__ yv, int B, int d, int k,
    const float* __restrict__ cent, float* __restrict__ sums, float* __restrict__ counts,
    int* __restrict__ assign, float* __restrict__ inertia) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int kp = (k + 31) & ~31;
  const int dp = (d + 1) & ~1;
  const int ldc = dp | 1;
  float* cs = reinterpret_cast<float*>(smem);  // [kp][ldc]
  float* cn = cs + (size_t)kp * ldc;           // [kp]  ‖c‖² (+inf for padding)
  float* s = cn + kp;                          // [k][d] cluster sums of this block
  float* n = s + (size_t)k * d;                // [k]
  __shared__ float part[4];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int i = tid; i < kp * ldc; i += 256) {
    const int r = i / ldc, c = i - r * ldc;
    cs[i] = (r < k && c < d) ? cent[(size_t)r * d + c] : 0.f;
  }
  for (int i = tid; i < k * d; i += 256) s[i] = 0.f;
  for (int i = tid; i < k; i += 256) n[i] = 0.f;
  __syncthreads();
  for (int r = tid; r < kp; r += 256) {
    float a = 0.f;
    for (int c = 0; c < d; ++c) a = fmaf(cs[r * ldc + c], cs[r * ldc + c], a);
    cn[r] = r < k ? a : INFINITY;
  }
  __syncthreads();
  const int j = lane & 31, h = lane >> 5;
  float my_in = 0.f;
  for (long long t = (long long)blockIdx.x * 4 + wave; t * 32 < B; t += (long long)gridDim.x * 4) {
    const long long row = t * 32 + j;
    const bool vrow = row < B;
    const float* xr = x + (vrow ? row : B - 1) * (long long)d;
    float xv[DMAX / 2];  // features h, h+2, h+4, ... of this lane's row (the B operand)
#pragma unroll
    for (int u = 0; u < DMAX / 2; ++u) {
      const int f = 2 * u + h;
      xv[u] = f < d ? xr[f < d ? f : 0] : 0.f;
    }
    float best = INFINITY;
    int bi = 0;
    for (int ct = 0; ct < kp; ct += 32) {
      f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const float* ca = cs + (size_t)(ct + j) * ldc + h;
#pragma unroll
      for (int u = 0; u < DMAX / 2; ++u)
        if (2 * u < dp) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[2 * u], xv[u], acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = ct + (q & 3) + 8 * (q >> 2) + 4 * h;
        const float dist = cn[i] - 2.f * acc[q];
        if (dist < best) {
          best = dist;
          bi = i;
        }
      }
    }
    // the other half-wave holds the same row's other 16 centroids of every tile
    const float ob = __shfl_xor(best, 32);
    const int oi = __shfl_xor(bi, 32);
    if (ob < best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
    if (h == 0 && vrow) {
      if (assign) assign[row] = bi;
      const bool train = yv == nullptr || !__builtin_isnan(yv[row]);
      if (train && sums) {
        float xx = 0.f;
        for (int f = 0; f < d; ++f) {
          const float v = xr[f];
          xx = fmaf(v, v, xx);
          atomicAdd(&s[bi * d + f], v);
        }
        atomicAdd(&n[bi], 1.f);
        my_in += fmaxf(0.f, xx + best);  // ‖x − c‖² ≥ 0 (rounding)
      }
    }
  }
  __syncthreads();
  if (sums) {
    for (int i = tid; i < k * d; i += 256)
      if (s[i] != 0.f) atomicAdd(&sums[i], s[i]);
    for (int i = tid; i < k; i += 256)
      if (n[i] != 0.f) atomicAdd(&counts[i], n[i]);
    const float w = wave_sum(my_in);
    if (lane == 0) part[wave] = w;
    __syncthreads();
    if (tid == 0 && inertia) atomicAdd(inertia, (part[0] + part[1]) + (part[2] + part[3]));
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

template <int NB, int EPT>
static int launch_gram_map(const float* x, const float* y, int B, int d0, const int* pairs,
                           int npairs, float* G, int ld, double* cnt, hipStream_t st) {
  // ≤ one block per CU, each ≥ one chunk: every block's image costs T·4 KiB of atomics
  long long rpb = ((long long)B + 255) / 256;
  rpb = ((rpb + 63) / 64) * 64;
  const int blocks = (int)(((long long)B + rpb - 1) / rpb);
  hipLaunchKernelGGL((gram_map_kernel<NB, EPT>), dim3(blocks), dim3(256), 0, st, x, y, B, d0, pairs,
                     npairs, (int)rpb, G, ld, cnt);
  const int n = NB * 32 < ld ? NB * 32 : ld;
  hipLaunchKernelGGL(gram_mirror_kernel, dim3((n * n + 255) / 256), dim3(256), 0, st, G, ld, n);
  return (int)hipGetLastError();
}

template <int NB>
static int gram_map_e(const float* x, const float* y, int B, int d0, const int* pairs, int npairs,
                      float* G, int ld, double* cnt, hipStream_t st) {
  // element slots per thread: 64 staged rows × d0 raw values over 256 threads
  if (d0 <= 16) return launch_gram_map<NB, 4>(x, y, B, d0, pairs, npairs, G, ld, cnt, st);
  if (d0 <= 32) return launch_gram_map<NB, 8>(x, y, B, d0, pairs, npairs, G, ld, cnt, st);
  if (d0 <= 64) return launch_gram_map<NB, 16>(x, y, B, d0, pairs, npairs, G, ld, cnt, st);
  return launch_gram_map<NB, 32>(x, y, B, d0, pairs, npairs, G, ld, cnt, st);
}

static int gram_map(const float* x, const float* y, int B, int d0, const int* pairs, int npairs,
                    float* G, int ld, double* cnt, hipStream_t st) {
  const int dz = d0 + npairs + 2;
  if (dz <= 32) return gram_map_e<1>(x, y, B, d0, pairs, npairs, G, ld, cnt, st);
  if (dz <= 64) return gram_map_e<2>(x, y, B, d0, pairs, npairs, G, ld, cnt, st);
  if (dz <= 96) return gram_map_e<3>(x, y, B, d0, pairs, npairs, G, ld, cnt, st);
  return gram_map_e<4>(x, y, B, d0, pairs, npairs, G, ld, cnt, st);
}

// G[ld×ld] += [X 1 y]ᵀ[X 1 y] over rows with finite y (ld ≥ d + 2).
// cnt (may be null): += number of rows with finite y.
OMLDM_API int omldm_gram_update(const float* x, const float* y, int B, int d, float* G, int ld,
                                double* cnt, void* stream) {
  if (B <= 0) return 0;
  const int dz = d + 2;
  if (ld < dz) return -1;
  static const int v1 = [] {
    const char* e = getenv("OMLDM_GRAM_V1");  // A/B: the one-tile-per-wave v1 kernel
    return e ? atoi(e) : 0;
  }();
  if (!v1 && dz <= 128) return gram_map(x, y, B, d, nullptr, 0, G, ld, cnt, (hipStream_t)stream);
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

template <int DMAX>
static int launch_kmeans_mfma(const float* x, const float* y, int B, int d, int k,
                              const float* cent, float* sums, float* counts, int* assign,
                              float* inertia, size_t lds, hipStream_t st) {
  auto fn = kmeans_assign_mfma_kernel<DMAX>;
  int e = check_dyn_lds((const void*)fn, lds);
  if (e) return e;
  const long long tiles = ((long long)B + 31) / 32;
  int blocks = (int)((tiles + 3) / 4);
  if (blocks > 512) blocks = 512;  // each block flushes k·d sums: keep the flush small
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), lds, st, x, y, B, d, k, cent, sums, counts,
                     assign, inertia);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_kmeans_assign(const float* x, const float* y, int B, int d, int k,
                                  const float* cent, float* sums, float* counts, int* assign,
                                  float* inertia, void* stream) {
  if (B <= 0) return 0;
  // matrix-core distances once there is a full 32-centroid tile and a few features
  // (OMLDM_KMEANS_MFMA=0: the scalar kernel, A/B)
  const char* mf = getenv("OMLDM_KMEANS_MFMA");
  if (k >= 32 && d >= 4 && d <= 128 && !(mf && atoi(mf) == 0)) {
    const int kp = (k + 31) & ~31, ldc = ((d + 1) & ~1) | 1;
    const size_t lds = ((size_t)kp * ldc + kp + (size_t)k * d + k) * 4;
    if (lds <= 150 * 1024) {
      hipStream_t st = (hipStream_t)stream;
      if (d <= 32) return launch_kmeans_mfma<32>(x, y, B, d, k, cent, sums, counts, assign, inertia, lds, st);
      if (d <= 64) return launch_kmeans_mfma<64>(x, y, B, d, k, cent, sums, counts, assign, inertia, lds, st);
      return launch_kmeans_mfma<128>(x, y, B, d, k, cent, sums, counts, assign, inertia, lds, st);
    }
  }
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

// G += Σ zzᵀ with z = [x, x_a·x_b for (a, b) in pairs, 1, y] over rows with finite y: the
// Gram of PolynomialFeatures(2)(x) without materialising the expansion (pairs: int32
// [npairs][2]; d0 + npairs + 2 ≤ 128, else -2: expand and call omldm_gram_update).
OMLDM_API int omldm_gram_update_poly2(const float* x, const float* y, int B, int d0,
                                      const int* pairs, int npairs, float* G, int ld, double* cnt,
                                      void* stream) {
  if (B <= 0) return 0;
  const int dz = d0 + npairs + 2;
  if (ld < dz) return -1;
  if (dz > 128) return -2;
  return gram_map(x, y, B, d0, pairs, npairs, G, ld, cnt, (hipStream_t)stream);
}
