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
constexpr int kKmeansMaxBlocks = 512;  // rows of the K-means partials image

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
// Element e of a tile-sum image (tile t, register r, lane l) → its (row, col) of G, added
// with an L2 atomic; entry (d, d) = Σ 1·1 is also the fitted-row count (fp64 total).
template <int NB>
__device__ __forceinline__ void gram_add_element(int e, float v, float* __restrict__ G, int ld,
                                                 int d, double* __restrict__ cnt) {
  const int t = e >> 10, r = (e >> 6) & 15, l = e & 63;
  int I = 0, k = t;
  while (k >= NB - I) {  // t-th upper-triangle tile in row-major order
    k -= NB - I;
    ++I;
  }
  const int J = I + k;
  const int row = I * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
  const int cl = J * 32 + (l & 31);
  if (v != 0.f && row < ld && cl < ld) {
    atomicAdd(&G[(size_t)row * ld + cl], v);
    if (cnt && row == d && cl == d) atomicAdd(cnt, (double)v);
  }
}

template <int NB, int EPT, int RC>
__global__ __launch_bounds__(256) void gram_map_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ y, int B, int d0,
                                                       const int* __restrict__ pairs, int npairs,
                                                       int rows_per_block, float* __restrict__ G,
                                                       int ld, double* __restrict__ cnt,
                                                       float* __restrict__ part) {
  constexpr int T = NB * (NB + 1) / 2;  // RC: rows per staged chunk
  const int d = d0 + npairs;     // z = [mapped features (d), 1, y]
  const int W = d0 + 3;          // staged row: x (d0), valid, y·valid, 0
  const int LDW = W | 1;         // odd row stride: the half-waves' rows on different banks
  const int ONE = d0, YC = d0 + 1, ZERO = d0 + 2;
  constexpr int RF = T * 1024;  // floats of the tile-sum image
  // dynamic: max(2 staging buffers of RC × LDW, the tile-sum image) floats
  extern __shared__ __attribute__((aligned(16))) float lds[];
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
    // software pipeline over the wave's row pairs: the LDS reads of pair p+1 are issued
    // before the MFMAs of pair p and consumed after them (instructions issue in order, so
    // reads placed after the MFMAs would leave the matrix core idle for their latency)
    float ra[NB], rb[NB], r1;
    auto issue = [&](int kp) {
      const float* xrow = xb + (size_t)(2 * kp + half) * LDW;
#pragma unroll
      for (int I = 0; I < NB; ++I) {
        ra[I] = xrow[fa[I]];
        rb[I] = xrow[fb[I]];
      }
      r1 = xrow[ONE];
    };
    issue(wave);
#pragma unroll
    for (int kp = wave; kp < RC / 2; kp += 4) {
      float a[NB];
#pragma unroll
      for (int I = 0; I < NB; ++I) a[I] = (ra[I] * rb[I]) * r1;
      if (kp + 4 < RC / 2) issue(kp + 4);
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
#ifdef OMLDM_GRAM_PROBE_NOFLUSH
  if (G) return;  // timing diagnostics only (csrc/tests/gram_probe.hip)
#endif
  if (part) {  // the block's image to its row of the partials (gram_colsum_kernel adds them)
    for (int e = tid; e < RF; e += 256) part[(size_t)blockIdx.x * RF + e] = red[e];
    return;
  }
  for (int e = tid; e < RF; e += 256) gram_add_element<NB>(e, red[e], G, ld, d, cnt);
}

// Sum of the blocks' tile images [nb][T·1024] per element into G: thread = element,
// blockIdx.y = a slab of 32 block rows (one atomic per element per slab instead of one
// per block: ≈ 2.6 M same-address atomics from 256 blocks serialised at the memory side).
template <int NB>
__global__ __launch_bounds__(256) void gram_colsum_kernel(const float* __restrict__ part, int nb,
                                                          float* __restrict__ G, int ld, int d,
                                                          double* __restrict__ cnt) {
  constexpr int RF = NB * (NB + 1) / 2 * 1024;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= RF) return;
  const int b0 = blockIdx.y * 32, b1 = min(nb, b0 + 32);
  float a = 0.f;
#pragma unroll 16
  for (int b = b0; b < b1; ++b) a += part[(size_t)b * RF + e];
  gram_add_element<NB>(e, a, G, ld, d, cnt);
}

// G[i][j] = G[j][i] for j < i < n (gram_map_kernel accumulates the upper triangle).
__global__ __launch_bounds__(256) void gram_mirror_kernel(float* __restrict__ G, int ld, int n) {
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n * n; e += gridDim.x * 256) {
    const int i = e / n, j = e % n;
    if (i > j) G[(size_t)i * ld + j] = G[(size_t)j * ld + i];
  }
}

// Block flush of the K-means partials. With `bpart`: the block's k·d sums, k counts and
// inertia go to its own row of the partials image with plain coalesced stores
// (kmeans_colsum_kernel adds the rows per column: a handful of atomics per address instead
// of one per block, which serialised at the memory side); without: atomics per block.
__device__ __forceinline__ void kmeans_flush(const float* s, const float* n, float my_in, int k,
                                             int d, float* __restrict__ sums,
                                             float* __restrict__ counts,
                                             float* __restrict__ inertia,
                                             float* __restrict__ bpart, float* red4) {
  const int tid = threadIdx.x;
  const float w = wave_sum(my_in);
  if ((tid & 63) == 0) red4[tid >> 6] = w;
  __syncthreads();
  const float tot = (red4[0] + red4[1]) + (red4[2] + red4[3]);
  const int kd = k * d;
  if (bpart) {
    float* row = bpart + (size_t)blockIdx.x * (kd + k + 1);
    for (int i = tid; i < kd; i += 256) row[i] = s[i];
    for (int i = tid; i < k; i += 256) row[kd + i] = n[i];
    if (tid == 0) row[kd + k] = tot;
    return;
  }
  for (int i = tid; i < kd; i += 256)
    if (s[i] != 0.f) atomicAdd(&sums[i], s[i]);
  for (int i = tid; i < k; i += 256)
    if (n[i] != 0.f) atomicAdd(&counts[i], n[i]);
  if (tid == 0 && inertia) atomicAdd(inertia, tot);
}

// Column sums of the partials image [nb][k·d + k + 1] into sums / counts / inertia: thread
// = column, blockIdx.y = a slab of 64 block rows (one atomic per column per slab).
__global__ __launch_bounds__(256) void kmeans_colsum_kernel(const float* __restrict__ part, int nb,
                                                            int k, int d, float* __restrict__ sums,
                                                            float* __restrict__ counts,
                                                            float* __restrict__ inertia) {
  const int kd = k * d, pw = kd + k + 1;
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= pw) return;
  const int b0 = blockIdx.y * 64, b1 = min(nb, b0 + 64);
  float a = 0.f;
#pragma unroll 16
  for (int b = b0; b < b1; ++b) a += part[(size_t)b * pw + col];
  if (a == 0.f) return;
  float* dst = col < kd ? &sums[col] : col < kd + k ? &counts[col - kd] : inertia;
  if (dst) atomicAdd(dst, a);
}

// ---- K-means -------------------------------------------------------------------------
// One thread per row: nearest centroid (centroids staged in LDS), per-block LDS sums of
// rows and counts per cluster, one atomic per (cluster, feature) per block.
// DMAX > 0 (d ≤ DMAX): the row is loaded into registers once (all loads in flight
// together, zero past d) and every distance and the sums read it from there; the
// centroids are staged zero-padded to DMAX columns, so the distance loop needs no masks.
// DMAX == 0: any d, the row is re-read through L1 per centroid.
template <int DMAX>
__global__ __launch_bounds__(256) void kmeans_assign_kernel(
    const float* __restrict__ x, const float* __restrict__ yv, int B, int d, int k,
    const float* __restrict__ cent, float* __restrict__ sums, float* __restrict__ counts,
    int* __restrict__ assign, float* __restrict__ inertia, float* __restrict__ bpart) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int kDm = DMAX > 0 ? DMAX : 1;
  const int cw = DMAX > 0 ? DMAX : d;          // centroid row width in LDS
  float* c = reinterpret_cast<float*>(smem);  // [k][cw]
  float* s = c + k * cw;                      // [k][d]
  float* n = s + k * d;                       // [k]
  __shared__ float part[4];
  for (int i = threadIdx.x; i < k * cw; i += 256) {
    const int r = i / cw, f = i - r * cw;
    c[i] = f < d ? cent[r * d + f] : 0.f;
  }
  for (int i = threadIdx.x; i < k * d; i += 256) s[i] = 0.f;
  for (int i = threadIdx.x; i < k; i += 256) n[i] = 0.f;
  __syncthreads();
  float my_in = 0.f;
  for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < B;
       r += (long long)gridDim.x * 256) {
    const float* xr = x + r * d;
    int best = 0;
    float bd = INFINITY;
    if constexpr (DMAX > 0) {
      float xv[kDm];
#pragma unroll
      for (int f = 0; f < kDm; ++f) xv[f] = xr[f < d ? f : 0];
#pragma unroll
      for (int f = 0; f < kDm; ++f) xv[f] = f < d ? xv[f] : 0.f;
      for (int j = 0; j < k; ++j) {
        float dd = 0.f;
#pragma unroll
        for (int f = 0; f < kDm; ++f) {  // zero-padded on both sides: no masks, no branches
          const float t = xv[f] - c[j * kDm + f];
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
#pragma unroll
        for (int f = 0; f < kDm; ++f)
          if (f < d) atomicAdd(&s[best * d + f], xv[f]);
        atomicAdd(&n[best], 1.f);
        my_in += bd;
      }
    } else {
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
  }
  __syncthreads();
  if (sums) kmeans_flush(s, n, my_in, k, d, sums, counts, inertia, bpart, part);
}

// Nearest-centroid assignment on the matrix cores (k ≥ 32 centroids): distances as
// ‖c‖² − 2·c·x (the row's own ‖x‖² does not change its argmin) with C·Xᵀ tiles on
// v_mfma_f32_32x32x2_f32 (exact fp32 products). A wave takes 32-row tiles; A = a 32-centroid
// tile staged in LDS (odd row stride: the 32 lanes of an operand column on distinct banks),
// B = the tile's rows, each lane keeping its row's features in registers across all
// centroid tiles. The operands are augmented so the product IS the distance: A row i =
// [c_i, ‖c_i‖²], B column j = [−2·x_j, 1] (−2 is exact), padded centroid rows carry +inf.
// Lane (j, h) ends a tile holding ‖c_i‖² − 2c_i·x_j for 16 centroids i of its half, so the
// argmin is an in-lane minimum plus one exchange with lane j ^ 32. Training rows then
// add x into the block's LDS cluster sums as the scalar kernel does.
template <int DMAX>
__global__ __launch_bounds__(256) void kmeans_assign_mfma_kernel(
    const float* __restrict__ x, const float* __restrict__ yv, int B, int d, int k,
    const float* __restrict__ cent, float* __restrict__ sums, float* __restrict__ counts,
    int* __restrict__ assign, float* __restrict__ inertia, float* __restrict__ bpart,
    int ablate) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int kp = (k + 31) & ~31;
  constexpr int ldc = DMAX | 1;  // ≥ DMAX + 1: every operand read stays inside its row
  float* cs = reinterpret_cast<float*>(smem);  // [kp][ldc]: c, ‖c‖² (+inf: padding), 0…
  float* s = cs + (size_t)kp * ldc;            // [k][d] cluster sums of this block
  float* n = s + (size_t)k * d;                // [k]
  __shared__ float part[4];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // padding (columns d..ldc-1 of every row, rows k..kp-1) is zero; the centroids are read
  // as one contiguous k·d run, 8 loads per thread in flight at a time (clamped, then masked)
  for (int i = tid; i < kp * ldc; i += 256) {
    const int r = i / ldc, c = i - r * ldc;
    if (r >= k || c >= d) cs[i] = 0.f;
  }
  const int kd = k * d;
  for (int base = 0; base < kd; base += 256 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * 256 + tid;
      v[u] = cent[i < kd ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * 256 + tid;
      if (i < kd) {
        const int r = i / d;
        cs[r * ldc + (i - r * d)] = v[u];
      }
    }
  }
  for (int i = tid; i < k * d; i += 256) s[i] = 0.f;
  for (int i = tid; i < k; i += 256) n[i] = 0.f;
  __syncthreads();
  for (int r = tid; r < kp; r += 256) {
    float a = 0.f;
    for (int c = 0; c < d; ++c) a = fmaf(cs[r * ldc + c], cs[r * ldc + c], a);
    cs[r * ldc + d] = r < k ? a : INFINITY;
  }
  __syncthreads();
  const int j = lane & 31, h = lane >> 5;
  float my_in = 0.f;
  // software pipeline: the next tile's row features and label are in flight while the
  // current tile computes (unconditional loads from clamped rows, masked afterwards)
  float nx[DMAX / 2], ny = 0.f;
  auto fetch = [&](long long t) {
    const long long row = t * 32 + j;
    const long long rr = row < B ? row : B - 1;
    const float* xr = x + rr * (long long)d;
#pragma unroll
    for (int u = 0; u < DMAX / 2; ++u) nx[u] = xr[2 * u + h < d ? 2 * u + h : 0];
    ny = yv ? yv[rr] : 0.f;
  };
  constexpr bool kPf = DMAX <= 48;  // wider rows: no room for a second row copy
  const long long tstride = (long long)gridDim.x * 4;
  long long t = (long long)blockIdx.x * 4 + wave;
  if (kPf && t * 32 < B) fetch(t);
  for (; t * 32 < B; t += tstride) {
    const long long row = t * 32 + j;
    const bool vrow = row < B;
    if (!kPf) fetch(t);
    // B operand: −2·x_f for f = h, h+2, … < d, then 1 at f = d (times ‖c‖²), then 0
    float xv[DMAX / 2];
#pragma unroll
    for (int u = 0; u < DMAX / 2; ++u) {
      const int f = 2 * u + h;
      xv[u] = f < d ? -2.f * nx[u] : (f == d ? 1.f : 0.f);
    }
    const float ycur = ny;
    if (kPf && (t + tstride) * 32 < B) fetch(t + tstride);
    float best = INFINITY;
    int bi = 0;
    auto argmin = [&](const f32x16& acc, int ct) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (acc[q] < best) {
          best = acc[q];
          bi = ct + (q & 3) + 8 * (q >> 2) + 4 * h;
        }
      }
    };
    // two centroid tiles per step: two independent MFMA chains in flight
    for (int ct = 0; ct < kp; ct += 64) {
      const bool two = ct + 32 < kp;
      f32x16 a0 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      f32x16 a1 = a0;
      const float* c0 = cs + (size_t)(ct + j) * ldc + h;
      const float* c1 = two ? c0 + 32 * (size_t)ldc : c0;
      // all DMAX/2 steps, no branches (a branch per step would wait for each operand
      // read): columns d+1..ldc-1 are zero in both operands
      float o0[DMAX / 2], o1[DMAX / 2];
#pragma unroll
      for (int u = 0; u < DMAX / 2; ++u) {
        o0[u] = c0[2 * u];
        o1[u] = c1[2 * u];
      }
#pragma unroll
      for (int u = 0; u < DMAX / 2; ++u) {
        a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(o0[u], xv[u], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(o1[u], xv[u], a1, 0, 0, 0);
      }
      argmin(a0, ct);
      if (two) argmin(a1, ct + 32);
    }
    // the other half-wave holds the same row's other 16 centroids of every tile
    const float ob = __shfl_xor(best, 32);
    const int oi = __shfl_xor(bi, 32);
    if (ob < best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
    // the sums come from the registers: each half adds its own features of the row
    // (x = −½·xv exactly)
#pragma unroll
    for (int u = 0; u < DMAX / 2; ++u) xv[u] = 2 * u + h < d ? -0.5f * xv[u] : 0.f;
    float xx = 0.f;
#pragma unroll
    for (int u = 0; u < DMAX / 2; ++u) xx = fmaf(xv[u], xv[u], xx);
    xx += __shfl_xor(xx, 32);
    if (vrow) {
      if (assign && h == 0) assign[row] = bi;
      const bool train = !__builtin_isnan(ycur);
      if (train && sums && !(ablate & 2)) {
#pragma unroll
        for (int u = 0; u < DMAX / 2; ++u)
          if (2 * u + h < d) atomicAdd(&s[bi * d + 2 * u + h], xv[u]);
        if (h == 0) {
          atomicAdd(&n[bi], 1.f);
          my_in += fmaxf(0.f, xx + best);  // ‖x − c‖² ≥ 0 (rounding)
        }
      }
    }
  }
  __syncthreads();
  if (sums && !(ablate & 1)) kmeans_flush(s, n, my_in, k, d, sums, counts, inertia, bpart, part);
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

template <int NB, int EPT, int RC>
static int launch_gram_map(const float* x, const float* y, int B, int d0, const int* pairs,
                           int npairs, float* G, int ld, double* cnt, float* part,
                           hipStream_t st) {
  // ≤ one block per CU, each ≥ one chunk: every block's image costs T·4 KiB of atomics
  long long rpb = ((long long)B + 255) / 256;
  rpb = ((rpb + RC - 1) / RC) * RC;
  const int blocks = (int)(((long long)B + rpb - 1) / rpb);
  const int ldw = (d0 + 3) | 1;
  const int T = NB * (NB + 1) / 2;
  const size_t lds = (size_t)(2 * RC * ldw > T * 1024 ? 2 * RC * ldw : T * 1024) * 4;
  auto fn = gram_map_kernel<NB, EPT, RC>;
  const int e = check_dyn_lds((const void*)fn, lds);
  if (e) return e;
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), lds, st, x, y, B, d0, pairs, npairs, (int)rpb, G,
                     ld, cnt, part);
  if (part)
    hipLaunchKernelGGL(gram_colsum_kernel<NB>, dim3(T * 4, (blocks + 31) / 32), dim3(256), 0, st,
                       part, blocks, G, ld, d0 + npairs, cnt);
  const int n = NB * 32 < ld ? NB * 32 : ld;
  hipLaunchKernelGGL(gram_mirror_kernel, dim3((n * n + 255) / 256), dim3(256), 0, st, G, ld, n);
  return (int)hipGetLastError();
}

template <int NB>
static int gram_map_e(const float* x, const float* y, int B, int d0, const int* pairs, int npairs,
                      float* G, int ld, double* cnt, float* part, hipStream_t st) {
  // element slots per thread: RC staged rows × d0 raw values over 256 threads (EPT ≥
  // RC·d0/256); 128-row chunks halve the per-chunk barriers where the registers allow
  if (d0 <= 8) return launch_gram_map<NB, 4, 128>(x, y, B, d0, pairs, npairs, G, ld, cnt, part, st);
  if (d0 <= 16) return launch_gram_map<NB, 8, 128>(x, y, B, d0, pairs, npairs, G, ld, cnt, part, st);
  if (d0 <= 32) return launch_gram_map<NB, 16, 128>(x, y, B, d0, pairs, npairs, G, ld, cnt, part, st);
  if (d0 <= 64) return launch_gram_map<NB, 16, 64>(x, y, B, d0, pairs, npairs, G, ld, cnt, part, st);
  return launch_gram_map<NB, 32, 64>(x, y, B, d0, pairs, npairs, G, ld, cnt, part, st);
}

static int gram_map(const float* x, const float* y, int B, int d0, const int* pairs, int npairs,
                    float* G, int ld, double* cnt, float* part, hipStream_t st) {
  const int dz = d0 + npairs + 2;
  if (dz <= 32) return gram_map_e<1>(x, y, B, d0, pairs, npairs, G, ld, cnt, part, st);
  if (dz <= 64) return gram_map_e<2>(x, y, B, d0, pairs, npairs, G, ld, cnt, part, st);
  if (dz <= 96) return gram_map_e<3>(x, y, B, d0, pairs, npairs, G, ld, cnt, part, st);
  return gram_map_e<4>(x, y, B, d0, pairs, npairs, G, ld, cnt, part, st);
}

// G[ld×ld] += [X 1 y]ᵀ[X 1 y] over rows with finite y (ld ≥ d + 2).
// cnt (may be null): += number of rows with finite y.
// part (optional): a [256][10240]-float scratch image for the per-block tile sums (v2
// kernel); nullptr: the blocks add into G with atomics.
OMLDM_API int omldm_gram_update(const float* x, const float* y, int B, int d, float* G, int ld,
                                double* cnt, float* part, void* stream) {
  if (B <= 0) return 0;
  const int dz = d + 2;
  if (ld < dz) return -1;
  static const int v1 = [] {
    const char* e = getenv("OMLDM_GRAM_V1");  // A/B: the one-tile-per-wave v1 kernel
    return e ? atoi(e) : 0;
  }();
  if (!v1 && dz <= 128) return gram_map(x, y, B, d, nullptr, 0, G, ld, cnt, part, (hipStream_t)stream);
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
                              float* inertia, float* bpart, size_t lds, hipStream_t st,
                              int* nblocks) {
  auto fn = kmeans_assign_mfma_kernel<DMAX>;
  int e = check_dyn_lds((const void*)fn, lds);
  if (e) return e;
  const long long tiles = ((long long)B + 31) / 32;
  int blocks = (int)((tiles + 3) / 4);
  int cap = kKmeansMaxBlocks;
  if (const char* e = getenv("OMLDM_KMEANS_BLOCKS")) cap = atoi(e) > 0 ? atoi(e) : cap;  // sweep
  if (blocks > cap) blocks = cap;
  if (blocks > kKmeansMaxBlocks) blocks = kKmeansMaxBlocks;  // the partials image's rows
  *nblocks = blocks;
  // timing diagnostics only: bit 0 skips the global flush, bit 1 the LDS cluster sums
  const char* ab = getenv("OMLDM_KMEANS_ABLATE");
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), lds, st, x, y, B, d, k, cent, sums, counts,
                     assign, inertia, bpart, ab ? atoi(ab) : 0);
  return (int)hipGetLastError();
}

static int kmeans_colsum(const float* bpart, int nb, int k, int d, float* sums, float* counts,
                         float* inertia, hipStream_t st) {
  const int pw = k * d + k + 1;
  hipLaunchKernelGGL(kmeans_colsum_kernel, dim3((pw + 255) / 256, (nb + 63) / 64), dim3(256), 0,
                     st, bpart, nb, k, d, sums, counts, inertia);
  return (int)hipGetLastError();
}

// bpart (optional, with sums): a [kKmeansMaxBlocks][k·d + k + 1] float scratch image for
// the per-block partials (see kmeans_flush); nullptr: per-block atomics.
OMLDM_API int omldm_kmeans_assign(const float* x, const float* y, int B, int d, int k,
                                  const float* cent, float* sums, float* counts, int* assign,
                                  float* inertia, float* bpart, void* stream) {
  if (B <= 0) return 0;
  if (!sums) bpart = nullptr;
  // matrix-core distances once there is a full 32-centroid tile and a few features
  // (OMLDM_KMEANS_MFMA=0: the scalar kernel, A/B)
  const char* mf = getenv("OMLDM_KMEANS_MFMA");
  if (k >= 32 && d >= 4 && d < 128 && !(mf && atoi(mf) == 0)) {
    // operand width: d + 1 (the ‖c‖² column) rounded up to the next of 16, 24, 32, 48, 64,
    // 96, 128 (the K loop runs DMAX/2 matrix-core steps unconditionally)
    const int da = d + 1;
    const int dm = da <= 16 ? 16 : da <= 24 ? 24 : da <= 32 ? 32 : da <= 48 ? 48 : da <= 64 ? 64
                 : da <= 96 ? 96 : 128;
    const int kp = (k + 31) & ~31, ldc = dm | 1;
    const size_t lds = ((size_t)kp * ldc + (size_t)k * d + k) * 4;
    if (lds <= 150 * 1024) {
      hipStream_t st = (hipStream_t)stream;
      int nb = 0, rc = -2;
#define OMLDM_KMM(DM)                                                                           \
  if (dm == DM)                                                                                 \
  rc = launch_kmeans_mfma<DM>(x, y, B, d, k, cent, sums, counts, assign, inertia, bpart, lds, st, \
                              &nb)
      OMLDM_KMM(16);
      OMLDM_KMM(24);
      OMLDM_KMM(32);
      OMLDM_KMM(48);
      OMLDM_KMM(64);
      OMLDM_KMM(96);
      OMLDM_KMM(128);
#undef OMLDM_KMM
      if (rc || !bpart) return rc;
      return kmeans_colsum(bpart, nb, k, d, sums, counts, inertia, st);
    }
  }
  const int dm = d <= 16 ? 16 : d <= 32 ? 32 : d <= 64 ? 64 : 0;
  const size_t lds = (size_t)(k * (dm ? dm : d) + k * d + k) * 4;
  if (lds > 150 * 1024) return -1;
  int blocks = (B + 255) / 256;
  if (blocks > kKmeansMaxBlocks) blocks = kKmeansMaxBlocks;
  hipStream_t st = (hipStream_t)stream;
#define OMLDM_KM(DM)                                                                        \
  do {                                                                                      \
    const int e_ = check_dyn_lds((const void*)kmeans_assign_kernel<DM>, lds);               \
    if (e_) return e_;                                                                      \
    hipLaunchKernelGGL(kmeans_assign_kernel<DM>, dim3(blocks), dim3(256), lds, st, x, y, B, d, \
                       k, cent, sums, counts, assign, inertia, bpart);                      \
  } while (0)
  if (dm == 16) OMLDM_KM(16);
  else if (dm == 32) OMLDM_KM(32);
  else if (dm == 64) OMLDM_KM(64);
  else OMLDM_KM(0);
#undef OMLDM_KM
  const int rc = (int)hipGetLastError();
  if (rc || !bpart) return rc;
  return kmeans_colsum(bpart, blocks, k, d, sums, counts, inertia, st);
}

// G += Σ zzᵀ with z = [x, x_a·x_b for (a, b) in pairs, 1, y] over rows with finite y: the
// Gram of PolynomialFeatures(2)(x) without materialising the expansion (pairs: int32
// [npairs][2]; d0 + npairs + 2 ≤ 128, else -2: expand and call omldm_gram_update).
OMLDM_API int omldm_gram_update_poly2(const float* x, const float* y, int B, int d0,
                                      const int* pairs, int npairs, float* G, int ld, double* cnt,
                                      float* part, void* stream) {
  if (B <= 0) return 0;
  const int dz = d0 + npairs + 2;
  if (ld < dz) return -1;
  if (dz > 128) return -2;
  return gram_map(x, y, B, d0, pairs, npairs, G, ld, cnt, part, (hipStream_t)stream);
}
