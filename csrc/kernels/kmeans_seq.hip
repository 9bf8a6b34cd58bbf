// Exact sequential (MacQueen) online k-means: the reference learner's per-point update
// (nearest centroid, c ← c + (x − c)/n_c; the spoke fits one point
// at a time, omldm/operators/spoke/FlinkSpoke.scala:92-107; K-means runs as SingleLearner,
// :203-209), at GPU speed for k ≤ 64.
//
// One wavefront owns the whole model in REGISTERS: lane j holds centroid j (its d ≤ DM
// coordinates) and its count n_j. Points stream in 64-row chunks, lane t holding point t
// of the chunk; step s broadcasts point s with v_readlane (scalar registers), every lane
// computes its centroid's squared distance, a DPP/readlane argmin picks j*, and lane j*
// moves its centroid — no LDS, no barrier, no memory access on the per-point chain.
// Seeding: while fewer than k centroids exist (n_j = 0), a point becomes the next
// centroid (n = 1). Rows with a NaN target are not training points and are skipped.
#include "common.h"

namespace omldm {
namespace {

// The lowest lane holding the wave's minimum of v (wave-uniform). The minimum climbs to
// lane 63 through DPP moves (row_shr 1/2/4/8 inside each 16-lane row, then row_bcast 15 /
// 31 across the rows: one VALU op per step, no LDS round trip — the ds_bpermute butterfly
// cost ~700 of the ~1000 cycles of a point's chain), then one compare + ballot finds its
// lowest lane.
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_min_step(float v) {
  const int o = __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                            CTRL, ROWS, 0xf, false);
  return fminf(v, __builtin_bit_cast(float, o));
}

__device__ __forceinline__ int wave_argmin(float v, float& vmin) {
  float m = v;
  m = dpp_min_step<0x111, 0xf>(m);  // row_shr:1
  m = dpp_min_step<0x112, 0xf>(m);  // row_shr:2
  m = dpp_min_step<0x114, 0xf>(m);  // row_shr:4
  m = dpp_min_step<0x118, 0xf>(m);  // row_shr:8  → lane 15 of each row: the row's minimum
  m = dpp_min_step<0x142, 0xa>(m);  // row_bcast:15 → lanes 31, 63: two rows' minimum
  m = dpp_min_step<0x143, 0xc>(m);  // row_bcast:31 → lane 63: the wave's minimum
  vmin = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, m), 63));
  const unsigned long long at = __builtin_amdgcn_ballot_w64(v == vmin);
  return at ? __builtin_ctzll(at) : 0;  // (no lane: every distance NaN)
}

template <int DM>
__global__ __launch_bounds__(64) void kmeans_seq_kernel(const float* __restrict__ x, int ldx,
                                                        const float* __restrict__ y, int B,
                                                        int d, int k, float* __restrict__ cent,
                                                        float* __restrict__ cnt,
                                                        double* __restrict__ cum) {
  const int lane = threadIdx.x;
  const bool mine = lane < k;
  float c[DM];
#pragma unroll
  for (int i = 0; i < DM; ++i) c[i] = (mine && i < d) ? cent[(size_t)lane * d + i] : 0.f;
  float n = mine ? cnt[lane] : 0.f;
  // seeded centroids: a prefix (seeding fills them in order)
  int seeded = __popcll(__builtin_amdgcn_ballot_w64(mine && n > 0.f));
  double inertia = 0.0, fitted = 0.0;
  float xr[DM];
  float yr;
  auto load = [&](int r0) {
    const int r = r0 + lane;
    const bool ok = r < B;
#pragma unroll
    for (int i = 0; i < DM; ++i) xr[i] = (ok && i < d) ? x[(size_t)r * ldx + i] : 0.f;
    yr = ok ? (y ? y[r] : 0.f) : __builtin_nanf("");
  };
  load(0);
  for (int r0 = 0; r0 < B; r0 += 64) {
    float xc[DM];
#pragma unroll
    for (int i = 0; i < DM; ++i) xc[i] = xr[i];
    const float yc = yr;
    if (r0 + 64 < B) load(r0 + 64);  // the next chunk's loads fly under this chunk's steps
    // training points of this chunk (non-NaN target, inside the batch)
    unsigned long long live = __builtin_amdgcn_ballot_w64(yc == yc);
    while (live) {
      const int s = __builtin_ctzll(live);
      live &= live - 1;
      float xs[DM];
#pragma unroll
      for (int i = 0; i < DM; ++i)
        xs[i] = i < d ? __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                      __builtin_bit_cast(int, xc[i]), s))
                      : 0.f;
      fitted += 1.0;
      if (seeded < k) {  // wave-uniform
        if (lane == seeded) {
#pragma unroll
          for (int i = 0; i < DM; ++i) c[i] = xs[i];
          n = 1.f;
        }
        ++seeded;
        continue;
      }
      // four independent partial sums: the distance is on the per-point chain
      float dp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < DM; ++i) {
        const float t = xs[i] - c[i];
        dp[i & 3] = fmaf(t, t, dp[i & 3]);
      }
      const float dist = (dp[0] + dp[1]) + (dp[2] + dp[3]);
      float dmin;
      const int j = wave_argmin(mine ? dist : __builtin_inff(), dmin);
      inertia += (double)dmin;
      if (lane == j) {
        n += 1.f;
        const float a = 1.f / n;
#pragma unroll
        for (int i = 0; i < DM; ++i) c[i] = fmaf(a, xs[i] - c[i], c[i]);
      }
    }
  }
  if (mine) {
#pragma unroll
    for (int i = 0; i < DM; ++i)
      if (i < d) cent[(size_t)lane * d + i] = c[i];
    cnt[lane] = n;
  }
  if (lane == 0 && cum) {
    cum[0] += inertia;
    cum[1] += fitted;
  }
}

// Larger models (k ≤ 1024 centroids, d ≤ 256 coordinates): one workgroup of NW waves,
// thread j owning centroid j, the centroids in LDS (row stride d + 1: the lanes' rows fall
// in different banks), each 64-point chunk staged in LDS. Per point: every thread's distance
// (the point's coordinates are LDS broadcasts), a DPP argmin per wave, the waves' minima
// through LDS (ties to the lowest index), the owner's update, two barriers — the same
// per-point order as the one-wave kernel, exact at any size that fits the LDS.
template <int NW>
__global__ __launch_bounds__(NW * 64) void kmeans_seq_wg_kernel(const float* __restrict__ x,
                                                                int ldx,
                                                                const float* __restrict__ y,
                                                                int B, int d, int k,
                                                                float* __restrict__ cent,
                                                                float* __restrict__ cnt,
                                                                double* __restrict__ cum) {
  extern __shared__ float smem[];
  const int ds = d + 1;
  float* C = smem;                        // [k][ds]
  float* xs = C + (size_t)k * ds;         // [64][d] the chunk's points
  float* ysh = xs + 64 * d;               // [64]
  float* rmin = ysh + 64;                 // [NW]
  int* ridx = reinterpret_cast<int*>(rmin + NW);  // [NW]
  int* sseed = ridx + NW;                 // [1]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool mine = tid < k;
  for (int i = tid; i < k * d; i += NW * 64) C[(i / d) * ds + i % d] = cent[i];
  float n = mine ? cnt[tid] : 0.f;
  if (tid == 0) *sseed = 0;
  __syncthreads();
  if (mine && n > 0.f) atomicAdd(sseed, 1);  // seeded centroids form a prefix
  __syncthreads();
  int seeded = *sseed;
  double inertia = 0.0, fitted = 0.0;
  for (int r0 = 0; r0 < B; r0 += 64) {
    __syncthreads();  // the previous chunk's points are consumed
    for (int i = tid; i < 64 * d; i += NW * 64) {
      const int r = r0 + i / d;
      xs[i] = r < B ? x[(size_t)r * ldx + i % d] : 0.f;
    }
    if (tid < 64) ysh[tid] = r0 + tid < B ? (y ? y[r0 + tid] : 0.f) : __builtin_nanf("");
    __syncthreads();
    const int np = B - r0 < 64 ? B - r0 : 64;
    for (int p = 0; p < np; ++p) {
      if (ysh[p] != ysh[p]) continue;  // not a training point (block-uniform)
      const float* xp = xs + p * d;
      fitted += 1.0;
      if (seeded < k) {  // block-uniform: the point becomes the next centroid
        if (tid == seeded) {
          for (int i = 0; i < d; ++i) C[tid * ds + i] = xp[i];
          n = 1.f;
        }
        ++seeded;
        __syncthreads();
        continue;
      }
      float dist = __builtin_inff();
      if (mine) {
        float dp[4] = {0.f, 0.f, 0.f, 0.f};
        const float* cr = C + tid * ds;
        for (int i = 0; i < d; ++i) {
          const float t = xp[i] - cr[i];
          dp[i & 3] = fmaf(t, t, dp[i & 3]);
        }
        dist = (dp[0] + dp[1]) + (dp[2] + dp[3]);
      }
      float wmin;
      const int wj = wave_argmin(dist, wmin);
      if (lane == 0) {
        rmin[wave] = wmin;
        ridx[wave] = wave * 64 + wj;
      }
      __syncthreads();
      float best = rmin[0];
      int j = ridx[0];
#pragma unroll
      for (int w = 1; w < NW; ++w)
        if (rmin[w] < best) {  // strictly: ties keep the lower wave (lower index)
          best = rmin[w];
          j = ridx[w];
        }
      if (tid == 0) inertia += (double)best;
      if (tid == j) {
        n += 1.f;
        const float a = 1.f / n;
        float* cr = C + tid * ds;
        for (int i = 0; i < d; ++i) cr[i] = fmaf(a, xp[i] - cr[i], cr[i]);
      }
      __syncthreads();  // the update is visible to the next point's distances
    }
  }
  __syncthreads();
  for (int i = tid; i < k * d; i += NW * 64) cent[i] = C[(i / d) * ds + i % d];
  if (mine) cnt[tid] = n;
  if (tid == 0 && cum) {
    cum[0] += inertia;
    cum[1] += fitted;
  }
}

size_t kmeans_wg_lds(int d, int k, int nw) {
  return ((size_t)k * (d + 1) + 64 * d + 64 + 2 * nw + 1) * sizeof(float);
}

}  // namespace
}  // namespace omldm

using namespace omldm;

static bool kmeans_one_wave(int d, int k) { return d >= 1 && d <= 64 && k >= 1 && k <= 64; }

OMLDM_API int omldm_kmeans_seq_fits(int d, int k) {
  if (kmeans_one_wave(d, k)) return 1;
  const int nw = (k + 63) / 64;
  return d >= 1 && d <= 256 && k >= 1 && k <= 1024 &&
         kmeans_wg_lds(d, k, nw <= 4 ? 4 : 16) <= 160 * 1024;
}

// x [B, ldx] fp32 (first d columns used), y [B] (NaN: not a training point; nullptr: all
// train), cent [k, d], cnt [k], cum (cum[0] += Σ squared distance to the chosen
// centroid, cum[1] += points fitted) — all device pointers; one wave, one launch.
OMLDM_API int omldm_kmeans_seq(const float* x, int ldx, const float* y, int B, int d, int k,
                               float* cent, float* cnt, double* cum, void* stream) {
  if (!omldm_kmeans_seq_fits(d, k) || ldx < d) return -1;
  if (B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (!kmeans_one_wave(d, k)) {  // the workgroup form
    const int nw = (k + 63) / 64 <= 4 ? 4 : 16;
    const size_t lds = kmeans_wg_lds(d, k, nw);
    if (nw == 4) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&kmeans_seq_wg_kernel<4>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      hipLaunchKernelGGL(kmeans_seq_wg_kernel<4>, dim3(1), dim3(256), lds, st, x, ldx, y, B, d,
                         k, cent, cnt, cum);
    } else {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&kmeans_seq_wg_kernel<16>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      hipLaunchKernelGGL(kmeans_seq_wg_kernel<16>, dim3(1), dim3(1024), lds, st, x, ldx, y, B,
                         d, k, cent, cnt, cum);
    }
    return (int)hipGetLastError();
  }
  if (d <= 16)
    hipLaunchKernelGGL(kmeans_seq_kernel<16>, dim3(1), dim3(64), 0, st, x, ldx, y, B, d, k, cent,
                       cnt, cum);
  else if (d <= 32)
    hipLaunchKernelGGL(kmeans_seq_kernel<32>, dim3(1), dim3(64), 0, st, x, ldx, y, B, d, k, cent,
                       cnt, cum);
  else
    hipLaunchKernelGGL(kmeans_seq_kernel<64>, dim3(1), dim3(64), 0, st, x, ldx, y, B, d, k, cent,
                       cnt, cum);
  return (int)hipGetLastError();
}
