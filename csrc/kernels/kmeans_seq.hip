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

#include <algorithm>
#include <cstdlib>

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

// ------------------------------------------------------------------------------------------
// Fast one-wave form (k ≤ 512, d ≤ 64): the per-point chain is issue-bound on one wave, so
// the layout spends every lane of the wave on it and keeps the instruction count per point
// minimal:
//  * G consecutive lanes own one centroid, DPL of its coordinates each (k ≤ 16, d = 13:
//    G = 4, DPL = 4 — the distance is four packed sub/fma pairs and two quad DPP adds, not
//    thirteen of each on a quarter of the wave); above 64 centroids a lane owns CPL of them
//    (lane l: centroids l + 64q);
//  * the point's coordinates are an LDS broadcast read (no v_readlane per coordinate), the
//    64-row chunk is staged by coalesced loads one chunk ahead, the next point's read is in
//    flight while this point's distances run, every LDS offset is an immediate (the chunk's
//    64 steps are unrolled);
//  * argmin: unsigned min over the distances' bits (squared distances are ≥ 0, so the bit
//    order is the value order) in fused DPP steps, then one ballot of the lanes equal to
//    the minimum: its lowest lane's centroid wins, the same lowest-index tie rule as the
//    oracle (all G lanes of a centroid hold the bitwise same sum: the DPP adds commute);
//  * the winning centroid's lanes move it: r = 1/n (v_rcp + one Newton step: the correctly
//    rounded reciprocal the oracle's 1.f/n gives), c ← fma(r, x − c, c).
// (the DPP moves' "old" operand is the operation's identity, so lanes with no source lane —
// or in rows the row mask leaves out — fold to a no-op and the move fuses into the VALU op)
template <int CTRL, int RM>
__device__ __forceinline__ unsigned dpp_umin(unsigned v) {
  const unsigned o = (unsigned)__builtin_amdgcn_update_dpp(-1, (int)v, CTRL, RM, 0xf, false);
  return v < o ? v : o;
}
template <int CTRL>
__device__ __forceinline__ float dpp_addf(float v) {
  const int o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false);
  return v + __builtin_bit_cast(float, o);
}

// Sum over the G consecutive lanes of a group (every lane of the group gets the same bits).
template <int G>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (G >= 2) v = dpp_addf<0xB1>(v);   // quad_perm [1,0,3,2]
  if constexpr (G >= 4) v = dpp_addf<0x4E>(v);   // quad_perm [2,3,0,1]
  if constexpr (G >= 8) v = dpp_addf<0x141>(v);  // row_half_mirror
  if constexpr (G >= 16) v = dpp_addf<0x140>(v); // row_mirror
  return v;
}

// Wave minimum of v (groups of G equal lanes), valid in lane 63.
template <int G>
__device__ __forceinline__ unsigned wave_umin_groups(unsigned v) {
  if constexpr (G <= 1) v = dpp_umin<0x111, 0xf>(v);  // row_shr:1
  if constexpr (G <= 2) v = dpp_umin<0x112, 0xf>(v);  // row_shr:2
  if constexpr (G <= 4) v = dpp_umin<0x114, 0xf>(v);  // row_shr:4
  if constexpr (G <= 8) v = dpp_umin<0x118, 0xf>(v);  // row_shr:8
  v = dpp_umin<0x142, 0xa>(v);                        // row_bcast:15
  v = dpp_umin<0x143, 0xc>(v);                        // row_bcast:31
  return v;
}

__device__ __forceinline__ float rcp_rn(float n) {
  float r = __builtin_amdgcn_rcpf(n);
  const float e = fmaf(-n, r, 1.f);
  return fmaf(e, r, r);
}

// Chunk staging shared by the fast forms: 64 rows × RS floats (coordinates ≥ d zero), NT
// threads, element e = tid + NT·u; branch-free (out-of-range elements load x[0]).
template <int RS, int NT>
struct ChunkStage {
  static constexpr int PER = 64 * RS / NT;
  float v[PER];
  __device__ __forceinline__ void fetch(const float* __restrict__ x, int ldx, int B, int d,
                                        int r0, int tid) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = tid + NT * u, row = e / RS, col = e % RS;
      const bool ok = col < d && r0 + row < B;
      const float t = x[ok ? (size_t)(r0 + row) * ldx + col : 0];
      v[u] = ok ? t : 0.f;
    }
  }
  __device__ __forceinline__ void put(float* buf, int tid) const {
#pragma unroll
    for (int u = 0; u < PER; ++u) buf[tid + NT * u] = v[u];
  }
};

// The training rows of chunk r0 (y not NaN, inside the batch) as a wave-uniform bit mask.
__device__ __forceinline__ unsigned long long live_rows(const float* __restrict__ y, int B,
                                                        int r0, int lane) {
  const bool ok = r0 + lane < B;
  const float yv = y ? y[ok ? r0 + lane : 0] : 0.f;
  return __builtin_amdgcn_ballot_w64(ok && yv == yv);
}

// ND of the lane's DPL coordinates from LDS (float4 broadcast reads).
template <int DPL, int ND>
__device__ __forceinline__ void lds_row(const float* p, float* o) {
#pragma unroll
  for (int i = 0; i < ND; i += 4) {
    const float4 v = *reinterpret_cast<const float4*>(p + i);
    o[i] = v.x;
    if (i + 1 < ND) o[i + 1] = v.y;
    if (i + 2 < ND) o[i + 2] = v.z;
    if (i + 3 < ND) o[i + 3] = v.w;
  }
}

// Squared distance over ND coordinates, two independent chains (plain fp32 ops: one wave
// issues a v_fma in 4 cycles and a packed one in 8, and a packed chain needs a wait state
// per dependent step — the file is built without SLP packing).
template <int ND>
__device__ __forceinline__ float sqdist(const float* x, const float* c) {
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int i = 0; i < ND; i += 2) {
    const float t0 = x[i] - c[i];
    a0 = fmaf(t0, t0, a0);
    if (i + 1 < ND) {
      const float t1 = x[i + 1] - c[i + 1];
      a1 = fmaf(t1, t1, a1);
    }
  }
  return a0 + a1;
}

// One wave; G lanes per centroid (k ≤ 64/G), DPL coordinates per lane of which the first
// ND are computed (d = 13 at G = 1 stores 16, computes 14).
template <int G, int DPL, int ND>
__global__ __launch_bounds__(64) void kmeans_fast_kernel(const float* __restrict__ x, int ldx,
                                                         const float* __restrict__ y, int B,
                                                         int d, int k, float* __restrict__ cent,
                                                         float* __restrict__ cnt,
                                                         double* __restrict__ cum) {
  constexpr int RS = G * DPL;
  static_assert(ND <= DPL && DPL % 4 == 0, "geometry");
  __shared__ float4 xs4[2 * 64 * RS / 4];
  float* xs = reinterpret_cast<float*>(xs4);
  const int lane = threadIdx.x;
  const int grp = lane / G, part = lane % G;
  const int c0 = part * DPL;  // this lane's first coordinate
  const bool mine = grp < k;
  float c[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) c[i] = (mine && c0 + i < d) ? cent[(size_t)grp * d + c0 + i] : 0.f;
  float n = mine ? cnt[grp] : 0.f;
  // seeded centroids form a prefix (seeding fills them in order)
  int seeded = __popcll(__builtin_amdgcn_ballot_w64(part == 0 && mine && n > 0.f));
  const unsigned pad = mine ? 0u : 0x7f800000u;  // OR-ed into a key: never the minimum
  double inertia = 0.0, fitted = 0.0;
  const int nchunks = (B + 63) / 64;
  ChunkStage<RS, 64> stage;
  stage.fetch(x, ldx, B, d, 0, lane);
  stage.put(xs, lane);
  unsigned long long live = live_rows(y, B, 0, lane);
  for (int ch = 0; ch < nchunks; ++ch) {
    const int buf = ch & 1;
    unsigned long long live_next = 0;
    if (ch + 1 < nchunks) {  // the next chunk's loads fly under this chunk
      stage.fetch(x, ldx, B, d, (ch + 1) * 64, lane);
      live_next = live_rows(y, B, (ch + 1) * 64, lane);
    }
    fitted += (double)__popcll(live);
    const float* xb = xs + buf * 64 * RS + c0;
    // seeding (the first k training points of the stream): a slow uniform path
    while (seeded < k && live) {
      const int s = __builtin_ctzll(live);
      live &= live - 1;
      float xr[DPL];
      lds_row<DPL, DPL>(xb + s * RS, xr);
      if (grp == seeded) {
#pragma unroll
        for (int i = 0; i < DPL; ++i) c[i] = xr[i];
        n = 1.f;
      }
      ++seeded;
    }
    float ich = 0.f;
    float xc[ND], xn[ND];
    lds_row<DPL, ND>(xb, xc);
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      if (s + 1 < 64) lds_row<DPL, ND>(xb + (s + 1) * RS, xn);
      // the distance unconditionally (a row that is not a training point wastes it), so the
      // next row's LDS read stays ahead of this row's chain
      const unsigned key = __builtin_bit_cast(unsigned, group_sum<G>(sqdist<ND>(xc, c))) | pad;
      // 1/(n + 1) ahead of the argmin (it does not depend on it): off the point's chain
      const float rn = rcp_rn(n + 1.f);
      if ((live >> s) & 1ull) {
        const unsigned mw = (unsigned)__builtin_amdgcn_readlane((int)wave_umin_groups<G>(key), 63);
        ich += __builtin_bit_cast(float, mw);
        // the lowest lane holding the minimum (some lane always does: the mask is ≠ 0)
        const unsigned long long eq = __builtin_amdgcn_ballot_w64(key == mw);
        // the winner's lanes move the centroid; selects, not a divergent branch (no exec
        // mask save / restore on the chain)
        const bool win = grp == (int)__builtin_ctzll(eq | (1ull << 63)) / G;
        n = win ? n + 1.f : n;
#pragma unroll
        for (int i = 0; i < ND; ++i) c[i] = win ? fmaf(rn, xc[i] - c[i], c[i]) : c[i];
      }
#pragma unroll
      for (int i = 0; i < ND; ++i) xc[i] = xn[i];
    }
    inertia += (double)ich;
    if (ch + 1 < nchunks) {
      stage.put(xs + (buf ^ 1) * 64 * RS, lane);
      live = live_next;
    }
  }
  if (mine) {
#pragma unroll
    for (int i = 0; i < DPL; ++i)
      if (c0 + i < d) cent[(size_t)grp * d + c0 + i] = c[i];
    if (part == 0) cnt[grp] = n;
  }
  if (lane == 0 && cum) {
    cum[0] += inertia;
    cum[1] += fitted;
  }
}

// 64 < k ≤ 1024: four waves (one per SIMD), lane l of wave w holding centroids
// j = 256q + 64w + l (CPL slots); each wave's minimum and its lowest index go through LDS
// (two parities: one barrier per point), every wave takes the lexicographic (distance,
// index) minimum of the four, the owner moves the centroid. The per-point work of the
// one-wave form spread over four instruction streams.
template <int CPL, int DPL, int ND>
__global__ __launch_bounds__(256) void kmeans_mw_kernel(const float* __restrict__ x, int ldx,
                                                        const float* __restrict__ y, int B,
                                                        int d, int k, float* __restrict__ cent,
                                                        float* __restrict__ cnt,
                                                        double* __restrict__ cum) {
  constexpr int NW = 4, RS = DPL;
  static_assert(ND <= DPL && DPL % 4 == 0, "geometry");
  __shared__ float4 xs4[2 * 64 * RS / 4];
  __shared__ uint4 red4[2][NW / 2];  // per parity: (key, index) of each wave
  __shared__ int s_seed;
  float* xs = reinterpret_cast<float*>(xs4);
  unsigned* red = reinterpret_cast<unsigned*>(red4);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  float c[CPL][DPL];
  float n[CPL];
  unsigned pad[CPL];
  if (tid == 0) s_seed = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int j = q * 256 + w * 64 + lane;
    const bool mine = j < k;
#pragma unroll
    for (int i = 0; i < DPL; ++i) c[q][i] = (mine && i < d) ? cent[(size_t)j * d + i] : 0.f;
    n[q] = mine ? cnt[j] : 0.f;
    pad[q] = mine ? 0u : 0x7f800000u;
    if (mine && n[q] > 0.f) atomicMax(&s_seed, j + 1);  // seeded centroids form a prefix
  }
  __syncthreads();
  int seeded = s_seed;
  double inertia = 0.0, fitted = 0.0;
  const int nchunks = (B + 63) / 64;
  ChunkStage<RS, 256> stage;
  stage.fetch(x, ldx, B, d, 0, tid);
  stage.put(xs, tid);
  unsigned long long live = live_rows(y, B, 0, lane);
  int par = 0;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int buf = ch & 1;
    __syncthreads();  // the chunk's rows are in LDS
    unsigned long long live_next = 0;
    if (ch + 1 < nchunks) {
      stage.fetch(x, ldx, B, d, (ch + 1) * 64, tid);
      live_next = live_rows(y, B, (ch + 1) * 64, lane);
    }
    fitted += (double)__popcll(live);
    const float* xb = xs + buf * 64 * RS;
    while (seeded < k && live) {
      const int s = __builtin_ctzll(live);
      live &= live - 1;
#pragma unroll
      for (int q = 0; q < CPL; ++q)
        if (q * 256 + w * 64 + lane == seeded) {
          lds_row<DPL, DPL>(xb + s * RS, c[q]);
          n[q] = 1.f;
        }
      ++seeded;
    }
    float ich = 0.f;
    float xc[ND], xn[ND];
    lds_row<DPL, ND>(xb, xc);
#pragma unroll 4
    for (int s = 0; s < 64; ++s) {
      if (s + 1 < 64) lds_row<DPL, ND>(xb + (s + 1) * RS, xn);
      unsigned key[CPL];
      float rn[CPL];  // 1/(n + 1) ahead of the argmin, off the point's chain
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        key[q] = __builtin_bit_cast(unsigned, sqdist<ND>(xc, c[q])) | pad[q];
        rn[q] = rcp_rn(n[q] + 1.f);
      }
      if ((live >> s) & 1ull) {
        unsigned m = key[0];
#pragma unroll
        for (int q = 1; q < CPL; ++q) m = key[q] < m ? key[q] : m;
        const unsigned mw = (unsigned)__builtin_amdgcn_readlane((int)wave_umin_groups<1>(m), 63);
        unsigned jw = 0xffffffffu;  // this wave's lowest centroid index at the minimum
#pragma unroll
        for (int q = CPL - 1; q >= 0; --q) {
          const unsigned long long b = __builtin_amdgcn_ballot_w64(key[q] == mw);
          if (b) jw = q * 256 + w * 64 + (unsigned)__builtin_ctzll(b);
        }
        if (lane == 0) {
          red[par * 2 * NW + 2 * w] = mw;
          red[par * 2 * NW + 2 * w + 1] = jw;
        }
        // (a bare barrier: only LDS is exchanged, so the chunk prefetch's global loads are
        // not waited for as __syncthreads' fence would)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // branch-free: the minimum key, then the lowest index among the waves holding it
        const uint4 r01 = red4[par][0], r23 = red4[par][1];
        const unsigned bk = __builtin_elementwise_min(__builtin_elementwise_min(r01.x, r01.z),
                                                      __builtin_elementwise_min(r23.x, r23.z));
        const unsigned j0 = r01.x == bk ? r01.y : ~0u, j1 = r01.z == bk ? r01.w : ~0u;
        const unsigned j2 = r23.x == bk ? r23.y : ~0u, j3 = r23.z == bk ? r23.w : ~0u;
        const unsigned bj = __builtin_elementwise_min(__builtin_elementwise_min(j0, j1),
                                                      __builtin_elementwise_min(j2, j3));
        ich += __builtin_bit_cast(float, bk);
        par ^= 1;
        if ((int)((bj >> 6) & 3) == w && (int)(bj & 63) == lane) {
#pragma unroll
          for (int q = 0; q < CPL; ++q)
            if ((int)(bj >> 8) == q) {
              n[q] += 1.f;
#pragma unroll
              for (int i = 0; i < ND; ++i) c[q][i] = fmaf(rn[q], xc[i] - c[q][i], c[q][i]);
            }
        }
      }
#pragma unroll
      for (int i = 0; i < ND; ++i) xc[i] = xn[i];
    }
    inertia += (double)ich;
    if (ch + 1 < nchunks) {
      stage.put(xs + (buf ^ 1) * 64 * RS, tid);
      live = live_next;
    }
  }
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int j = q * 256 + w * 64 + lane;
    if (j < k) {
#pragma unroll
      for (int i = 0; i < DPL; ++i)
        if (i < d) cent[(size_t)j * d + i] = c[q][i];
      cnt[j] = n[q];
    }
  }
  if (tid == 0 && cum) {
    cum[0] += inertia;
    cum[1] += fitted;
  }
}

// Any size (past the LDS budget of the forms above): the centroids stay in HBM (L2-resident
// when they fit its 4 MiB), one workgroup of 1024 threads. Per point: the point's
// coordinates are staged in LDS, thread t scans centroids t, t + 1024, … keeping its lowest
// (distance, index), the block minimum goes through LDS (ties: lowest index), then every
// thread moves a slice of the winner's coordinates — the same per-point order and update
// as the CPU oracle, at any (k, d). Counts stay in LDS up to 32768 centroids, else in HBM.
constexpr int kBigNT = 1024;
constexpr int kBigDMax = 8192;  // staged coordinates per point (32 KiB)

__global__ __launch_bounds__(kBigNT) void kmeans_seq_big_kernel(
    const float* __restrict__ x, int ldx, const float* __restrict__ y, int B, int d, int k,
    float* __restrict__ cent, float* __restrict__ cnt, double* __restrict__ cum) {
  __shared__ float xp[kBigDMax];
  __shared__ unsigned rk[kBigNT / 64], rj[kBigNT / 64];
  __shared__ int s_seed, s_win;
  __shared__ float s_r;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_seed = 0;
  __syncthreads();
  for (int j = tid; j < k; j += kBigNT)
    if (cnt[j] > 0.f) atomicMax(&s_seed, j + 1);  // seeded centroids form a prefix
  __syncthreads();
  int seeded = s_seed;
  double inertia = 0.0, fitted = 0.0;
  for (int p = 0; p < B; ++p) {
    const float yp = y ? y[p] : 0.f;
    if (yp != yp) continue;  // not a training point (uniform)
    fitted += 1.0;
    for (int i = tid; i < d; i += kBigNT) xp[i] = x[(size_t)p * ldx + i];
    __syncthreads();
    if (seeded < k) {
      for (int i = tid; i < d; i += kBigNT) cent[(size_t)seeded * d + i] = xp[i];
      if (tid == 0) cnt[seeded] = 1.f;
      ++seeded;
      __syncthreads();
      continue;
    }
    unsigned best = 0xffffffffu, bj = 0xffffffffu;
    for (int j = tid; j < k; j += kBigNT) {
      const float* cr = cent + (size_t)j * d;
      float a0 = 0.f, a1 = 0.f;
      int i = 0;
      for (; i + 1 < d; i += 2) {
        const float t0 = xp[i] - cr[i], t1 = xp[i + 1] - cr[i + 1];
        a0 = fmaf(t0, t0, a0);
        a1 = fmaf(t1, t1, a1);
      }
      if (i < d) {
        const float t0 = xp[i] - cr[i];
        a0 = fmaf(t0, t0, a0);
      }
      const unsigned key = __builtin_bit_cast(unsigned, a0 + a1);
      if (key < best) best = key, bj = (unsigned)j;  // j ascends: ties keep the lowest
    }
    const unsigned wmin = (unsigned)__builtin_amdgcn_readlane((int)wave_umin_groups<1>(best), 63);
    unsigned wj = best == wmin ? bj : 0xffffffffu;
    for (int o = 32; o >= 1; o >>= 1) wj = __builtin_elementwise_min(wj, (unsigned)__shfl_xor((int)wj, o));
    if (lane == 0) rk[wave] = wmin, rj[wave] = wj;
    __syncthreads();
    if (tid == 0) {
      unsigned bk = rk[0], bjj = rj[0];
      for (int w = 1; w < kBigNT / 64; ++w)
        if (rk[w] < bk || (rk[w] == bk && rj[w] < bjj)) bk = rk[w], bjj = rj[w];
      inertia += (double)__builtin_bit_cast(float, bk);
      const float nn = cnt[bjj] + 1.f;
      cnt[bjj] = nn;
      s_win = (int)bjj;
      s_r = 1.f / nn;
    }
    __syncthreads();
    const int wj2 = s_win;
    const float r = s_r;
    float* cw = cent + (size_t)wj2 * d;
    for (int i = tid; i < d; i += kBigNT) cw[i] = fmaf(r, xp[i] - cw[i], cw[i]);
    __syncthreads();  // (workgroup scope: the moved centroid is read back on this CU only)
  }
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

static int pow2_at_least(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// The fast forms' geometry for (d, k): one wave with G lanes per centroid (k ≤ 64), or
// four waves with CPL centroids per lane (k ≤ 1024); DPL stored / ND computed coordinates
// per lane. False when (d, k) is outside both.
static bool kmeans_fast_geometry(int d, int k, int& G, int& DPL, int& CPL, int& ND) {
  if (d < 1 || d > 64 || k < 1) return false;
  if (k <= 64) {
    const int gmax = 64 / pow2_at_least(k);
    G = std::min(gmax, pow2_at_least((d + 3) / 4));
    DPL = std::max(4, pow2_at_least((d + G - 1) / G));
    CPL = 0;  // (the one-wave form)
  } else {
    G = 1;
    DPL = std::max(4, pow2_at_least(d));
    CPL = (k + 255) / 256;
    if (CPL == 3) CPL = 4;
    if (CPL > 4 || CPL * DPL > 128) return false;
  }
  // (G > 1: the first part holds min(DPL, d) coordinates, so all DPL are computed)
  ND = (G == 1 && DPL >= 8 && d <= DPL - 2) ? DPL - 2 : DPL;
  return G * DPL <= 64;
}

template <int G, int DPL, int ND>
static bool launch_one(int g, int dpl, int cpl, int nd, hipStream_t st, const float* x, int ldx,
                       const float* y, int B, int d, int k, float* cent, float* cnt, double* cum) {
  if (cpl != 0 || g != G || dpl != DPL || nd != ND) return false;
  hipLaunchKernelGGL((kmeans_fast_kernel<G, DPL, ND>), dim3(1), dim3(64), 0, st, x, ldx, y, B, d,
                     k, cent, cnt, cum);
  return true;
}

template <int CPL, int DPL, int ND>
static bool launch_mw(int cpl, int dpl, int nd, hipStream_t st, const float* x, int ldx,
                      const float* y, int B, int d, int k, float* cent, float* cnt, double* cum) {
  if (cpl != CPL || dpl != DPL || nd != ND) return false;
  hipLaunchKernelGGL((kmeans_mw_kernel<CPL, DPL, ND>), dim3(1), dim3(256), 0, st, x, ldx, y, B,
                     d, k, cent, cnt, cum);
  return true;
}

static bool kmeans_fast(hipStream_t st, const float* x, int ldx, const float* y, int B, int d,
                        int k, float* cent, float* cnt, double* cum) {
  int g, dpl, cpl, nd;
  if (!kmeans_fast_geometry(d, k, g, dpl, cpl, nd)) return false;
#define K1(G, DPL, ND) launch_one<G, DPL, ND>(g, dpl, cpl, nd, st, x, ldx, y, B, d, k, cent, cnt, cum)
#define KM(CPL, DPL, ND) launch_mw<CPL, DPL, ND>(cpl, dpl, nd, st, x, ldx, y, B, d, k, cent, cnt, cum)
  return K1(16, 4, 4) || K1(8, 4, 4) || K1(8, 8, 8) || K1(4, 4, 4) || K1(4, 8, 8) ||
         K1(4, 16, 16) || K1(2, 4, 4) || K1(2, 8, 8) || K1(2, 16, 16) || K1(2, 32, 32) ||
         K1(1, 4, 4) || K1(1, 8, 8) || K1(1, 8, 6) || K1(1, 16, 16) ||
         K1(1, 16, 14) || K1(1, 32, 32) || K1(1, 32, 30) || K1(1, 64, 64) || K1(1, 64, 62) ||
         KM(1, 4, 4) || KM(1, 8, 8) || KM(1, 8, 6) || KM(1, 16, 16) || KM(1, 16, 14) ||
         KM(1, 32, 32) || KM(1, 32, 30) || KM(1, 64, 64) || KM(1, 64, 62) || KM(2, 4, 4) ||
         KM(2, 8, 8) || KM(2, 8, 6) || KM(2, 16, 16) || KM(2, 16, 14) || KM(2, 32, 32) ||
         KM(2, 32, 30) || KM(2, 64, 64) || KM(2, 64, 62) || KM(4, 4, 4) || KM(4, 8, 8) ||
         KM(4, 8, 6) || KM(4, 16, 16) || KM(4, 16, 14) || KM(4, 32, 32) || KM(4, 32, 30);
#undef K1
#undef KM
}

static int g_kmeans_form = -1;  // -1 unset; 0 the earlier forms; 1 the fast one-wave form

// 1: the fast one-wave form wherever its geometry holds (default); 0: the earlier one-wave
// / workgroup forms (the A/B of the fast form). Returns the form in use.
OMLDM_API int omldm_kmeans_seq_form(int form) {
  if (form >= 0) g_kmeans_form = form ? 1 : 0;
  if (g_kmeans_form < 0) {
    const char* e = getenv("OMLDM_KMEANS_FAST");
    g_kmeans_form = (e && e[0] == '0') ? 0 : 1;
  }
  return g_kmeans_form;
}

static bool kmeans_wg_fits(int d, int k) {
  const int nw = (k + 63) / 64;
  return d >= 1 && d <= 256 && k >= 1 && k <= 1024 &&
         kmeans_wg_lds(d, k, nw <= 4 ? 4 : 16) <= 160 * 1024;
}

// Every (d, k) with d ≤ 8192 runs exactly: the register / LDS forms where they fit, the
// HBM-resident form past them.
OMLDM_API int omldm_kmeans_seq_fits(int d, int k) {
  return d >= 1 && k >= 1 && d <= kBigDMax;
}

// x [B, ldx] fp32 (first d columns used), y [B] (NaN: not a training point; nullptr: all
// train), cent [k, d], cnt [k], cum (cum[0] += Σ squared distance to the chosen
// centroid, cum[1] += points fitted) — all device pointers; one wave, one launch.
OMLDM_API int omldm_kmeans_seq(const float* x, int ldx, const float* y, int B, int d, int k,
                               float* cent, float* cnt, double* cum, void* stream) {
  if (!omldm_kmeans_seq_fits(d, k) || ldx < d) return -1;
  if (B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (omldm_kmeans_seq_form(-1) && kmeans_fast(st, x, ldx, y, B, d, k, cent, cnt, cum))
    return (int)hipGetLastError();
  if (!kmeans_one_wave(d, k) && !kmeans_wg_fits(d, k)) {  // past the LDS: centroids in HBM
    hipLaunchKernelGGL(kmeans_seq_big_kernel, dim3(1), dim3(kBigNT), 0, st, x, ldx, y, B, d, k,
                       cent, cnt, cum);
    return (int)hipGetLastError();
  }
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
