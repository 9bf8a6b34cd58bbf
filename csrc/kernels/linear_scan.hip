// Exact sequential online linear learners, v2: the chunk Grams are built by the WHOLE GPU,
// the per-spoke sequential part runs on one workgroup per spoke with no global-memory
// latency and no device-wide fence on its path.
//
// Reference semantics as in linear_seq.hip: P spokes, spoke s fits rows [s·R, (s+1)·R) of
// the round strictly one example at a time on its own model replica
// (omldm/operators/spoke/FlinkSpoke.scala:92-107), the Synchronous PS averages the
// replicas. For additive learners the margin of row t of chunk k is
//     m_t = x_t·w_start(k) + Σ_{s<t in k} c_s G_k[t][s],   G_k = X_k X_kᵀ,
// with w_start(k) = the replica after chunks < k. Three passes per round:
//
//  1. hash:  every raw 32-bit category token → field-aware signed slot (hash_raw_kernel).
//  2. prep:  one workgroup per (spoke, chunk) over all CUs: G_k (strictly lower: the scan
//     then leaves every lane's margin frozen after its own step), the cross Grams
//     X1_k = X_k X_{k−1}ᵀ and X2_k = X_k X_{k−2}ᵀ, and ‖x‖². Categorical products are
//     exact integer counts of equal field slots (signed), dense products fp32 FMAs.
//  3. scan:  one workgroup per spoke, 8 waves, chunks of 64 rows, one barrier per chunk:
//       * wave 0 (the scanner) runs the recurrence of chunk k: per step one closed-form
//         candidate per lane, a v_readlane of lane t's, one FMA with G_k — and one more FMA
//         with X1_{k+1} that folds c_k into chunk k+1's margins on the fly (off the
//         dependency chain);
//       * waves 1-7 (helpers) own disjoint FIELDS (field-aware slots are disjoint ranges)
//         and disjoint dense columns, so every global access of the replica a helper makes
//         depends on its own earlier accesses only: it waits for its own atomics
//         (s_waitcnt), never for a fence or another wave. In chunk k's iteration a helper
//         gathers chunk k+1's round-start margins from the replica (which then holds
//         chunks ≤ k−2), adds X2_{k+1}·c_{k−1} and its dense columns' x·w, scatters chunk
//         k−1's update (fp32 L2 atomics) and updates its dense weights, and stages G_{k+1}
//         and X1_{k+2} into LDS.
// Replicas [S][dim] fp32 in HBM; round end as in linear_seq.hip (linear_seq_reduce).
#include "common.h"
#include "hash_dev.h"
#include "seq_common.h"

namespace omldm {

namespace scan {
constexpr int CH = 64;                     // rows per chunk = scanner lanes
constexpr int NH = 7;                      // helper waves
constexpr int NT = 64 * (NH + 1);
constexpr int GS = CH + 4;                 // LDS row stride of G / X1 (16-B aligned, b128 reads spread)
constexpr int MAXF = 32;                   // categorical fields per row
constexpr int NF = (MAXF + NH - 1) / NH;   // fields per helper lane
constexpr int KNMAX = 32;
constexpr int NJ = (KNMAX + NH - 1) / NH;  // dense columns per helper lane
constexpr int GXB = (CH + NH - 1) / NH;    // X2 columns per helper wave
constexpr int MAT = CH * CH;
constexpr int PREP = 3 * MAT + CH;         // G | X1 | X2 | ‖x‖² per chunk (floats)
constexpr int NV4 = (2 * MAT / 4 + 64 * NH - 1) / (64 * NH);  // float4 of G+X1 per helper lane
constexpr int WS = 8;
constexpr int ABSENT_A = 0x7ffffffe;       // never equal to a slot (slots < 2^31 − 2)
}  // namespace scan

// ------------------------------------------------------------------------ pass 2: prep
// grid (chunks per spoke, S); 256 threads; thread (bi, bj) computes the 4×4 block of rows
// 4bi.. of chunk c against rows 4bj.. of chunk c − d, for d = 0 (G), 1 (X1), 2 (X2).
template <int KN>
__global__ __launch_bounds__(256) void scan_prep_kernel(const int* __restrict__ slots, int dc,
                                                        const float* __restrict__ num, int dn,
                                                        int B, int R, int bias,
                                                        float* __restrict__ prep, int nchs) {
  const int c = blockIdx.x, s = blockIdx.y;
  const long long t0ll = (long long)s * R;
  const int t0 = t0ll > B ? B : (int)t0ll;
  const int t1 = (t0ll + R) > B ? B : (int)(t0ll + R);
  if (t0 + c * scan::CH >= t1) return;  // chunk past the spoke's shard
  float* out = prep + ((size_t)s * nchs + c) * scan::PREP;
  // row stride 68: the field-fastest fill (coalesced global reads) hits 16 banks, not 1
  __shared__ alignas(16) int sl[3][scan::MAXF][scan::CH + 4];
  __shared__ float xn[3][scan::CH][KN + 1];
  const int tid = threadIdx.x;
  for (int i = tid; i < 3 * dc * scan::CH; i += 256) {
    const int d = i / (dc * scan::CH), rem = i - d * dc * scan::CH;
    const int r = rem / dc, f = rem - r * dc;  // consecutive threads: consecutive fields of a row
    const int cc = c - d, row = t0 + cc * scan::CH + r;
    sl[d][f][r] = (cc >= 0 && row < t1) ? slots[(size_t)row * dc + f] : -1;
  }
  for (int i = tid; i < 3 * scan::CH * KN; i += 256) {
    const int d = i / (scan::CH * KN), rem = i - d * scan::CH * KN;
    const int r = rem / KN, j = rem - r * KN;
    const int cc = c - d, row = t0 + cc * scan::CH + r;
    float x = 0.f;
    if (cc >= 0 && row < t1) x = j < dn ? num[(size_t)row * dn + j] : ((bias && j == dn) ? 1.f : 0.f);
    xn[d][r][j] = x;
  }
  __syncthreads();
  if (tid < scan::CH) {  // ‖x‖² over the feature list (dense values, ±1 categorical)
    float n2 = 0.f;
    for (int j = 0; j < KN; ++j) n2 = fmaf(xn[0][tid][j], xn[0][tid][j], n2);
    for (int f = 0; f < dc; ++f) n2 += sl[0][f][tid] != -1 ? 1.f : 0.f;
    out[3 * scan::MAT + tid] = n2;
  }
  const int bi = tid >> 4, bj = tid & 15;
#pragma unroll 1
  for (int d = 0; d < 3; ++d) {
    float acc[4][4] = {};
    // G keeps its strictly lower triangle only: blocks right of the diagonal stay 0
    if (c - d >= 0 && !(d == 0 && bj > bi)) {
      int cnt[4][4] = {};
      for (int f = 0; f < dc; ++f) {
        const int4 a4 = *reinterpret_cast<const int4*>(&sl[0][f][4 * bi]);
        const int4 b4 = *reinterpret_cast<const int4*>(&sl[d][f][4 * bj]);
        const int av[4] = {a4.x, a4.y, a4.z, a4.w}, bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int a = av[i] == -1 ? scan::ABSENT_A : av[i];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int x = a ^ bv[j];
            cnt[i][j] += (x & 0x7fffffff) ? 0 : (x < 0 ? -1 : 1);  // same slot: ±1 (signs)
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (float)cnt[i][j];
      for (int q = 0; q < KN; ++q) {
        float xa[4], xb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          xa[i] = xn[0][4 * bi + i][q];
          xb[i] = xn[d][4 * bj + i][q];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(xa[i], xb[j], acc[i][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 4 * bi + i;
      float4 v = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
      if (d == 0) {  // G strictly lower: column s ≥ row t → 0
        if (4 * bj + 0 >= t) v.x = 0.f;
        if (4 * bj + 1 >= t) v.y = 0.f;
        if (4 * bj + 2 >= t) v.z = 0.f;
        if (4 * bj + 3 >= t) v.w = 0.f;
      }
      *reinterpret_cast<float4*>(&out[d * scan::MAT + t * scan::CH + 4 * bj]) = v;
    }
  }
}

// ------------------------------------------------------------------------ pass 3: scan
// The update c(m) of one lane's row with its per-row constants folded in ahead of the
// chunk, so the recurrence's dependency chain per step is fma → med3 → v_readlane → fma.
template <int RULE>
struct ScanCand {
  float a, b, lo, hi, b2;
  float y, inv;
  __device__ __forceinline__ void prepare(float y_, float inv_, const SeqParams& p) {
    y = y_;
    inv = inv_;
    a = -inv_;
    if constexpr (RULE == kSeqHinge) {
      // y·min(C, max(0, 1 − y·m)·inv) = clamp(inv·(y − m)·|y|…): y = +1 → [0, C] of
      // inv − inv·m; y = −1 → [−C, 0] of −inv − inv·m; y = 0 (padding row) → 0
      b = y_ * inv_;
      lo = y_ < 0.f ? -p.cclip : 0.f;
      hi = y_ < 0.f ? 0.f : p.cclip;
    } else if constexpr (RULE == kSeqEps) {
      // sign(e)·min(C, max(0, |e| − ε)·inv), e = y − m: one of two one-sided clamps
      b = (y_ - p.eps) * inv_;
      b2 = (y_ + p.eps) * inv_;
      lo = -p.cclip;
      hi = p.cclip;
    }
  }
  __device__ __forceinline__ float operator()(float m, const SeqParams& p) const {
    if constexpr (RULE == kSeqHinge) {
      return __builtin_amdgcn_fmed3f(fmaf(a, m, b), lo, hi);
    } else if constexpr (RULE == kSeqEps) {
      return __builtin_amdgcn_fmed3f(fmaf(a, m, b), 0.f, hi) +
             __builtin_amdgcn_fmed3f(fmaf(a, m, b2), lo, 0.f);
    } else {
      return seq_candidate<RULE>(m, y, inv, p);
    }
  }
};

struct ScanSmem {
  alignas(16) float G[2][scan::CH][scan::GS];    // G_k, by chunk parity
  alignas(16) float X1[2][scan::CH][scan::GS];   // X1_{k+1} (read by the scanner in chunk k)
  alignas(16) float X2[2][scan::CH][scan::GS];   // X2_{k+2} (read by the scanner in chunk k)
  float part[2][scan::NH][scan::CH];             // base-margin partials per helper wave
  float cb[2][scan::CH];                         // c of the chunk, by parity
};
// + dynamic LDS: a ring of 4 chunks' raw inputs as loaded (coalesced), row-major:
//   int slots[64][dc] | float num[64][dn]

// The replica is private to one workgroup (one CU): workgroup-scope atomics keep every
// wave's gathers coherent with its own scatters without the device-scope (sc1) path that
// bypasses the XCD's L2.
__device__ __forceinline__ float ld_rep(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void add_rep(float* p, float v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Diagnostics (omldm_linear_scan_stamps): per-phase s_memtime cycles into
// g_scan_stamps[spoke][16]: 0 scanner scan, 1 scanner barrier wait; helper wave 1:
// 2 top wait, 3 issue, 4 margins (incl. gather wait), 5 LDS staging, 6 scatter, 7 barrier;
// 8 iterations.
__device__ unsigned long long* g_scan_stamps;

constexpr int kStageF4 = (3 * scan::MAT / 4 + 64 * scan::NH - 1) / (64 * scan::NH);  // 7
constexpr int kRawMaxDw = 50 * scan::CH;   // (dc + dn) ≤ 50: raw dwords of one chunk
constexpr int kRawLd = (kRawMaxDw + 64 * scan::NH - 1) / (64 * scan::NH);           // 8

template <int RULE, int KN>
__global__ __launch_bounds__(scan::NT, 1) void scan_round_kernel(
    const int* __restrict__ slots, int dc, const float* __restrict__ num, int dn,
    const void* __restrict__ yv, int B, int R, const float* __restrict__ prep, int nchs,
    float* __restrict__ rep, int dim, float* __restrict__ ws, SeqParams p) {
  __shared__ ScanSmem sm;
  extern __shared__ int ring[];  // [4][(dc + dn) · 64]
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int s = blockIdx.x;
  float* W = rep + (size_t)s * dim;
  const long long t0ll = (long long)s * R;
  const int t0 = t0ll > B ? B : (int)t0ll;
  const int t1 = (t0ll + R) > B ? B : (int)(t0ll + R);
  float* wrow = ws + (size_t)s * scan::WS;
  if (t0 >= t1) {
    if (tid < scan::WS) wrow[tid] = 0.f;
    return;
  }
  const int nch = (t1 - t0 + scan::CH - 1) / scan::CH;
  const float* P0 = prep + (size_t)s * nchs * scan::PREP;
  auto chunk_prep = [&](int k) { return P0 + (size_t)k * scan::PREP; };
  const int rdw = (dc + dn) * scan::CH;  // dwords of one ring slot
  auto ring_sl = [&](int k) { return ring + (k & 3) * rdw; };
  auto ring_x = [&](int k) { return reinterpret_cast<const float*>(ring + (k & 3) * rdw + dc * scan::CH); };

  unsigned long long* stamps = g_scan_stamps;
  unsigned long long st_acc[9] = {};
  unsigned long long st_t = stamps ? clock64() : 0;
  auto stamp = [&](int k) {
    if (stamps) {
      const unsigned long long now = clock64();
      st_acc[k] += now - st_t;
      st_t = now;
    }
  };
  auto flush_stamps = [&]() {
    if (stamps && lane == 0 && wave <= 1)
      for (int k = 0; k < 9; ++k)
        if ((wave == 0) == (k < 2)) atomicAdd(&stamps[(size_t)s * 16 + k], st_acc[k]);
  };

  if (wave == 0) {
    // ------------------------------------------------------------------ scanner
    // the recurrence is the round's critical path: it wins VALU issue arbitration over
    // the helper wave sharing its SIMD
    __builtin_amdgcn_s_setprio(3);
    float loss = 0.f, nex = 0.f, mist = 0.f, sqe = 0.f;
    float f1 = 0.f;   // c_{k−1}·X1_k for this lane's row of chunk k
    float f2 = 0.f;   // c_{k−2}·X2_k
    float f2n = 0.f;  // c_{k−1}·X2_{k+1}
    float ynx = load_y(yv, min(t0 + lane, t1 - 1), p.y8);
    float n2nx = chunk_prep(0)[3 * scan::MAT + lane];
    for (int k = -2; k <= nch; ++k) {
      if (k >= 0 && k < nch) {
        const int b = k & 1;
        const int row = t0 + k * scan::CH + lane;
        const bool valid = row < t1 && ynx == ynx;  // a NaN target: not fitted
        const float y = valid ? ynx : 0.f;
        const float n2 = valid ? n2nx : 0.f;
        if (k + 1 < nch) {
          ynx = load_y(yv, min(row + scan::CH, t1 - 1), p.y8);
          n2nx = chunk_prep(k + 1)[3 * scan::MAT + lane];
        }
        float m = f1 + f2;
#pragma unroll
        for (int q = 0; q < scan::NH; ++q) m += sm.part[b][q][lane];
        const float inv = n2 > 0.f ? __builtin_amdgcn_rcpf(n2 + p.kadd) : 0.f;
        ScanCand<RULE> cf;
        cf.prepare(y, inv, p);
        const float* grow = &sm.G[b][lane][0];
        const float* x1row = &sm.X1[b ^ 1][lane][0];
        const float* x2row = &sm.X2[b][lane][0];
        float n1 = 0.f, n2f = 0.f;
#pragma unroll
        for (int t4 = 0; t4 < scan::CH; t4 += 4) {
          const float4 g4 = *reinterpret_cast<const float4*>(grow + t4);
          const float4 a4 = *reinterpret_cast<const float4*>(x1row + t4);
          const float4 c4 = *reinterpret_cast<const float4*>(x2row + t4);
          const float gg[4] = {g4.x, g4.y, g4.z, g4.w};
          const float aa[4] = {a4.x, a4.y, a4.z, a4.w};
          const float cc[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float ct = readlane_f(cf(m, p), t4 + u);
            m = fmaf(ct, gg[u], m);   // G strictly lower: lane t frozen after step t
            n1 = fmaf(ct, aa[u], n1);  // → chunk k+1 (off the dependency chain)
            n2f = fmaf(ct, cc[u], n2f);  // → chunk k+2
          }
        }
        const float c = cf(m, p);
        sm.cb[b][lane] = c;
        if (valid) {
          seq_stats<RULE>(m, y, p, loss, mist, sqe);
          nex += 1.f;
        }
        f1 = n1;
        f2 = f2n;
        f2n = n2f;
      }
      stamp(0);
      __syncthreads();
      stamp(1);
    }
    flush_stamps();
    loss = wave_sum(loss);
    nex = wave_sum(nex);
    mist = wave_sum(mist);
    sqe = wave_sum(sqe);
    if (lane == 0) {
      wrow[0] = loss;
      wrow[1] = nex;
      wrow[2] = mist;
      wrow[3] = sqe;
      wrow[4] = 1.f;
      wrow[5] = 0.f;
      wrow[6] = 0.f;
      wrow[7] = 0.f;
    }
    return;
  }

  // ------------------------------------------------------------------- helpers
  // wave q owns categorical fields f ≡ q and dense columns j ≡ q (mod NH); lane r = row.
  const int q = wave - 1, r = lane;
  const int hl = tid - 64;  // 0 .. 64·NH − 1
  float wn[scan::NJ];       // this wave's dense weights (wave-uniform)
#pragma unroll
  for (int i = 0; i < scan::NJ; ++i) {
    const int j = q + scan::NH * i;
    wn[i] = (j < KN) ? (j < dn ? W[j] : ((p.bias && j == dn) ? W[dim - 1] : 0.f)) : 0.f;
  }
  const int slot_dw = dc * scan::CH;
  // this lane's dwords of a chunk's raw image (slots then num): d = hl + 64·NH·u, the
  // same in every chunk, so the (row, column) split is done once (integer division is
  // ~40 VALU instructions)
  int rrow[kRawLd], rcol[kRawLd];
#pragma unroll
  for (int u = 0; u < kRawLd; ++u) {
    const int d = min(hl + 64 * scan::NH * u, rdw - 1);
    if (d < slot_dw) {
      rrow[u] = d / dc;
      rcol[u] = d - rrow[u] * dc;
    } else {
      const int e = d - slot_dw, dd = max(dn, 1);
      rrow[u] = e / dd;
      rcol[u] = -1 - (e - rrow[u] * dd);  // < 0: a numerical column
    }
  }
  // raw inputs of chunk kc: the lane's dword u, clamped source
  auto raw_src = [&](int kc, int u) -> const int* {
    const int row = min(t0 + min(kc, nch - 1) * scan::CH + rrow[u], t1 - 1);
    return rcol[u] >= 0 ? slots + (size_t)row * dc + rcol[u]
                        : reinterpret_cast<const int*>(num) + (size_t)row * dn + (-1 - rcol[u]);
  };
  // its row validity (rows past the shard: absent slots, zero features)
  auto raw_fix = [&](int kc, int u, int v) -> int {
    if (t0 + kc * scan::CH + rrow[u] < t1) return v;
    return rcol[u] >= 0 ? -1 : 0;
  };
  int rv[kRawLd];

  auto iteration = [&](int k) __attribute__((always_inline)) {
    const int cn = k + 1;  // the chunk whose round-start margins this iteration builds
    if (wave == 1) stamp(7);
    // own atomics of the previous iteration (chunk k − 2) have landed in L2
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (wave == 1) stamp(2);
    // ---- gather chunk cn's categorical weights (the replica holds chunks ≤ k − 2)
    const int* csl = ring_sl(cn);
    float g[scan::NF];
    int code[scan::NF];
#pragma unroll
    for (int i = 0; i < scan::NF; ++i) {
      const int f = q + scan::NH * i;
      code[i] = (cn >= 0 && cn < nch && f < dc) ? csl[r * dc + f] : -1;
      g[i] = ld_rep(&W[code[i] != -1 ? (code[i] & 0x7fffffff) : 0]);
    }
    // ---- stage G_{cn}, X1_{cn+1}, X2_{cn+2} (float4 registers; LDS at the end)
    auto stage_src = [&](int u) {
      const int i = min(hl + 64 * scan::NH * u, 3 * scan::MAT / 4 - 1);
      const int mtx = i >> 10, e = i & 1023;
      const int kc = max(0, min(cn + mtx, nch - 1));  // cn = −1 in the first iteration
      return reinterpret_cast<const float4*>(chunk_prep(kc) + mtx * scan::MAT) + e;
    };
    const float4 v0 = *stage_src(0), v1 = *stage_src(1), v2 = *stage_src(2), v3 = *stage_src(3),
                 v4 = *stage_src(4), v5 = *stage_src(5), v6 = *stage_src(6);
    // ---- raw inputs of chunk cn + 1 (coalesced dwords; LDS ring at the end)
    const int kr = cn + 1;
#pragma unroll
    for (int u = 0; u < kRawLd; ++u) rv[u] = *raw_src(kr, u);
    if (wave == 1) stamp(3);
    if (cn >= 0 && cn < nch) {
      // ---- dense part of chunk cn's margins (w_dense after chunks ≤ k − 2)
      const float* cx = ring_x(cn);
      float base = 0.f;
#pragma unroll
      for (int i = 0; i < scan::NJ; ++i) {
        const int j = q + scan::NH * i;
        if (j < KN) {
          const float x = j < dn ? cx[r * dn + j] : ((p.bias && j == dn) ? 1.f : 0.f);
          base = fmaf(x, wn[i], base);
        }
      }
      // ---- gathered weights (in flight since the top of the iteration)
#pragma unroll
      for (int i = 0; i < scan::NF; ++i) base += code[i] == -1 ? 0.f : (code[i] < 0 ? -g[i] : g[i]);
      sm.part[cn & 1][q][r] = base;
    }
    if (wave == 1) stamp(4);
    // ---- G_cn → G[cn & 1], X1_{cn+1} → X1[(cn+1) & 1], X2_{cn+2} → X2[cn & 1]
    auto stage_put = [&](int u, const float4& v) {
      const int i = hl + 64 * scan::NH * u;
      const int mtx = i >> 10, e = i & 1023;
      if (i < 3 * scan::MAT / 4 && cn >= 0 && cn + mtx < nch) {
        const int row = e >> 4, col = (e & 15) * 4;
        float* dst = mtx == 0 ? &sm.G[cn & 1][row][col]
                   : mtx == 1 ? &sm.X1[(cn + 1) & 1][row][col] : &sm.X2[cn & 1][row][col];
        *reinterpret_cast<float4*>(dst) = v;
      }
    };
    stage_put(0, v0);
    stage_put(1, v1);
    stage_put(2, v2);
    stage_put(3, v3);
    stage_put(4, v4);
    stage_put(5, v5);
    stage_put(6, v6);
    if (wave == 1) stamp(5);
    // ---- scatter chunk k − 1 (c known since the last barrier) and its dense update
    const int ks = k - 1;
    if (ks >= 0 && ks < nch) {
      const int* ssl = ring_sl(ks);
      const float* sx = ring_x(ks);
      const float cv = sm.cb[ks & 1][r];
#pragma unroll
      for (int i = 0; i < scan::NF; ++i) {
        const int f = q + scan::NH * i;
        if (f < dc) {
          const int cd = ssl[r * dc + f];
          if (cd != -1 && cv != 0.f) add_rep(&W[cd & 0x7fffffff], cd < 0 ? -cv : cv);
        }
      }
#pragma unroll
      for (int i = 0; i < scan::NJ; ++i) {
        const int j = q + scan::NH * i;
        if (j < KN) {
          const float x = j < dn ? sx[r * dn + j] : ((p.bias && j == dn) ? 1.f : 0.f);
          wn[i] += wave_sum(cv * x);
        }
      }
    }
    // ---- raw inputs of chunk cn + 1 → ring (its slot held chunk k − 2, scattered last
    // iteration; the ring holds chunks k − 1 … k + 2)
    if (kr < nch) {
      int* dst = ring_sl(kr);
#pragma unroll
      for (int u = 0; u < kRawLd; ++u) {
        const int d = hl + 64 * scan::NH * u;
        if (d < rdw) dst[d] = raw_fix(kr, u, rv[u]);
      }
    }
    if (wave == 1) {
      stamp(6);
      st_acc[8] += 1;
    }
    __syncthreads();
  };

  for (int k = -2; k <= nch; ++k) iteration(k);
  if (wave == 1) stamp(7);
  flush_stamps();
  // round end: this wave's dense weights back into the replica
#pragma unroll
  for (int i = 0; i < scan::NJ; ++i) {
    const int j = q + scan::NH * i;
    if (lane == 0 && j < KN) {
      if (j < dn) W[j] = wn[i];
      else if (p.bias && j == dn) W[dim - 1] = wn[i];
    }
  }
}

// dynamic LDS of the scan: the 4-chunk ring of raw inputs (slots [64][dc] | num [64][dn])
static size_t scan_dyn_lds(int dc, int dn) {
  return (size_t)4 * (dc + dn) * scan::CH * sizeof(int);
}

template <int RULE, int KN>
static int launch_scan(const int* slots, int dc, const float* num, int dn, const void* y, int B,
                       int R, int S, const float* prep, int nchs, float* rep, int dim, float* ws,
                       const SeqParams& p, hipStream_t st) {
  const size_t ring_bytes = scan_dyn_lds(dc, dn);
  static bool attr_set = false;  // the ring is dynamic LDS on top of ~106 KiB static
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&scan_round_kernel<RULE, KN>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - (int)sizeof(ScanSmem));
    attr_set = true;
  }
  hipLaunchKernelGGL((scan_round_kernel<RULE, KN>), dim3(S), dim3(scan::NT), ring_bytes, st, slots,
                     dc, num, dn, y, B, R, prep, nchs, rep, dim, ws, p);
  return (int)hipGetLastError();
}

template <int KN>
static int dispatch_scan(int rule, const int* slots, int dc, const float* num, int dn,
                         const void* y, int B, int R, int S, const float* prep, int nchs,
                         float* rep, int dim, float* ws, const SeqParams& p, hipStream_t st) {
  if (rule == kSeqHinge)
    return launch_scan<kSeqHinge, KN>(slots, dc, num, dn, y, B, R, S, prep, nchs, rep, dim, ws, p, st);
  if (rule == kSeqEps)
    return launch_scan<kSeqEps, KN>(slots, dc, num, dn, y, B, R, S, prep, nchs, rep, dim, ws, p, st);
  return launch_scan<kSeqLogistic, KN>(slots, dc, num, dn, y, B, R, S, prep, nchs, rep, dim, ws, p, st);
}

}  // namespace omldm

using namespace omldm;

OMLDM_API int omldm_hash_raw(const void* tok, long long B, int dc, int dn, long long dim, int* out,
                             void* stream);
OMLDM_API int omldm_linear_seq_reduce(const float* rep, const float* w, int S_act, int dim,
                                      float* dacc, float inv_p, const float* ws, double* cum,
                                      void* stream);

OMLDM_API int omldm_linear_scan_stamps(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_scan_stamps), &buf, sizeof(buf));
}

// 1 when the v2 round supports this (dn, dc) shape (its LDS fits), else 0.
OMLDM_API int omldm_linear_scan_fits(int dn, int dc) {
  return dc > 0 && dc <= scan::MAXF && dc + dn <= 50 &&
         scan_dyn_lds(dc, dn) + sizeof(ScanSmem) <= 160 * 1024;
}

// Floats of prep workspace one round needs (S spokes of R rows).
OMLDM_API long long omldm_linear_scan_prep_floats(int R, int S) {
  const long long nchs = (R + scan::CH - 1) / scan::CH;
  return (long long)S * nchs * scan::PREP;
}

static int scan_check(int dc, int dn, int dim, int bias, int rule, int R) {
  if (R <= 0 || dc > scan::MAXF || dc <= 0 || dn < 0 || dim <= dn + 1) return -2;
  if (rule < 0 || rule > 2) return -5;
  if (dn + (bias ? 1 : 0) > scan::KNMAX) return -2;
  if ((long long)(dim - dn - 1) / dc < 1) return -2;
  // the LDS ring of raw chunk inputs must fit beside the static LDS: else use linear_seq
  if (dc + dn > 50 || scan_dyn_lds(dc, dn) + sizeof(ScanSmem) > 160 * 1024) return -3;
  return 0;
}

// Passes 1-2 (hash, chunk Grams) of a round into (slots_ws, prep_ws) — independent of the
// model, so they may run ahead on another stream while the previous round scans.
OMLDM_API int omldm_linear_scan_prepare(const float* num, int dn, const void* tok, int dc, int B,
                                        int R, int S, int dim, int bias, int* slots_ws,
                                        float* prep_ws, void* stream) {
  if (S <= 0 || B <= 0) return 0;
  int e = scan_check(dc, dn, dim, bias, 0, R);
  if (e) return e;
  hipStream_t st = (hipStream_t)stream;
  e = omldm_hash_raw(tok, B, dc, dn, dim, slots_ws, stream);
  if (e) return e;
  const int nchs = (R + scan::CH - 1) / scan::CH;
  const long long sact = ((long long)B + R - 1) / R;
  const int S_act = sact < S ? (int)sact : S;
  if (dn + (bias ? 1 : 0) <= 16)
    hipLaunchKernelGGL(scan_prep_kernel<16>, dim3(nchs, S_act), dim3(256), 0, st, slots_ws, dc,
                       num, dn, B, R, bias, prep_ws, nchs);
  else
    hipLaunchKernelGGL(scan_prep_kernel<32>, dim3(nchs, S_act), dim3(256), 0, st, slots_ws, dc,
                       num, dn, B, R, bias, prep_ws, nchs);
  return (int)hipGetLastError();
}

// Pass 2 alone, on slots that are already hashed (the engine's field-aware batches:
// HashedBatch.to_wide() int32 signed slots, dn + f·span + local).
OMLDM_API int omldm_linear_scan_prepare_slots(const float* num, int dn, const int* slots, int dc,
                                              int B, int R, int S, int dim, int bias,
                                              float* prep_ws, void* stream) {
  if (S <= 0 || B <= 0) return 0;
  int e = scan_check(dc, dn, dim, bias, 0, R);
  if (e) return e;
  const int nchs = (R + scan::CH - 1) / scan::CH;
  const long long sact = ((long long)B + R - 1) / R;
  const int S_act = sact < S ? (int)sact : S;
  if (dn + (bias ? 1 : 0) <= 16)
    hipLaunchKernelGGL(scan_prep_kernel<16>, dim3(nchs, S_act), dim3(256), 0, (hipStream_t)stream,
                       slots, dc, num, dn, B, R, bias, prep_ws, nchs);
  else
    hipLaunchKernelGGL(scan_prep_kernel<32>, dim3(nchs, S_act), dim3(256), 0, (hipStream_t)stream,
                       slots, dc, num, dn, B, R, bias, prep_ws, nchs);
  return (int)hipGetLastError();
}

// Pass 3 (the scan) + the round end, on a prepared round.
OMLDM_API int omldm_linear_scan_run(const float* w, const float* num, int dn, int dc, const void* y,
                                    int y8, int B, int R, int S, float* rep, float* dacc, int dim,
                                    float* ws, double* cum, int rule, int variant, float C,
                                    float eps, float lr, float inv_p, int bias,
                                    const int* slots_ws, const float* prep_ws, void* stream) {
  if (S <= 0 || B <= 0) return 0;
  int e = scan_check(dc, dn, dim, bias, rule, R);
  if (e) return e;
  hipStream_t st = (hipStream_t)stream;
  const SeqParams p{rule, variant, variant == 1 ? C : INFINITY, variant == 2 ? 0.5f / C : 0.f,
                    eps, lr, inv_p, bias, y8, (uint32_t)((dim - dn - 1) / dc)};
  const int nchs = (R + scan::CH - 1) / scan::CH;
  const long long sact = ((long long)B + R - 1) / R;
  const int S_act = sact < S ? (int)sact : S;
  e = dn + (bias ? 1 : 0) <= 16
          ? dispatch_scan<16>(rule, slots_ws, dc, num, dn, y, B, R, S, prep_ws, nchs, rep, dim, ws, p, st)
          : dispatch_scan<32>(rule, slots_ws, dc, num, dn, y, B, R, S, prep_ws, nchs, rep, dim, ws, p, st);
  if (e) return e;
  return omldm_linear_seq_reduce(rep, w, S_act, dim, dacc, inv_p, ws, cum, stream);
}

// One Synchronous round of S exact sequential spokes on the raw wire (see the file
// comment): prepare + run on one stream. Same contract as omldm_linear_seq_round, plus
// workspaces: slots_ws [B·dc] int32, prep_ws [omldm_linear_scan_prep_floats(R, S)] fp32.
OMLDM_API int omldm_linear_scan_round(const float* w, const float* num, int dn, const void* tok,
                                      int dc, const void* y, int y8, int B, int R, int S,
                                      float* rep, float* dacc, int dim, float* ws, double* cum,
                                      int rule, int variant, float C, float eps, float lr,
                                      float inv_p, int bias, int* slots_ws, float* prep_ws,
                                      void* stream) {
  int e = omldm_linear_scan_prepare(num, dn, tok, dc, B, R, S, dim, bias, slots_ws, prep_ws,
                                    stream);
  if (e) return e;
  return omldm_linear_scan_run(w, num, dn, dc, y, y8, B, R, S, rep, dacc, dim, ws, cum, rule,
                               variant, C, eps, lr, inv_p, bias, slots_ws, prep_ws, stream);
}
