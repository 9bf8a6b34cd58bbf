// Exact sequential online linear learners at GPU speed: the Gram-scan round.
//
// Reference semantics (what every spoke computes): a Flink spoke fits its stream shard
// strictly one example at a time on its own full model replica
// (omldm/operators/spoke/FlinkSpoke.scala:92-107 → BufferingWrapper.receiveTuple →
// MLPipeline.pipePoint → learner.fit); the Synchronous parameter server then averages the
// replicas. The reference runs P = 16 spokes by default
// (omldm/utils/DefaultJobParameters.scala:5). Averaging many more replicas per example
// learns measurably slower per example (bench/accuracy_sweep.py: 16 spokes reach 0.866
// holdout accuracy after 16 M examples, 8192 spokes 0.792), so the headline runs the
// reference's 16 sequential spokes per GPU and makes each of them fast instead.
//
// Blocked-exact sequential scan. For additive learners the model after
// row s of a chunk is w_s = w_0 + Σ_{r<s} c_r x_r, so the margin of row t is
//     m_t = x_t·w_0 + Σ_{s<t} c_s G_st,   G = X Xᵀ (the chunk's Gram matrix),
// and only the scalar recurrence c_t = rule(m_t) is sequential. Per chunk of 64 rows:
//   * producers (waves 1-3) hash the raw 32-bit category tokens (murmur3, hash_dev.h),
//     group equal slots per field in LDS hash tables, and build G on the matrix cores:
//     the dense part [numerical | intercept] with fp32-in/fp32-acc MFMA (exact f32
//     products), the categorical part G_cat[t][s] = Σ_f [slot_tf = slot_sf]·x_tf·x_sf as
//     U·Uᵀ with bf16 MFMA over a ±1 one-hot "shared group" matrix U in LDS —
//     all of it for chunk k+1 while
//   * the scanner (wave 0, lane t = row t) runs the recurrence of chunk k: per step one
//     closed-form candidate per lane, a v_readlane of lane t's, one FMA with row t of G.
//   * then all 4 waves scatter chunk k's update into the spoke's replica (hardware fp32
//     atomics in L2) and gather the round-start margins of chunk k+1.
// One workgroup per spoke, replicas [S][dim] fp32 in HBM (4 MiB each at 2^20 dims).
// Round end: linear_seq_reduce_kernel averages the replicas into the round accumulator
// (the RCCL all-reduce runs on it for N > 1) and linear_seq_apply_kernel folds it into w
// and refreshes every replica.
#include "common.h"
#include "hash_dev.h"

namespace omldm {

namespace seq {
constexpr int CH = 64;     // rows per chunk = scanner lanes
constexpr int NT = 256;    // threads per workgroup
constexpr int MAXF = 32;   // categorical fields per row
constexpr int TB = 128;    // per-field group table entries (≥ 2× the chunk's rows)
constexpr int KU = 256;    // shared-group columns of U handled on the matrix cores
constexpr int UPAD = 8;    // bf16 row padding of U (spreads the 16-B operand reads over banks)
constexpr int GPAD = 4;    // G row stride 68 floats: 16-B aligned rows, ds_read_b128 spread over banks
constexpr int WS = 8;      // per-spoke stat row: loss, n, mistakes, sq_err, 1, 0, 0, 0
}  // namespace seq

enum SeqRule : int { kSeqHinge = 0, kSeqEps = 1, kSeqLogistic = 2 };

struct SeqParams {
  int rule, variant;
  float cclip;  // τ clip: C for PA-I, +inf otherwise
  float kadd;   // τ denominator offset: 1/(2C) for PA-II
  float eps, lr, inv_p;
  int bias, y8;
  uint32_t span;  // dim − dn − 1
};

// v_writelane_b32 (no clang builtin in this toolchain: the LLVM intrinsic by name)
extern "C" __device__ int omldm_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int KN>
struct SeqSmem {
  float xn[2][seq::CH][KN + 1];                   // dense block [numerical | 1 | 0 pad]
  int slots[2][seq::MAXF][seq::CH];               // slot | sign << 31, −1 absent
  alignas(16) float G[2][seq::CH][seq::CH + seq::GPAD];  // Gram of the chunk, lower triangle
  alignas(16) unsigned short U[seq::CH][seq::KU + seq::UPAD];  // bf16 ±1 one-hot of shared groups
  int tkey[seq::MAXF][seq::TB];                   // group tables: slot (−1 empty)
  int tcnt[seq::MAXF][seq::TB];                   // members
  int tcol[seq::MAXF][seq::TB];                   // U column (−1: none yet)
  float part_p[4][seq::CH];                       // round-start margin partials
  float part_n[2][3][seq::CH];                    // ‖x‖² partials
  float cval[seq::CH];                            // the chunk's c_t
  float wn[KN];                                   // dense weights (numerical, intercept)
  int ncols[2];
  int ovf[2];
  int pbar;                                       // producer-wave barrier counter
  int stuck;                                      // a producer barrier timed out
};

// Barrier of the three producer waves only (the scanner wave keeps running): a monotonic
// LDS counter, one increment per wave, spin until all three arrived. The spin is bounded
// (≈ 2^22 sleeps, far beyond any legitimate wait): a broken invariant ends the kernel with
// a wrong result flagged in the spoke's stat row instead of hanging the GPU.
__device__ __forceinline__ bool producer_barrier(int* ctr, int& target) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) atomicAdd(ctr, 1);
  target += 3;
  int spins = 0;
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 22)) return false;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return true;
}

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
  if constexpr (RULE == kSeqHinge) {
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

// Producer state carried between chunks: the raw inputs of the next chunk, in registers.
template <int KN>
struct ProdRegs {
  static constexpr int NF = (seq::MAXF + 2) / 3;  // fields per producer thread
  static constexpr int NJ = (KN + 2) / 3;         // dense columns per producer thread
  uint32_t tk[NF];
  float xv[NJ];
};

// Branch-free: every load is issued unconditionally from a clamped address (a load in a
// lane-divergent branch is waited for inside the branch), invalid lanes are masked after.
template <int KN>
__device__ __forceinline__ void prod_load(ProdRegs<KN>& R, const float* __restrict__ num, int dn,
                                          const uint32_t* __restrict__ tok, int dc, int row,
                                          bool valid, int q, int bias, int last_row) {
  const size_t rc = (size_t)(valid ? row : last_row);
#pragma unroll
  for (int k = 0; k < ProdRegs<KN>::NF; ++k) {
    const int f = q + 3 * k;
    R.tk[k] = dc > 0 ? tok[rc * dc + min(f, dc - 1)] : kAbsentToken;
  }
#pragma unroll
  for (int k = 0; k < ProdRegs<KN>::NJ; ++k) {
    const int j = q + 3 * k;
    R.xv[k] = dn > 0 ? num[rc * dn + min(j, dn - 1)] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < ProdRegs<KN>::NF; ++k)
    if (!valid || q + 3 * k >= dc) R.tk[k] = kAbsentToken;
#pragma unroll
  for (int k = 0; k < ProdRegs<KN>::NJ; ++k) {
    const int j = q + 3 * k;
    R.xv[k] = !valid ? 0.f : (j < dn ? R.xv[k] : ((bias && j == dn) ? 1.f : 0.f));
  }
}

// Builds chunk k of the spoke in buffer b: dense block, hashed slots, ‖x‖², group tables,
// U, and G on the matrix cores. Waves 1..3 only (pw = wave − 1, pt = thread − 64).
template <int KN>
__device__ void produce(SeqSmem<KN>& sm, const ProdRegs<KN>& R, int b, int dn, int dc,
                        const SeqParams& p, int& pbt) {
  const int pt = (int)threadIdx.x - 64;
  const int r = pt & 63, q = __builtin_amdgcn_readfirstlane(pt >> 6);  // wave-uniform
  const int lane = threadIdx.x & 63;
  float n2 = 0.f;
#pragma unroll
  for (int k = 0; k < ProdRegs<KN>::NJ; ++k) {
    const int j = q + 3 * k;
    if (j < KN) {
      sm.xn[b][r][j] = R.xv[k];
      n2 = fmaf(R.xv[k], R.xv[k], n2);
    }
  }
  // hash + group: insert the slot into its field's table, count members; the member that
  // makes a group shared (second arrival) claims its U column
  int ent[ProdRegs<KN>::NF];
  int code[ProdRegs<KN>::NF];
#pragma unroll
  for (int k = 0; k < ProdRegs<KN>::NF; ++k) {
    const int f = q + 3 * k;
    ent[k] = -1;
    code[k] = -1;
    if (f < dc) {
      code[k] = hash_token_dev(R.tk[k], f, dn, p.span);
      sm.slots[b][f][r] = code[k];
    }
  }
#pragma unroll
  for (int k = 0; k < ProdRegs<KN>::NF; ++k) {
    const int f = q + 3 * k;
    if (f < dc) {
      if (code[k] != -1) {
        n2 += 1.f;
        const int key = code[k] & 0x7fffffff;
        uint32_t h = ((uint32_t)key * 0x9E3779B1u) >> 25;  // TB = 128
        for (int probe = 0; probe < seq::TB; ++probe) {
          int cur = __hip_atomic_load(&sm.tkey[f][h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (cur == -1) {
            const int prev = atomicCAS(&sm.tkey[f][h], -1, key);
            cur = prev == -1 ? key : prev;
          }
          if (cur == key) {
            ent[k] = (int)h;
            break;
          }
          h = (h + 1) & (seq::TB - 1);
        }
        // ≤ 64 keys in 128 entries: the probe always terminates with a slot
        if (atomicAdd(&sm.tcnt[f][ent[k]], 1) == 1) sm.tcol[f][ent[k]] = atomicAdd(&sm.ncols[b], 1);
      }
    }
  }
  sm.part_n[b][q][r] = n2;
  if (!producer_barrier(&sm.pbar, pbt)) sm.stuck = 1;
  // members of shared groups set their one-hot entry: the feature value ±1 (two tokens of
  // a field that collide on a slot may carry opposite hash signs, so U·Uᵀ = Σ x_t·x_s);
  // columns ≥ KU take the exact slow path
  int col[ProdRegs<KN>::NF];
  bool slow = false;
#pragma unroll
  for (int k = 0; k < ProdRegs<KN>::NF; ++k) {
    const int f = q + 3 * k;
    col[k] = -1;
    if (f < dc && ent[k] >= 0 && sm.tcnt[f][ent[k]] >= 2) {
      col[k] = sm.tcol[f][ent[k]];
      if (col[k] < seq::KU) sm.U[r][col[k]] = code[k] < 0 ? 0xBF80 : 0x3F80;  // bf16 ∓1
      else slow = true;
    }
  }
  if (slow) sm.ovf[b] = 1;
  if (!producer_barrier(&sm.pbar, pbt)) sm.stuck = 1;
  // G tiles (I, J) ∈ {(0,0), (1,0), (1,1)}: the scan reads row s of G at columns t < s
  // (G is symmetric; its upper-right tile stays 0)
  {
    const int I0 = q == 0 ? 0 : 32, J0 = q == 2 ? 32 : 0;
    const int l31 = lane & 31, hi = lane >> 5;
    f32x16 acc = {};
#pragma unroll
    for (int k0 = 0; k0 < KN; k0 += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sm.xn[b][I0 + l31][k0 + hi],
                                                 sm.xn[b][J0 + l31][k0 + hi], acc, 0, 0, 0);
    const int nc = min(__builtin_amdgcn_readfirstlane(sm.ncols[b]), seq::KU);
    for (int k0 = 0; k0 < nc; k0 += 16) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(&sm.U[I0 + l31][k0 + 8 * hi]);
      const bf16x8 bb = *reinterpret_cast<const bf16x8*>(&sm.U[J0 + l31][k0 + 8 * hi]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, acc, 0, 0, 0);
    }
#pragma unroll
    for (int reg = 0; reg < 16; ++reg)
      sm.G[b][I0 + (reg & 3) + 8 * (reg >> 2) + 4 * hi][J0 + l31] = acc[reg];
  }
  if (!producer_barrier(&sm.pbar, pbt)) sm.stuck = 1;
  if (__builtin_amdgcn_readfirstlane(sm.ovf[b])) {
    // more shared groups than U columns: the overflowed ones add their counts directly
#pragma unroll
    for (int k = 0; k < ProdRegs<KN>::NF; ++k) {
      const int f = q + 3 * k;
      if (col[k] >= seq::KU) {
        const int key = code[k] & 0x7fffffff;
        for (int t = 0; t < seq::CH; ++t) {
          const int ct = sm.slots[b][f][t];
          if (t != r && ct != -1 && (ct & 0x7fffffff) == key)
            atomicAdd(&sm.G[b][r][t], (ct ^ code[k]) < 0 ? -1.f : 1.f);
        }
      }
    }
  }
  // leave U, the tables and the other buffer's counters clean for the next chunk
#pragma unroll
  for (int k = 0; k < ProdRegs<KN>::NF; ++k) {
    const int f = q + 3 * k;
    if (col[k] >= 0 && col[k] < seq::KU) sm.U[r][col[k]] = 0;
    if (f < dc && ent[k] >= 0) {
      sm.tkey[f][ent[k]] = -1;  // several members may clear the same entry: same values
      sm.tcnt[f][ent[k]] = 0;
      sm.tcol[f][ent[k]] = -1;
    }
  }
  if (pt == 0) {
    sm.ncols[b ^ 1] = 0;
    sm.ovf[b ^ 1] = 0;
  }
}

template <int RULE, int KN>
__global__ __launch_bounds__(seq::NT, 1) void linear_seq_kernel(
    const float* __restrict__ num, int dn, const uint32_t* __restrict__ tok, int dc,
    const void* __restrict__ yv, int B, int R, float* __restrict__ rep, int dim,
    float* __restrict__ ws, SeqParams p) {
  __shared__ SeqSmem<KN> sm;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int s = blockIdx.x;
  float* W = rep + (size_t)s * dim;
  const long long t0ll = (long long)s * R;
  const int t0 = t0ll > B ? B : (int)t0ll;
  const int t1 = (t0ll + R) > B ? B : (int)(t0ll + R);
  float* wrow = ws + (size_t)s * seq::WS;
  if (t0 >= t1) {  // idle spoke: not a worker of this round
    if (tid < seq::WS) wrow[tid] = 0.f;
    return;
  }
  const int nch = (t1 - t0 + seq::CH - 1) / seq::CH;

  // ---- init: tables empty, U zero, dense weights from the replica, G's lower-left tile 0
  for (int i = tid; i < seq::MAXF * seq::TB; i += seq::NT) {
    (&sm.tkey[0][0])[i] = -1;
    (&sm.tcnt[0][0])[i] = 0;
    (&sm.tcol[0][0])[i] = -1;
  }
  for (int i = tid; i < seq::CH * (seq::KU + seq::UPAD); i += seq::NT) (&sm.U[0][0])[i] = 0;
  for (int i = tid; i < 2 * 32 * 32; i += seq::NT) {
    const int b = i >> 10, t = (i >> 5) & 31, c = 32 + (i & 31);
    sm.G[b][t][c] = 0.f;
  }
  for (int i = tid; i < 2 * seq::CH * (KN + 1); i += seq::NT) (&sm.xn[0][0][0])[i] = 0.f;
  if (tid < KN) sm.wn[tid] = tid < dn ? W[tid] : ((p.bias && tid == dn) ? W[dim - 1] : 0.f);
  if (tid < 2) {
    sm.ncols[tid] = 0;
    sm.ovf[tid] = 0;
  }
  if (tid == 0) {
    sm.pbar = 0;
    sm.stuck = 0;
  }
  __syncthreads();

  // gather of chunk k into buffer b: round-start margins from the replica + dense weights
  auto gather = [&](int b) {
    const int r = tid & 63, q4 = __builtin_amdgcn_readfirstlane(tid >> 6);
    float acc = 0.f;
    float wv[(seq::MAXF + 3) / 4];
    int code[(seq::MAXF + 3) / 4];
#pragma unroll
    for (int k = 0; k < (seq::MAXF + 3) / 4; ++k) {
      const int f = q4 + 4 * k;
      code[k] = f < dc ? sm.slots[b][f][r] : -1;
      wv[k] = W[code[k] != -1 ? (code[k] & 0x7fffffff) : 0];  // unconditional (see prod_load)
    }
#pragma unroll
    for (int k = 0; k < (seq::MAXF + 3) / 4; ++k)
      acc += code[k] == -1 ? 0.f : (code[k] < 0 ? -wv[k] : wv[k]);
#pragma unroll
    for (int k = q4; k < KN; k += 4) acc = fmaf(sm.xn[b][r][k], sm.wn[k], acc);
    sm.part_p[q4][r] = acc;
  };

  int pbt = 0;  // producer barrier target
  ProdRegs<KN> PR;
  const int pq = __builtin_amdgcn_readfirstlane((tid - 64) >> 6), pr = (tid - 64) & 63;
  // scanner state
  float loss = 0.f, nex = 0.f, mist = 0.f, sqe = 0.f;
  float ynext = 0.f;
  if (wave == 0) {
    ynext = load_y(yv, min(t0 + lane, t1 - 1), p.y8);
  } else {
    const int row = t0 + pr;
    prod_load<KN>(PR, num, dn, tok, dc, row, row < t1, pq, p.bias, t1 - 1);
  }

  // Software pipeline over chunks: iteration c scans chunk c (wave 0) while waves 1-3
  // build chunk c + 1; then everyone scatters chunk c and gathers chunk c + 1's margins.
  // c = −1 is the prologue (build + gather of chunk 0 only).
  for (int c = -1; c < nch; ++c) {
    const int b = c & 1;  // buffer of chunk c (c = −1 → 1, unused)
    if (wave == 0) {
      if (c >= 0) {
        // ---------------- scan chunk c
        const int row = t0 + c * seq::CH + lane;
        const bool valid = row < t1;
        // invalid rows (past the spoke's shard) get y = 0 and 1/‖x‖² = 0: c = 0 exactly
        const float y = valid ? ynext : 0.f;
        if (c + 1 < nch) {
          const int r1 = row + seq::CH;
          ynext = load_y(yv, min(r1, t1 - 1), p.y8);
        }
        float m = (sm.part_p[0][lane] + sm.part_p[1][lane]) + (sm.part_p[2][lane] + sm.part_p[3][lane]);
        const float n2 = sm.part_n[b][0][lane] + sm.part_n[b][1][lane] + sm.part_n[b][2][lane];
        const float inv = (valid && n2 > 0.f) ? __builtin_amdgcn_rcpf(n2 + p.kadd) : 0.f;
        // the recurrence: step t broadcasts lane t's c_t (v_readlane) and every lane s adds
        // c_t·G[s][t] (row s of the symmetric G, four steps per ds_read_b128). c_t and m_t
        // are written back into lane t (v_writelane, off the dependency chain).
        int cvec = 0, mvec = 0;
        const float* grow = &sm.G[b][lane][0];
#pragma unroll
        for (int t4 = 0; t4 < seq::CH; t4 += 4) {
          const float4 g4 = *reinterpret_cast<const float4*>(grow + t4);
          const float gg[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int t = t4 + u;
            const float cand = seq_candidate<RULE>(m, y, inv, p);
            const int ct = __builtin_amdgcn_readlane(__builtin_bit_cast(int, cand), t);
            const int mt = __builtin_amdgcn_readlane(__builtin_bit_cast(int, m), t);
            cvec = omldm_writelane(ct, t, cvec);
            mvec = omldm_writelane(mt, t, mvec);
            m = fmaf(__builtin_bit_cast(float, ct), gg[u], m);
          }
        }
        sm.cval[lane] = __builtin_bit_cast(float, cvec);
        if (valid) {
          seq_stats<RULE>(__builtin_bit_cast(float, mvec), y, p, loss, mist, sqe);
          nex += 1.f;
        }
      }
    } else if (c + 1 < nch) {
      // ---------------- build chunk c + 1 (the inputs of c + 2 load meanwhile)
      const ProdRegs<KN> cur = PR;
      const int r2 = t0 + (c + 2) * seq::CH + pr;
      if (c + 2 < nch) prod_load<KN>(PR, num, dn, tok, dc, r2, r2 < t1, pq, p.bias, t1 - 1);
      produce<KN>(sm, cur, b ^ 1, dn, dc, p, pbt);
    }
    __syncthreads();
    if (c >= 0) {
      // ---------------- scatter chunk c into the replica (L2 fp32 atomics) + dense weights
      const int r = tid & 63, q4 = __builtin_amdgcn_readfirstlane(tid >> 6);
      const float cv = sm.cval[r];
      if (cv != 0.f) {
#pragma unroll
        for (int k = 0; k < (seq::MAXF + 3) / 4; ++k) {
          const int f = q4 + 4 * k;
          const int code = f < dc ? sm.slots[b][f][r] : -1;
          if (code != -1) unsafeAtomicAdd(&W[code & 0x7fffffff], code < 0 ? -cv : cv);
        }
      }
      constexpr int PARTS = seq::NT / KN;
      constexpr int RPP = seq::CH / PARTS;
      const int kcol = tid % KN, part = tid / KN;
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < RPP; ++i) {
        const int rr = part * RPP + i;
        d = fmaf(sm.cval[rr], sm.xn[b][rr][kcol], d);
      }
      if (d != 0.f) atomicAdd(&sm.wn[kcol], d);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    if (c + 1 < nch) gather(b ^ 1);
    __syncthreads();
  }

  // ---- round end: dense weights back into the replica, spoke statistics
  if (tid < dn && tid < KN) W[tid] = sm.wn[tid];
  if (p.bias && tid == 0) W[dim - 1] = sm.wn[dn];
  if (wave == 0) {
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
      wrow[5] = sm.stuck ? 1.f : 0.f;  // → running totals "overflow": must stay 0
      wrow[6] = 0.f;
      wrow[7] = 0.f;
    }
  }
}

// dacc[j] = inv_p · Σ_{s < S_act} (rep[s][j] − w[j]); dacc[dim] = dacc[dim+1] = S_act·inv_p;
// block 0 also folds the spoke statistics into the fp64 running totals.
__global__ __launch_bounds__(256) void linear_seq_reduce_kernel(
    const float* __restrict__ rep, const float* __restrict__ w, int S_act, int dim,
    float* __restrict__ dacc, float inv_p, const float* __restrict__ ws, double* __restrict__ cum) {
  const int n4 = dim >> 2;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int stride = gridDim.x * blockDim.x;
  const float4* w4 = reinterpret_cast<const float4*>(w);
  float4* d4 = reinterpret_cast<float4*>(dacc);
  for (int i = tid; i < n4; i += stride) {
    const float4 wv = w4[i];
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < S_act; ++s) {
      const float4 r = reinterpret_cast<const float4*>(rep + (size_t)s * dim)[i];
      a.x += r.x - wv.x;
      a.y += r.y - wv.y;
      a.z += r.z - wv.z;
      a.w += r.w - wv.w;
    }
    d4[i] = make_float4(a.x * inv_p, a.y * inv_p, a.z * inv_p, a.w * inv_p);
  }
  for (int i = (n4 << 2) + tid; i < dim; i += stride) {
    float a = 0.f;
    for (int s = 0; s < S_act; ++s) a += rep[(size_t)s * dim + i] - w[i];
    dacc[i] = a * inv_p;
  }
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) {
      dacc[dim] = (float)S_act * inv_p;
      dacc[dim + 1] = (float)S_act * inv_p;
    }
    if (cum && threadIdx.x < 6 && threadIdx.x != 4) {
      double t = 0.0;
      for (int s = 0; s < S_act; ++s) t += (double)ws[(size_t)s * seq::WS + threadIdx.x];
      cum[threadIdx.x] += t;
    }
  }
}

// w = (a·w + D)/n (the model average, a = D[dim], n = D[dim+1]); every replica ← w; D ← 0.
__global__ __launch_bounds__(256) void linear_seq_apply_kernel(float* __restrict__ w,
                                                               float* __restrict__ rep, int S,
                                                               float* __restrict__ dacc, int dim) {
  const float n = dacc[dim + 1];
  const float a = n > 0.f ? dacc[dim] : 1.f;
  const float rn = n > 0.f ? 1.f / n : 1.f;
  const int n4 = dim >> 2;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int stride = gridDim.x * blockDim.x;
  float4* w4 = reinterpret_cast<float4*>(w);
  float4* d4 = reinterpret_cast<float4*>(dacc);
  for (int i = tid; i < n4; i += stride) {
    float4 wv = w4[i];
    const float4 dv = d4[i];
    wv.x = fmaf(a, wv.x, dv.x) * rn;
    wv.y = fmaf(a, wv.y, dv.y) * rn;
    wv.z = fmaf(a, wv.z, dv.z) * rn;
    wv.w = fmaf(a, wv.w, dv.w) * rn;
    w4[i] = wv;
    d4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < S; ++s) reinterpret_cast<float4*>(rep + (size_t)s * dim)[i] = wv;
  }
  for (int i = (n4 << 2) + tid; i < dim; i += stride) {
    const float v = fmaf(a, w[i], dacc[i]) * rn;
    w[i] = v;
    dacc[i] = 0.f;
    for (int s = 0; s < S; ++s) rep[(size_t)s * dim + i] = v;
  }
}

// every replica ← w (after the model changed outside a round: restore, Create, Update)
__global__ __launch_bounds__(256) void linear_seq_broadcast_kernel(const float* __restrict__ w,
                                                                   float* __restrict__ rep, int S,
                                                                   int dim) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int stride = gridDim.x * blockDim.x;
  for (int i = tid; i < dim; i += stride) {
    const float v = w[i];
    for (int s = 0; s < S; ++s) rep[(size_t)s * dim + i] = v;
  }
}

__global__ __launch_bounds__(256) void hash_raw_kernel(const uint32_t* __restrict__ tok, long long n,
                                                       int dc, int dn, uint32_t span,
                                                       int* __restrict__ out) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = hash_token_dev(tok[i], (int)(i % dc), dn, span);
}

template <int RULE, int KN>
static int launch_seq(const float* num, int dn, const uint32_t* tok, int dc, const void* y, int B,
                      int R, int S, float* rep, int dim, float* ws, const SeqParams& p,
                      hipStream_t st) {
  hipLaunchKernelGGL((linear_seq_kernel<RULE, KN>), dim3(S), dim3(seq::NT), 0, st, num, dn, tok,
                     dc, y, B, R, rep, dim, ws, p);
  return (int)hipGetLastError();
}

template <int KN>
static int dispatch_seq(int rule, const float* num, int dn, const uint32_t* tok, int dc,
                        const void* y, int B, int R, int S, float* rep, int dim, float* ws,
                        const SeqParams& p, hipStream_t st) {
  if (rule == kSeqHinge) return launch_seq<kSeqHinge, KN>(num, dn, tok, dc, y, B, R, S, rep, dim, ws, p, st);
  if (rule == kSeqEps) return launch_seq<kSeqEps, KN>(num, dn, tok, dc, y, B, R, S, rep, dim, ws, p, st);
  return launch_seq<kSeqLogistic, KN>(num, dn, tok, dc, y, B, R, S, rep, dim, ws, p, st);
}

static int grid_for(int dim) {
  int blocks = (dim / 4 + 255) / 256;
  return blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
}

}  // namespace omldm

using namespace omldm;

// One Synchronous round of S sequential spokes on the raw wire (see the file comment).
// rep: [S, dim] fp32 replicas, equal to w at entry (linear_seq_apply / _broadcast keep
// them so); ws: [S, 8] scratch; cum: fp64 running totals (loss, n, mistakes, sq_err) or
// NULL. Leaves the round delta in dacc [dim + 2] for the collective + apply.
OMLDM_API int omldm_linear_seq_round(const float* w, const float* num, int dn, const void* tok,
                                     int dc, const void* y, int y8, int B, int R, int S,
                                     float* rep, float* dacc, int dim, float* ws, double* cum,
                                     int rule, int variant, float C, float eps, float lr,
                                     float inv_p, int bias, void* stream) {
  if (S <= 0 || B <= 0) return 0;
  if (R <= 0 || dc > seq::MAXF || dc < 0 || dn < 0 || dim <= dn + 1) return -2;
  if (rule < 0 || rule > 2) return -5;
  const int kn_need = dn + (bias ? 1 : 0);
  if (kn_need > 32) return -2;
  const SeqParams p{rule, variant, variant == 1 ? C : INFINITY, variant == 2 ? 0.5f / C : 0.f,
                    eps, lr, inv_p, bias, y8, (uint32_t)(dim - dn - 1)};
  hipStream_t st = (hipStream_t)stream;
  int e = kn_need <= 16 ? dispatch_seq<16>(rule, num, dn, (const uint32_t*)tok, dc, y, B, R, S, rep, dim, ws, p, st)
                        : dispatch_seq<32>(rule, num, dn, (const uint32_t*)tok, dc, y, B, R, S, rep, dim, ws, p, st);
  if (e) return e;
  const long long sact = ((long long)B + R - 1) / R;
  const int S_act = sact < S ? (int)sact : S;
  hipLaunchKernelGGL(linear_seq_reduce_kernel, dim3(grid_for(dim)), dim3(256), 0, st, rep, w,
                     S_act, dim, dacc, inv_p, ws, cum);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_linear_seq_apply(float* w, float* rep, int S, float* dacc, int dim,
                                     void* stream) {
  hipLaunchKernelGGL(linear_seq_apply_kernel, dim3(grid_for(dim)), dim3(256), 0,
                     (hipStream_t)stream, w, rep, S, dacc, dim);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_linear_seq_broadcast(const float* w, float* rep, int S, int dim, void* stream) {
  hipLaunchKernelGGL(linear_seq_broadcast_kernel, dim3(grid_for(dim)), dim3(256), 0,
                     (hipStream_t)stream, w, rep, S, dim);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_hash_raw(const void* tok, long long B, int dc, int dn, long long dim, int* out,
                             void* stream) {
  if (B <= 0 || dc <= 0) return 0;
  const long long n = B * dc;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(hash_raw_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     (const uint32_t*)tok, n, dc, dn, (uint32_t)(dim - dn - 1), out);
  return (int)hipGetLastError();
}
