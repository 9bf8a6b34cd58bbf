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
// and only the scalar recurrence c_t = rule(m_t) is sequential. One workgroup per spoke,
// 8 waves; chunks of 64 rows are software-pipelined:
//   * the scanner (wave 0, lane t = row t) runs the recurrence of chunk k: per step one
//     closed-form candidate per lane, a v_readlane of lane t's, one FMA with row t of G;
//   * meanwhile the 7 producer waves build chunk k+1: murmur3-hash the raw 32-bit
//     category tokens (field-aware, hash_dev.h), group each field's equal slots
//     wave-locally (no atomics), build G on the matrix cores — the dense block
//     [numerical | intercept] with fp32-in/fp32-acc MFMA (exact f32 products), the
//     categorical part G_cat[t][s] = Σ_f [slot_tf = slot_sf]·x_tf·x_sf as U·Uᵀ with bf16
//     MFMA over a ±1 one-hot "shared group" matrix U in LDS — and GATHER chunk k+1's
//     round-start margins from the spoke's replica BEFORE chunk k's update lands;
//   * after the scan, chunk k's update is scattered into the replica (L2 fp32 atomics,
//     not waited for) and chunk k+1's margins get the exact correction for what they
//     missed: Σ_f x_sf · Σ_{t ∈ k, slot_tf = slot_sf} c_t x_tf + x_s,dense · Δw_dense,k
//     (the producers link chunk k's entries to chunk k+1's groups while grouping).
// So no global-memory latency (gather, scatter completion) sits on the scanner's path.
// Replicas [S][dim] fp32 in HBM (4 MiB each at 2^20 dims). Round end:
// linear_seq_reduce_kernel averages the replicas into the round accumulator (the RCCL
// all-reduce runs on it for N > 1) and linear_seq_apply_kernel folds it into w and
// refreshes every replica.
#include "common.h"
#include "hash_dev.h"
#include "seq_common.h"

namespace omldm {

namespace seq {
constexpr int CH = 64;     // rows per chunk = scanner lanes
constexpr int NP = 7;      // producer waves (wave 0 is the scanner)
constexpr int NW = NP + 1; // waves per workgroup
constexpr int NT = 64 * NW;
constexpr int MAXF = 32;   // categorical fields per row
constexpr int CPW = 32;    // U columns owned by each producer wave
constexpr int KU = NP * CPW;  // shared-group columns of U on the matrix cores
constexpr int UPAD = 8;    // bf16 row padding of U (spreads the 16-B operand reads over banks)
constexpr int GPAD = 4;    // G row stride 68 floats: 16-B aligned rows, b128 reads over banks
constexpr int TB1 = 512;   // per-wave grouping table, first hash
constexpr int TB2 = 256;   // second hash (keys that lost the first)
constexpr int WS = 8;      // per-spoke stat row: loss, n, mistakes, sq_err, 1, stuck, 0, 0
}  // namespace seq

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
  int tab[seq::NP][seq::TB1 + seq::TB2];          // per producer wave: (local slot << 6) | row
  int flag[seq::NP][seq::CH];                     // per wave: row is a shared group's rep
  int gcol[seq::NP][seq::CH];                     // per wave: rep row → its U column
  int ovl[seq::NP][seq::CH];                      // per wave: third-chance groups (slot)
  signed char rep[2][seq::MAXF][seq::CH];         // chunk row → its group's representative row
  signed char xlink[seq::MAXF][seq::CH];          // chunk-k row → chunk-(k+1) group rep (−1)
  float cgrp[seq::MAXF][seq::CH];                 // Σ c_t x_t of chunk k per chunk-(k+1) group
  float part_p[seq::NP][seq::CH];                 // round-start margin partials
  float part_n[2][seq::NP][seq::CH];              // ‖x‖² partials
  float cval[seq::CH];                            // the chunk's c_t
  float wn[KN];                                   // dense weights (numerical, intercept)
  float dwn[KN];                                  // the last chunk's dense update
  int ucnt[2][seq::NP];                           // U columns used per wave
  int ovf[2];
  int pbar;                                       // producer-wave barrier counter
  int stuck;                                      // a producer barrier timed out
};

// Barrier of the producer waves only (the scanner wave keeps running): a monotonic LDS
// counter, one increment per wave, spin until all arrived. The spin is bounded (≈ 2^22
// sleeps, far beyond any legitimate wait): a broken invariant ends the kernel with a wrong
// result flagged in the spoke's stat row instead of hanging the GPU.
__device__ __forceinline__ bool producer_barrier(int* ctr, int& target) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) atomicAdd(ctr, 1);
  target += seq::NP;
  int spins = 0;
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 22)) return false;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return true;
}

// Producer state carried between chunks: the raw inputs of the next chunk, in registers.
template <int KN>
struct ProdRegs {
  static constexpr int NF = (seq::MAXF + seq::NP - 1) / seq::NP;  // fields per producer thread
  static constexpr int NJ = (KN + seq::NP - 1) / seq::NP;         // dense columns per thread
  uint32_t tk[NF];
  float xv[NJ];
};

// Issues the loads of one chunk's inputs into registers and returns at once: every load
// comes from a clamped (always valid) address and NOTHING reads the values here — masking
// them (rows past the shard, fields ≥ dc) right after the loads made the compiler wait
// for them, which turned the one-chunk-ahead prefetch into a synchronous HBM round trip
// per chunk. produce() masks when it consumes the registers, a chunk later.
template <int KN>
__device__ __forceinline__ void prod_load(ProdRegs<KN>& R, const float* __restrict__ num, int dn,
                                          const uint32_t* __restrict__ tok, int dc, int row,
                                          int q, int last_row) {
  const size_t rc = (size_t)min(row, last_row);
  if (dc > 0) {
#pragma unroll
    for (int k = 0; k < ProdRegs<KN>::NF; ++k)
      R.tk[k] = tok[rc * dc + min(q + seq::NP * k, dc - 1)];
  }
  if (dn > 0) {
#pragma unroll
    for (int k = 0; k < ProdRegs<KN>::NJ; ++k)
      R.xv[k] = num[rc * dn + min(q + seq::NP * k, dn - 1)];
  }
}

// Diagnostics: when set (omldm_linear_seq_stamps), lane 0 of wave 0 and of wave 1 add
// per-phase cycle counts (s_memtime) into g_seq_stamps[spoke][16]:
//   0 scan, 1 scanner wait for producers, 2 post-scan (scatter/link/correct) (wave 0);
//   4 produce (wave 1), 5 chunks, 6 wave-1 wait at the first barrier;
//   8.. produce sub-phases (wave 1): 8 fence + dense + hash, 9 gather issue,
//   10 grouping + links + U, 11 barrier, 12 MFMA + G, 13 barrier, 14 slow path + reset,
//   15 gather consume.
__device__ unsigned long long* g_seq_stamps;

__device__ __forceinline__ void sub_stamp(unsigned long long* acc, unsigned long long& t, int k) {
  if (acc) {
    const unsigned long long now = clock64();
    if (k >= 0) acc[k] += now - t;
    t = now;
  }
}

// Wave-local grouping of one field of the chunk being built (lane = row). Returns the
// row's group representative (−1 when absent). tab holds (local slot << 6) | row; a lane
// only trusts an entry it verified, so the table is never cleared.
__device__ __forceinline__ int group_rows(volatile int* tab, volatile int* ovl, int& novl,
                                          bool present, int loc) {
  int rep = -1;
  const int h1 = (int)(((uint32_t)loc * 0x9E3779B1u) >> 23);          // TB1 = 512
  if (present) tab[h1] = (loc << 6) | (int)(threadIdx.x & 63);
  const int e1 = present ? tab[h1] : 0;
  if (present && (e1 >> 6) == loc) rep = e1 & 63;
  novl = 0;
  if (__ballot(present && rep < 0)) {
    const int h2 = seq::TB1 + (int)(((uint32_t)loc * 0x85EBCA77u + 0x27D4EB2Fu) >> 24);  // TB2
    const bool again = present && rep < 0;
    if (again) tab[h2] = (loc << 6) | (int)(threadIdx.x & 63);
    const int e2 = again ? tab[h2] : 0;
    if (again && (e2 >> 6) == loc) rep = e2 & 63;
    // third chance: the first unresolved lane of each remaining slot represents it; its
    // slot goes to the wave's overflow list (what chunk lookups check last)
    unsigned long long m = __ballot(present && rep < 0);
    while (m) {
      const int u = __builtin_ctzll(m);
      const int lu = __builtin_amdgcn_readlane(loc, u);
      if (present && rep < 0 && loc == lu) rep = u;
      if ((int)(threadIdx.x & 63) == 0) ovl[novl] = (lu << 6) | u;
      ++novl;
      m = __ballot(present && rep < 0);
    }
  }
  return rep;
}

// The representative row of `loc` among the chunk grouped last into tab/ovl (−1: the
// slot does not occur there). Table entries may be stale (earlier fields or chunks), so
// a hit is verified against that chunk's slots.
__device__ __forceinline__ int lookup_rows(volatile int* tab, const volatile int* ovl, int novl,
                                           const int* slots_f, int base_f, bool present, int loc) {
  if (!present) return -1;
  const int h1 = (int)(((uint32_t)loc * 0x9E3779B1u) >> 23);
  const int e1 = tab[h1];
  if ((e1 >> 6) == loc && (slots_f[e1 & 63] & 0x7fffffff) == base_f + loc) return e1 & 63;
  const int h2 = seq::TB1 + (int)(((uint32_t)loc * 0x85EBCA77u + 0x27D4EB2Fu) >> 24);
  const int e2 = tab[h2];
  if ((e2 >> 6) == loc && (slots_f[e2 & 63] & 0x7fffffff) == base_f + loc) return e2 & 63;
  for (int i = 0; i < novl; ++i)
    if ((ovl[i] >> 6) == loc) return ovl[i] & 63;
  return -1;
}

// Builds chunk n (buffer bn) while the scanner works on chunk o (buffer bo, has_o):
// dense block, hashed slots, ‖x‖², the gather of the round-start margins from the
// replica, the field groups of chunk n and the links of chunk o's entries into them, U,
// and G on the matrix cores. Producer waves only (q = wave − 1, r = row).
template <int KN>
__device__ void produce(SeqSmem<KN>& sm, const ProdRegs<KN>& R, ProdRegs<KN>& next,
                        int next_row, bool load_next, const float* __restrict__ num,
                        const uint32_t* __restrict__ tok, int last_row, bool valid, int bn,
                        bool has_o, int dn, int dc, const SeqParams& p, int& pbt,
                        const float* W, int (&code)[ProdRegs<KN>::NF], float& pacc,
                        unsigned long long* sacc) {
  constexpr int NF = ProdRegs<KN>::NF;
  const int bo = bn ^ 1;
  unsigned long long st_t = 0;
  sub_stamp(sacc, st_t, -1);
  const int pt = (int)threadIdx.x - 64;
  const int r = pt & 63, q = __builtin_amdgcn_readfirstlane(pt >> 6);  // wave-uniform
  const int lane = threadIdx.x & 63;
  // ---- every earlier chunk's scatter has completed before this chunk's gather: each
  // producer wave waits for its own atomics, then the producers meet (the scanner scans
  // meanwhile); only then the next chunk's inputs are requested (a release fence waits
  // for every outstanding load as well)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  if (!producer_barrier(&sm.pbar, pbt)) sm.stuck = 1;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (load_next) prod_load<KN>(next, num, dn, tok, dc, next_row, q, last_row);
  // ---- dense block + the dense part of the round-start margin
  float n2 = 0.f, pd = 0.f;
#pragma unroll
  for (int k = 0; k < ProdRegs<KN>::NJ; ++k) {
    const int j = q + seq::NP * k;
    if (j < KN) {  // dense block: features, then the intercept column, then zero padding
      const float x = !valid ? 0.f : (j < dn ? R.xv[k] : ((p.bias && j == dn) ? 1.f : 0.f));
      sm.xn[bn][r][j] = x;
      n2 = fmaf(x, x, n2);
      pd = fmaf(x, sm.wn[j], pd);
    }
  }
  // ---- hash; the previous link targets of this row are cleared for the new chunk
#pragma unroll
  for (int k = 0; k < NF; ++k) {
    const int f = q + seq::NP * k;
    code[k] = -1;
    if (f < dc) {
      code[k] = hash_token_dev(valid ? R.tk[k] : kAbsentToken, f, dn, p.span);
      sm.slots[bn][f][r] = code[k];
      sm.cgrp[f][r] = 0.f;
    }
    n2 += code[k] != -1 ? 1.f : 0.f;  // ‖x‖² over the feature list (CPU oracle semantics)
  }
  sm.part_n[bn][q][r] = n2;
  sub_stamp(sacc, st_t, 8);
  // ---- gather (chunk o's update has not been scattered yet: corrected after the scan)
  float wv[NF];
#pragma unroll
  for (int k = 0; k < NF; ++k) wv[k] = W[code[k] != -1 ? (code[k] & 0x7fffffff) : 0];
  sub_stamp(sacc, st_t, 9);
  // ---- group each field of chunk n; link chunk o's entries of the field to them
  volatile int* tab = sm.tab[q];
  volatile int* ovl = sm.ovl[q];
  volatile int* flg = sm.flag[q];
  volatile int* gcl = sm.gcol[q];
  int col[NF];
  int used = 0;  // this wave's U columns (wave-uniform)
  bool slow = false;
#pragma unroll
  for (int k = 0; k < NF; ++k) {
    const int f = q + seq::NP * k;
    col[k] = -1;
    if (f >= dc) continue;  // wave-uniform
    const int base_f = dn + f * (int)p.span;
    const bool present = code[k] != -1;
    const int loc = (code[k] & 0x7fffffff) - base_f;
    int novl = 0;
    const int rp = group_rows(tab, ovl, novl, present, loc);
    sm.rep[bn][f][r] = (signed char)rp;
    if (has_o) {
      const int co = sm.slots[bo][f][r];
      sm.xlink[f][r] = (signed char)lookup_rows(tab, ovl, novl, sm.slots[bn][f], base_f,
                                                co != -1, (co & 0x7fffffff) - base_f);
    }
    // shared groups: flagged by a non-representative member; flagged representatives take
    // this wave's next U columns (ballot + mbcnt), members store ±1 at U[row][column]
    flg[r] = 0;
    if (present && rp != r) flg[rp] = 1;
    const bool lead = present && rp == r && flg[r] != 0;
    const unsigned long long m = __ballot(lead);
    if (lead)
      gcl[r] = q * seq::CPW + used + (int)__builtin_amdgcn_mbcnt_hi(
                   (unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
    used += __builtin_popcountll(m);
    if (present && (rp != r || lead)) {
      col[k] = gcl[rp];
      if (col[k] < (q + 1) * seq::CPW) sm.U[r][col[k]] = code[k] < 0 ? 0xBF80 : 0x3F80;
      else slow = true;  // more than CPW shared groups in this wave: exact slow path
    }
  }
  if (lane == 0) sm.ucnt[bn][q] = min(used, seq::CPW);
  if (__ballot(slow) && lane == 0) sm.ovf[bn] = 1;
  sub_stamp(sacc, st_t, 10);
  if (!producer_barrier(&sm.pbar, pbt)) sm.stuck = 1;
  sub_stamp(sacc, st_t, 11);
  // ---- G tiles (I, J) ∈ {(0,0), (1,0), (1,1)}: the scan reads row s of G at columns t < s
  // (G is symmetric; its upper-right tile stays 0). Producer waves 0-2, one tile each.
  if (q < 3) {
    const int I0 = q == 0 ? 0 : 32, J0 = q == 2 ? 32 : 0;
    const int l31 = lane & 31, hi = lane >> 5;
    f32x16 acc = {};
#pragma unroll
    for (int k0 = 0; k0 < KN; k0 += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sm.xn[bn][I0 + l31][k0 + hi],
                                                 sm.xn[bn][J0 + l31][k0 + hi], acc, 0, 0, 0);
    for (int w = 0; w < seq::NP; ++w) {
      const int nc = __builtin_amdgcn_readfirstlane(sm.ucnt[bn][w]);
      for (int k0 = w * seq::CPW; k0 < w * seq::CPW + nc; k0 += 16) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&sm.U[I0 + l31][k0 + 8 * hi]);
        const bf16x8 bb = *reinterpret_cast<const bf16x8*>(&sm.U[J0 + l31][k0 + 8 * hi]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int reg = 0; reg < 16; ++reg)
      sm.G[bn][I0 + (reg & 3) + 8 * (reg >> 2) + 4 * hi][J0 + l31] = acc[reg];
  }
  sub_stamp(sacc, st_t, 12);
  if (!producer_barrier(&sm.pbar, pbt)) sm.stuck = 1;
  sub_stamp(sacc, st_t, 13);
  if (__builtin_amdgcn_readfirstlane(sm.ovf[bn])) {
    // groups past a wave's CPW columns: each such entry adds its products with every
    // other row of the same slot in its field into its own row of G
#pragma unroll
    for (int k = 0; k < NF; ++k) {
      if (col[k] >= (q + 1) * seq::CPW) {
        const int f = q + seq::NP * k;
        const int key = code[k] & 0x7fffffff;
        for (int t = 0; t < seq::CH; ++t) {
          const int ct = sm.slots[bn][f][t];
          if (t != r && ct != -1 && (ct & 0x7fffffff) == key)
            atomicAdd(&sm.G[bn][r][t], (ct ^ code[k]) < 0 ? -1.f : 1.f);
        }
      }
    }
  }
  // leave U and the other buffer's overflow flag clean for the next chunk
#pragma unroll
  for (int k = 0; k < NF; ++k)
    if (col[k] >= 0 && col[k] < (q + 1) * seq::CPW) sm.U[r][col[k]] = 0;
  if (pt == 0) sm.ovf[bo] = 0;
  sub_stamp(sacc, st_t, 14);
  // ---- the gathered categorical weights (in flight since the gather)
  float pc = 0.f;
#pragma unroll
  for (int k = 0; k < NF; ++k) pc += code[k] == -1 ? 0.f : (code[k] < 0 ? -wv[k] : wv[k]);
  pacc = pd + pc;
  sub_stamp(sacc, st_t, 15);
}

template <int RULE, int KN>
__global__ __launch_bounds__(seq::NT, 1) void linear_seq_kernel(
    const float* __restrict__ num, int dn, const uint32_t* __restrict__ tok, int dc,
    const void* __restrict__ yv, int B, int R, float* __restrict__ rep, int dim,
    float* __restrict__ ws, SeqParams p) {
  constexpr int NF = ProdRegs<KN>::NF;
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

  // ---- init: tables, U zero, dense weights from the replica, G's upper-right tiles 0
  for (int i = tid; i < seq::NP * (seq::TB1 + seq::TB2); i += seq::NT) (&sm.tab[0][0])[i] = -1;
  for (int i = tid; i < seq::CH * (seq::KU + seq::UPAD); i += seq::NT) (&sm.U[0][0])[i] = 0;
  for (int i = tid; i < 2 * 32 * 32; i += seq::NT) {
    const int b = i >> 10, t = (i >> 5) & 31, c = 32 + (i & 31);
    sm.G[b][t][c] = 0.f;
  }
  for (int i = tid; i < 2 * seq::CH * (KN + 1); i += seq::NT) (&sm.xn[0][0][0])[i] = 0.f;
  for (int i = tid; i < 2 * seq::MAXF * seq::CH; i += seq::NT) (&sm.slots[0][0][0])[i] = -1;
  for (int i = tid; i < seq::MAXF * seq::CH; i += seq::NT) {
    (&sm.cgrp[0][0])[i] = 0.f;
    (&sm.xlink[0][0])[i] = -1;
  }
  if (tid < KN) {
    sm.wn[tid] = tid < dn ? W[tid] : ((p.bias && tid == dn) ? W[dim - 1] : 0.f);
    sm.dwn[tid] = 0.f;
  }
  if (tid < 2) sm.ovf[tid] = 0;
  if (tid == 0) {
    sm.pbar = 0;
    sm.stuck = 0;
  }
  __syncthreads();

  unsigned long long* stamps = g_seq_stamps;
  unsigned long long st_acc[16] = {};
  unsigned long long st_t = 0;
  auto stamp = [&](int k) {
    if (stamps) {
      const unsigned long long now = clock64();
      if (k >= 0) st_acc[k] += now - st_t;
      st_t = now;
    }
  };

  int pbt = 0;  // producer barrier target
  ProdRegs<KN> PR;
  const int pq = __builtin_amdgcn_readfirstlane((tid - 64) >> 6), pr = (tid - 64) & 63;
  float loss = 0.f, nex = 0.f, mist = 0.f, sqe = 0.f;
  float ynext = 0.f;
  if (wave == 0) {
    ynext = load_y(yv, min(t0 + lane, t1 - 1), p.y8);
  } else {
    prod_load<KN>(PR, num, dn, tok, dc, t0 + pr, pq, t1 - 1);
  }

  // Iteration c: the scanner scans chunk c while the producers build chunk c + 1; then
  // chunk c is scattered and chunk c + 1's margins corrected. c = −1 is the prologue.
  // The two roles run separate loops with the same barrier sequence (s_barrier counts
  // waves), so each loop carries only its own outstanding loads in the compiler's wait
  // analysis.
  if (wave == 0) {
    for (int c = -1; c < nch; ++c) {
      const int b = c & 1;  // buffer of chunk c
      stamp(-1);
      if (c >= 0) {
        const int row = t0 + c * seq::CH + lane;
        const bool valid = row < t1;
        // invalid rows (past the spoke's shard) get y = 0 and 1/‖x‖² = 0: c = 0 exactly
        const float y = valid ? ynext : 0.f;
        if (c + 1 < nch) ynext = load_y(yv, min(row + seq::CH, t1 - 1), p.y8);
        float m = 0.f, n2 = 0.f;
#pragma unroll
        for (int q = 0; q < seq::NP; ++q) {
          m += sm.part_p[q][lane];
          n2 += sm.part_n[b][q][lane];
        }
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
        stamp(0);
        if (valid) {
          seq_stats<RULE>(__builtin_bit_cast(float, mvec), y, p, loss, mist, sqe);
          nex += 1.f;
        }
      }
      __syncthreads();  // B1: chunk c scanned, chunk c + 1 built
      stamp(1);
      __syncthreads();  // B2: chunk c's links and dense update accumulated
      __syncthreads();  // B3: chunk c + 1's margins corrected
      stamp(2);
      st_acc[5] += 1;
    }
  } else {
    const int q = pq, r = pr;
    int code[NF];
    float pacc = 0.f;
    for (int c = -1; c < nch; ++c) {
      const int b = c & 1;
      const bool more = c + 1 < nch;
      stamp(-1);
      if (more) {
        const ProdRegs<KN> cur = PR;
        produce<KN>(sm, cur, PR, t0 + (c + 2) * seq::CH + r, c + 2 < nch, num, tok, t1 - 1,
                    t0 + (c + 1) * seq::CH + r < t1, b ^ 1, c >= 0, dn, dc, p, pbt, W, code,
                    pacc, stamps ? st_acc : nullptr);
        stamp(4);
      }
      __syncthreads();  // B1
      stamp(6);
      if (c >= 0) {
        // ---- chunk c: scatter its update into the replica (not waited for: the next
        // gather fences), link it into chunk c + 1's groups, accumulate the dense update
        const float cv = sm.cval[r];
#pragma unroll
        for (int k = 0; k < NF; ++k) {
          const int f = q + seq::NP * k;
          if (f < dc) {
            const int co = sm.slots[b][f][r];
            if (co != -1 && cv != 0.f) {
              const float u = co < 0 ? -cv : cv;
              unsafeAtomicAdd(&W[co & 0x7fffffff], u);
              const int xl = sm.xlink[f][r];
              if (xl >= 0 && more) atomicAdd(&sm.cgrp[f][xl], u);
            }
          }
        }
        for (int j = q; j < KN; j += seq::NP) {  // Δw_dense of chunk c (lane = row)
          const float d = wave_sum(cv * sm.xn[b][r][j]);
          if (lane == 0) sm.dwn[j] = d;
        }
      }
      __syncthreads();  // B2
      if (more) {
        // ---- chunk c + 1's exact round-start margins: raw gather + what chunk c changed
        float corr = 0.f;
        if (c >= 0) {
#pragma unroll
          for (int k = 0; k < NF; ++k) {
            const int f = q + seq::NP * k;
            if (f < dc && code[k] != -1) {
              const float g = sm.cgrp[f][sm.rep[b ^ 1][f][r]];
              corr += code[k] < 0 ? -g : g;
            }
          }
          for (int j = q; j < KN; j += seq::NP) corr = fmaf(sm.xn[b ^ 1][r][j], sm.dwn[j], corr);
        }
        sm.part_p[q][r] = pacc + corr;
      }
      if (c >= 0) {
        for (int j = q; j < KN; j += seq::NP)
          if (lane == 0) sm.wn[j] += sm.dwn[j];  // w_dense after chunk c
      }
      __syncthreads();  // B3
    }
  }

  if (stamps && lane == 0 && wave <= 1) {
    for (int k = 0; k < 16; ++k)
      if ((wave == 0) == (k < 4 || k == 5)) atomicAdd(&stamps[(size_t)s * 16 + k], st_acc[k]);
  }
  __syncthreads();
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
  // grouping tables pack (local slot << 6 | row) in an int: ≤ 2^25 slots per field
  if (dc > 0 && (long long)(dim - dn - 1) / dc >= (1LL << 25)) return -2;
  const SeqParams p{rule, variant, variant == 1 ? C : INFINITY, variant == 2 ? 0.5f / C : 0.f,
                    eps, lr, inv_p, bias, y8, dc > 0 ? (uint32_t)((dim - dn - 1) / dc) : 1u};
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

// Round end of the v1 round: replicas of the S_act active spokes averaged into
// the round accumulator, spoke statistics into the running totals.
OMLDM_API int omldm_linear_seq_reduce(const float* rep, const float* w, int S_act, int dim,
                                      float* dacc, float inv_p, const float* ws, double* cum,
                                      void* stream) {
  hipLaunchKernelGGL(linear_seq_reduce_kernel, dim3(grid_for(dim)), dim3(256), 0,
                     (hipStream_t)stream, rep, w, S_act, dim, dacc, inv_p, ws, cum);
  return (int)hipGetLastError();
}

// Diagnostics: per-phase cycle accumulation into buf [S][16] (nullptr: off).
OMLDM_API int omldm_linear_seq_stamps(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_seq_stamps), &buf, sizeof(buf));
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
                     (const uint32_t*)tok, n, dc, dn, (uint32_t)((dim - dn - 1) / dc), out);
  return (int)hipGetLastError();
}
