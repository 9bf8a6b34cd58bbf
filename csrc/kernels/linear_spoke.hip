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
//  * At round end each spoke stores its bucketed table (σ·Δ/P per slot) with plain
//    coalesced stores; linear_reduce_kernel sums the tables per key range in LDS and
//    adds them to the dense round accumulator, while its finish blocks sum the per-spoke
//    dense columns and σ/P (the w0 weight, accumulator[dim]). The accumulator is then
//    all-reduced over xGMI by RCCL and folded into w by linear_apply (below) — that is
//    the Synchronous PS round.
#include "spoke_table.h"

namespace omldm {

enum LinRule : int { kHinge = 0, kEpsInsensitive = 1, kLogistic = 2, kPegasos = 3 };
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
  int cspan;      // > 0: compact uint16 categorical wire format (spoke_table.h)
  float cclip;   // τ clip: C for PA-I, +inf otherwise
  float kadd;     // τ denominator offset: 1/(2C) for PA-II, 0 otherwise
  float shrink;   // per-step multiplicative L2 shrink of w (1 when λ = 0)
  float rshrink;  // 1 / shrink
  int y_i8;       // labels on the wire as int8 (classification streams: ±1 exactly)
  float tbase;    // Pegasos: step index T of the spoke's first row this round (≥ 2)
};

// Per-spoke workspace row: [loss, n, mistakes, sq_err, sigma, overflow, σ/P, 1/P,
//                           Δ(dense slot 0..dn-1)·σ/P, Δ(intercept)·σ/P]
constexpr int kWsStat = 8;

// Dense column of feature j: numerical slot j → j, intercept → dn; hashed features → -1.
// Dense features live in a register per lane for the whole round (every example has
// them), so they never touch the LDS table and never hit the same global address from
// every spoke: they are reduced by the finish blocks of linear_reduce_kernel instead of by atomics.
__device__ __forceinline__ int dense_col(int j, int dn, int dc, int bias) {
  if (j < dn) return j;
  if (bias && j == dn + dc) return dn;
  return -1;
}

// Per-row L2 shrink of w (σ ← σ·sh, 1/σ ← 1/σ·rsh) and step size. Pegasos (Shalev-Shwartz
// et al. 2007, the SVM option of SURVEY Appendix D): at step T, η = 1/(λT) and
// w ← (1 − ηλ)·w + η·y·x·[y·w·x < 1], so sh = (T − 1)/T; T counts the spoke's rows
// (p.tbase ≥ 2 keeps σ > 0). Every other rule: the constant shrink of λ.
template <int RULE>
__device__ __forceinline__ void row_rate(const LinParams& p, int row, float& sh, float& rsh,
                                         float& eta) {
  if constexpr (RULE == kPegasos) {
    const float T = p.tbase + (float)row;
    sh = (T - 1.f) / T;
    rsh = T / (T - 1.f);
    eta = 1.f / (p.lam * T);
  } else {
    sh = p.shrink;
    rsh = p.rshrink;
    eta = 0.f;
  }
}

template <int RULE>
struct Step {
  // returns (loss, c) for margin m, label y, ‖x‖² n2; updates counters
  __device__ __forceinline__ static void run(float m, float y, float n2, float eta,
                                             const LinParams& p, float& loss_sum, float& mist,
                                             float& sqe, float& c) {
    if constexpr (RULE == kPegasos) {  // hinge sub-gradient step
      const float ym = y * m;
      loss_sum += fmaxf(0.f, 1.f - ym);
      mist += ym <= 0.f ? 1.f : 0.f;
      c = ym < 1.f ? eta * y : 0.f;
    } else if constexpr (RULE == kHinge) {
      const float ym = y * m;
      const float loss = fmaxf(0.f, 1.f - ym);
      loss_sum += loss;
      mist += ym <= 0.f ? 1.f : 0.f;
      const float tau = n2 > 0.f ? fminf(p.cclip, loss * __builtin_amdgcn_rcpf(n2 + p.kadd)) : 0.f;
      c = tau * y;
    } else if constexpr (RULE == kEpsInsensitive) {
      const float err = y - m;
      const float loss = fmaxf(0.f, fabsf(err) - p.eps);
      loss_sum += loss;
      sqe = fmaf(err, err, sqe);
      const float tau = n2 > 0.f ? fminf(p.cclip, loss * __builtin_amdgcn_rcpf(n2 + p.kadd)) : 0.f;
      c = err >= 0.f ? tau : -tau;
    } else {
      const float z = y * m;
      const float ez = __expf(-fabsf(z));
      loss_sum += fmaxf(-z, 0.f) + __logf(1.f + ez);
      mist += z <= 0.f ? 1.f : 0.f;
      // σ(−z) = 1/(1+e^z), computed from e^{−|z|} without overflow
      const float sg = z >= 0.f ? ez * __builtin_amdgcn_rcpf(1.f + ez) : __builtin_amdgcn_rcpf(1.f + ez);
      c = p.lr * y * sg;
    }
  }
};

// ablate (timing diagnostics only): bit0 skip the table flush, bit1 skip the sequential
// phase, bit2 skip the w0 gathers, bit3 skip the LDS table probes; bit4 selects this
// kernel where the register-dedup kernel (below) would run (exact either way).
template <int FPL, int CH, int RULE, typename NumT, typename WT>
__global__ __launch_bounds__(64) void linear_round_kernel(
    const WT* __restrict__ w, const NumT* __restrict__ num, int dn, const void* __restrict__ cat,
    int dc, const void* __restrict__ yv, int B, int R, int dim, float* __restrict__ ws,
    int2* __restrict__ tables, float* __restrict__ dacc, LinParams p, TableGeom g, int ablate,
    Spill sp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int cap = 1 << g.log2cap;
  const int tsz = cap + kOvf;
  int* keys = reinterpret_cast<int*>(smem);
  float* vals = reinterpret_cast<float*>(smem + (size_t)tsz * sizeof(int));
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
  for (int i = lane; i < tsz; i += kWave) {
    keys[i] = kEmptyKey;
    vals[i] = 0.f;
  }
  __syncthreads();

  const int bs_log2 = g.log2cap - g.log2nb;
  const uint32_t bmask = (1u << bs_log2) - 1u;
  int dcol[FPL];
  float dreg[FPL];
#pragma unroll
  for (int f = 0; f < FPL; ++f) {
    dcol[f] = dense_col(lane + kWave * f, dn, dc, p.bias);
    dreg[f] = 0.f;
  }
  float sigma = 1.f, rsig = 1.f, loss_sum = 0.f, nex = 0.f, mist = 0.f, sqe = 0.f, ovf = 0.f;

  // Software pipeline: the features of chunk c+1 are in flight while chunk c computes.
  int nidx[CH][FPL];
  float nxv[CH][FPL];
  float nyy[CH];
  // every load of a chunk is issued before any is decoded (branch-free, clamped rows)
  auto load_chunk = [&](int tc) {
    FeatRaw raw[CH][FPL];
    float yr[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int t = min(tc + e, t1 - 1);
      yr[e] = load_label(yv, t, p.y_i8);
#pragma unroll
      for (int f = 0; f < FPL; ++f)
        raw[e][f] = load_feature_raw(num, dn, cat, dc, t, lane + kWave * f, p.cspan);
    }
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const bool ok = tc + e < t1;
      nyy[e] = ok ? yr[e] : __builtin_nanf("");
#pragma unroll
      for (int f = 0; f < FPL; ++f)
        decode_feature(raw[e][f], dn, dc, lane + kWave * f, dim, p.bias, p.cspan, ok, nidx[e][f],
                       nxv[e][f]);
    }
  };
  load_chunk(t0);

  for (int tc = t0; tc < t1; tc += CH) {
    int slot[CH][FPL];
    float xv[CH][FPL];
    float wv[CH][FPL];
    float yy[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      yy[e] = nyy[e];
#pragma unroll
      for (int f = 0; f < FPL; ++f) {
        slot[e][f] = nidx[e][f];
        xv[e][f] = nxv[e][f];
      }
    }
    // Gather w0 for the whole chunk (read-only during the round).
#pragma unroll
    for (int e = 0; e < CH; ++e)
#pragma unroll
      for (int f = 0; f < FPL; ++f)
        wv[e][f] = (slot[e][f] >= 0 && !(ablate & 4)) ? to_f(w[slot[e][f]]) : 0.f;
    if (tc + CH < t1) load_chunk(tc + CH);
    // Resolve the LDS slots of hashed features. First probe: ONE 16-byte ds_read of the
    // four slots at the key's 4-aligned hashed start in its bucket per (row, feature), all
    // issued for the whole
    // chunk before any is consumed; a hit or a first-empty CAS settles almost every key,
    // the full-bucket / lost-race case takes the slow path (which scans the whole bucket,
    // so keys are found wherever either path inserted them).
    int b0[CH][FPL];
    int4 kq[CH][FPL];
#pragma unroll
    for (int e = 0; e < CH; ++e)
#pragma unroll
      for (int f = 0; f < FPL; ++f) {
        const int key = slot[e][f];
        b0[e][f] = ((key >> g.kshift) << bs_log2) + (int)((hmix((uint32_t)key) & bmask) & ~3u);
        kq[e][f] = (dcol[f] < 0 && key >= 0 && !(ablate & 8))
                       ? *reinterpret_cast<const int4*>(&keys[b0[e][f]])
                       : make_int4(0, 0, 0, 0);
      }
#pragma unroll
    for (int e = 0; e < CH; ++e)
#pragma unroll
      for (int f = 0; f < FPL; ++f) {
        const int key = slot[e][f];
        if (dcol[f] < 0 && key >= 0 && (ablate & 8)) {
          slot[e][f] = -1;  // diagnostics: no table slot
        } else if (dcol[f] < 0 && key >= 0) {
          const int4 q = kq[e][f];
          const int b = b0[e][f];
          int sl = q.x == key ? b : q.y == key ? b + 1 : q.z == key ? b + 2 : q.w == key ? b + 3 : -2;
          if (sl == -2) {
            const int j = q.x == kEmptyKey ? 0 : q.y == kEmptyKey ? 1 : q.z == kEmptyKey ? 2
                        : q.w == kEmptyKey ? 3 : -1;
            if (j >= 0) {
              const int prev = atomicCAS(&keys[b + j], kEmptyKey, key);
              if (prev == kEmptyKey || prev == key) sl = b + j;
            }
          }
          // lost a race to an earlier row of the chunk (stale view): re-read the four
          // slots and retry inline — rows of one chunk often share a bucket
          for (int r = 0; r < 3 && sl == -2; ++r) {
            const int4 q2 = *reinterpret_cast<const int4*>(&keys[b]);
            sl = q2.x == key ? b : q2.y == key ? b + 1 : q2.z == key ? b + 2
               : q2.w == key ? b + 3 : -2;
            if (sl != -2) break;
            const int j = q2.x == kEmptyKey ? 0 : q2.y == kEmptyKey ? 1 : q2.z == kEmptyKey ? 2
                        : q2.w == kEmptyKey ? 3 : -1;
            if (j < 0) break;  // the four slots are full: slow path
            const int prev = atomicCAS(&keys[b + j], kEmptyKey, key);
            if (prev == kEmptyKey || prev == key) sl = b + j;
          }
          if (sl == -2) sl = table_find_or_insert(keys, key, g);
          if (sl < 0) sl = spill_slot(sp, s, key, ovf);  // LDS table full: HBM spill
          slot[e][f] = sl;
        }
      }
    if (ablate & 2) {
#pragma unroll
      for (int e = 0; e < CH; ++e)
#pragma unroll
        for (int f = 0; f < FPL; ++f) loss_sum += wv[e][f] + xv[e][f] + (float)slot[e][f];
      continue;
    }
    // Exact sequential online updates. A chunk with spilled keys takes its own copy of
    // the loop (global reads and atomics on the chain, ordered row to row by vmcnt(0)); the
    // in-LDS copy keeps no global access between the rows.
    bool spl = false;
#pragma unroll
    for (int e = 0; e < CH; ++e)
#pragma unroll
      for (int f = 0; f < FPL; ++f) spl = spl || is_spill(slot[e][f]);
    auto rows = [&](auto spill_tag) {
      constexpr bool SPL = decltype(spill_tag)::value;
#pragma unroll
      for (int e = 0; e < CH; ++e) {
        const float y = yy[e];
        if (__builtin_isnan(y)) continue;  // wave-uniform
        float pm = 0.f, pn = 0.f;
#pragma unroll
        for (int f = 0; f < FPL; ++f) {
          const int sl = slot[e][f];
          float d = dcol[f] >= 0 ? dreg[f] : (sl >= 0 ? vals[sl] : 0.f);
          if constexpr (SPL)
            if (is_spill(sl)) d = spill_load(spill_vals<1>(sp, s, spill_index(sl)));
          pm = fmaf(xv[e][f], wv[e][f] + d, pm);
          pn = fmaf(xv[e][f], xv[e][f], pn);
        }
        wave_sum2(pm, pn);
        float c, sh, rsh, eta;
        row_rate<RULE>(p, tc - t0 + e, sh, rsh, eta);
        Step<RULE>::run(sigma * pm, y, pn, eta, p, loss_sum, mist, sqe, c);
        nex += 1.f;
        sigma *= sh;
        rsig *= rsh;
        if (c != 0.f) {  // wave-uniform
          const float cv = c * rsig;
#pragma unroll
          for (int f = 0; f < FPL; ++f) {
            const int sl = slot[e][f];
            if (dcol[f] >= 0) dreg[f] = fmaf(cv, xv[e][f], dreg[f]);
            else if (sl >= 0) atomicAdd(&vals[sl], cv * xv[e][f]);
            else if (SPL && is_spill(sl))
              atomicAdd(spill_vals<1>(sp, s, spill_index(sl)), cv * xv[e][f]);
          }
          if constexpr (SPL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
    };
    if (__builtin_amdgcn_ballot_w64(spl)) rows(SpillTag<true>{});
    else rows(SpillTag<false>{});
  }
  __syncthreads();
  // Round end: the bucketed table (σ·Δ/P per slot) goes out with plain coalesced stores
  // and linear_reduce_kernel sums it per key range — no global atomics on the hot path;
  // the (rare) overflow-area entries are added to the accumulator directly.
  const float scale = sigma * p.inv_p;
  if (!(ablate & 1)) {
    // group-major layout: the reducer of group q then streams one contiguous region
    // (slot i of spoke s → [q = i >> seg][s][i & (2^seg − 1)], full-line segments)
    const int seg_log2 = (g.log2cap - g.log2nb) + g.lgg;
    const size_t S_tot = gridDim.x;
    const int used = (int)min((long long)g.qused << seg_log2, (long long)cap);
    for (int i = lane; i < used; i += kWave) {
      const size_t q = (size_t)(i >> seg_log2);
      tables[((q * S_tot + s) << seg_log2) + (i & ((1 << seg_log2) - 1))] =
          make_int2(keys[i], __float_as_int(vals[i] * scale));
    }
    for (int i = cap + lane; i < tsz; i += kWave) {
      const int k = keys[i];
      const float v = vals[i] * scale;
      if (k >= 0 && v != 0.f) atomicAdd(&dacc[k], v);
    }
  }
  spill_flush<1>(sp, s, 1, dim, scale, dacc, lane);  // (restores the region even under ablate)
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

// Diagnostics only (csrc/tests/rd_stamp_probe.hip builds with OMLDM_RD_STAMPS): per-spoke
// phase timestamps of linear_round_rd_kernel, each after a full wait on the wave's
// memory operations, so a phase's time includes its latency.
#ifdef OMLDM_RD_STAMPS
__device__ unsigned long long* g_rd_stamps;
#define RD_STAMP(k)                                                              \
  do {                                                                           \
    __builtin_amdgcn_s_waitcnt(0);                                               \
    if (lane == 0) g_rd_stamps[(size_t)s * 8 + (k)] = (k) == 0 ? wall_clock64() : clock64(); \
  } while (0)
#else
#define RD_STAMP(k) \
  do {              \
  } while (0)
#endif

// Register-dedup round (field-aware compact wire, ≤ RMAX rows per spoke, ≤ 64 features).
//
// On the field-aware wire lane f only ever sees keys of field f (slot ranges of different
// fields, the numerical slots and the intercept are disjoint), so a spoke's delta for a
// key lives with ONE lane, and a spoke's R rows are few: the whole spoke fits in
// registers. Each lane keeps its R keys, values and round-start weights, and d[e] = the
// delta of row e's key as row e sees it. After row e's closed-form step u = c·x_e, the
// lane adds u to d[e'] of every later row e' with the same key (compile-time indices:
// plain VALU compares/selects, no LDS on the sequential chain, no hash probes, no CAS,
// no table overflow). This is the same per-key accumulation order as the LDS table, so
// the deltas are bitwise those of linear_round_kernel.
// At round end the last occurrence of each key holds its total delta; those go into an
// LDS staging image with the round kernel's bucketed layout (one LDS atomic counter per
// bucket; a bucket that is full sends its extra keys to the accumulator with an L2
// atomic — exact, nothing is dropped) and leave with the same coalesced group-major flush,
// so linear_reduce_kernel is unchanged.
#ifndef OMLDM_RD_OCC
#define OMLDM_RD_OCC 5  // waves per SIMD the register budget is sized for (diagnostics sweep)
#endif
template <int RMAX, int RULE, typename NumT, typename WT>
__global__ __launch_bounds__(64, OMLDM_RD_OCC) void linear_round_rd_kernel(
    const WT* __restrict__ w, const NumT* __restrict__ num, int dn, const void* __restrict__ cat,
    int dc, const void* __restrict__ yv, int B, int R, int dim, float* __restrict__ ws,
    int2* __restrict__ tables, float* __restrict__ dacc, LinParams p, TableGeom g, int ablate) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int cap = 1 << g.log2cap;
  const int nbk = 1 << g.log2nb;
  const int bs_log2 = g.log2cap - g.log2nb;
  int2* tab = reinterpret_cast<int2*>(smem);                     // [cap] staging image
  int* bcnt = reinterpret_cast<int*>(smem + (size_t)cap * 8);     // [nbk / 2] bucket fill
  int* dummy = bcnt + ((nbk + 1) >> 1);                           // [64] no-op atomics
  const int lane = threadIdx.x;
  const int s = blockIdx.x;
  const int wsw = kWsStat + dn + 1;
  float* wrow = ws + (size_t)s * wsw;
  RD_STAMP(0);
  RD_STAMP(1);
  const long long t0ll = (long long)s * R;
  const int t0 = t0ll > B ? B : (int)t0ll;
  const int t1 = (t0ll + R) > B ? B : (int)(t0ll + R);
  if (t0 >= t1) {  // idle spoke: not a worker of this round
    for (int k = lane; k < wsw; k += kWave) wrow[k] = k == 4 ? 1.f : 0.f;
    return;
  }
  // the spoke's rows, every load in flight at once (spoke_table.h: load_spoke_rows) — a
  // load inside a lane-divergent branch is waited for inside it, which serialised the
  // rows of the first version. Row e's label sits in lane e (one VGPR for all labels,
  // v_readlane on the chain).
  const float yraw = load_label(yv, min(t0 + lane, t1 - 1), p.y_i8);  // unconditional
  int key[RMAX];
  float xv[RMAX], wv[RMAX], d[RMAX];
  load_spoke_rows<RMAX>(num, dn, cat, dc, t0, t1, lane, dim, p.bias, p.cspan, key, xv);
#pragma unroll
  for (int e = 0; e < RMAX; ++e) d[e] = 0.f;
  const float ylane = lane < t1 - t0 ? yraw : __builtin_nanf("");
  RD_STAMP(2);
  // staging image init overlaps the gathers
  for (int i = lane; i < cap; i += kWave) tab[i] = make_int2(kEmptyKey, 0);
  for (int i = lane; i < (nbk + 1) >> 1; i += kWave) bcnt[i] = 0;
  // round-start weights (read-only for the round; the bf16 shadow sits in L2), gathered
  // unconditionally (absent features read slot 0 and are zeroed after)
  WT wraw[RMAX];
#pragma unroll
  for (int e = 0; e < RMAX; ++e) wraw[e] = w[key[e] >= 0 ? key[e] : 0];
#pragma unroll
  for (int e = 0; e < RMAX; ++e) wv[e] = key[e] >= 0 ? to_f(wraw[e]) : 0.f;
  RD_STAMP(3);
  const int dcol = dense_col(lane, dn, dc, p.bias);
  float sigma = 1.f, rsig = 1.f, loss_sum = 0.f, nex = 0.f, mist = 0.f, sqe = 0.f;
  // ‖x_e‖² does not depend on the updates: every row's norm first (independent
  // reductions, off the sequential chain)
  float pn[RMAX];
#pragma unroll
  for (int e = 0; e < RMAX; ++e) pn[e] = wave_sum(xv[e] * xv[e]);
  // exact sequential online updates, all in registers
#pragma unroll
  for (int e = 0; e < RMAX; ++e) {
    const float y = readlane_f(ylane, e);
    if (__builtin_isnan(y)) continue;  // wave-uniform (rows past t1 are NaN too)
    const float pm = wave_sum(xv[e] * (wv[e] + d[e]));
    float c, sh, rsh, eta;
    row_rate<RULE>(p, e, sh, rsh, eta);
    Step<RULE>::run(sigma * pm, y, pn[e], eta, p, loss_sum, mist, sqe, c);
    nex += 1.f;
    sigma *= sh;
    rsig *= rsh;
    if (c != 0.f) {  // wave-uniform
      const float u = (c * rsig) * xv[e];
      d[e] += u;
#pragma unroll
      for (int e2 = e + 1; e2 < RMAX; ++e2) d[e2] += key[e2] == key[e] ? u : 0.f;
    }
  }
  RD_STAMP(4);
  __syncthreads();  // staging image initialised
  const float scale = sigma * p.inv_p;
  float dense_total = 0.f, ovf = 0.f;
  // The last occurrence of a key carries its total delta. Its bucket position comes from
  // an LDS counter; every lane issues all RMAX counter atomics back to back (lanes with
  // nothing to place add 0 to a private dummy word: no branch to wait inside, no
  // same-address serialisation), then places its entries.
  int pos[RMAX];
  bool emit[RMAX];
#pragma unroll
  for (int e = 0; e < RMAX; ++e) {
    bool last = key[e] >= 0;
#pragma unroll
    for (int e2 = e + 1; e2 < RMAX; ++e2) last = last && key[e2] != key[e];
    last = last && d[e] != 0.f;
    if (dcol >= 0 && last) dense_total = d[e];
    emit[e] = last && dcol < 0 && !(ablate & 1);
    const int b = emit[e] ? key[e] >> g.kshift : 0;
    const int sh = 16 * (b & 1);
    // 16-bit counters, two buckets per word: a spoke has at most 64 × RMAX ≤ 1024 keys,
    // so a half-word never carries into its neighbour
    int* ctr = emit[e] ? &bcnt[b >> 1] : &dummy[lane];
    pos[e] = (atomicAdd(ctr, emit[e] ? 1 << sh : 0) >> sh) & 0xffff;
  }
#pragma unroll
  for (int e = 0; e < RMAX; ++e) {
    if (emit[e]) {
      const int b = key[e] >> g.kshift;
      const float v = d[e] * scale;
      if (pos[e] < (1 << bs_log2)) {
        tab[(b << bs_log2) + pos[e]] = make_int2(key[e], __float_as_int(v));
      } else {  // bucket full: straight to the accumulator (exact)
        unsafeAtomicAdd(&dacc[key[e]], v);
        ovf += 1.f;
      }
    }
  }
  __syncthreads();
  RD_STAMP(5);
  if (!(ablate & 1)) {
    const int seg_log2 = bs_log2 + g.lgg;
    const size_t S_tot = gridDim.x;
    const int used = min(cap, (int)min((long long)g.qused << seg_log2, (long long)cap));
    for (int i = lane; i < used; i += kWave) {
      const size_t q = (size_t)(i >> seg_log2);
      tables[((q * S_tot + s) << seg_log2) + (i & ((1 << seg_log2) - 1))] = tab[i];
    }
  }
  if (dcol >= 0) wrow[kWsStat + dcol] = dense_total * scale;
  (void)ovf;  // spilled keys went to the accumulator: nothing was dropped
  if (lane == 0) {
    wrow[0] = loss_sum;
    wrow[1] = nex;
    wrow[2] = mist;
    wrow[3] = sqe;
    wrow[4] = sigma;
    wrow[5] = 0.f;  // dropped updates (none on this path)
    wrow[6] = scale;
    wrow[7] = p.inv_p;
    if (!p.bias) wrow[kWsStat + dn] = 0.f;
  }
  RD_STAMP(6);
}

// Column sums of the per-spoke workspace (one block per column) → accumulator slots
// that every spoke would otherwise hit with same-address atomics:
//   dense columns → dacc[0:dn], intercept → dacc[dim-1], Σσ/P → dacc[dim],
//   Σ1/P → dacc[dim+1], loss/n/mistakes/sq_err/overflow → cum (device running totals).
template <int NT>
__device__ __forceinline__ void finish_column(int c, const float* __restrict__ ws, int S, int dn,
                                              int dim, float* __restrict__ dacc,
                                              double* __restrict__ cum) {
  __shared__ float part[NT / 64];
  const int wsw = kWsStat + dn + 1;
  float acc = 0.f;
  for (int s = threadIdx.x; s < S; s += NT) acc += ws[(size_t)s * wsw + c];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) t += part[k];
    if (c < kWsStat) {
      if (c == 6) dacc[dim] = t;       // the round's counters (apply does not clear them)
      else if (c == 7) dacc[dim + 1] = t;
      else if (c != 4 && cum) cum[c] += (double)t;
    } else {
      const int j = c - kWsStat;
      dacc[j < dn ? j : dim - 1] += t;
    }
  }
}

// One launch after the round kernel (or `parts` launches, see launch_reduce). Blocks
// [0, nb): `split` blocks per key group, group q0 + b / split; bucket b owns keys
// [b·2^kshift, (b+1)·2^kshift); it streams bucket b of every active spoke's table (BS
// consecutive int2 per spoke), accumulates into an LDS image with ds_add_f32 and adds its
// non-zero slots to the accumulator (which the apply pass left at zero; overflow entries
// were added by the round kernel). Blocks [nb, nb + wsw): workspace column sums. Hashed
// keys never map to dense / intercept slots, so the two block kinds touch disjoint slots.
template <int NT>
__global__ __launch_bounds__(NT) void linear_reduce_kernel(
    const int2* __restrict__ tables, int S_act, TableGeom g, int dim, float* __restrict__ dacc,
    int nb, int split, int q0, const float* __restrict__ ws, int S, int dn,
    double* __restrict__ cum, int hot) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if ((int)blockIdx.x >= nb) {
    finish_column<NT>(blockIdx.x - nb, ws, S, dn, dim, dacc, cum);
    return;
  }
  float* acc = reinterpret_cast<float*>(smem);
  const int span = 1 << (g.kshift + g.lgg);  // keys of the 2^lgg buckets of this group
  const int q = q0 + (int)blockIdx.x / split;  // key group
  const int part = (int)blockIdx.x % split;    // this block's share of the spokes
  const int s_lo = (int)(((long long)S_act * part) / split);
  const int s_hi = (int)(((long long)S_act * (part + 1)) / split);
  for (int i = threadIdx.x; i < span; i += NT) acc[i] = 0.f;
  __syncthreads();
  const int seg_log2 = (g.log2cap - g.log2nb) + g.lgg;
  const int lo = q << (g.kshift + g.lgg);
  // the group's region is contiguous ([group][spoke][segment]), so is every part of it:
  // (s_hi − s_lo) segments of 2^seg int2 → 16-byte loads (two slots), four in flight per
  // thread
  const long long items = (long long)(s_hi - s_lo) << (seg_log2 - 1);
  const int4* t4 = reinterpret_cast<const int4*>(tables) +
                   (((size_t)q * S + s_lo) << (seg_log2 - 1));
  // Software-pipelined: the next batch of 4 loads is in flight while this batch's entries
  // are added. Empty slots (key −1, most of a table) are skipped: LDS atomics are this
  // kernel's bound, and adding 0 to a dummy word for them instead (branch-free) measured
  // 26 → 46 µs.
  auto add = [&](int key, int val) {
    if (key >= 0) atomicAdd(&acc[key - lo], __int_as_float(val));
  };
  // Hot keys: a popular category sits in nearly every spoke's table, so the lanes of a
  // wave (consecutive spokes' segments of one bucket) often carry the same key, and the
  // LDS atomic serialises them. The wave takes its first valid lane's key; when at least
  // `hot` lanes share it, their values are summed across the wave (DPP) and added once.
  // Needs every lane of the wave active (the main loop below runs a wave-uniform count).
  const int lane = threadIdx.x & 63;
  auto add_wave = [&](int key, int val) {
    const unsigned long long vm = __ballot(key >= 0);
    if (vm == 0) return;
    const int first = __builtin_ctzll(vm);
    const int kc = __builtin_amdgcn_readlane(key, first);
    const unsigned long long hm = __ballot(key == kc);
    const float fv = __int_as_float(val);
    if (__builtin_popcountll(hm) >= hot) {
      const float sum = wave_sum(key == kc ? fv : 0.f);
      if (lane == first) atomicAdd(&acc[kc - lo], sum);
      if (key >= 0 && key != kc) atomicAdd(&acc[key - lo], fv);
    } else if (key >= 0) {
      atomicAdd(&acc[key - lo], fv);
    }
  };
  long long it = threadIdx.x;
  // full batches: it + 4·NT·b + 3·NT < items (the old loop's condition), evaluated for
  // the wave's last lane (the smallest count in the wave), so the count is wave-uniform;
  // the other lanes' remaining items go to the tail loop
  const long long full_t = items - it - 3 * NT > 0 ? (items - it - 3 * NT - 1) / (4 * NT) + 1 : 0;
  const long long full = (long long)__builtin_amdgcn_readlane((int)full_t, 63);
  int4 v[4];
  if (full > 0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = t4[it + u * NT];
  }
  for (long long b = 0; b < full; ++b) {
    int4 cur[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = v[u];
    it += 4 * NT;
    if (b + 1 < full) {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = t4[it + u * NT];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      add_wave(cur[u].x, cur[u].y);
      add_wave(cur[u].z, cur[u].w);
    }
  }
  for (; it < items; it += NT) {
    const int4 w4 = t4[it];
    add(w4.x, w4.y);
    add(w4.z, w4.w);
  }
  __syncthreads();
  if (split == 1) {  // sole owner of the key range
    for (int i = threadIdx.x; i < span; i += NT) {
      const int k = lo + i;
      const float v = acc[i];
      if (k < dim && v != 0.f) dacc[k] += v;
    }
  } else {  // the group's parts meet in L2 (hardware fp32 atomics, no return value)
    for (int i = threadIdx.x; i < span; i += NT) {
      const int k = lo + i;
      const float v = acc[i];
      if (k < dim && v != 0.f) unsafeAtomicAdd(&dacc[k], v);
    }
  }
}

// Buckets per reduce group (2^lgg). Measured at 8192 spokes × 1K tables, dim 2^20:
// lgg 0 → 0.135 ms/step (256 reduce blocks, each streaming its 256 KiB region), lgg 1 →
// 0.149, lgg 2 → 0.195 (64 blocks: too few to pull HBM bandwidth), so one bucket per group.
// Reduce blocks per key group. One block per group gives 256 blocks at dim 2^20: one per
// CU, four waves each, too few loads in flight to stream the 64 MiB of tables at HBM rate.
// Splitting the spokes of a group over several blocks (partial LDS images, combined with
// L2 atomics) raises the memory-level parallelism; see profiles/round1_ablation.md.
static inline int reduce_split(int ngroups, int S_act) {
  int sp = ngroups >= 1024 ? 1 : 4;
  if (const char* e = getenv("OMLDM_REDUCE_SPLIT")) sp = atoi(e);  // diagnostics sweep
  if (sp < 1) sp = 1;
  if (sp > 16) sp = 16;
  while (sp > 1 && sp > S_act) sp >>= 1;
  return sp;
}

// Lanes of a wave that must share a key before the reducer sums them across the wave
// instead of one LDS atomic each (OMLDM_REDUCE_HOT: A/B; 65 = never).
static inline int reduce_hot() {
  static const int h = [] {
    const char* e = getenv("OMLDM_REDUCE_HOT");
    return e ? atoi(e) : 4;
  }();
  return h;
}

// Threads per reduce block (diagnostics sweep: OMLDM_REDUCE_THREADS = 256 | 512 | 1024).
static inline int reduce_threads() {
  int nt = 256;
  if (const char* e = getenv("OMLDM_REDUCE_THREADS")) nt = atoi(e);
  return nt == 1024 ? 1024 : nt == 512 ? 512 : 256;
}

template <int NT>
static int launch_reduce_t(dim3 grid, size_t lds, hipStream_t st, const int2* tables, int S_act,
                           TableGeom g, int dim, float* dacc, int nb, int split, int q0,
                           const float* ws, int S, int dn, double* cum) {
  int e = check_dyn_lds((const void*)linear_reduce_kernel<NT>, lds);
  if (e) return e;
  hipLaunchKernelGGL(linear_reduce_kernel<NT>, grid, dim3(NT), lds, st, tables, S_act, g, dim, dacc,
                     nb, split, q0, ws, S, dn, cum, reduce_hot());
  return (int)hipGetLastError();
}

static int launch_reduce_nt(int nt, dim3 grid, size_t lds, hipStream_t st, const int2* tables,
                            int S_act, TableGeom g, int dim, float* dacc, int nb, int split, int q0,
                            const float* ws, int S, int dn, double* cum) {
  if (nt == 1024)
    return launch_reduce_t<1024>(grid, lds, st, tables, S_act, g, dim, dacc, nb, split, q0, ws, S,
                                 dn, cum);
  if (nt == 512)
    return launch_reduce_t<512>(grid, lds, st, tables, S_act, g, dim, dacc, nb, split, q0, ws, S,
                                dn, cum);
  return launch_reduce_t<256>(grid, lds, st, tables, S_act, g, dim, dacc, nb, split, q0, ws, S, dn,
                              cum);
}

static inline int reduce_lgg(int kshift, int log2nb) {
  (void)kshift;
  int lgg = 0;
  if (const char* e = getenv("OMLDM_REDUCE_LGG")) lgg = atoi(e);  // diagnostics sweep
  if (lgg < 0) lgg = 0;
  return lgg < log2nb ? lgg : log2nb;
}

// One wavefront per example; M stacked models (w + m*wstride) → out[t*M + m].
template <int FPL, typename NumT, typename WT>
__global__ __launch_bounds__(256) void linear_predict_kernel(
    const WT* __restrict__ w, long long wstride, int M, const NumT* __restrict__ num, int dn,
    const void* __restrict__ cat, int dc, int B, int dim, int bias, int cspan,
    const float* __restrict__ wscale, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int m = blockIdx.y;
  const WT* wm = w + (size_t)m * wstride;
  const float sc = wscale ? wscale[m] : 1.f;
  for (int t = wv; t < B; t += nwaves) {
    float acc = 0.f;
    FeatRaw raw[FPL];
#pragma unroll
    for (int f = 0; f < FPL; ++f) raw[f] = load_feature_raw(num, dn, cat, dc, t, lane + kWave * f, cspan);
#pragma unroll
    for (int f = 0; f < FPL; ++f) {
      int idx;
      float v;
      decode_feature(raw[f], dn, dc, lane + kWave * f, dim, bias, cspan, true, idx, v);
      acc = fmaf(v, to_f(wm[idx >= 0 ? idx : 0]), acc);  // v = 0 when absent
    }
    acc = wave_sum(acc);
    if (lane == 0) out[(size_t)t * M + m] = acc * sc;
  }
}

// Model average over the round's active workers:
//   w = (a·w + D) / n,  a = D[dim] = Σσ/P, n = D[dim+1] = Σ1/P  (n == 0: no change;
//   n < 0: a round its kernel marked failed — w unchanged, D cleared);
// D[0:dim] = 0 (D[dim:dim+2] are overwritten by the next round's finish kernel);
// optional bf16 shadow of w for the gathers of the next round.
__device__ __forceinline__ void linear_apply_body(float* __restrict__ w32,
                                                  __hip_bfloat16* __restrict__ w16,
                                                  float* __restrict__ dacc, int dim) {
  const float n = dacc[dim + 1];
  const float a = n > 0.f ? dacc[dim] : 1.f;
  const float r = n > 0.f ? 1.f / n : 1.f;
  const bool keep = !(n < 0.f);  // (discard: D counts for nothing, NaN garbage included)
  const int n4 = dim >> 2;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int stride = gridDim.x * blockDim.x;
  float4* w4 = reinterpret_cast<float4*>(w32);
  float4* d4 = reinterpret_cast<float4*>(dacc);
  for (int i = tid; i < n4; i += stride) {
    float4 wv = w4[i];
    float4 dv = d4[i];
    if (!keep) dv = make_float4(0.f, 0.f, 0.f, 0.f);
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
    const float v = fmaf(a, w32[i], keep ? dacc[i] : 0.f) * r;
    w32[i] = v;
    dacc[i] = 0.f;
    if (w16) w16[i] = __float2bfloat16(v);
  }
}

__global__ __launch_bounds__(256) void linear_apply_kernel(float* __restrict__ w32,
                                                           __hip_bfloat16* __restrict__ w16,
                                                           float* __restrict__ dacc, int dim) {
  linear_apply_body(w32, w16, dacc, dim);
}

// M models of one dimension in one launch (grid.y = model): the pipelines of one fused
// round (BASELINE config 5) — M launches of ~5 µs each, with the gaps between them, were
// ~85 µs of a 16-pipeline step.
constexpr int kApplyMaxM = 16;
struct ApplyPtrs {
  float* w32[kApplyMaxM];
  __hip_bfloat16* w16[kApplyMaxM];
  float* dacc[kApplyMaxM];
};
__global__ __launch_bounds__(256) void linear_apply_multi_kernel(ApplyPtrs P, int dim) {
  const int m = blockIdx.y;
  linear_apply_body(P.w32[m], P.w16[m], P.dacc[m], dim);
}

// Key range [lo, hi) of the accumulator that reduce part `part` of `parts` completes:
// part k owns key groups [ng·k/parts, ng·(k+1)/parts). Part 0 also runs the workspace
// column sums, so it completes dacc[0:dn], and the last part extends to dim + 2 (the
// intercept slot dim − 1 and the round counters dacc[dim:dim+2], written by part 0's
// finish blocks earlier in stream order). Independent of the table size: every rank
// derives the same slices from dim alone.
static void part_bounds(int dim, TableGeom g, int part, int parts, long long* lo, long long* hi) {
  const int gspan_log2 = g.kshift + g.lgg;
  const long long ng = ((long long)dim + (1LL << gspan_log2) - 1) >> gspan_log2;
  const long long q0 = ng * part / parts, q1 = ng * (part + 1) / parts;
  *lo = part == 0 ? 0 : q0 << gspan_log2;
  *hi = part == parts - 1 ? (long long)dim + 2 : q1 << gspan_log2;
  if (*hi > (long long)dim + 2) *hi = (long long)dim + 2;
}

// Reduce part `part` of `parts` (parts == 1: the whole reduce in one launch). With
// parts > 1 the caller issues the collective of each part's key range right after that
// part's launch, so the all-reduce of part k runs on the RCCL stream while part k+1
// reduces (protocols.Synchronous, reduce_parts).
static int launch_reduce(const int2* tables, int B, int R, int S, TableGeom g, int dim,
                         float* dacc, const float* ws, int dn, double* cum, int part, int parts,
                         int ablate, hipStream_t st) {
  const long long sact_ll = R > 0 ? ((long long)B + R - 1) / R : 0;
  const int S_act = sact_ll < S ? (int)sact_ll : S;
  const int gspan_log2 = g.kshift + g.lgg;
  const int ng = (!(ablate & 1) && S_act > 0) ? (dim + (1 << gspan_log2) - 1) >> gspan_log2 : 0;
  const int q0 = (int)((long long)ng * part / parts);
  // part slices follow dim alone (every rank agrees); groups past qused hold no keys
  const int q1 = min((int)((long long)ng * (part + 1) / parts), max(q0, g.qused));
  const int split = ng ? reduce_split(ng, S_act) : 1;
  const int nb = (q1 - q0) * split;
  const int nfin = part == 0 ? kWsStat + dn + 1 : 0;
  if (nb + nfin == 0) return 0;
  const size_t rlds = nb ? (size_t(1) << gspan_log2) * 4 : 0;
  return launch_reduce_nt(reduce_threads(), dim3(nb + nfin), rlds, st, tables, S_act, g, dim, dacc,
                          nb, split, q0, ws, S, dn, cum);
}

int bucket_reduce_launch(const int2* tables, int S_act, int S, TableGeom g, int dim,
                         float* dacc, int q0, int q1, hipStream_t st) {
  if (S_act <= 0 || q1 <= q0) return 0;
  const int gspan_log2 = g.kshift + g.lgg;
  const int ng = (dim + (1 << gspan_log2) - 1) >> gspan_log2;
  const int split = reduce_split(ng, S_act);
  const int nb = (q1 - q0) * split;
  const size_t rlds = (size_t(1) << gspan_log2) * 4;
  return launch_reduce_nt(256, dim3(nb), rlds, st, tables, S_act, g, dim, dacc, nb, split, q0,
                          (const float*)nullptr, S, 0, (double*)nullptr);
}

template <int FPL, int CH, int RULE, typename NumT, typename WT>
static int launch_round(const void* w, const void* num, int dn, const void* cat, int dc,
                        const void* y, int B, int R, int S, float* dacc, int dim, float* ws,
                        int2* tables, double* cum, const LinParams& p, TableGeom g, int ablate,
                        int parts, const Spill& sp, hipStream_t st) {
  auto fn = linear_round_kernel<FPL, CH, RULE, NumT, WT>;
  const size_t lds = ((size_t(1) << g.log2cap) + kOvf) * 8;
  int e = check_dyn_lds((const void*)fn, lds);
  if (e) return e;
  hipLaunchKernelGGL(fn, dim3(S), dim3(64), lds, st, (const WT*)w, (const NumT*)num, dn, cat, dc,
                     y, B, R, dim, ws, tables, dacc, p, g, ablate, sp);
  e = (int)hipGetLastError();
  if (e) return e;
  return launch_reduce(tables, B, R, S, g, dim, dacc, ws, dn, cum, 0, parts, ablate, st);
}

template <int RMAX, int RULE, typename NumT, typename WT>
static int launch_round_rd(const void* w, const void* num, int dn, const void* cat, int dc,
                           const void* y, int B, int R, int S, float* dacc, int dim, float* ws,
                           int2* tables, double* cum, const LinParams& p, TableGeom g, int ablate,
                           int parts, hipStream_t st) {
  auto fn = linear_round_rd_kernel<RMAX, RULE, NumT, WT>;
  const size_t lds =
      (size_t(1) << g.log2cap) * 8 + (((size_t(1) << g.log2nb) + 1) / 2) * 4 + kWave * 4;
  int e = check_dyn_lds((const void*)fn, lds);
  if (e) return e;
  hipLaunchKernelGGL(fn, dim3(S), dim3(64), lds, st, (const WT*)w, (const NumT*)num, dn, cat, dc,
                     y, B, R, dim, ws, tables, dacc, p, g, ablate);
  e = (int)hipGetLastError();
  if (e) return e;
  return launch_reduce(tables, B, R, S, g, dim, dacc, ws, dn, cum, 0, parts, ablate, st);
}

// Register-dedup path (linear_round_rd_kernel): field-aware compact wire, ≤ 64 features,
// ≤ 16 rows per spoke. ablate bit 4 (or OMLDM_LINEAR_RD=0) forces the LDS-hash-table
// kernel (A/B and equality tests).
static bool use_rd_path(int cspan, int F, int R, int ablate) {
  if (cspan <= 0 || F > 64 || R > 16 || R < 1 || (ablate & 16)) return false;
  const char* e = getenv("OMLDM_LINEAR_RD");
  return !(e && atoi(e) == 0);
}

template <int RULE>
static int dispatch_round_rd(const void* w, int w_bf16, const void* num, int num_bf16, int dn,
                             const void* cat, int dc, const void* y, int B, int R, int S,
                             float* dacc, int dim, float* ws, int2* tables, double* cum,
                             const LinParams& p, TableGeom g, int ablate, int parts,
                             const Spill& sp, hipStream_t st) {
  (void)sp;  // the register-dedup round never drops: a full bucket adds to dacc directly
#define OMLDM_RD(RM, NT, WTT)                                                                  \
  return launch_round_rd<RM, RULE, NT, WTT>(w, num, dn, cat, dc, y, B, R, S, dacc, dim, ws,  \
                                            tables, cum, p, g, ablate, parts, st)
#define OMLDM_RD_R(NT, WTT) \
  if (R <= 8) OMLDM_RD(8, NT, WTT); \
  OMLDM_RD(16, NT, WTT)
  if (num_bf16) {
    if (w_bf16) { OMLDM_RD_R(__hip_bfloat16, __hip_bfloat16); }
    OMLDM_RD_R(__hip_bfloat16, float);
  }
  if (w_bf16) { OMLDM_RD_R(float, __hip_bfloat16); }
  OMLDM_RD_R(float, float);
#undef OMLDM_RD_R
#undef OMLDM_RD
}

template <int FPL, int CH, int RULE>
static int dispatch_round(const void* w, int w_bf16, const void* num, int num_bf16, int dn,
                          const void* cat, int dc, const void* y, int B, int R, int S, float* dacc,
                          int dim, float* ws, int2* tables, double* cum, const LinParams& p,
                          TableGeom g, int ablate, int parts, const Spill& sp, hipStream_t st) {
#define OMLDM_LR(NT, WTT)                                                                      \
  return launch_round<FPL, CH, RULE, NT, WTT>(w, num, dn, cat, dc, y, B, R, S, dacc, dim, ws, \
                                              tables, cum, p, g, ablate, parts, sp, st)
  if (num_bf16) {
    if (w_bf16) OMLDM_LR(__hip_bfloat16, __hip_bfloat16);
    OMLDM_LR(__hip_bfloat16, float);
  }
  if (w_bf16) OMLDM_LR(float, __hip_bfloat16);
  OMLDM_LR(float, float);
#undef OMLDM_LR
}

template <int FPL, int CH>
static int dispatch_rule(int rule, const void* w, int w_bf16, const void* num, int num_bf16,
                         int dn, const void* cat, int dc, const void* y, int B, int R, int S,
                         float* dacc, int dim, float* ws, int2* tables, double* cum,
                         const LinParams& p, TableGeom g, int ablate, int parts,
                         const Spill& sp, hipStream_t st) {
  if (FPL == 1 && use_rd_path(p.cspan, dn + dc + (p.bias ? 1 : 0), R, ablate)) {
    if (rule == kHinge)
      return dispatch_round_rd<kHinge>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc,
                                       dim, ws, tables, cum, p, g, ablate, parts, sp, st);
    if (rule == kEpsInsensitive)
      return dispatch_round_rd<kEpsInsensitive>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S,
                                                dacc, dim, ws, tables, cum, p, g, ablate, parts,
                                                sp, st);
    if (rule == kPegasos)
      return dispatch_round_rd<kPegasos>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc,
                                         dim, ws, tables, cum, p, g, ablate, parts, sp, st);
    return dispatch_round_rd<kLogistic>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc,
                                        dim, ws, tables, cum, p, g, ablate, parts, sp, st);
  }
  if (rule == kHinge)
    return dispatch_round<FPL, CH, kHinge>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc,
                                           dim, ws, tables, cum, p, g, ablate, parts, sp, st);
  if (rule == kEpsInsensitive)
    return dispatch_round<FPL, CH, kEpsInsensitive>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R,
                                                    S, dacc, dim, ws, tables, cum, p, g, ablate,
                                                    parts, sp, st);
  if (rule == kPegasos)
    return dispatch_round<FPL, CH, kPegasos>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S,
                                             dacc, dim, ws, tables, cum, p, g, ablate, parts, sp, st);
  return dispatch_round<FPL, CH, kLogistic>(w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S,
                                            dacc, dim, ws, tables, cum, p, g, ablate, parts, sp, st);
}

template <int FPL, typename NumT, typename WT>
static int launch_predict(const void* w, long long wstride, int M, const void* num, int dn,
                          const void* cat, int dc, int B, int dim, int bias, int cspan,
                          const float* wscale,
                          float* out, hipStream_t st) {
  const int waves = B < 1 ? 1 : B;
  int blocks = (waves + 3) / 4;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL((linear_predict_kernel<FPL, NumT, WT>), dim3(blocks, M), dim3(256), 0, st,
                     (const WT*)w, wstride, M, (const NumT*)num, dn, cat, dc, B, dim, bias, cspan, wscale, out);
  return (int)hipGetLastError();
}

template <int FPL>
static int dispatch_predict(const void* w, int w_bf16, long long wstride, int M, const void* num,
                            int num_bf16, int dn, const void* cat, int dc, int B, int dim, int bias,
                            int cspan, const float* wscale, float* out, hipStream_t st) {
  if (num_bf16) {
    if (w_bf16)
      return launch_predict<FPL, __hip_bfloat16, __hip_bfloat16>(w, wstride, M, num, dn, cat, dc,
                                                                 B, dim, bias, cspan, wscale, out,
                                                                 st);
    return launch_predict<FPL, __hip_bfloat16, float>(w, wstride, M, num, dn, cat, dc, B, dim, bias, cspan,
                                                      wscale, out, st);
  }
  if (w_bf16)
    return launch_predict<FPL, float, __hip_bfloat16>(w, wstride, M, num, dn, cat, dc, B, dim, bias, cspan,
                                                      wscale, out, st);
  return launch_predict<FPL, float, float>(w, wstride, M, num, dn, cat, dc, B, dim, bias, cspan, wscale,
                                           out, st);
}

}  // namespace omldm

using namespace omldm;

static int ceil_log2(long long x) {
  int k = 0;
  while ((1LL << k) < x) ++k;
  return k;
}

// Key groups that can hold hashed keys: all of them, except on the field-aware wire
// (cspan > 0), whose categorical slots end at dn + dc·cspan.
static int used_groups(int dim, int dn, int dc, int cspan, const TableGeom& g) {
  const int gl = g.kshift + g.lgg;
  const long long hi = cspan > 0 ? (long long)dn + (long long)dc * cspan : (long long)dim;
  const long long lim = hi < dim ? hi : dim;
  return (int)((lim + (1LL << gl) - 1) >> gl);
}

// Table geometry for a hash dimension: bucket span ≤ 4096 keys (16 KiB LDS in the
// reducer), ≥ 4 slots per bucket. Returns false when log2cap is too small.
OMLDM_API int omldm_linear_table_geom(int dim, int log2cap, int* out3) {
  const int ld = ceil_log2(dim);
  int kbase = 12;
  if (const char* e = getenv("OMLDM_KSHIFT")) kbase = atoi(e);  // diagnostics sweep
  const int kshift = ld < kbase ? ld : kbase;
  const int log2nb = ld - kshift;
  if (log2cap - log2nb < 2) return -1;
  out3[0] = log2cap;
  out3[1] = log2nb;
  out3[2] = kshift;
  return 0;
}

namespace omldm {
int bucket_geom(int dim, int log2cap, TableGeom* g) {
  int geo[3];
  if (omldm_linear_table_geom(dim, log2cap, geo)) return -1;
  *g = TableGeom{geo[0], geo[1], geo[2], reduce_lgg(geo[2], geo[1])};
  if ((g->log2cap - g->log2nb) + g->lgg < 1) return -1;
  return 0;
}
}  // namespace omldm

// 4-byte words of the HBM spill of S spokes (spoke_table.h: Spill), VK floats per entry.
OMLDM_API long long omldm_spill_words(int S, int log2gcap, int VK) {
  return (long long)spill_words(S, log2gcap, VK);
}

// tables: device scratch of S * ((1 << log2cap) + 64) int2; spill: omldm_spill_words(S,
// log2gcap, 1) words (keys −1, the rest 0 when allocated; every round leaves it so).
OMLDM_API int omldm_linear_round(const void* w, int w_bf16, const void* num, int num_bf16, int dn,
                                 const void* cat, int dc, const void* y, int y_i8, int B,
                                 int R, int S, float* dacc, int dim, float* ws, void* tables,
                                 double* cum, int rule, int variant, float C, float eps, float lr,
                                 float lam, float inv_p, int bias, int cspan, int log2cap,
                                 int chunk, int ablate, int parts, float tbase, void* spill,
                                 int log2gcap, void* stream) {
  if (S <= 0) return 0;
  if (spill == nullptr || log2gcap < 6 || log2gcap > 24) return -6;  // the HBM spill is required
  if (log2cap < 4 || log2cap > 14) return -1;  // ≤ 128 KiB of LDS per spoke
  if (rule == kPegasos && !(lam > 0.f && tbase >= 2.f)) return -5;
  if (parts < 1 || parts > 64) return -4;
  int geo[3];
  if (omldm_linear_table_geom(dim, log2cap, geo)) return -3;
  TableGeom g{geo[0], geo[1], geo[2], reduce_lgg(geo[2], geo[1])};
  if ((g.log2cap - g.log2nb) + g.lgg < 1) return -3;  // ≥ 2 slots per segment (int4 loads)
  g.qused = used_groups(dim, dn, dc, cspan, g);
  const float shrink = rule == kLogistic ? 1.f - lr * lam : 1.f - lam;
  const LinParams p{rule, variant, C, eps, lr, lam, inv_p, bias, cspan,
                    variant == kPA1 ? C : INFINITY, variant == kPA2 ? 0.5f / C : 0.f, shrink,
                    1.f / shrink, y_i8 ? 1 : 0, tbase};
  const int F = dn + dc + (bias ? 1 : 0);
  hipStream_t st = (hipStream_t)stream;
  int2* tb = (int2*)tables;
  const Spill sp = make_spill(spill, S, log2gcap, 1);
  if (F <= 64 && chunk <= 8) return dispatch_rule<1, 8>(rule, w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc, dim, ws, tb, cum, p, g, ablate, parts, sp, st);
  if (F <= 64) return dispatch_rule<1, 16>(rule, w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc, dim, ws, tb, cum, p, g, ablate, parts, sp, st);
  if (F <= 128) return dispatch_rule<2, 8>(rule, w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc, dim, ws, tb, cum, p, g, ablate, parts, sp, st);
  if (F <= 256) return dispatch_rule<4, 4>(rule, w, w_bf16, num, num_bf16, dn, cat, dc, y, B, R, S, dacc, dim, ws, tb, cum, p, g, ablate, parts, sp, st);
  return -2;
}

// Reduce part `part` (1 ≤ part < parts) of the round launched by omldm_linear_round with
// the same arguments; part 0 was launched by the round call itself.
OMLDM_API int omldm_linear_reduce_part(void* tables, float* ws, double* cum, float* dacc, int dim,
                                       int dn, int dc, int cspan, int B, int R, int S,
                                       int log2cap, int part, int parts, int ablate,
                                       void* stream) {
  if (S <= 0) return 0;
  if (parts < 1 || parts > 64 || part < 1 || part >= parts) return -4;
  int geo[3];
  if (omldm_linear_table_geom(dim, log2cap, geo)) return -3;
  TableGeom g{geo[0], geo[1], geo[2], reduce_lgg(geo[2], geo[1])};
  g.qused = used_groups(dim, dn, dc, cspan, g);
  return launch_reduce((const int2*)tables, B, R, S, g, dim, dacc, ws, dn, cum, part, parts,
                       ablate, (hipStream_t)stream);
}

// Accumulator slice [lo, hi) completed by reduce part `part` of `parts` (see part_bounds).
OMLDM_API int omldm_linear_part_bounds(int dim, int part, int parts, long long* lo_hi) {
  if (parts < 1 || part < 0 || part >= parts) return -4;
  int geo[3];
  const int ld = ceil_log2(dim);
  if (omldm_linear_table_geom(dim, ld + 2, geo)) return -3;  // kshift/log2nb depend on dim only
  const TableGeom g{geo[0], geo[1], geo[2], reduce_lgg(geo[2], geo[1])};
  part_bounds(dim, g, part, parts, &lo_hi[0], &lo_hi[1]);
  return 0;
}

OMLDM_API int omldm_linear_predict(const void* w, int w_bf16, long long wstride, int M,
                                   const void* num, int num_bf16, int dn, const void* cat, int dc,
                                   int B, int dim, int bias, int cspan, const float* wscale,
                                   float* out, void* stream) {
  if (B <= 0 || M <= 0) return 0;
  const int F = dn + dc + (bias ? 1 : 0);
  hipStream_t st = (hipStream_t)stream;
  if (F <= 64) return dispatch_predict<1>(w, w_bf16, wstride, M, num, num_bf16, dn, cat, dc, B, dim, bias, cspan, wscale, out, st);
  if (F <= 128) return dispatch_predict<2>(w, w_bf16, wstride, M, num, num_bf16, dn, cat, dc, B, dim, bias, cspan, wscale, out, st);
  if (F <= 256) return dispatch_predict<4>(w, w_bf16, wstride, M, num, num_bf16, dn, cat, dc, B, dim, bias, cspan, wscale, out, st);
  return -2;
}

OMLDM_API int omldm_linear_apply_multi(int M, float* const* w32, void* const* w16,
                                       float* const* dacc, int dim, void* stream) {
  if (M < 1 || M > kApplyMaxM) return -2;
  ApplyPtrs P{};
  for (int m = 0; m < M; ++m) {
    P.w32[m] = w32[m];
    P.w16[m] = static_cast<__hip_bfloat16*>(w16[m]);
    P.dacc[m] = dacc[m];
  }
  int blocks = (dim / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(linear_apply_multi_kernel, dim3(blocks, M), dim3(256), 0,
                     (hipStream_t)stream, P, dim);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_linear_apply(float* w32, void* w16, float* dacc, int dim, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int blocks = (dim / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(linear_apply_kernel, dim3(blocks), dim3(256), 0, st, w32,
                     (__hip_bfloat16*)w16, dacc, dim);
  return (int)hipGetLastError();
}
