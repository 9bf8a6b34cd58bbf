// MultiClassPA on hashed features — K prototype vectors W[K][dim], virtual spokes.
//
// Reference learner name "MultiClassPA" (omldm/utils/parsers/requestStream/
// PipelineMap.scala:68); rule (Crammer et al. 2006):
//   r = argmax_{k≠y} w_k·x,  ℓ = max(0, 1 − (w_y − w_r)·x),
//   τ = ℓ/(2‖x‖²) (PA), min(C, ℓ/(2‖x‖²)) (PA-I), ℓ/(2‖x‖² + 1/(2C)) (PA-II),
//   w_y += τx,  w_r −= τx.
//
// Same machinery as the binary learners (linear_spoke.hip, spoke_table.h): one wavefront
// per virtual spoke, lane = feature, exact sequential updates over the spoke's rows.
//  * The spoke's private deltas live in a bucketed LDS table keyed by feature with K
//    floats per slot, so the K deltas of a feature come back in one vector LDS read on
//    the sequential chain.
//  * Rows, the K round-start prototype gathers and the slot probes (16-byte first probe
//    of four slots, inline retry, slow path) of a chunk of CH rows are issued before the
//    chunk's sequential part, rows one chunk ahead.
//  * Dense features (numerical + intercept) keep their K deltas in registers and leave
//    through a per-spoke workspace row whose columns one small kernel sums — no
//    same-address atomics from thousands of spokes.
//  * Round end: class k of the table is flushed group-major into its own region and
//    summed by the shared bucket reducer into dacc[k]; multiclass_apply then averages
//    over the active spokes.
#include "spoke_table.h"

namespace omldm {

constexpr int kMcStat = 8;  // ws row: loss, n, mistakes, active, -, overflow, -, -, K×(dn+1) dense

// Slot of hashed key `key` (find or insert): one 16-byte read of the four slots at the
// key's 4-aligned hashed start in its bucket, CAS into the first empty one, inline
// re-reads when another lane won it, then the slow path (same probe order, so a key is
// never inserted twice); a key the LDS table cannot take goes to the spoke's HBM spill
// (spoke_table.h), so no update is dropped.
__device__ __forceinline__ int mc_slot(int* keys, int key, int b, int4 q, TableGeom g,
                                       const Spill& sp, int s, float& ovf) {
  int sl = q.x == key ? b : q.y == key ? b + 1 : q.z == key ? b + 2 : q.w == key ? b + 3 : -2;
  if (sl == -2) {
    const int j = q.x == kEmptyKey ? 0 : q.y == kEmptyKey ? 1 : q.z == kEmptyKey ? 2
                : q.w == kEmptyKey ? 3 : -1;
    if (j >= 0) {
      const int prev = atomicCAS(&keys[b + j], kEmptyKey, key);
      if (prev == kEmptyKey || prev == key) sl = b + j;
    }
  }
  for (int r = 0; r < 3 && sl == -2; ++r) {
    const int4 q2 = *reinterpret_cast<const int4*>(&keys[b]);
    sl = q2.x == key ? b : q2.y == key ? b + 1 : q2.z == key ? b + 2 : q2.w == key ? b + 3 : -2;
    if (sl != -2) break;
    const int j = q2.x == kEmptyKey ? 0 : q2.y == kEmptyKey ? 1 : q2.z == kEmptyKey ? 2
                : q2.w == kEmptyKey ? 3 : -1;
    if (j < 0) break;
    const int prev = atomicCAS(&keys[b + j], kEmptyKey, key);
    if (prev == kEmptyKey || prev == key) sl = b + j;
  }
  if (sl == -2) sl = table_find_or_insert(keys, key, g);
  if (sl < 0) sl = spill_slot(sp, s, key, ovf);  // LDS table full: the HBM spill
  return sl;
}

// The K round-start prototype weights of one key from the key-major shadow Wt[dim][K]
// (fp32 or bf16): one or a few vector loads, one cache line, instead of K gathers 4 MiB
// apart in W[K][dim].
template <int K>
__device__ __forceinline__ void load_protos(const float* __restrict__ Wt, int idx, float (&o)[K]) {
  if constexpr (K == 2) {
    const float2 v = *reinterpret_cast<const float2*>(Wt + (size_t)idx * 2);
    o[0] = v.x;
    o[1] = v.y;
  } else {
#pragma unroll
    for (int k = 0; k < K; k += 4) {
      const float4 v = *reinterpret_cast<const float4*>(Wt + (size_t)idx * K + k);
      o[k] = v.x; o[k + 1] = v.y; o[k + 2] = v.z; o[k + 3] = v.w;
    }
  }
}
template <int K>
__device__ __forceinline__ void load_protos(const __hip_bfloat16* __restrict__ Wt, int idx,
                                            float (&o)[K]) {
  auto lo = [](uint32_t u) { return __uint_as_float(u << 16); };
  auto hi = [](uint32_t u) { return __uint_as_float(u & 0xffff0000u); };
  if constexpr (K == 2) {
    const uint32_t v = *reinterpret_cast<const uint32_t*>(Wt + (size_t)idx * 2);
    o[0] = lo(v);
    o[1] = hi(v);
  } else {
#pragma unroll
    for (int k = 0; k < K; k += 4) {
      const uint2 v = *reinterpret_cast<const uint2*>(Wt + (size_t)idx * K + k);
      o[k] = lo(v.x); o[k + 1] = hi(v.x); o[k + 2] = lo(v.y); o[k + 3] = hi(v.y);
    }
  }
}

template <int K, int CH, typename NumT, typename WT>
__global__ __launch_bounds__(64) void multiclass_round_kernel(
    const WT* __restrict__ Wt, const NumT* __restrict__ num, int dn, const void* __restrict__ cat,
    int dc, int cspan, const void* __restrict__ yv, int y_i8, int B, int R, int dim, int nclass,
    int variant, float C, int bias, float* __restrict__ ws, int2* __restrict__ tables,
    float* __restrict__ dacc, TableGeom g, int ablate, int compact, Spill sp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int cap = 1 << g.log2cap;
  const int tsz = cap + kOvf;
  int* keys = reinterpret_cast<int*>(smem);
  float* vals = reinterpret_cast<float*>(smem + (size_t)tsz * sizeof(int));  // [tsz][K]
  const int lane = threadIdx.x;
  const int s = blockIdx.x;
  const int wsw = kMcStat + nclass * (dn + 1);
  float* wrow = ws + (size_t)s * wsw;
  const long long t0ll = (long long)s * R;
  const int t0 = t0ll > B ? B : (int)t0ll;
  const int t1 = (t0ll + R) > B ? B : (int)(t0ll + R);
  if (t0 >= t1) {  // idle spoke: not a worker this round
    for (int k = lane; k < wsw; k += kWave) wrow[k] = 0.f;
    return;
  }
  for (int i = lane; i < tsz; i += kWave) {
    keys[i] = kEmptyKey;
#pragma unroll
    for (int k = 0; k < K; ++k) vals[(size_t)i * K + k] = 0.f;
  }
  __syncthreads();
  const int bs_log2 = g.log2cap - g.log2nb;
  const uint32_t bmask = (1u << bs_log2) - 1u;
  const int dcol = lane < dn ? lane : ((bias && lane == dn + dc) ? dn : -1);
  float dreg[K];
#pragma unroll
  for (int k = 0; k < K; ++k) dreg[k] = 0.f;
  float loss_sum = 0.f, nex = 0.f, mist = 0.f, ovf = 0.f;

  int nidx[CH];
  float nxv[CH], nyy[CH];
  // every load of a chunk is issued before any is decoded (branch-free, clamped rows)
  auto load_chunk = [&](int tc) {
    FeatRaw raw[CH];
    float yr[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int t = min(tc + e, t1 - 1);
      yr[e] = load_label(yv, t, y_i8);
      raw[e] = load_feature_raw(num, dn, cat, dc, t, lane, cspan);
    }
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const bool ok = tc + e < t1;
      nyy[e] = ok ? yr[e] : __builtin_nanf("");
      decode_feature(raw[e], dn, dc, lane, dim, bias, cspan, ok, nidx[e], nxv[e]);
    }
  };
  load_chunk(t0);
  for (int tc = t0; tc < t1; tc += CH) {
    int idx[CH], slot[CH];
    float xv[CH], yy[CH], wv[CH][K];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      idx[e] = nidx[e];
      xv[e] = nxv[e];
      yy[e] = nyy[e];
    }
    // round-start prototypes of the whole chunk (read-only during the round)
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      if (idx[e] >= 0) {
        load_protos<K>(Wt, idx[e], wv[e]);
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) wv[e][k] = 0.f;
      }
    }
    if (tc + CH < t1) load_chunk(tc + CH);
    // slots of the chunk's hashed features: all first probes issued, then resolved
    int b0[CH];
    int4 kq[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int key = idx[e];
      b0[e] = ((key >> g.kshift) << bs_log2) + (int)((hmix((uint32_t)key) & bmask) & ~3u);
      kq[e] = (dcol < 0 && key >= 0) ? *reinterpret_cast<const int4*>(&keys[b0[e]])
                                     : make_int4(0, 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < CH; ++e)
      slot[e] = (dcol < 0 && idx[e] >= 0) ? mc_slot(keys, idx[e], b0[e], kq[e], g, sp, s, ovf) : -1;
    // exact sequential updates (a chunk with spilled keys: its own copy of the loop, global
    // reads / atomics on the chain ordered row to row by vmcnt(0))
    bool spl = false;
#pragma unroll
    for (int e = 0; e < CH; ++e) spl = spl || is_spill(slot[e]);
    auto rows = [&](auto spill_tag) {
    constexpr bool SPL = decltype(spill_tag)::value;
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const float y = yy[e];
      if (__builtin_isnan(y) || (ablate & 2)) continue;  // wave-uniform
      const int yc = (int)y;
      float d[K];
      if (dcol >= 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) d[k] = dreg[k];
      } else if (SPL && is_spill(slot[e])) {
        const float* gv = spill_vals<K>(sp, s, spill_index(slot[e]));
#pragma unroll
        for (int k = 0; k < K; ++k) d[k] = spill_load(gv + k);
      } else if (slot[e] >= 0) {
        if constexpr (K % 4 == 0) {
#pragma unroll
          for (int k = 0; k < K; k += 4) {
            const float4 v = *reinterpret_cast<const float4*>(&vals[(size_t)slot[e] * K + k]);
            d[k] = v.x; d[k + 1] = v.y; d[k + 2] = v.z; d[k + 3] = v.w;
          }
        } else {
          const float2 v = *reinterpret_cast<const float2*>(&vals[(size_t)slot[e] * K]);
          d[0] = v.x;
          d[1] = v.y;
        }
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) d[k] = 0.f;
      }
      float sc[K];
#pragma unroll
      for (int k = 0; k < K; ++k) sc[k] = (k < nclass) ? xv[e] * (wv[e][k] + d[k]) : 0.f;
      float n2 = xv[e] * xv[e];
#pragma unroll
      for (int k = 0; k < K; k += 2) wave_sum2(sc[k], sc[k + 1]);
      n2 = wave_sum(n2);
      int r = -1;
      float best = -INFINITY, sy = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (k < nclass && k != yc && sc[k] > best) {
          best = sc[k];
          r = k;
        }
        if (k == yc) sy = sc[k];
      }
      const float margin = sy - best;
      const float loss = fmaxf(0.f, 1.f - margin);
      loss_sum += loss;
      nex += 1.f;
      mist += margin <= 0.f ? 1.f : 0.f;
      float tau = 0.f;
      if (loss > 0.f && n2 > 0.f && r >= 0) {
        const float den = 2.f * n2;
        tau = variant == 0 ? loss * __builtin_amdgcn_rcpf(den)
            : variant == 1 ? fminf(C, loss * __builtin_amdgcn_rcpf(den))
                           : loss * __builtin_amdgcn_rcpf(den + 0.5f / C);
      }
      if (tau != 0.f && idx[e] >= 0) {  // wave-uniform τ
        const float gy = tau * xv[e];
        if (dcol >= 0) {
#pragma unroll
          for (int k = 0; k < K; ++k) {
            if (k == yc) dreg[k] += gy;
            if (k == r) dreg[k] -= gy;
          }
        } else if (slot[e] >= 0) {
          if (yc >= 0 && yc < nclass) atomicAdd(&vals[(size_t)slot[e] * K + yc], gy);
          atomicAdd(&vals[(size_t)slot[e] * K + r], -gy);
        } else if (SPL && is_spill(slot[e])) {
          float* gv = spill_vals<K>(sp, s, spill_index(slot[e]));
          if (yc >= 0 && yc < nclass) atomicAdd(gv + yc, gy);
          atomicAdd(gv + r, -gy);
        }
        if constexpr (SPL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    };
    if (__builtin_amdgcn_ballot_w64(spl)) rows(SpillTag<true>{});
    else rows(SpillTag<false>{});
  }
  __syncthreads();
  // Round end: class k of slot i of spoke s → region k, [i >> seg][s][i & seg mask]
  // (group-major, the shared bucket reducer's layout); overflow-area entries go straight
  // to dacc.
  const int seg_log2 = bs_log2 + g.lgg;
  const size_t S_tot = gridDim.x;
  const size_t region = S_tot << g.log2cap;
  const int used = (int)min((long long)g.qused << seg_log2, (long long)cap);  // see TableGeom
  if (compact) {
    // One record per slot: the key once ([group][spoke][segment] int32 region) and its
    // K deltas as one vector ([group][spoke][segment][K] floats after it) — 4 + 4K bytes
    // instead of 8 per class, one reduce launch for all classes (multiclass_reduce_kernel).
    int* kout = reinterpret_cast<int*>(tables);
    float* vout = reinterpret_cast<float*>(kout + region);
    for (int i = lane; i < used && !(ablate & 1); i += kWave) {
      const size_t q = (size_t)(i >> seg_log2);
      const size_t o = ((q * S_tot + s) << seg_log2) + (i & ((1 << seg_log2) - 1));
      kout[o] = keys[i];
      if constexpr (K % 4 == 0) {
#pragma unroll
        for (int k = 0; k < K; k += 4)
          *reinterpret_cast<float4*>(vout + o * K + k) =
              *reinterpret_cast<const float4*>(&vals[(size_t)i * K + k]);
      } else {
        *reinterpret_cast<float2*>(vout + o * K) =
            *reinterpret_cast<const float2*>(&vals[(size_t)i * K]);
      }
    }
  } else {
    for (int i = lane; i < used && !(ablate & 1); i += kWave) {
      const size_t q = (size_t)(i >> seg_log2);
      const size_t o = ((q * S_tot + s) << seg_log2) + (i & ((1 << seg_log2) - 1));
      const int key = keys[i];
      for (int k = 0; k < nclass; ++k)
        tables[(size_t)k * region + o] = make_int2(key, __float_as_int(vals[(size_t)i * K + k]));
    }
  }
  for (int i = cap + lane; i < tsz; i += kWave) {
    const int key = keys[i];
    if (key >= 0)
      for (int k = 0; k < nclass; ++k) {
        const float v = vals[(size_t)i * K + k];
        if (v != 0.f) atomicAdd(&dacc[(size_t)k * dim + key], v);
      }
  }
  spill_flush<K>(sp, s, nclass, dim, 1.f, dacc, lane);
  if (dcol >= 0)
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < nclass) wrow[kMcStat + k * (dn + 1) + dcol] = dreg[k];
  const float ovf_total = wave_sum(ovf);
  if (lane == 0) {
    wrow[0] = loss_sum;
    wrow[1] = nex;
    wrow[2] = mist;
    wrow[3] = 1.f;  // active worker
    wrow[4] = 0.f;
    wrow[5] = ovf_total;
    wrow[6] = 0.f;
    wrow[7] = 0.f;
    if (!bias)
      for (int k = 0; k < nclass; ++k) wrow[kMcStat + k * (dn + 1) + dn] = 0.f;
  }
}

// Register-dedup MultiClassPA round (field-aware compact wire, ≤ RMAX rows per spoke, ≤ 64
// features, compact flush): the binary register-dedup idea (linear_spoke.hip,
// linear_round_rd_kernel) with K deltas per row. On the field-aware wire lane f only sees
// keys of field f, so a spoke's K deltas for a key belong to one lane: per lane its
// rows' keys, values, K round-start prototype weights and d[e][k] (the delta of row e's
// key for class k as row e sees it). Row e's step touches classes y and r (wave-uniform):
// u = τ·x_e is added to d[e'][y] and subtracted from d[e'][r] of row e and every later row
// with the same key (compile-time row and class indices: selects, no LDS, no probes, no
// overflow on the chain). The per-key accumulation order is the LDS table's, so the round
// equals multiclass_round_kernel's. The last occurrence of each key carries its K totals
// into the compact staging image (bucket positions from LDS counters; a full bucket adds
// straight to the accumulator) and the unchanged compact flush / reducer.
template <int K, int RMAX, typename NumT, typename WT>
__global__ __launch_bounds__(64) void multiclass_round_rd_kernel(
    const WT* __restrict__ Wt, const NumT* __restrict__ num, int dn, const void* __restrict__ cat,
    int dc, int cspan, const void* __restrict__ yv, int y_i8, int B, int R, int dim, int nclass,
    int variant, float C, int bias, float* __restrict__ ws, int* __restrict__ tables,
    float* __restrict__ dacc, TableGeom g, int ablate) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int cap = 1 << g.log2cap;
  const int nbk = 1 << g.log2nb;
  const int bs_log2 = g.log2cap - g.log2nb;
  int* keys = reinterpret_cast<int*>(smem);                               // [cap]
  float* vals = reinterpret_cast<float*>(smem + (size_t)cap * 4);         // [cap][K]
  int* bcnt = reinterpret_cast<int*>(vals + (size_t)cap * K);             // [nbk / 2]
  int* dummy = bcnt + ((nbk + 1) >> 1);                                   // [64]
  const int lane = threadIdx.x;
  const int s = blockIdx.x;
  const int wsw = kMcStat + nclass * (dn + 1);
  float* wrow = ws + (size_t)s * wsw;
  const long long t0ll = (long long)s * R;
  const int t0 = t0ll > B ? B : (int)t0ll;
  const int t1 = (t0ll + R) > B ? B : (int)(t0ll + R);
  if (t0 >= t1) {  // idle spoke: not a worker this round
    for (int k = lane; k < wsw; k += kWave) wrow[k] = 0.f;
    return;
  }
  const float yraw = load_label(yv, min(t0 + lane, t1 - 1), y_i8);  // row e's class in lane e
  int key[RMAX];
  float xv[RMAX];
  load_spoke_rows<RMAX>(num, dn, cat, dc, t0, t1, lane, dim, bias, cspan, key, xv);
  const float ylane = lane < t1 - t0 ? yraw : __builtin_nanf("");
  for (int i = lane; i < cap; i += kWave) {
    keys[i] = kEmptyKey;
#pragma unroll
    for (int k = 0; k < K; ++k) vals[(size_t)i * K + k] = 0.f;
  }
  for (int i = lane; i < (nbk + 1) >> 1; i += kWave) bcnt[i] = 0;
  // round-start prototypes (key-major shadow, one vector load per row), unconditional
  float wv[RMAX][K], d[RMAX][K];
#pragma unroll
  for (int e = 0; e < RMAX; ++e) load_protos<K>(Wt, key[e] >= 0 ? key[e] : 0, wv[e]);
#pragma unroll
  for (int e = 0; e < RMAX; ++e)
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (key[e] < 0) wv[e][k] = 0.f;
      d[e][k] = 0.f;
    }
  float pn[RMAX];  // ‖x_e‖²: off the sequential chain
#pragma unroll
  for (int e = 0; e < RMAX; ++e) pn[e] = wave_sum(xv[e] * xv[e]);
  const int dcol = lane < dn ? lane : ((bias && lane == dn + dc) ? dn : -1);
  float loss_sum = 0.f, nex = 0.f, mist = 0.f;
#pragma unroll
  for (int e = 0; e < RMAX; ++e) {
    const float y = readlane_f(ylane, e);
    if (__builtin_isnan(y) || (ablate & 2)) continue;  // wave-uniform
    const int yc = (int)y;
    float sc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) sc[k] = (k < nclass) ? xv[e] * (wv[e][k] + d[e][k]) : 0.f;
#pragma unroll
    for (int k = 0; k < K; k += 2) wave_sum2(sc[k], sc[k + 1]);
    int r = -1;
    float best = -INFINITY, sy = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (k < nclass && k != yc && sc[k] > best) {
        best = sc[k];
        r = k;
      }
      if (k == yc) sy = sc[k];
    }
    const float margin = sy - best;
    const float loss = fmaxf(0.f, 1.f - margin);
    loss_sum += loss;
    nex += 1.f;
    mist += margin <= 0.f ? 1.f : 0.f;
    float tau = 0.f;
    if (loss > 0.f && pn[e] > 0.f && r >= 0) {
      const float den = 2.f * pn[e];
      tau = variant == 0 ? loss * __builtin_amdgcn_rcpf(den)
          : variant == 1 ? fminf(C, loss * __builtin_amdgcn_rcpf(den))
                         : loss * __builtin_amdgcn_rcpf(den + 0.5f / C);
    }
    if (tau != 0.f) {  // wave-uniform
      const float u = tau * xv[e];
      float du[K];
#pragma unroll
      for (int k = 0; k < K; ++k)
        du[k] = (k == yc && yc < nclass ? u : 0.f) - (k == r ? u : 0.f);
#pragma unroll
      for (int k = 0; k < K; ++k) d[e][k] += du[k];
#pragma unroll
      for (int e2 = e + 1; e2 < RMAX; ++e2) {
        const bool m = key[e2] == key[e];
#pragma unroll
        for (int k = 0; k < K; ++k) d[e2][k] += m ? du[k] : 0.f;
      }
    }
  }
  __syncthreads();  // staging image initialised
  float dreg[K];
#pragma unroll
  for (int k = 0; k < K; ++k) dreg[k] = 0.f;
  int pos[RMAX];
  bool emit[RMAX];
#pragma unroll
  for (int e = 0; e < RMAX; ++e) {
    bool last = key[e] >= 0;
#pragma unroll
    for (int e2 = e + 1; e2 < RMAX; ++e2) last = last && key[e2] != key[e];
    bool nz = false;
#pragma unroll
    for (int k = 0; k < K; ++k) nz = nz || d[e][k] != 0.f;
    last = last && nz;
    if (dcol >= 0 && last)
#pragma unroll
      for (int k = 0; k < K; ++k) dreg[k] = d[e][k];
    emit[e] = last && dcol < 0 && !(ablate & 1);
    const int b = emit[e] ? key[e] >> g.kshift : 0;
    const int sh = 16 * (b & 1);
    int* ctr = emit[e] ? &bcnt[b >> 1] : &dummy[lane];  // 16-bit counters, see linear_spoke
    pos[e] = (atomicAdd(ctr, emit[e] ? 1 << sh : 0) >> sh) & 0xffff;
  }
#pragma unroll
  for (int e = 0; e < RMAX; ++e) {
    if (emit[e]) {
      if (pos[e] < (1 << bs_log2)) {
        const int sl = ((key[e] >> g.kshift) << bs_log2) + pos[e];
        keys[sl] = key[e];
#pragma unroll
        for (int k = 0; k < K; ++k) vals[(size_t)sl * K + k] = d[e][k];
      } else {  // bucket full: straight to the accumulator (exact)
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (k < nclass && d[e][k] != 0.f) unsafeAtomicAdd(&dacc[(size_t)k * dim + key[e]], d[e][k]);
      }
    }
  }
  __syncthreads();
  // compact flush (multiclass_round_kernel's layout): key once, K deltas as one vector
  const int seg_log2 = bs_log2 + g.lgg;
  const size_t S_tot = gridDim.x;
  const size_t region = S_tot << g.log2cap;
  float* vout = reinterpret_cast<float*>(tables + region);
  const int used = (int)min((long long)g.qused << seg_log2, (long long)cap);
  for (int i = lane; i < used && !(ablate & 1); i += kWave) {
    const size_t q = (size_t)(i >> seg_log2);
    const size_t o = ((q * S_tot + s) << seg_log2) + (i & ((1 << seg_log2) - 1));
    tables[o] = keys[i];
    if constexpr (K % 4 == 0) {
#pragma unroll
      for (int k = 0; k < K; k += 4)
        *reinterpret_cast<float4*>(vout + o * K + k) =
            *reinterpret_cast<const float4*>(&vals[(size_t)i * K + k]);
    } else {
      *reinterpret_cast<float2*>(vout + o * K) = *reinterpret_cast<const float2*>(&vals[(size_t)i * K]);
    }
  }
  if (dcol >= 0)
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < nclass) wrow[kMcStat + k * (dn + 1) + dcol] = dreg[k];
  if (lane == 0) {
    wrow[0] = loss_sum;
    wrow[1] = nex;
    wrow[2] = mist;
    wrow[3] = 1.f;  // active worker
    wrow[4] = 0.f;
    wrow[5] = 0.f;  // dropped updates (none on this path)
    wrow[6] = 0.f;
    wrow[7] = 0.f;
    if (!bias)
      for (int k = 0; k < nclass; ++k) wrow[kMcStat + k * (dn + 1) + dn] = 0.f;
  }
}

// Compact-flush reducer: `split` blocks per key group (group = blockIdx / split) sum the
// (key, K-vector) records of their share of the active spokes into an LDS image
// acc[span][K] (ds_add_f32), then add its non-zero entries to dacc[k][key] — plainly when
// a block owns the group, with L2 fp32 atomics when the group is split. Same invariants as
// linear_reduce_kernel: slot i of a table lies in group i >> seg, and its key in that
// group's key range (overflow-area keys never reach the flushed region).
template <int K>
__global__ __launch_bounds__(256) void multiclass_reduce_kernel(
    const int* __restrict__ keys, const float* __restrict__ vals, int S_act, int S, TableGeom g,
    int dim, int nclass, float* __restrict__ dacc, int split) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* acc = reinterpret_cast<float*>(smem);
  const int gl = g.kshift + g.lgg;
  const int span = 1 << gl;
  const int q = (int)blockIdx.x / split;
  const int part = (int)blockIdx.x % split;
  const int s_lo = (int)(((long long)S_act * part) / split);
  const int s_hi = (int)(((long long)S_act * (part + 1)) / split);
  for (int i = threadIdx.x; i < span * K; i += 256) acc[i] = 0.f;
  __syncthreads();
  const int seg_log2 = (g.log2cap - g.log2nb) + g.lgg;
  const int lo = q << gl;
  const size_t base = ((size_t)q * S + s_lo) << seg_log2;
  const long long items = (long long)(s_hi - s_lo) << seg_log2;
  auto add = [&](int key, const float (&v)[K]) {
    const unsigned off = (unsigned)(key - lo);
    if (key < 0 || off >= (unsigned)span) return;
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < nclass && v[k] != 0.f) atomicAdd(&acc[off * K + k], v[k]);
  };
  auto load = [&](long long it, int& key, float (&v)[K]) {
    const size_t o = base + (size_t)it;
    key = keys[o];
    if constexpr (K % 4 == 0) {
#pragma unroll
      for (int k = 0; k < K; k += 4) {
        const float4 f = *reinterpret_cast<const float4*>(vals + o * K + k);
        v[k] = f.x; v[k + 1] = f.y; v[k + 2] = f.z; v[k + 3] = f.w;
      }
    } else {
      const float2 f = *reinterpret_cast<const float2*>(vals + o * K);
      v[0] = f.x;
      v[1] = f.y;
    }
  };
  long long it = threadIdx.x;
  for (; it + 3 * 256 < items; it += 4 * 256) {
    int key[4];
    float v[4][K];
#pragma unroll
    for (int u = 0; u < 4; ++u) load(it + u * 256, key[u], v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) add(key[u], v[u]);
  }
  for (; it < items; it += 256) {
    int key;
    float v[K];
    load(it, key, v);
    add(key, v);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < span * K; i += 256) {
    const int k = i % K;
    const int key = lo + i / K;
    const float v = acc[i];
    if (k < nclass && key < dim && v != 0.f) {
      if (split == 1) dacc[(size_t)k * dim + key] += v;
      else unsafeAtomicAdd(&dacc[(size_t)k * dim + key], v);
    }
  }
}

template <int K>
static int launch_mc_reduce(const void* tables, int S_act, int S, TableGeom g, int dim,
                            int nclass, float* dacc, hipStream_t st) {
  if (S_act <= 0) return 0;
  const int gl = g.kshift + g.lgg;
  const int ng = min((dim + (1 << gl) - 1) >> gl, g.qused);
  // Spokes of a key group split over 2 blocks: measured at 4 classes, 8192 spokes, 2^20
  // dims (256 groups): split 1 / 2 / 4 / 8 → 0.370 / 0.348 / 0.361 / 0.385 ms per round
  // (the 64 KiB image allows 2 blocks per CU; wider splits pay in L2 atomics).
  int split = ng >= 1024 ? 1 : 2;
  if (const char* e = getenv("OMLDM_REDUCE_SPLIT")) split = atoi(e);
  if (split < 1) split = 1;
  if (split > 16) split = 16;
  while (split > 1 && split > S_act) split >>= 1;
  const size_t lds = (size_t(1) << gl) * K * sizeof(float);
  auto fn = multiclass_reduce_kernel<K>;
  int e = check_dyn_lds((const void*)fn, lds);
  if (e) return e;
  const size_t region = (size_t)S << g.log2cap;
  const int* keys = static_cast<const int*>(tables);
  hipLaunchKernelGGL(fn, dim3(ng * split), dim3(256), lds, st, keys,
                     reinterpret_cast<const float*>(keys + region), S_act, S, g, dim, nclass,
                     dacc, split);
  return (int)hipGetLastError();
}

// Workspace column sums (one block per column): stats[c] += Σ_s ws[s][c] for c < 8;
// dense column (k, j) → dacc[k][j] (j < dn) or dacc[k][dim-1] (intercept).
__global__ __launch_bounds__(256) void multiclass_finish_kernel(const float* __restrict__ ws,
                                                                int S, int dn, int nclass, int dim,
                                                                float* __restrict__ dacc,
                                                                float* __restrict__ stats) {
  __shared__ float part[4];
  const int wsw = kMcStat + nclass * (dn + 1);
  const int c = blockIdx.x;
  float acc = 0.f;
  for (int s = threadIdx.x; s < S; s += 256) acc += ws[(size_t)s * wsw + c];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = (part[0] + part[1]) + (part[2] + part[3]);
    if (c < kMcStat) {
      if (c != 4 && c < 6) stats[c] += t;
    } else {
      const int j = c - kMcStat, k = j / (dn + 1), jj = j % (dn + 1);
      dacc[(size_t)k * dim + (jj < dn ? jj : dim - 1)] += t;
    }
  }
}

// W[k][i] += dacc[k][i] / n_active ; dacc = 0 ; key-major shadow Wt[i][k] = W[k][i]
// (fp32 or bf16, row stride kp) for the next round's gathers.
// fold != 0 also folds the round's statistics into the running totals (block 0, one
// lane; `st` is not read by any other block — nact is its own buffer):
//   fold 1: cum[k] += st[k], k < 3;  fold 2 (NN regression): cum[0..1] += st[0..1];
//   fold 3 (NN classification): as 2 plus cum[2] += st[1] − st[2];  then st[0..3] = 0.
// This replaces four small elementwise launches per round.
__global__ __launch_bounds__(256) void multiclass_apply_kernel(float* __restrict__ W,
                                                               float* __restrict__ dacc, int dim,
                                                               int nclass, void* __restrict__ Wt,
                                                               int wt_bf16, int kp,
                                                               const float* __restrict__ nact,
                                                               float* __restrict__ st,
                                                               double* __restrict__ cum, int fold,
                                                               float* __restrict__ nact_next) {
  // nact_next (optional, ≠ nact): the divisor buffer of the NEXT round, zeroed here so the
  // next round kernel can count into it (callers alternate two buffers)
  if (nact_next && blockIdx.x == 0 && threadIdx.x == 0) *nact_next = 0.f;
  if (fold && blockIdx.x == 0 && threadIdx.x == 0) {
    const float a = st[0], b = st[1], c = st[2];
    cum[0] += (double)a;
    cum[1] += (double)b;
    if (fold == 1) cum[2] += (double)c;
    if (fold == 3) cum[2] += (double)(b - c);
    st[0] = st[1] = st[2] = st[3] = 0.f;
  }
  const float na = *nact;
  const float r = na > 0.f ? 1.f / na : 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < dim; i += gridDim.x * 256) {
    for (int k = 0; k < nclass; ++k) {
      const size_t o = (size_t)k * dim + i;
      const float v = fmaf(dacc[o], r, W[o]);
      W[o] = v;
      dacc[o] = 0.f;
      if (Wt) {
        if (wt_bf16) static_cast<__hip_bfloat16*>(Wt)[(size_t)i * kp + k] = __float2bfloat16(v);
        else static_cast<float*>(Wt)[(size_t)i * kp + k] = v;
      }
    }
  }
}

template <int K, typename NumT, typename WT>
static void launch_mc(const void* Wt, const void* num, int dn, const void* cat, int dc, int cspan,
                      const void* y, int y_i8, int B, int R, int S, int dim, int nclass,
                      int variant, float C, int bias, float* ws, int2* tables, float* dacc,
                      TableGeom g, size_t lds, int compact, const Spill& sp, hipStream_t st,
                      int* err) {
  int ablate = 0;  // timing diagnostics only: bit0 no flush, bit1 no sequential part
  if (const char* e = getenv("OMLDM_MC_ABLATE")) ablate = atoi(e);
  // register-dedup path: field-aware wire, ≤ 16 rows per spoke, K ≤ 4, compact flush
  // (OMLDM_MC_RD=0: the LDS-table kernel, A/B)
  const char* rd_env = getenv("OMLDM_MC_RD");
  if constexpr (K <= 4) {
  if (compact && cspan > 0 && R <= 16 && !(rd_env && atoi(rd_env) == 0)) {
    const int nbk = 1 << g.log2nb;
    const size_t lds_rd =
        (size_t(1) << g.log2cap) * (4 + 4 * (size_t)K) + (size_t)((nbk + 1) / 2) * 4 + kWave * 4;
    auto run = [&](auto fn) {
      *err = check_dyn_lds((const void*)fn, lds_rd);
      if (*err) return;
      hipLaunchKernelGGL(fn, dim3(S), dim3(64), lds_rd, st, (const WT*)Wt, (const NumT*)num, dn,
                         cat, dc, cspan, y, y_i8, B, R, dim, nclass, variant, C, bias, ws,
                         (int*)tables, dacc, g, ablate);
    };
    if (R <= 8) run(multiclass_round_rd_kernel<K, 8, NumT, WT>);
    else run(multiclass_round_rd_kernel<K, 16, NumT, WT>);
    return;
  }
  }
  auto fn = multiclass_round_kernel<K, 4, NumT, WT>;
  *err = check_dyn_lds((const void*)fn, lds);
  if (*err) return;
  hipLaunchKernelGGL(fn, dim3(S), dim3(64), lds, st, (const WT*)Wt, (const NumT*)num, dn, cat, dc,
                     cspan, y, y_i8, B, R, dim, nclass, variant, C, bias, ws, tables, dacc, g,
                     ablate, compact, sp);
}

}  // namespace omldm

using namespace omldm;

// One round of S spokes: dacc[nclass][dim] += Σ_s Δ_s, stats[0..5] += (loss, n, mistakes,
// active spokes, -, overflow). ws: S·(8 + nclass·(dn+1)) floats; tables: nclass·S·2^log2cap
// int2.
OMLDM_API int omldm_multiclass_round(const void* Wt, int wt_bf16, const void* num, int num_bf16,
                                     int dn, const void* cat, int dc, int cspan, const void* y, int y_i8,
                                     int B, int R, int S, int dim, int nclass, int variant,
                                     float C, int bias, float* dacc, float* stats, int log2cap,
                                     float* ws, void* tables, void* spill, int log2gcap,
                                     void* stream) {
  if (S <= 0 || B <= 0) return 0;
  if (spill == nullptr || log2gcap < 6 || log2gcap > 24) return -6;  // the HBM spill is required
  if (dn + dc + (bias ? 1 : 0) > 64) return -2;
  if (nclass < 2 || nclass > 16) return -3;
  if (log2cap < 6 || log2cap > 13) return -1;
  TableGeom g;
  if (bucket_geom(dim, log2cap, &g)) return -4;  // per-class key space: the linear geometry
  if (cspan > 0) {  // field-aware wire: no hashed key at or above dn + dc·cspan
    const int gl = g.kshift + g.lgg;
    const long long hi = (long long)dn + (long long)dc * cspan;
    g.qused = (int)(((hi < dim ? hi : dim) + (1LL << gl) - 1) >> gl);
  }
  const int K = nclass <= 2 ? 2 : nclass <= 4 ? 4 : nclass <= 8 ? 8 : 16;
  const Spill sp = make_spill(spill, S, log2gcap, K);  // K floats per entry
  const size_t lds = ((size_t(1) << log2cap) + kOvf) * (4 + 4 * (size_t)K);
  if (lds > 160 * 1024) return -1;
  hipStream_t st = (hipStream_t)stream;
  // Compact flush + one reduce launch when the reducer's LDS image acc[span][K] fits
  // (K ≤ 8 at the default 4096-key groups); per-class int2 regions otherwise. Both fit
  // the caller's nclass·S·2^log2cap int2 scratch, since 1 + K ≤ 2·nclass.
  int compact = ((size_t(1) << (g.kshift + g.lgg)) * K * sizeof(float)) <= 160 * 1024;
  if (const char* ev = getenv("OMLDM_MC_COMPACT")) compact = compact && atoi(ev) != 0;  // A/B
  int e = 0;
#define OMLDM_MC(KK)                                                                         \
  {                                                                                          \
    if (num_bf16 && wt_bf16)                                                                 \
      launch_mc<KK, __hip_bfloat16, __hip_bfloat16>(Wt, num, dn, cat, dc, cspan, y, y_i8, B, R, \
          S, dim, nclass, variant, C, bias, ws, (int2*)tables, dacc, g, lds, compact, sp, st, &e);           \
    else if (num_bf16)                                                                       \
      launch_mc<KK, __hip_bfloat16, float>(Wt, num, dn, cat, dc, cspan, y, y_i8, B, R, S, dim,  \
          nclass, variant, C, bias, ws, (int2*)tables, dacc, g, lds, compact, sp, st, &e);                   \
    else if (wt_bf16)                                                                        \
      launch_mc<KK, float, __hip_bfloat16>(Wt, num, dn, cat, dc, cspan, y, y_i8, B, R, S, dim,  \
          nclass, variant, C, bias, ws, (int2*)tables, dacc, g, lds, compact, sp, st, &e);                   \
    else                                                                                     \
      launch_mc<KK, float, float>(Wt, num, dn, cat, dc, cspan, y, y_i8, B, R, S, dim, nclass,   \
          variant, C, bias, ws, (int2*)tables, dacc, g, lds, compact, sp, st, &e);                           \
  }
  if (K == 2) OMLDM_MC(2) else if (K == 4) OMLDM_MC(4) else if (K == 8) OMLDM_MC(8) else OMLDM_MC(16)
#undef OMLDM_MC
  if (e) return e;
  e = (int)hipGetLastError();
  if (e) return e;
  const long long sact_ll = ((long long)B + R - 1) / R;
  const int S_act = sact_ll < S ? (int)sact_ll : S;
  const int gspan = g.kshift + g.lgg;
  const int ng = min((dim + (1 << gspan) - 1) >> gspan, g.qused);  // unflushed groups are empty
  const size_t region = (size_t)S << log2cap;
  if (compact) {
    e = K == 2 ? launch_mc_reduce<2>(tables, S_act, S, g, dim, nclass, dacc, st)
      : K == 4 ? launch_mc_reduce<4>(tables, S_act, S, g, dim, nclass, dacc, st)
      : K == 8 ? launch_mc_reduce<8>(tables, S_act, S, g, dim, nclass, dacc, st)
               : launch_mc_reduce<16>(tables, S_act, S, g, dim, nclass, dacc, st);
    if (e) return e;
  } else {
    for (int k = 0; k < nclass; ++k) {
      e = bucket_reduce_launch((const int2*)tables + k * region, S_act, S, g, dim,
                               dacc + (size_t)k * dim, 0, ng, st);
      if (e) return e;
    }
  }
  hipLaunchKernelGGL(multiclass_finish_kernel, dim3(kMcStat + nclass * (dn + 1)), dim3(256), 0, st,
                     ws, S, dn, nclass, dim, dacc, stats);
  return (int)hipGetLastError();
}

// Wt: key-major shadow [dim][kp] (nullptr: none).
OMLDM_API int omldm_multiclass_apply(float* W, float* dacc, int dim, int nclass, void* Wt,
                                     int wt_bf16, int kp, const float* nact, float* st,
                                     double* cum, int fold, float* nact_next, void* stream) {
  if (fold && (!st || !cum || st == nact)) return -1;
  if (nact_next && nact_next == nact) return -1;
  int blocks = (dim + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(multiclass_apply_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, W,
                     dacc, dim, nclass, Wt, wt_bf16, kp, nact, st, cum, fold, nact_next);
  return (int)hipGetLastError();
}
