// Hashed-feature spoke tables shared by the virtual-spoke learners (linear_spoke.hip,
// multiclass_spoke.hip): wire decoding of one feature / label, the bucketed LDS delta
// table (geometry, slow-path probe) and the round-end bucket reducer's launcher.
#pragma once
#include "common.h"

namespace omldm {

// Label of example t: fp32, or int8 on the compact classification wire (1 B instead of 4
// per example over PCIe; ±1 and class ids are exact). One unconditional aligned dword load
// (the word holding the int8 label, tensor allocations being ≥ 4-byte granular): a
// y_i8 branch around two loads made the wave wait inside the branch.
__device__ __forceinline__ float load_label(const void* __restrict__ yv, int t, int y_i8) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(yv) + (y_i8 ? (uintptr_t)t : (uintptr_t)t * 4);
  const uint32_t w = *reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  return y_i8 ? (float)(signed char)(w >> (8 * (a & 3))) : __uint_as_float(w);
}

// Bucketed LDS delta table geometry (host-computed, see omldm_linear_round):
//   keys/vals [cap + kOvf]; bucket(key) = key >> kshift owns slots
//   [bucket·BS, (bucket+1)·BS), BS = cap >> log2nb; the kOvf tail is a shared overflow area.
struct TableGeom {
  int log2cap;
  int log2nb;
  int kshift;
  int lgg;  // log2 buckets per reduce group (flush layout: [group][spoke][2^lgg · BS])
  // key groups that can hold hashed keys at all: on the field-aware wire the categorical
  // slots end at dn + dc·cspan, so the groups above are empty in every table — neither
  // flushed nor reduced
  int qused = 1 << 30;
};
constexpr int kOvf = 64;

// Feature f of example t for this lane (wire format). Numeric features occupy slots [0, dn);
// categorical features carry their hashed slot in the low 31 bits and the hash sign in
// bit 31; -1 marks an absent categorical feature.
// With bias != 0 the feature right after the categorical ones is the intercept: slot
// dim-1 (reserved by the hasher) with constant value 1 (reference VectorBias, U23).
// Compact wire format (cspan > 0): categorical field f is a uint16 {sign:1, local:15}
// with slot = dn + f·cspan + local (field-aware hashing), 0xFFFF = absent — half the
// PCIe bytes of the int32 form for Criteo-shaped streams.
// Loading is split in two so a caller can issue the loads of many rows before decoding
// any (a load inside a lane-divergent or per-row branch is waited for
// inside that branch, which serialised the rows of the spoke kernels):
//   load_feature_raw — unconditional loads from always-valid addresses (t must be a valid
//     row; absent numerical/categorical blocks read a zero word): the numerical value and
//     the categorical word (the aligned dword holding a 16-bit compact slot — tensor
//     allocations are at least 4-byte granular — or the int32 slot of the wide format);
//   decode_feature — (idx, v) of the format above, or (-1, 0) when !ok or out of range.
__device__ const uint32_t kZeroWords[4] = {0u, 0u, 0u, 0u};

struct FeatRaw {
  float nv;
  uint32_t c;
};

template <typename NumT>
__device__ __forceinline__ FeatRaw load_feature_raw(const NumT* __restrict__ num, int dn,
                                                    const void* __restrict__ cat, int dc, int t,
                                                    int j, int cspan) {
  const bool is_num = j < dn;
  const bool is_cat = j >= dn && j < dn + dc;
  const NumT* np = dn > 0 ? num + ((size_t)t * dn + (is_num ? j : 0))
                          : reinterpret_cast<const NumT*>(kZeroWords);
  const uintptr_t ca =
      dc > 0 ? reinterpret_cast<uintptr_t>(cat) +
                   ((size_t)t * dc + (is_cat ? j - dn : 0)) * (cspan > 0 ? 2u : 4u)
             : reinterpret_cast<uintptr_t>(kZeroWords);
  const uint32_t cw = *reinterpret_cast<const uint32_t*>(ca & ~uintptr_t(3));
  FeatRaw r;
  r.nv = to_f(*np);
  r.c = cspan > 0 ? (cw >> (8 * (ca & 3))) & 0xffffu : cw;
  return r;
}

__device__ __forceinline__ void decode_feature(FeatRaw r, int dn, int dc, int j, int dim,
                                               int bias, int cspan, bool ok, int& idx,
                                               float& v) {
  const bool is_num = j < dn;
  const bool is_cat = j >= dn && j < dn + dc;
  const bool is_bias = bias && j == dn + dc;
  int ci;
  float cv;
  if (cspan > 0) {  // wave-uniform; no loads inside
    ci = r.c != 0xFFFFu ? dn + (j - dn) * cspan + (int)(r.c & 0x7fffu) : -1;
    cv = (r.c & 0x8000u) ? -1.f : 1.f;
  } else {
    ci = r.c != 0xFFFFFFFFu ? (int)(r.c & 0x7fffffffu) : -1;
    cv = (r.c & 0x80000000u) ? -1.f : 1.f;
  }
  idx = is_num ? j : is_cat ? ci : is_bias ? dim - 1 : -1;
  v = is_num ? r.nv : is_cat ? cv : 1.f;
  if (!ok || (unsigned)idx >= (unsigned)dim) idx = -1;
  if (idx < 0) v = 0.f;
}

// The ≤ RMAX rows [t0, t1) of a register-dedup spoke on the field-aware compact wire
// (cspan > 0; ≤ 64 features, lane = feature): key[e] / xv[e] of row e for this lane, -1 / 0
// for absent features and rows past t1. Every load is in flight before any is decoded:
// one 16-bit load per row and lane when the numericals are bf16 (lane-dependent base and
// stride: numerical slot or categorical field), two loads otherwise.
template <int RMAX, typename NumT>
__device__ __forceinline__ void load_spoke_rows(const NumT* __restrict__ num, int dn,
                                                const void* __restrict__ cat, int dc, int t0,
                                                int t1, int lane, int dim, int bias, int cspan,
                                                int (&key)[RMAX], float (&xv)[RMAX]) {
  const bool is_num = lane < dn;
  const bool is_cat = lane >= dn && lane < dn + dc;
  const bool is_bias = bias && lane == dn + dc;
  const int jn = is_num ? lane : 0;
  const int jc = is_cat ? lane - dn : 0;
  unsigned short raw[RMAX];
  NumT nraw[sizeof(NumT) == 2 ? 1 : RMAX];
  if constexpr (sizeof(NumT) == 2) {
    const unsigned short* base = is_num ? reinterpret_cast<const unsigned short*>(num) + jn
                                        : static_cast<const unsigned short*>(cat) + jc;
    const int stride = is_num ? dn : dc;
#pragma unroll
    for (int e = 0; e < RMAX; ++e) raw[e] = base[(size_t)min(t0 + e, t1 - 1) * stride];
  } else {
#pragma unroll
    for (int e = 0; e < RMAX; ++e) {
      const int t = min(t0 + e, t1 - 1);
      nraw[e] = num[(size_t)t * dn + jn];
      raw[e] = static_cast<const unsigned short*>(cat)[(size_t)t * dc + jc];
    }
  }
  const int cbase = dn + jc * cspan;
#pragma unroll
  for (int e = 0; e < RMAX; ++e) {
    const unsigned c = raw[e];
    float nv;
    if constexpr (sizeof(NumT) == 2) nv = __uint_as_float(c << 16);  // bf16 bits
    else nv = to_f(nraw[e]);
    int idx = is_num ? lane : is_bias ? dim - 1 : (is_cat && c != 0xFFFFu) ? cbase + (int)(c & 0x7fffu) : -1;
    const float v = is_num ? nv : is_bias ? 1.f : (c & 0x8000u) ? -1.f : 1.f;
    if ((unsigned)idx >= (unsigned)dim || t0 + e >= t1) idx = -1;
    key[e] = idx;
    xv[e] = idx >= 0 ? v : 0.f;
  }
}

__device__ __forceinline__ uint32_t hmix(uint32_t k) { return k * 0x9E3779B1u; }

// Slow path of the bucketed table: probe the whole bucket, then the overflow area.
static __device__ __noinline__ int table_find_or_insert(int* keys, int key, TableGeom g) {
  const int bs_log2 = g.log2cap - g.log2nb;
  const uint32_t bmask = (1u << bs_log2) - 1u;
  const int base = (key >> g.kshift) << bs_log2;
  const uint32_t h = hmix((uint32_t)key);
  // linear probing from the 4-aligned hashed start — the same order as the vector first
  // probe in the round kernel (which covers start..start+3), so a key is never inserted
  // twice: it sits after its start only if every slot in between was taken at insertion
  const uint32_t s0 = (h & bmask) & ~3u;
  for (uint32_t q = 0; q <= bmask; ++q) {
    const int i = base + (int)((s0 + q) & bmask);
    const int k = __hip_atomic_load(&keys[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (k == key) return i;
    if (k == kEmptyKey) {
      const int prev = atomicCAS(&keys[i], kEmptyKey, key);
      if (prev == kEmptyKey || prev == key) return i;
    }
  }
  const int ob = 1 << g.log2cap;
  for (int q = 0; q < kOvf; ++q) {
    const int i = ob + (int)((h + q) & (kOvf - 1));
    const int k = __hip_atomic_load(&keys[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (k == key) return i;
    if (k == kEmptyKey) {
      const int prev = atomicCAS(&keys[i], kEmptyKey, key);
      if (prev == kEmptyKey || prev == key) return i;
    }
  }
  return -1;  // table full: the caller takes the key to the global spill (below)
}

// ---------------------------------------------------------------- global spill
// A spoke whose distinct keys outgrow its LDS table (bucket and overflow area full) keeps
// the rest in HBM, so no update is ever dropped: per spoke an open-addressing table
// keys[gcap] (kEmptyKey when free), vals[gcap][VK] and the list of the entries it took
// this round (count[s] of them). Round end: every listed entry is flushed into the
// accumulator and restored to empty, so the region is clean for the next round without
// a memset. Only the spoke's own wave touches its region: device-scope atomics keep the
// lanes of one row coherent, and a row's reads of a spilled delta (agent-scope loads,
// past L1) follow a vmcnt(0) after the previous row's atomics.
// Slot encoding on the sequential chain: ≥ 0 LDS slot, −1 no key, ≤ −3: spill entry
// (−3 − index).
struct Spill {
  int* keys;    // [S][gcap], every entry kEmptyKey when allocated
  float* vals;  // [S][gcap][VK], zero when allocated
  int* list;    // [S][gcap]
  int* count;   // [S], zero when allocated
  int log2gcap;
};
constexpr int kSpillBase = -3;
// One contiguous caller buffer: keys [S·gcap] | vals [S·gcap·VK] | list [S·gcap] | count [S]
// (spill_words(S, log2gcap, VK) 4-byte words; keys = −1, vals = count = 0 when allocated).
inline size_t spill_words(int S, int log2gcap, int VK) {
  return (size_t)S * ((size_t)1 << log2gcap) * (2 + (size_t)VK) + (size_t)S;
}
inline Spill make_spill(void* base, int S, int log2gcap, int VK) {
  const size_t n = (size_t)S << log2gcap;
  int* keys = static_cast<int*>(base);
  float* vals = reinterpret_cast<float*>(keys + n);
  int* list = reinterpret_cast<int*>(vals + n * VK);
  return Spill{keys, vals, list, list + n, log2gcap};
}
template <bool B>
struct SpillTag {
  static constexpr bool value = B;
};

__device__ __forceinline__ bool is_spill(int sl) { return sl <= kSpillBase; }
__device__ __forceinline__ int spill_index(int sl) { return kSpillBase - sl; }

// Entry of `key` in spoke s's spill (find or insert); -1 only when all gcap entries are
// taken (the host sizes gcap ≥ 2 × the spoke's key occurrences, so never).
static __device__ __noinline__ int spill_find_or_insert(const Spill& sp, int s, int key) {
  const int gcap = 1 << sp.log2gcap;
  int* keys = sp.keys + (size_t)s * gcap;
  uint32_t i = hmix((uint32_t)key) >> (32 - sp.log2gcap);
  for (int q = 0; q < gcap; ++q) {
    const int k = __hip_atomic_load(&keys[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) return (int)i;
    if (k == kEmptyKey) {
      const int prev = atomicCAS(&keys[i], kEmptyKey, key);
      if (prev == kEmptyKey) {
        const int at = atomicAdd(&sp.count[s], 1);
        sp.list[(size_t)s * gcap + at] = (int)i;
        return (int)i;
      }
      if (prev == key) return (int)i;
    }
    i = (i + 1) & (uint32_t)(gcap - 1);
  }
  return -1;
}

// The slot of a key the LDS table could not take: a spill entry, or -1 (counted in `ovf`).
__device__ __forceinline__ int spill_slot(const Spill& sp, int s, int key, float& ovf) {
  const int gi = spill_find_or_insert(sp, s, key);
  if (gi < 0) {
    ovf += 1.f;
    return -1;
  }
  return kSpillBase - gi;
}

template <int VK>
__device__ __forceinline__ float* spill_vals(const Spill& sp, int s, int gi) {
  return sp.vals + ((size_t)s * (1 << sp.log2gcap) + gi) * VK;
}

__device__ __forceinline__ float spill_load(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Round end of one spoke wave (all 64 lanes): every listed entry → dacc[k·dim + key] +=
// scale·vals[k] for k < nv, then the entry is restored (key empty, values 0).
template <int VK>
__device__ __forceinline__ void spill_flush(const Spill& sp, int s, int nv, int dim, float scale,
                                            float* __restrict__ dacc, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int gcap = 1 << sp.log2gcap;
  const int n = __hip_atomic_load(&sp.count[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (n == 0) return;
  int* keys = sp.keys + (size_t)s * gcap;
  for (int j = lane; j < n; j += kWave) {
    const int gi = __hip_atomic_load(&sp.list[(size_t)s * gcap + j], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
    const int key = __hip_atomic_load(&keys[gi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float* v = spill_vals<VK>(sp, s, gi);
#pragma unroll
    for (int k = 0; k < VK; ++k) {
      const float x = spill_load(v + k);
      if (k < nv && x != 0.f) atomicAdd(&dacc[(size_t)k * dim + key], x * scale);
      v[k] = 0.f;
    }
    keys[gi] = kEmptyKey;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) sp.count[s] = 0;
}

// Bucket reduce of flushed spoke tables into dacc (linear_spoke.hip): key groups
// [q0, q1) of the geometry `g` over `dim` keys, no workspace columns. `S` is the spoke
// count of the flush layout, `S_act` the spokes that flushed.
int bucket_reduce_launch(const int2* tables, int S_act, int S, TableGeom g, int dim,
                         float* dacc, int q0, int q1, hipStream_t st);
// reduce_lgg-adjusted geometry for `dim` keys and a 2^log2cap-entry table (-1: too small)
int bucket_geom(int dim, int log2cap, TableGeom* g);

}  // namespace omldm
