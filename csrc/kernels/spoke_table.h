// Hashed-feature spoke tables shared by the virtual-spoke learners (linear_spoke.hip,
// multiclass_spoke.hip): wire decoding of one feature / label, the bucketed LDS delta
// table (geometry, slow-path probe) and the round-end bucket reducer's launcher.
#pragma once
#include "common.h"

namespace omldm {

// Label of example t: fp32, or int8 on the compact classification wire (1 B instead of 4
// per example over PCIe; ±1 and class ids are exact).
__device__ __forceinline__ float load_label(const void* __restrict__ yv, int t, int y_i8) {
  return y_i8 ? (float)static_cast<const signed char*>(yv)[t] : static_cast<const float*>(yv)[t];
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

// Loads feature f of example t for this lane. Numeric features occupy slots [0, dn);
// categorical features carry their hashed slot in the low 31 bits and the hash sign in
// bit 31; -1 marks an absent categorical feature.
// With bias != 0 the feature right after the categorical ones is the intercept: slot
// dim-1 (reserved by the hasher) with constant value 1 (reference VectorBias, U23).
// Compact wire format (cspan > 0): categorical field f is a uint16 {sign:1, local:15}
// with slot = dn + f·cspan + local (field-aware hashing), 0xFFFF = absent — half the
// PCIe bytes of the int32 form for Criteo-shaped streams.
template <typename NumT>
__device__ __forceinline__ void load_feature(const NumT* __restrict__ num, int dn,
                                             const void* __restrict__ cat, int dc, int t, int j,
                                             int dim, int bias, int cspan, int& idx, float& v) {
  idx = -1;
  v = 0.f;
  if (j == dn + dc && bias) {
    idx = dim - 1;
    v = 1.f;
  } else if (j < dn) {
    idx = j;
    v = to_f(num[(size_t)t * dn + j]);
  } else if (j < dn + dc) {
    if (cspan > 0) {
      const unsigned c = static_cast<const unsigned short*>(cat)[(size_t)t * dc + (j - dn)];
      if (c != 0xFFFFu) {
        idx = dn + (j - dn) * cspan + (int)(c & 0x7fffu);
        v = (c & 0x8000u) ? -1.f : 1.f;
      }
    } else {
      const int c = static_cast<const int*>(cat)[(size_t)t * dc + (j - dn)];
      if (c != -1) {
        idx = c & 0x7fffffff;
        v = c < 0 ? -1.f : 1.f;
      }
    }
  }
  if ((unsigned)idx >= (unsigned)dim) {  // never gather out of bounds
    idx = -1;
    v = 0.f;
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
  return -1;  // table full: the update is dropped and counted as overflow
}

// Bucket reduce of flushed spoke tables into dacc (linear_spoke.hip): key groups
// [q0, q1) of the geometry `g` over `dim` keys, no workspace columns. `S` is the spoke
// count of the flush layout, `S_act` the spokes that flushed.
int bucket_reduce_launch(const int2* tables, int S_act, int S, TableGeom g, int dim,
                         float* dacc, int q0, int q1, hipStream_t st);
// reduce_lgg-adjusted geometry for `dim` keys and a 2^log2cap-entry table (-1: too small)
int bucket_geom(int dim, int log2cap, TableGeom* g);

}  // namespace omldm
