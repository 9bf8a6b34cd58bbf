// Shared device helpers for the OMLDM-AMD CDNA4 (gfx950) kernels.
//
// Everything here is written for 64-lane wavefronts: reductions use DPP row
// rotations inside 16-lane rows plus four v_readlane ops (no LDS round trip),
// which keeps the per-example critical path of the sequential online learners
// short (see linear_spoke.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define OMLDM_API extern "C" __attribute__((visibility("default")))

namespace omldm {

constexpr int kWave = 64;
constexpr int kEmptyKey = -1;

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

// Full-wave sum. Every lane must be active (callers pass 0 for inactive lanes).
// quad_perm[1,0,3,2], quad_perm[2,3,0,1], row_ror:4, row_ror:8 leave the
// 16-lane row sum in every lane of the row; the four row sums are combined
// through scalar readlanes, so the result is wave-uniform.
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x124>(v);
  v += dpp_mov<0x128>(v);
  return (readlane_f(v, 0) + readlane_f(v, 16)) + (readlane_f(v, 32) + readlane_f(v, 48));
}

// Two independent sums interleaved for ILP (margin and squared norm).
__device__ __forceinline__ void wave_sum2(float& a, float& b) {
  a += dpp_mov<0xB1>(a);
  b += dpp_mov<0xB1>(b);
  a += dpp_mov<0x4E>(a);
  b += dpp_mov<0x4E>(b);
  a += dpp_mov<0x124>(a);
  b += dpp_mov<0x124>(b);
  a += dpp_mov<0x128>(a);
  b += dpp_mov<0x128>(b);
  a = (readlane_f(a, 0) + readlane_f(a, 16)) + (readlane_f(a, 32) + readlane_f(a, 48));
  b = (readlane_f(b, 0) + readlane_f(b, 16)) + (readlane_f(b, 32) + readlane_f(b, 48));
}

__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x124>(v));
  v = fmaxf(v, dpp_mov<0x128>(v));
  return fmaxf(fmaxf(readlane_f(v, 0), readlane_f(v, 16)), fmaxf(readlane_f(v, 32), readlane_f(v, 48)));
}

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(__hip_bfloat16 x) { return __bfloat162float(x); }

// Multiplicative (Fibonacci) hash into a power-of-two table.
__device__ __forceinline__ uint32_t hslot(uint32_t key, int log2cap) {
  return (key * 0x9E3779B1u) >> (32 - log2cap);
}

// Lane-parallel insert-or-find in an LDS open-addressing table (linear probing).
// Returns the slot or -1 when the table is full (bounded: never spins forever).
__device__ __forceinline__ int lds_find_or_insert(int* keys, int key, int log2cap) {
  const uint32_t mask = (1u << log2cap) - 1u;
  uint32_t h = hslot((uint32_t)key, log2cap);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    int k = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (k == key) return (int)h;
    if (k == kEmptyKey) {
      int prev = atomicCAS(&keys[h], kEmptyKey, key);
      if (prev == kEmptyKey || prev == key) return (int)h;
    }
    h = (h + 1u) & mask;
  }
  return -1;
}

// Lookup only (no insert). Returns -1 if absent.
__device__ __forceinline__ int lds_find(const int* keys, int key, int log2cap) {
  const uint32_t mask = (1u << log2cap) - 1u;
  uint32_t h = hslot((uint32_t)key, log2cap);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    int k = keys[h];
    if (k == key) return (int)h;
    if (k == kEmptyKey) return -1;
    h = (h + 1u) & mask;
  }
  return -1;
}

inline int check_dyn_lds(const void* fn, size_t bytes) {
  // Up to 160 KiB of LDS per workgroup on gfx950; above 64 KiB the attribute is required.
  if (bytes > 65536) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

}  // namespace omldm
