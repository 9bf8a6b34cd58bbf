// Exact sequential online linear learners, v3 ("table scan"): every spoke keeps the
// weights it re-reads during a round in an LDS slot table, so the per-spoke workgroup
// issues no global atomics and a third of v2's global gathers; the round end adds the
// spokes' updates straight into the round accumulator over the whole GPU instead of
// averaging dense replicas.
//
// Semantics as linear_seq.hip (the reference's spoke,
// omldm/operators/spoke/FlinkSpoke.scala:92-107, with the Synchronous PS averaging the
// replicas): P spokes, spoke s fits rows [s·R, (s+1)·R) strictly one example at a time on
// its own replica of w, the round's model is the replica average. For additive learners
// the margin of row t of chunk k (64 rows) is
//     m_t = x_t·w + Σ_{s<t in the round} c_s·(x_s·x_t)
// and is split by distance:
//   * s in chunk k:        the scanner's recurrence over G_k (strictly lower Gram);
//   * s in chunk k − 1:    folded by the scanner while it scans chunk k − 1, through
//                          X1_k = X_k X_{k−1}ᵀ;
//   * s in chunks ≤ k − 2: the base margin the helper waves assemble before the chunk:
//                          dense columns from their running dense weights, categorical
//                          fields from the spoke's SLOT TABLE (LDS) for every slot that
//                          recurs two or more chunks apart, else from w itself.
// A slot that occurs only inside a window of two consecutive chunks never needs a table
// entry: G and X1 carry all its in-round updates. On the bench stream that leaves ~17.7 K
// table slots per 8192-row spoke (fits LDS), ~580 global gathers per chunk (v2: 1664) and
// no global atomics in the scan (v2: 1664 per chunk).
//
// The scanner keeps each row's affine candidate u = a·m + b instead of m (a = −1/(‖x‖² +
// kadd), b = y/(‖x‖² + kadd) for the hinge rule): with the Grams pre-scaled by the row's a
// (prep), one step of the recurrence is med3 → v_readlane → fma, on rows held in VGPRs.
//
// Passes of a round (1-3 model-independent: they run ahead on another stream):
//   1. s3_slots_kernel   tokens (or slots) → field-aware signed slots, FIELD-MAJOR [dc][B]
//   2. s3_flags_kernel   one workgroup per (field, spoke): an LDS hash table of the
//                        field's slots (first / last row), table ids, per-occurrence
//                        flags → occurrence records {slot, meta} [dc][B] (one 8-B load
//                        per occurrence in the scan)
//   3. s3_gram_kernel    one workgroup per (spoke, chunk): a_t, G_k and X1_k (categorical
//                        match counts and the dense block), scaled by a_t; the chunk's
//                        dense columns transposed for the helpers
//   4. s3_scan_kernel    one workgroup per spoke: scanner wave + 11 helper waves; in the
//                        same launch, combiner workgroups (one per spoke by default) fold
//                        dacc[slot] += inv_p·c·sign per occurrence WHILE the spoke scans:
//                        the scanner publishes each row's c as an {epoch, c} 8-B granule
//                        (write-through), the combiner polls the granules chunk by chunk,
//                        sums per slot in an LDS hash and adds each sum to dacc at the end
//   5. s3_tail_kernel    one block: the dense columns, scalars and statistics
//      (s3_scatter_kernel: the earlier whole-GPU combine after the scan, kept as the A/B
//      reference — omldm_scan3_set_comb(0))
#include "common.h"
#include "hash_dev.h"
#include "seq_common.h"

#include <mutex>
#include <unordered_map>

namespace omldm {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace s3 {
constexpr int CH = 64;                     // rows per chunk = scanner lanes
#ifndef OMLDM_S3_NH
#define OMLDM_S3_NH 11
#endif
// helper waves: 11 + the scanner = 12 waves, 3 per SIMD (≤ 168 VGPRs each): with 7 the
// helpers' ~6 K cycles per chunk matched the scanner's and set the chunk period
constexpr int NH = OMLDM_S3_NH;
constexpr int NT = 64 * (NH + 1);
constexpr int WPE = (NH + 1 + 3) / 4;      // waves per SIMD
// (idling the two helpers that share the scanner's SIMD left the chain as slow: 317 vs
// 303 µs per round — the SIMD's other waves are not what slows the scanner)
constexpr int NHA = NH;
constexpr int GS = CH + 4;                 // LDS row stride of G / X1
constexpr int MAXF = 32;                   // categorical fields per row
constexpr int NF = (MAXF + NHA - 1) / NHA;  // fields per working helper wave
constexpr int KNMAX = 32;                  // dense columns (numerical + intercept)
constexpr int NJ = (KNMAX + NHA - 1) / NHA;  // dense columns per working helper wave
constexpr int MAT = CH * CH;
constexpr int RMAX = 8192;                 // rows per spoke (16-bit rows in the flags table)
constexpr int WS = 8;                      // per-spoke stat row
constexpr int DS = KNMAX;                  // per-spoke dense delta row
// meta word of one occurrence: flags | sign | table id
constexpr uint32_t F_TG = 1u;              // margin reads the table (else w)
constexpr uint32_t F_INIT = 2u;            // first occurrence: writes w[slot] into the table
constexpr uint32_t F_SCAT = 4u;            // the slot recurs ≥ 2 chunks later: add c·sign
constexpr uint32_t F_SIGN = 8u;
// a non-table occurrence (its slot's occurrences span < 2 chunks) with the slot itself in
// the id bits: the in-scan combine adds its c·sign straight to the accumulator
constexpr uint32_t F_PRES = 16u;
constexpr uint32_t F_TAB = F_TG | F_INIT | F_SCAT;  // any occurrence of a table slot
constexpr int LID_SHIFT = 10;
}  // namespace s3

// floats of one chunk's prep block: aG | aX1 | a | dense columns transposed [KN][64] | y
// (the target as fp32, NaN for a row without one or past the shard: the scanner reads it
// a chunk ahead with no conversion — an int8 label's convert made it wait for the load)
// | σ_t | 1/σ_{t+1} (shrinking rules: the model scale before / after the row's step,
// s3_sigma_kernel). After the last spoke's blocks: σ at the end of each spoke [S].
template <int KN>
__host__ __device__ constexpr int s3_prep_floats() {
  return 2 * s3::MAT + s3::CH + KN * s3::CH + 3 * s3::CH;
}
template <int KN>
__host__ __device__ constexpr int s3_prep_y() {
  return 2 * s3::MAT + s3::CH + KN * s3::CH;
}
template <int KN>
__host__ __device__ constexpr int s3_prep_sg() {
  return s3_prep_y<KN>() + s3::CH;
}
template <int KN>
__host__ __device__ constexpr int s3_prep_hh() {
  return s3_prep_y<KN>() + 2 * s3::CH;
}
// the shrink of the model over row t of a spoke (local index i; y NaN: no step, no shrink)
__device__ __forceinline__ float s3_shrink(int shr, float r, float tbase, int i, float y) {
  if (shr == 0 || y != y) return 1.f;
  if (shr == 2) {
    const float T = tbase + (float)i;
    return (T - 1.f) / T;
  }
  return r;
}

__device__ __forceinline__ void spoke_rows(int s, int R, int B, int& t0, int& t1) {
  const long long a = (long long)s * R;
  t0 = a > B ? B : (int)a;
  t1 = (a + R) > B ? B : (int)(a + R);
}

// ------------------------------------------------------------------ pass 1: slots
// 256 rows per block through an LDS tile: coalesced row-major reads, coalesced
// field-major writes. hashed = 0: 32-bit tokens (murmur3 per field); 1: int32 signed
// slots; 2: the engine's compact uint16 {sign, local} (0xFFFF absent), slot = cbase +
// f·span + local (cbase: the feature space's dense slot count, which a preprocessor
// that widens the numerical block leaves unchanged) — the wire trains without widening.
__global__ __launch_bounds__(256) void s3_slots_kernel(const void* __restrict__ src, int B,
                                                       int dc, int dn, uint32_t span, int hashed,
                                                       int cbase, int* __restrict__ slotsT) {
  __shared__ int tile[256][s3::MAXF + 1];
  const int r0 = blockIdx.x * 256, tid = threadIdx.x;
  const int nr = min(256, B - r0);
  for (int i = tid; i < nr * dc; i += 256) {
    const int r = i / dc, f = i - r * dc;
    int slot;
    if (hashed == 2) {
      const uint32_t v = reinterpret_cast<const uint16_t*>(src)[(size_t)r0 * dc + i];
      slot = v == 0xFFFFu ? -1
                          : (int)(((uint32_t)cbase + (uint32_t)f * span + (v & 0x7FFFu)) |
                                  ((v & 0x8000u) << 16));
    } else {
      const uint32_t v = reinterpret_cast<const uint32_t*>(src)[(size_t)r0 * dc + i];
      slot = hashed ? (int)v : hash_token_dev(v, f, dn, span);
    }
    tile[r][f] = slot;
  }
  __syncthreads();
  if (tid < nr)
    for (int f = 0; f < dc; ++f) slotsT[(size_t)f * B + r0 + tid] = tile[tid][f];
}

// ------------------------------------------------------------------ pass 2: flags
// One workgroup per (field, spoke): every present occurrence of the field in the spoke's
// rows is inserted into an LDS hash table keyed by its slot, which keeps the slot's first
// and last row (LDS atomic min / max: a compare-and-swap loop on one packed word retried
// under contention — thousands of rows of a low-cardinality field on one entry). A slot
// whose first and last occurrence are two or more chunks apart gets a table id (one LDS
// add per wave, then a block base from the spoke's counter lidcount[s], zeroed before the
// launch); every occurrence gets its meta word: F_TG (the margin reads the table: a table
// slot seen in an earlier chunk), F_INIT (the table slot's first occurrence), F_SCAT (the
// slot recurs ≥ 2 chunks later), the sign and the table id; 0 for absent occurrences. No
// sort: the table ids only need to be unique within the spoke.
namespace s3 {
constexpr int FT = 1024;                   // flags threads
constexpr int HCAP = 12288;                // hash entries (≤ 8192 distinct slots: load ≤ 2/3)
constexpr int RPT = RMAX / FT;             // rows per thread (8)
}  // namespace s3

// Output: the meta words, [dc][B] uint32 (the slots stay in slotsT). enc: non-table
// occurrences carry F_PRES and their slot (slots < 2^22); l2s (or null): each table id's slot,
// [S][gs] (the in-scan combine's flush).
__global__ __launch_bounds__(s3::FT) void s3_flags_kernel(const int* __restrict__ slotsT, int B,
                                                          int R, uint32_t* __restrict__ meta,
                                                          int* __restrict__ lidcount, int enc,
                                                          int* __restrict__ l2s, long long gs) {
  __shared__ int hkey[s3::HCAP];        // slot, −1 empty; after the inserts: local table id
  __shared__ uint32_t hfirst[s3::HCAP];  // first row (atomic min)
  __shared__ uint32_t hlast[s3::HCAP];   // last row (atomic max)
  __shared__ int s_cnt, s_base;
  const int f = blockIdx.x, s = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  int t0, t1;
  spoke_rows(s, R, B, t0, t1);
  const int n = t1 - t0;
  if (n <= 0) return;
  for (int i = tid; i < s3::HCAP; i += s3::FT) {
    hkey[i] = -1;
    hfirst[i] = 0xFFFFFFFFu;
    hlast[i] = 0u;
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  const int* col = slotsT + (size_t)f * B + t0;
  int v[s3::RPT], h[s3::RPT];
#pragma unroll
  for (int q = 0; q < s3::RPT; ++q) {
    const int i = tid + q * s3::FT;
    v[q] = i < n ? col[i] : -1;
    h[q] = -1;
  }
#pragma unroll
  for (int q = 0; q < s3::RPT; ++q) {
    if (v[q] == -1) continue;
    const int i = tid + q * s3::FT;
    const int key = v[q] & 0x7fffffff;
    uint32_t at = __umulhi((uint32_t)key * 0x9E3779B1u, (uint32_t)s3::HCAP);
    for (int probe = 0; probe < s3::HCAP; ++probe) {  // bounded: load ≤ 2/3
      const int prev = atomicCAS(&hkey[at], -1, key);
      if (prev == -1 || prev == key) break;
      at = at + 1 == (uint32_t)s3::HCAP ? 0u : at + 1;
    }
    h[q] = (int)at;
    atomicMin(&hfirst[at], (uint32_t)i);
    atomicMax(&hlast[at], (uint32_t)i);
  }
  __syncthreads();
  // table ids: the first occurrence of every table slot takes one (one LDS add per wave)
  int lloc[s3::RPT];
#pragma unroll
  for (int q = 0; q < s3::RPT; ++q) {
    const int i = tid + q * s3::FT;
    bool take = false;
    if (h[q] >= 0) {
      const int first = (int)hfirst[h[q]], last = (int)hlast[h[q]];
      take = i == first && (last >> 6) - (first >> 6) >= 2;
    }
    const unsigned long long mask = __ballot(take);
    int wbase = 0;
    if (mask) {
      const int leader = __ffsll((long long)mask) - 1;
      if (lane == leader) wbase = atomicAdd(&s_cnt, __popcll(mask));
      wbase = __shfl(wbase, leader);
    }
    const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
    lloc[q] = take ? wbase + rank : -1;
  }
  __syncthreads();
  if (tid == 0) s_base = atomicAdd(&lidcount[s], s_cnt);
#pragma unroll
  for (int q = 0; q < s3::RPT; ++q)
    if (lloc[q] >= 0) hkey[h[q]] = lloc[q];  // the slot's key is no longer looked up
  __syncthreads();
  const int base = s_base;
#pragma unroll
  for (int q = 0; q < s3::RPT; ++q) {
    const int i = tid + q * s3::FT;
    if (i >= n) continue;
    uint32_t m = 0u;
    if (h[q] >= 0) {
      const int first = (int)hfirst[h[q]], last = (int)hlast[h[q]];
      const int ch = i >> 6;
      m = v[q] < 0 ? s3::F_SIGN : 0u;
      if ((last >> 6) - (first >> 6) >= 2) {
        if (ch > (first >> 6)) m |= s3::F_TG;
        if (i == first) m |= s3::F_INIT;
        if ((last >> 6) >= ch + 2) m |= s3::F_SCAT;
        m |= (uint32_t)(base + hkey[h[q]]) << s3::LID_SHIFT;
        if (l2s && lloc[q] >= 0) l2s[(size_t)s * gs + base + lloc[q]] = v[q] & 0x7fffffff;
      } else if (enc) {
        m |= s3::F_PRES | ((uint32_t)(v[q] & 0x7fffffff) << s3::LID_SHIFT);
      }
    }
    meta[(size_t)f * B + t0 + i] = m;
  }
}

// ------------------------------------------------------------------ pass 3: Grams
// Column factors of the Grams (logistic without shrink, cscale = lr): column t of aG_k and
// aX1_{k+1} is the effect of row t's step c_t = lr·y_t·ρ_t (ρ_t = 1/(1 + e^{y_t·u_t})), so
// with the columns scaled by lr·y_t the scanner's chain steps on ρ_t alone: two dependent
// multiplies fewer per row on the chain (scol[d][t]: row t of chunk c − d; 0 past the shard
// or without a target). The scan takes it from cb's rule: s3_scan_body, RULE logistic, !shr.
__device__ __forceinline__ void s3_gram_colscale(float (*scol)[s3::CH], float cscale,
                                                 const void* __restrict__ yv, int y8, int t0,
                                                 int t1, int c, int tid) {
  if (cscale == 0.f || tid >= 2 * s3::CH) return;
  const int d = tid / s3::CH, r = tid - d * s3::CH;
  const int row = t0 + (c - d) * s3::CH + r;
  const float y = (c - d >= 0 && row < t1) ? load_y(yv, row, y8) : 0.f;
  scol[d][r] = y == y ? cscale * y : 0.f;
}

// grid (chunks, S_act), 256 threads. Row scale a_t: −1/(‖x‖² + kadd) for the affine rules
// (hinge, ε-insensitive), 1 for logistic; 0 for rows past the shard. Out, per chunk:
// aG (strictly lower) | aX1 | a | dense [KN][64] (numerical columns, then the intercept).
template <int KN>
__global__ __launch_bounds__(256) void s3_gram_kernel(const int* __restrict__ slotsT, int dc,
                                                      const float* __restrict__ num, int dn,
                                                      const void* __restrict__ yv, int y8,
                                                      int B, int R, int bias, int affine,
                                                      float kadd, float* __restrict__ prep,
                                                      int nchs, int shr, float shr_r,
                                                      float cscale) {
  const int c = blockIdx.x, s = blockIdx.y;
  int t0, t1;
  spoke_rows(s, R, B, t0, t1);
  if (t0 + c * s3::CH >= t1) return;
  constexpr int PF = s3_prep_floats<KN>();
  float* out = prep + ((size_t)s * nchs + c) * PF;
  __shared__ alignas(16) int sl[2][s3::MAXF][s3::CH + 4];
  __shared__ float xn[2][s3::CH][KN + 1];
  __shared__ float sa[s3::CH];
  __shared__ float scol[2][s3::CH];  // column factors (s3_gram_colscale)
  const int tid = threadIdx.x;
  s3_gram_colscale(scol, cscale, yv, y8, t0, t1, c, tid);
  for (int i = tid; i < 2 * dc * s3::CH; i += 256) {
    const int d = i / (dc * s3::CH), rem = i - d * dc * s3::CH;
    const int f = rem / s3::CH, r = rem - f * s3::CH;  // field-major: coalesced per field
    const int cc = c - d, row = t0 + cc * s3::CH + r;
    sl[d][f][r] = (cc >= 0 && row < t1) ? slotsT[(size_t)f * B + row] : -1;
  }
  for (int i = tid; i < 2 * s3::CH * KN; i += 256) {
    const int d = i / (s3::CH * KN), rem = i - d * s3::CH * KN;
    const int r = rem / KN, j = rem - r * KN;
    const int cc = c - d, row = t0 + cc * s3::CH + r;
    float x = 0.f;
    if (cc >= 0 && row < t1) x = j < dn ? num[(size_t)row * dn + j] : ((bias && j == dn) ? 1.f : 0.f);
    xn[d][r][j] = x;
  }
  __syncthreads();
  if (tid < s3::CH) {
    float n2 = 0.f;
    for (int j = 0; j < KN; ++j) n2 = fmaf(xn[0][tid][j], xn[0][tid][j], n2);
    for (int f = 0; f < dc; ++f) n2 += sl[0][f][tid] != -1 ? 1.f : 0.f;
    const bool live = t0 + c * s3::CH + tid < t1;
    const float yt = live ? load_y(yv, t0 + c * s3::CH + tid, y8) : __builtin_nanf("");
    // a: −1/(‖x‖² + kadd) (affine 1: hinge, ε), 1 (0: logistic), y (2: Pegasos, u = y·v).
    // Shrinking affine rules scale the Grams by a·σ_t/σ_{t+1} = a/r (the scanner's u is
    // (a·m + b)/σ_{t+1}); the others keep u in v-space units
    // affine 3 (MultiClassPA, s3mc_scan_kernel): a = 1/(2‖x‖² + kadd), the Grams unscaled
    float a = 0.f, g = 1.f;
    if (live) {
      a = affine == 1 ? (n2 > 0.f ? -1.f / (n2 + kadd) : 0.f)
        : affine == 2 ? (yt == yt ? yt : 0.f)
        : affine == 3 ? (n2 > 0.f ? 1.f / (2.f * n2 + kadd) : 0.f) : 1.f;
      if (affine == 1 && shr == 1 && yt == yt) g = 1.f / shr_r;
    }
    sa[tid] = affine == 3 ? (live ? 1.f : 0.f) : a * g;
    out[2 * s3::MAT + tid] = a;
    out[s3_prep_y<KN>() + tid] = yt;
  }
  // dense columns transposed for the helper waves (coalesced per column)
  for (int i = tid; i < KN * s3::CH; i += 256) {
    const int j = i / s3::CH, r = i - j * s3::CH;
    out[2 * s3::MAT + s3::CH + i] = xn[0][r][j];
  }
  __syncthreads();
  const int bi = tid >> 4, bj = tid & 15;
#pragma unroll 1
  for (int d = 0; d < 2; ++d) {
    float acc[4][4] = {};
    if (c - d >= 0 && !(d == 0 && bj > bi)) {
      int cnt[4][4] = {};
      for (int f = 0; f < dc; ++f) {
        const int4 a4 = *reinterpret_cast<const int4*>(&sl[0][f][4 * bi]);
        const int4 b4 = *reinterpret_cast<const int4*>(&sl[d][f][4 * bj]);
        const int av[4] = {a4.x, a4.y, a4.z, a4.w}, bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int a = av[i] == -1 ? 0x7ffffffe : av[i];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int x = a ^ bv[j];
            cnt[i][j] += (x & 0x7fffffff) ? 0 : (x < 0 ? -1 : 1);
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
      const float a = sa[t];
      float4 v = make_float4(a * acc[i][0], a * acc[i][1], a * acc[i][2], a * acc[i][3]);
      if (cscale != 0.f) {
        v.x *= scol[d][4 * bj + 0];
        v.y *= scol[d][4 * bj + 1];
        v.z *= scol[d][4 * bj + 2];
        v.w *= scol[d][4 * bj + 3];
      }
      if (d == 0) {  // strictly lower: column ≥ row → 0
        if (4 * bj + 0 >= t) v.x = 0.f;
        if (4 * bj + 1 >= t) v.y = 0.f;
        if (4 * bj + 2 >= t) v.z = 0.f;
        if (4 * bj + 3 >= t) v.w = 0.f;
      }
      *reinterpret_cast<float4*>(&out[d * s3::MAT + t * s3::CH + 4 * bj]) = v;
    }
  }
}

// Diagnostics: bit 0 skips the categorical match counts, bit 1 the dense MFMA, bit 2 the
// output stores of s3_gram_mfma_kernel (scripts/gram_ablate.py; 0 in production)
__device__ int g_s3_gram_ablate = 0;

// Pass 3 on the matrix cores (the default; s3_gram_kernel above is the VALU reference the
// GPU test compares it with). grid (chunks, S_act), 256 threads = 4 waves. Every load of the
// chunk pair (slots of chunks c and c − 1, their numerical rows) is issued before the first
// LDS write — the VALU kernel's strided load loops waited on global memory once per
// iteration. Each wave then owns two 32 × 32 tiles of the output in the MFMA C layout
// (lane: column J0 + l31; register reg: row I0 + (reg & 3) + 8·(reg >> 2) + 4·(l >> 5)):
// the categorical ±1 match counts of its 16 (row, column) pairs go into the accumulator
// (exact small integers), then v_mfma_f32_32x32x2_f32 adds the dense Gram x_i·x_j over
// the KN columns. Tiles: aX1 (d = 1) tile (w >> 1, w & 1); aG (d = 0) tiles (0,0), (1,0),
// (1,1) on waves 0-2 (wave 3's upper-right aG tile is all zero).
template <int KN>
__global__ __launch_bounds__(256) void s3_gram_mfma_kernel(const int* __restrict__ slotsT, int dc,
                                                           const float* __restrict__ num, int dn,
                                                           const void* __restrict__ yv, int y8,
                                                           int B, int R, int bias, int affine,
                                                           float kadd, float* __restrict__ prep,
                                                           int nchs, int shr, float shr_r,
                                                           float cscale) {
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  const int c = blockIdx.x, s = blockIdx.y;
  int t0, t1;
  spoke_rows(s, R, B, t0, t1);
  if (t0 + c * s3::CH >= t1) return;
  constexpr int PF = s3_prep_floats<KN>();
  float* out = prep + ((size_t)s * nchs + c) * PF;
  __shared__ alignas(16) int sl[2][s3::MAXF][s3::CH + 4];
  __shared__ float xn[2][s3::CH][KN + 1];
  __shared__ float sa[s3::CH];
  __shared__ float scol[2][s3::CH];  // column factors (s3_gram_colscale)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  s3_gram_colscale(scol, cscale, yv, y8, t0, t1, c, tid);
  // ---- all loads in flight at once (clamped addresses, results selected after)
  constexpr int NSL = 2 * s3::MAXF * s3::CH / 256, NXN = 2 * s3::CH * KN / 256;
  int sv[NSL];
  float xv[NXN];
#pragma unroll
  for (int u = 0; u < NSL; ++u) {
    const int i = tid + 256 * u;  // [d][f][r], r fastest: coalesced per field
    const int d = i / (s3::MAXF * s3::CH), rem = i - d * s3::MAXF * s3::CH;
    const int f = rem / s3::CH, r = rem - f * s3::CH;
    const int cc = c - d, row = t0 + cc * s3::CH + r;
    const bool ok = f < dc && cc >= 0 && row < t1;
    const int v = slotsT[ok ? (size_t)f * B + row : 0];
    sv[u] = ok ? v : -1;
  }
#pragma unroll
  for (int u = 0; u < NXN; ++u) {
    const int i = tid + 256 * u;  // [d][r][j]
    const int d = i / (s3::CH * KN), rem = i - d * s3::CH * KN;
    const int r = rem / KN, j = rem - r * KN;
    const int cc = c - d, row = t0 + cc * s3::CH + r;
    const bool in = cc >= 0 && row < t1;
    const float x = dn > 0 ? num[(in && j < dn) ? (size_t)row * dn + j : 0] : 0.f;
    xv[u] = in ? (j < dn ? x : ((bias && j == dn) ? 1.f : 0.f)) : 0.f;
  }
#pragma unroll
  for (int u = 0; u < NSL; ++u) {
    const int i = tid + 256 * u;
    const int d = i / (s3::MAXF * s3::CH), rem = i - d * s3::MAXF * s3::CH;
    sl[d][rem / s3::CH][rem % s3::CH] = sv[u];
  }
#pragma unroll
  for (int u = 0; u < NXN; ++u) {
    const int i = tid + 256 * u;
    const int d = i / (s3::CH * KN), rem = i - d * s3::CH * KN;
    xn[d][rem / KN][rem % KN] = xv[u];
  }
  __syncthreads();
  if (tid < s3::CH) {
    float n2 = 0.f;
    for (int j = 0; j < KN; ++j) n2 = fmaf(xn[0][tid][j], xn[0][tid][j], n2);
    for (int f = 0; f < dc; ++f) n2 += sl[0][f][tid] != -1 ? 1.f : 0.f;
    const bool live = t0 + c * s3::CH + tid < t1;
    const float yt = live ? load_y(yv, t0 + c * s3::CH + tid, y8) : __builtin_nanf("");
    // a: −1/(‖x‖² + kadd) (affine 1: hinge, ε), 1 (0: logistic), y (2: Pegasos, u = y·v).
    // Shrinking affine rules scale the Grams by a·σ_t/σ_{t+1} = a/r (the scanner's u is
    // (a·m + b)/σ_{t+1}); the others keep u in v-space units
    // affine 3 (MultiClassPA, s3mc_scan_kernel): a = 1/(2‖x‖² + kadd), the Grams unscaled
    float a = 0.f, g = 1.f;
    if (live) {
      a = affine == 1 ? (n2 > 0.f ? -1.f / (n2 + kadd) : 0.f)
        : affine == 2 ? (yt == yt ? yt : 0.f)
        : affine == 3 ? (n2 > 0.f ? 1.f / (2.f * n2 + kadd) : 0.f) : 1.f;
      if (affine == 1 && shr == 1 && yt == yt) g = 1.f / shr_r;
    }
    sa[tid] = affine == 3 ? (live ? 1.f : 0.f) : a * g;
    out[2 * s3::MAT + tid] = a;
    out[s3_prep_y<KN>() + tid] = yt;
  }
  for (int i = tid; i < KN * s3::CH; i += 256) {
    const int j = i / s3::CH, r = i - j * s3::CH;
    out[2 * s3::MAT + s3::CH + i] = xn[0][r][j];
  }
  __syncthreads();
  const int l31 = lane & 31, hi = lane >> 5;
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    // pass 0: the aX1 tile (d = 1) of this wave; pass 1: its aG tile (d = 0)
    const int d = pass == 0 ? 1 : 0;
    // aG tiles: wave 0 (0,0), 1 (32,0), 2 (32,32), 3 (0,32) — the all-zero upper right
    const int I0 = pass == 0 ? 32 * (wave >> 1) : ((wave == 1 || wave == 2) ? 32 : 0);
    const int J0 = pass == 0 ? 32 * (wave & 1) : (wave >= 2 ? 32 : 0);
    const bool zero = (pass == 1 && wave == 3) || c - d < 0;
    f32x16 acc;
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[g] = 0.f;
    const int abl = g_s3_gram_ablate;
    if (!zero) {
      int cnt[16];
#pragma unroll
      for (int g = 0; g < 16; ++g) cnt[g] = 0;
      for (int f = 0; f < ((abl & 1) ? 0 : dc); ++f) {
        const int b = sl[d][f][J0 + l31];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int4 a4 = *reinterpret_cast<const int4*>(&sl[0][f][I0 + 8 * g + 4 * hi]);
          const int av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int a = av[e] == -1 ? 0x7ffffffe : av[e];
            const int x = a ^ b;
            cnt[4 * g + e] += (x & 0x7fffffff) ? 0 : (x < 0 ? -1 : 1);
          }
        }
      }
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[g] = (float)cnt[g];
      if (!(abl & 2)) {
#pragma unroll
        for (int k0 = 0; k0 < KN; k0 += 2)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xn[0][I0 + l31][k0 + hi],
                                                     xn[d][J0 + l31][k0 + hi], acc, 0, 0, 0);
      }
    }
    if (abl & 4) continue;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int t = I0 + (g & 3) + 8 * (g >> 2) + 4 * hi, col = J0 + l31;
      float v = sa[t] * acc[g];
      if (cscale != 0.f) v *= scol[d][col];
      if (d == 0 && col >= t) v = 0.f;  // aG strictly lower
      out[d * s3::MAT + t * s3::CH + col] = v;
    }
  }
}

// Pass 3b (shrinking rules only): per spoke, the model scale σ_t before and 1/σ_{t+1} after
// each row's step (σ ×= the row's shrink; rows without a target leave it alone) into the
// chunks' prep blocks, and σ at the spoke's end into sig[s]. One wave per spoke: each lane
// multiplies its run of rows, an exclusive product across the lanes, then each lane walks its
// run again from that prefix.
template <int KN>
__global__ __launch_bounds__(64) void s3_sigma_kernel(float* __restrict__ prep, int nchs, int B,
                                                      int R, int shr, float shr_r, float tbase,
                                                      float* __restrict__ sig) {
  constexpr int PF = s3_prep_floats<KN>();
  const int s = blockIdx.x, lane = threadIdx.x;
  int t0, t1;
  spoke_rows(s, R, B, t0, t1);
  const int n = t1 - t0;
  if (n <= 0) return;
  float* P0 = prep + (size_t)s * nchs * PF;
  auto at = [&](int i) -> float* { return P0 + (size_t)(i >> 6) * PF + (i & 63); };
  const int L = (n + 63) / 64, i0 = lane * L, i1 = min(n, i0 + L);
  float pr = 1.f;
  for (int i = i0; i < i1; ++i) pr *= s3_shrink(shr, shr_r, tbase, i, at(i)[s3_prep_y<KN>()]);
  float incl = pr;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float o = __shfl_up(incl, d, 64);
    if (lane >= d) incl *= o;
  }
  float sg = __shfl_up(incl, 1, 64);
  if (lane == 0) sg = 1.f;
  for (int i = i0; i < i1; ++i) {
    float* b = at(i);
    b[s3_prep_sg<KN>()] = sg;
    sg *= s3_shrink(shr, shr_r, tbase, i, b[s3_prep_y<KN>()]);
    b[s3_prep_hh<KN>()] = 1.f / sg;
  }
  const int tail = (64 - (n & 63)) & 63;  // rows past the shard in the last chunk
  if (lane < tail) {
    float* b = at(n + lane);
    b[s3_prep_sg<KN>()] = 1.f;
    b[s3_prep_hh<KN>()] = 1.f;
  }
  if (lane == 63) sig[s] = incl;
}

// ------------------------------------------------------------------ pass 4: scan
struct S3Smem {
  alignas(16) float G[2][s3::CH][s3::GS];   // aG_k by chunk parity
  alignas(16) float X1[2][s3::CH][s3::GS];  // aX1_{k+1} (read by the scanner in chunk k)
  float part[2][s3::NHA][s3::CH];           // base-margin partials per working helper
  float cb[2][s3::CH];                      // c of the chunk, by parity
  int last;                                 // s3_scan_arrive: this block arrived last
};
// + dynamic LDS: the slot table, `cap` floats

template <int RULE>
struct S3Cand {
  float lo, hi, d;
  __device__ __forceinline__ float operator()(float u, const SeqParams& p, float y) const {
    if constexpr (RULE == kSeqHinge) {
      return __builtin_amdgcn_fmed3f(u, lo, hi);
    } else if constexpr (RULE == kSeqEps) {
      return __builtin_amdgcn_fmed3f(u, 0.f, hi) + __builtin_amdgcn_fmed3f(u + d, lo, 0.f);
    } else if constexpr (RULE == kSeqPegasos) {  // u = y·v: a step below the threshold 1/σ_t
      return u < lo ? hi : 0.f;
    } else {  // lo = y·σ_t, hi = lr·y/σ_{t+1}
      return hi * __builtin_amdgcn_rcpf(1.f + __expf(lo * u));
    }
  }
};

__device__ unsigned long long* g_s3_stamps;
__device__ int g_s3_debug;  // diagnostics: 1 = every gather reads w[0] (latency experiment)
__device__ unsigned long long* g_s3mc_dbg;  // MultiClassPA scan phase cycles (null: off)
__device__ int g_s3_comb_err;  // a combiner gave up waiting for its spoke (bounded spin)
__device__ int g_s3_dense_order = 0;  // helpers' dense column ownership (see s3_scan_kernel)
__device__ int g_s3_hprio = 0;         // helpers' issue priorities by age (A/B: see s3_scan_body)

// The in-launch combine (Guideline 16, R2 "the data is the flag"): the scanner stores row
// t's c as one 8-B granule {epoch << 32 | bits(c)} with a relaxed agent-scope atomic store
// (global_store_dwordx2 sc1: write-through, no release fence), the combiner re-reads a
// chunk's 64 granules with agent-scope atomic loads (sc1, past its L1) until every tag is
// this round's epoch. The granule buffer is zeroed when allocated and every round on it
// takes the next epoch (never 0), so no granule of an earlier round can match.
typedef __attribute__((address_space(1))) unsigned long long s3_gu64;
template <bool B>
struct S3Tag {
  static constexpr bool value = B;
};
struct S3Comb {
  const int* lidcount;       // [S] table entries per spoke (the flags pass)
  unsigned long long* gran;  // [B] granules: the scanner's c per row
  uint32_t epoch;
  int S_act;                 // blocks [0, S_act) scan, the rest combine
  float* dacc;
  float inv_p;
  // the round's tail (dense columns, scalars, statistics) run by the last scan block to
  // finish: an epoch-tagged arrival word {epoch, count} (never zeroed: a word of an older
  // epoch restarts at 1), null → s3_tail_kernel / the scatter grid's extra row instead
  unsigned long long* arrive;
  double* cum;
  const float* sig;  // shrinking rules: σ at each spoke's end (its c's scale), else null
  int wbf;           // the model w is bf16 (modelDtype bf16: margins on the bf16 weights)
  int cns;           // spokes per combiner workgroup (> 1: one part, chunks interleaved)
  // in-scan combine (no combiner workgroups): the helpers add every table occurrence's
  // c·sign to the table and the scan workgroup flushes it through l2s ([S][gs]: each table
  // id's slot) at its end; a non-table occurrence's (F_PRES) goes to dacc from the helpers
  // (1: no c granules) or from the spoke's w0 workgroup after its pass (2: s3_fold_pres)
  const int* l2s;
  long long gs;
  int inscan;
};

// workgroups of one pipeline: its w0-margin (RARE) and scan workgroups, then its combiners
__host__ __device__ inline int s3_nper(int S_act, bool rare, int ncomb, int cns) {
  const int nc = cns > 1 ? (S_act + cns - 1) / cns : ncomb * S_act;
  return S_act * (rare ? 2 : 1) + (ncomb > 0 ? nc : 0);
}

// w[i] of a bf16 model (wbf) or an fp32 one
__device__ __forceinline__ float s3_w16(const float* w, long long i) {
  return __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(w)[i] << 16);
}
namespace s3 {
constexpr int CHASH = 8192;          // combiner LDS hash entries (keys in G, sums in X1)
constexpr unsigned SPIN_MAX = 1u << 21;      // polls before a combiner gives up (~1 s)
}  // namespace s3

// One combiner workgroup: spoke i mod S_act, part i / S_act. Its waves take the spoke's
// chunks round-robin (wave w of part j: chunks j·12 + w, then + 12·parts), every field of
// the chunk: a wave has 12 chunk periods to fold its chunk, so the combine keeps pace with
// the scanner and only the last chunk is left when the scan ends (one wave per field, every
// chunk, fell behind: its slot loads and its poll were one round trip each per chunk). All
// of a chunk's slot loads are issued before the poll. Rows with c = 0 add nothing.
// ns > 1: one combiner for spokes s .. s + ns − 1, their chunks interleaved in time order
// (chunk k of each spoke in turn: the spokes scan at the same pace) — fewer workgroups when
// a launch holds more pipelines than the GPU has CUs.
__device__ __forceinline__ void s3_combine_spoke(const int* __restrict__ slotsT, int dc, int B,
                                                 int R, const S3Comb& cb, S3Smem& sm, int s,
                                                 int part, int nparts, int ns = 1) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int* hk = reinterpret_cast<int*>(&sm.G[0][0][0]);
  float* hv = &sm.X1[0][0][0];
  for (int j = tid; j < s3::CHASH; j += s3::NT) {
    hk[j] = -1;
    hv[j] = 0.f;
  }
  __syncthreads();
  const int nchs = (R + s3::CH - 1) / s3::CH;  // chunks of a full spoke
  const int wstride = nparts * (s3::NH + 1);
  const unsigned long long want = (unsigned long long)cb.epoch;
  for (int kk = part * (s3::NH + 1) + wave; kk < nchs * ns; kk += wstride) {
    const int si = s + kk % ns, k = kk / ns;
    if (si >= cb.S_act) continue;
    int t0, t1;
    spoke_rows(si, R, B, t0, t1);
    // σ_end·Σ c·x: the spoke's Δ
    const float sc = cb.inv_p * (cb.sig ? cb.sig[si] : 1.f);
    const int row = t0 + k * s3::CH + lane;
    const bool in = row < t1;
    int v[s3::MAXF];
#pragma unroll
    for (int f = 0; f < s3::MAXF; ++f) {
      const bool ok = in && f < dc;
      const int x = slotsT[ok ? (size_t)f * B + row : 0];
      v[f] = ok ? x : -1;
    }
    unsigned long long g = 0;
    bool ready = false;
    for (unsigned spins = 0; spins < s3::SPIN_MAX; ++spins) {
      g = in ? __hip_atomic_load((s3_gu64*)(cb.gran + row), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT)
             : (want << 32);
      if (__builtin_amdgcn_ballot_w64((g >> 32) != want) == 0ull) {
        ready = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ready) {
      if (lane == 0) atomicExch(&g_s3_comb_err, 1);
      break;
    }
    const float c = __uint_as_float((uint32_t)g);
    if (__builtin_amdgcn_ballot_w64(c != 0.f) == 0ull) continue;
#pragma unroll
    for (int f = 0; f < s3::MAXF; ++f) {
      if (c == 0.f || v[f] == -1) continue;
      const int key = v[f] & 0x7fffffff;
      const float val = v[f] < 0 ? -c * sc : c * sc;
      uint32_t at = ((uint32_t)key * 0x9E3779B1u) >> (32 - 13);
      bool done = false;
      for (int probe = 0; probe < 8; ++probe) {
        const int prev = atomicCAS(&hk[at], -1, key);
        if (prev == -1 || prev == key) {
          atomicAdd(&hv[at], val);
          done = true;
          break;
        }
        at = (at + 1) & (s3::CHASH - 1);
      }
      if (!done) atomicAdd(&cb.dacc[key], val);
    }
  }
  __syncthreads();
  for (int j = tid; j < s3::CHASH; j += s3::NT) {
    const int key = hk[j];
    if (key != -1) atomicAdd(&cb.dacc[key], hv[j]);
  }
}

// The w0-margin workgroup of a spoke (round mode 4). Mode 4's slot table holds the spoke's
// DELTAS (zeroed at a slot's first occurrence, c·sign added by the scatter), so every
// occurrence's round-start weight w0[slot] is model-independent within the round: this
// workgroup gathers them for every chunk of its spoke, sums them per row and publishes the sum
// as a granule {epoch, Σ ±w0} — it depends on nothing in the round and runs ahead of the
// scan. The scan workgroup's helpers then issue no global gathers at all and read 4-byte meta
// words (flags, sign, table id) instead of {slot, meta}. Fields f ≡ wave (mod 12); a chunk's
// slots are loaded and its gathers issued a chunk ahead of their sum.
namespace s3 {
constexpr int NWR = NH + 1;                   // waves of the w0 workgroup (the block's)
constexpr int NFR = (MAXF + NWR - 1) / NWR;  // fields per wave
}  // namespace s3

__device__ __forceinline__ void s3_rare(const int* __restrict__ slotsT, int dc, int B, int R,
                                        const float* __restrict__ w, const S3Comb& cb,
                                        unsigned long long* __restrict__ rgran, S3Smem& sm, int s) {
  const int tid = threadIdx.x, r = tid & 63;
  const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
  int t0, t1;
  spoke_rows(s, R, B, t0, t1);
  if (t0 >= t1) return;
  const int nch = (t1 - t0 + s3::CH - 1) / s3::CH;
  float (*part)[s3::NWR][s3::CH] = reinterpret_cast<float (*)[s3::NWR][s3::CH]>(&sm.G[0][0][0]);
  const unsigned long long tag = (unsigned long long)cb.epoch << 32;
  struct Set {
    int cs[s3::NFR];
    float g[s3::NFR];
  };
  auto load_slots = [&](int ch, Set& S) {
#pragma unroll
    for (int i = 0; i < s3::NFR; ++i) {
      const int f = q + s3::NWR * i;
      const int row = t0 + ch * s3::CH + r;
      const bool ok = ch < nch && f < dc && row < t1;
      const int v = slotsT[ok ? (size_t)f * B + row : 0];
      S.cs[i] = ok ? v : -1;
    }
  };
  auto issue_gathers = [&](Set& S) {
    if (cb.wbf) {
#pragma unroll
      for (int i = 0; i < s3::NFR; ++i) S.g[i] = s3_w16(w, S.cs[i] != -1 ? (S.cs[i] & 0x7fffffff) : 0);
    } else {
#pragma unroll
      for (int i = 0; i < s3::NFR; ++i) S.g[i] = w[S.cs[i] != -1 ? (S.cs[i] & 0x7fffffff) : 0];
    }
  };
  auto body = [&](int k, Set& CUR, Set& NXT) {
    load_slots(k + 1, NXT);
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < s3::NFR; ++i)
      if (CUR.cs[i] != -1) m += CUR.cs[i] < 0 ? -CUR.g[i] : CUR.g[i];
    part[k & 1][q][r] = m;
    issue_gathers(NXT);
    __syncthreads();
    if (q == 0) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < s3::NWR; ++j) v += part[k & 1][j][r];
      const int row = t0 + k * s3::CH + r;
      if (row < t1)
        __hip_atomic_store((s3_gu64*)(rgran + row), tag | __float_as_uint(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  Set A, Bs;
  load_slots(0, A);
  issue_gathers(A);
  for (int k = 0; k < nch; k += 2) {
    body(k, A, Bs);
    if (k + 1 < nch) body(k + 1, Bs, A);
  }
}

// In-scan combine with the w0-margin workgroups (S3Comb::inscan 2): once its w0 pass is
// done, the spoke's w0 workgroup adds the non-table occurrences' c·sign (F_PRES: slots whose
// occurrences span < 2 chunks, each a few adds) straight to the accumulator as the scanner's
// granules arrive — chunks round-robin over its waves, every field of the chunk. (From the
// helpers, one global atomic of 64 distinct lines per field and chunk took ~700 cycles of
// the scan workgroup's memory pipeline per chunk.)
__device__ __forceinline__ void s3_fold_pres(const uint32_t* __restrict__ meta, int dc, int B,
                                             int R, const S3Comb& cb, int s) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int t0, t1;
  spoke_rows(s, R, B, t0, t1);
  const int nch = (t1 - t0 + s3::CH - 1) / s3::CH;
  const float sc = cb.inv_p * (cb.sig ? cb.sig[s] : 1.f);
  const unsigned long long want = (unsigned long long)cb.epoch;
  for (int k = wave; k < nch; k += s3::NH + 1) {
    const int row = t0 + k * s3::CH + lane;
    const bool in = row < t1;
    uint32_t m[s3::MAXF];
#pragma unroll
    for (int f = 0; f < s3::MAXF; ++f) {
      const bool ok = in && f < dc;
      const uint32_t x = meta[ok ? (size_t)f * B + row : 0];
      m[f] = ok ? x : 0u;
    }
    unsigned long long g = 0;
    bool ready = false;
    for (unsigned spins = 0; spins < s3::SPIN_MAX; ++spins) {
      g = in ? __hip_atomic_load((s3_gu64*)(cb.gran + row), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT)
             : (want << 32);
      if (__builtin_amdgcn_ballot_w64((g >> 32) != want) == 0ull) {
        ready = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ready) {
      if (lane == 0) atomicExch(&g_s3_comb_err, 1);
      return;
    }
    const float c = __uint_as_float((uint32_t)g) * sc;
    if (__builtin_amdgcn_ballot_w64(c != 0.f) == 0ull) continue;
#pragma unroll
    for (int f = 0; f < s3::MAXF; ++f)
      if (c != 0.f && (m[f] & s3::F_PRES))
        atomicAdd(&cb.dacc[m[f] >> s3::LID_SHIFT], (m[f] & s3::F_SIGN) ? -c : c);
  }
}

// A combiner workgroup: ns = 1: spoke i mod S_act, part i / S_act of the combiner blocks;
// ns > 1 (one part): spokes ns·i .. ns·i + ns − 1.
__device__ __forceinline__ void s3_combine(const int* __restrict__ slotsT, int dc, int B, int R,
                                           const S3Comb& cb, S3Smem& sm, int base, int bid,
                                           int nblk, int ns) {
  const int i = bid - base;
  if (ns > 1) {
    s3_combine_spoke(slotsT, dc, B, R, cb, sm, ns * i, 0, 1, ns);
    return;
  }
  s3_combine_spoke(slotsT, dc, B, R, cb, sm, i % cb.S_act, i / cb.S_act, (nblk - base) / cb.S_act);
}

// Forward: the tail body (defined with the combine pass below).
__device__ void s3_dense_body(const float* __restrict__ ws, const float* __restrict__ wsd,
                              const float* __restrict__ sig, int S_act, int dn, int dim, int bias,
                              float inv_p, float* __restrict__ dacc, double* __restrict__ cum);

// End of a scan workgroup (every wave comes here): with cb.arrive set, the block's spoke
// statistics / dense deltas are published (each wave drains its stores, the workgroup
// meets, one lane releases at agent scope and counts the block in), and the block that
// arrives last acquires and runs the round's tail (Guideline 16: release → counter,
// last arriver → acquire → plain loads). Saves the tail kernel's launch after the scan.
// (the flag lives in S3Smem: the kernel's static + dynamic LDS is exactly 160 KB)
__device__ __forceinline__ void s3_scan_arrive(const S3Comb& cb, const float* __restrict__ ws,
                                               const float* __restrict__ wsd, int dn, int dim,
                                               const SeqParams& p, S3Smem& sm) {
  if (cb.arrive == nullptr) return;
  int& s_last = sm.last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s3_gu64* a = (s3_gu64*)cb.arrive;
    unsigned long long old = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long nw;
    do {
      nw = (uint32_t)(old >> 32) == cb.epoch ? old + 1
                                             : (((unsigned long long)cb.epoch << 32) | 1ull);
    } while (!__hip_atomic_compare_exchange_weak(a, &old, nw, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    s_last = (int)(uint32_t)nw == cb.S_act;
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (s_last)
    s3_dense_body(ws, wsd, cb.sig, cb.S_act, dn, dim, p.bias, p.inv_p, cb.dacc, cb.cum);
}

// In-scan combine, the scan workgroup's end: its table's deltas into the accumulator, one
// atomic per table slot (mode 4's table holds deltas; mode 3's the running weights, so the
// round-start weight is taken off), ids past the LDS from the global spill.
template <bool RARE>
__device__ __forceinline__ void s3_inscan_flush(const S3Comb& cb, const float* tab,
                                                float* ag, int cap,
                                                const float* __restrict__ w, int s) {
  __syncthreads();  // the helpers' last scatter is in the table
  const int n = cb.lidcount[s];
  const float sc = cb.inv_p * (cb.sig ? cb.sig[s] : 1.f);
  const int* l2 = cb.l2s + (size_t)s * cb.gs;
  // FB entries per thread in flight: every slot load issued before the first atomic (one
  // entry at a time, each atomic waited for its slot's load: ~1 µs per entry)
  constexpr int FB = 8;
  for (int i0 = threadIdx.x; i0 < n; i0 += FB * s3::NT) {
    int slot[FB];
    float d[FB];
#pragma unroll
    for (int u = 0; u < FB; ++u) {
      const int i = i0 + u * s3::NT;
      slot[u] = l2[i < n ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < FB; ++u) {
      const int i = i0 + u * s3::NT;
      d[u] = i < min(n, cap) ? tab[i] : 0.f;
    }
    if (n > cap) {
#pragma unroll
      for (int u = 0; u < FB; ++u) {
        const int i = i0 + u * s3::NT;
        if (i >= cap && i < n)
          d[u] = __hip_atomic_load(&ag[i - cap], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if constexpr (!RARE) {
#pragma unroll
      for (int u = 0; u < FB; ++u) {
        const int i = i0 + u * s3::NT;
        const int sl = i < n ? slot[u] : 0;
        d[u] -= i < n ? (cb.wbf ? s3_w16(w, sl) : w[sl]) : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < FB; ++u) {
      const int i = i0 + u * s3::NT;
      if (i < n && d[u] != 0.f) atomicAdd(&cb.dacc[slot[u]], sc * d[u]);
    }
  }
}

// RARE (round mode 4): blocks [S_act, 2·S_act) are the spokes' rare-slot workgroups
// (s3_rare above) and the combiners follow them; the scanner adds each row's rare margin
// from its granule (rgran), the helpers gather only the table slots' first occurrences.
// One pipeline's workgroup `bid` of the round (`nblk` per pipeline): [0, S_act) the scan
// workgroups, [S_act, 2·S_act) the rare-slot ones (RARE), then the combiners.
// End of a scan workgroup with rows (every wave): with `tail` (a launch too large for
// in-launch combiners) the workgroup folds its own spoke's c·sign into the accumulator now
// that its scan is done (s3_combine_spoke over its LDS, free after the last chunk), then
// the arrival / round tail.
__device__ __forceinline__ void s3_spoke_end(bool tail, const int* __restrict__ slotsT, int dc,
                                             int B, int R, const S3Comb& cb,
                                             const float* __restrict__ ws,
                                             const float* __restrict__ wsd, int dn, int dim,
                                             const SeqParams& p, S3Smem& sm, int s) {
  if (tail) {
    __syncthreads();  // the scanner is done with G / X1
    s3_combine_spoke(slotsT, dc, B, R, cb, sm, s, 0, 1);
  }
  s3_scan_arrive(cb, ws, wsd, dn, dim, p, sm);
}

template <int RULE, int KN, bool RARE>
__device__ __forceinline__ void s3_scan_body(
    int bid, int nblk, int tail, S3Smem& sm, float* tab,
    const int* __restrict__ slotsT, const uint32_t* __restrict__ meta, int dc, int dn,
    const void* __restrict__ yv, int B, int R, const float* __restrict__ prep, int nchs,
    const float* __restrict__ w, int dim, float* __restrict__ aglob, int cap, long long gstride,
    const S3Comb& cb, float* __restrict__ ws, float* __restrict__ wsd, const SeqParams& p,
    unsigned long long* __restrict__ rgran) {
  constexpr int PF = s3_prep_floats<KN>();
  if (bid >= cb.S_act) {
    if (RARE && bid < 2 * cb.S_act) {  // a rare-slot workgroup
      s3_rare(slotsT, dc, B, R, w, cb, rgran, sm, bid - cb.S_act);
      if (cb.inscan == 2) s3_fold_pres(meta, dc, B, R, cb, bid - cb.S_act);
      if (tail == 2) {  // then the spoke's combiner: its w0 pass ends long before the scan
        __syncthreads();
        s3_combine_spoke(slotsT, dc, B, R, cb, sm, bid - cb.S_act, 0, 1);
      }
      return;
    }
    s3_combine(slotsT, dc, B, R, cb, sm, (RARE ? 2 : 1) * cb.S_act, bid, nblk, cb.cns);
    return;
  }
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int s = bid;
  int t0, t1;
  spoke_rows(s, R, B, t0, t1);
  if (t0 >= t1) {
    if (tid < s3::WS) ws[(size_t)s * s3::WS + tid] = 0.f;
    if (tid < s3::DS) wsd[(size_t)s * s3::DS + tid] = 0.f;
    s3_scan_arrive(cb, ws, wsd, dn, dim, p, sm);
    return;
  }
  const int nch = (t1 - t0 + s3::CH - 1) / s3::CH;
  const float* P0 = prep + (size_t)s * nchs * PF;
  auto chunk_prep = [&](int k) { return P0 + (size_t)k * PF; };
  float* ag = aglob + (size_t)s * gstride;

  unsigned long long* stamps = g_s3_stamps;
  const bool dbg_gather = g_s3_debug == 1;
  unsigned long long st_acc[12] = {};
  unsigned long long st_t = stamps ? clock64() : 0;
  auto stamp = [&](int k) {
    if (stamps) {
      const unsigned long long now = clock64();
      st_acc[k] += now - st_t;
      st_t = now;
    }
  };

  if (wave == 0) {
    // ---------------------------------------------------------------- scanner
    __builtin_amdgcn_s_setprio(3);
    float loss = 0.f, nex = 0.f, mist = 0.f, sqe = 0.f;
    float f1 = 0.f;  // a·(X1_k · c_{k−1}) for this lane's row of chunk k
    float ynx = chunk_prep(0)[s3_prep_y<KN>() + lane];
    float anx = chunk_prep(0)[2 * s3::MAT + lane];
    // shrinking rules (p.shr): the row's σ_t and 1/σ_{t+1} (s3_sigma_kernel), a chunk ahead
    const bool shr = p.shr != 0;
    float snx = shr ? chunk_prep(0)[s3_prep_sg<KN>() + lane] : 1.f;
    float hnx = shr ? chunk_prep(0)[s3_prep_hh<KN>() + lane] : 1.f;
    for (int k = -1; k <= nch; ++k) {
      if (k >= 0 && k < nch) {
        const int b = k & 1;
        const int row = t0 + k * s3::CH + lane;
        const bool valid = row < t1 && ynx == ynx;
        const float y = valid ? ynx : 0.f;
        const float a = valid ? anx : 0.f;
        const float sg = valid ? snx : 1.f, hh = valid ? hnx : 1.f;
        if (k + 1 < nch) {
          ynx = chunk_prep(k + 1)[s3_prep_y<KN>() + lane];
          anx = chunk_prep(k + 1)[2 * s3::MAT + lane];
          if (shr) {
            snx = chunk_prep(k + 1)[s3_prep_sg<KN>() + lane];
            hnx = chunk_prep(k + 1)[s3_prep_hh<KN>() + lane];
          }
        }
        float m0 = 0.f;
#pragma unroll
        for (int q = 0; q < s3::NHA; ++q) m0 += sm.part[b][q][lane];
        S3Cand<RULE> cf;
        float u, bc = 0.f;
        const float inv = -a;
        // shrinking rules keep v (w = σ·v) and step c' = c/σ_{t+1}: the affine rules' u is
        // (a·σ_t·v + b)/σ_{t+1} (Grams scaled by a/r in the prep), so b and the clamps take
        // the factor hh = 1/σ_{t+1} and the round-start margin a·σ_t·hh (sg = hh = 1 without)
        if constexpr (RULE == kSeqHinge) {
          bc = y * inv * hh;
          cf.lo = y < 0.f ? -p.cclip * hh : 0.f;
          cf.hi = y < 0.f ? 0.f : (y > 0.f ? p.cclip * hh : 0.f);
          u = fmaf(a * (sg * hh), m0, bc) + f1;
        } else if constexpr (RULE == kSeqEps) {
          bc = (y - p.eps) * inv * hh;
          cf.d = 2.f * p.eps * inv * hh;
          cf.lo = valid ? -p.cclip * hh : 0.f;
          cf.hi = valid ? p.cclip * hh : 0.f;
          u = fmaf(a * (sg * hh), m0, bc) + f1;
        } else if constexpr (RULE == kSeqPegasos) {
          // u = y·v (a = y): a step c' = y/(λ·T·σ_{t+1}) when y·σ_t·v < 1
          const float T = p.tbase + (float)(row - t0);
          cf.lo = valid ? 1.f / sg : 0.f;
          cf.hi = valid ? y * hh / (p.lam * T) : 0.f;
          u = fmaf(a, m0, 0.f) + f1;
        } else {
          cf.lo = y * sg;
          cf.hi = p.lr * y * hh;
          u = m0 + f1;
        }
        // the lane's rows of aG_k and aX1_{k+1} in VGPRs before the chain starts: an LDS
        // read inside the chain cost ~20 of its ~48 cycles per step (scan_chain_probe)
        const float* grow = &sm.G[b][lane][0];
        const float* xrow = &sm.X1[b ^ 1][lane][0];
        float gg[s3::CH], xx[s3::CH];
#pragma unroll
        for (int t4 = 0; t4 < s3::CH; t4 += 4) {
          const float4 g4 = *reinterpret_cast<const float4*>(grow + t4);
          const float4 x4 = *reinterpret_cast<const float4*>(xrow + t4);
          gg[t4] = g4.x, gg[t4 + 1] = g4.y, gg[t4 + 2] = g4.z, gg[t4 + 3] = g4.w;
          xx[t4] = x4.x, xx[t4 + 1] = x4.y, xx[t4 + 2] = x4.z, xx[t4 + 3] = x4.w;
        }
        stamp(8);
        float n1 = 0.f;
        // one step per row: lane t's step (its c, or for the logistic rule without shrink
        // ρ_t = 1/(1 + e^{y_t·u_t}) with lr·y_t in the Grams' columns, s3_gram_colscale)
        // broadcast, every later row's u and the next chunk's fold updated
        auto chain = [&](auto step) {
#pragma unroll
          for (int t = 0; t < s3::CH; ++t) {
            const float ct = readlane_f(step(u), t);
            u = fmaf(ct, gg[t], u);     // aG strictly lower: lane t frozen after step t
            n1 = fmaf(ct, xx[t], n1);   // → chunk k+1 (off the dependency chain)
            // pin the fold beside its step: left to itself the compiler parks the 64 c's
            // in SGPRs and runs the fold as a serial tail after the chunk
            asm volatile("" : "+v"(u), "+v"(n1));
          }
        };
        if constexpr (RULE == kSeqLogistic) {
          if (!shr) {
            const float lo2 = y * 1.44269504088896341f;  // e^{y·u} = 2^{y·log2(e)·u}
            chain([&](float v) {
              return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(lo2 * v));
            });
          } else {
            chain([&](float v) { return cf(v, p, y); });
          }
        } else {
          chain([&](float v) { return cf(v, p, y); });
        }
        stamp(9);
        const float c = cf(u, p, y);
        sm.cb[b][lane] = c;
        if (row < t1 && cb.inscan != 1)  // the row's granule (write-through): a combiner polls it
          __hip_atomic_store((s3_gu64*)(cb.gran + row),
                             ((unsigned long long)cb.epoch << 32) | __float_as_uint(c),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (valid) {
          float m;
          if constexpr (RULE == kSeqLogistic) m = sg * u;
          else if constexpr (RULE == kSeqPegasos) m = sg * y * u;
          else m = inv > 0.f ? (bc - u) * __builtin_amdgcn_rcpf(inv * hh) : 0.f;
          seq_stats<RULE>(m, y, p, loss, mist, sqe);
          nex += 1.f;
        }
        f1 = n1;
      }
      stamp(0);
      __syncthreads();
      stamp(1);
    }
    if (stamps && lane == 0)
      for (int q = 0; q < 12; ++q)
        if (q < 2 || q >= 8) atomicAdd(&stamps[(size_t)s * 16 + q], st_acc[q]);
    loss = wave_sum(loss);
    nex = wave_sum(nex);
    mist = wave_sum(mist);
    sqe = wave_sum(sqe);
    if (lane == 0) {
      float* wr = ws + (size_t)s * s3::WS;
      wr[0] = loss;
      wr[1] = nex;
      wr[2] = mist;
      wr[3] = sqe;
      wr[4] = 1.f;
      wr[5] = 0.f;
      wr[6] = 0.f;
      wr[7] = 0.f;
    }
    if (cb.inscan) s3_inscan_flush<RARE>(cb, tab, ag, cap, w, s);
    s3_spoke_end(tail == 1, slotsT, dc, B, R, cb, ws, wsd, dn, dim, p, sm, s);
    return;
  }

  // ------------------------------------------------------------------- helpers
  // helper q owns categorical fields f ≡ q and dense columns j ≡ q (mod NHA); lane r = row
  const int q = wave - 1, r = lane;
  const int swave = g_s3_debug >= 16 ? g_s3_debug - 16 : 1;  // the stamped helper wave
  // A/B (off): issue priority by age on each SIMD. With equal priorities the oldest wave
  // issues first and the youngest helpers (waves 8-11) set the chunk period; lifting them
  // moves the starvation to the oldest (profiles/round5/probe_helpers_prio.txt: 0.263-0.266
  // vs 0.270-0.274 ms) — the helpers share the SIMDs' issue slots, so only fewer helper
  // instructions shorten the period
  if (g_s3_hprio) {
    if (q >= 7) __builtin_amdgcn_s_setprio(2);
    else if (q >= 3) __builtin_amdgcn_s_setprio(1);
  }
  // dense column ownership: j ≡ q (mod NHA) (order 0), or in the reverse order of the
  // fields (order 1: the helpers that own a third categorical field do not also own a
  // second dense column)
  const int qd = g_s3_dense_order ? s3::NHA - 1 - q : q;
  const int kd = dn + (p.bias ? 1 : 0);  // real dense columns (KN pads them to 16 / 32)
  const int hl = q * 64 + lane;
  const bool inscan = cb.inscan != 0, inscan1 = cb.inscan == 1;  // 2: s3_fold_pres
  const uint32_t tmask = inscan ? s3::F_TAB : s3::F_SCAT;
  const float isc = inscan1 ? cb.inv_p * (cb.sig ? cb.sig[s] : 1.f) : 0.f;
  float wn[s3::NJ], w0[s3::NJ];  // running dense weights of this wave's columns, round start
#pragma unroll
  for (int i = 0; i < s3::NJ; ++i) {
    const int j = qd + s3::NHA * i;
    const int jw = j < dn ? j : dim - 1;
    const float wj = cb.wbf ? s3_w16(w, jw) : w[jw];
    w0[i] = (j < KN && (j < dn || (p.bias && j == dn))) ? wj : 0.f;
    wn[i] = w0[i];
  }
  // Software pipeline, one chunk ahead. Iteration k margins chunk cn = k + 1 and scatters
  // chunk k − 1 from the CUR set of registers while it fills the NXT set for chunk cn + 1:
  // its words (slot, meta), the Gram staging, the dense columns, and — once the words are
  // in, after this iteration's scatter and margins — the w gathers. Everything loaded is
  // model-independent (w is the round-start model), so no load waits on the chain. The
  // loop is unrolled by two with the sets swapping roles (a register rotation would make
  // every NXT load complete before the barrier), and every load is issued unconditionally
  // (clamped address, result selected after): loads under exec-masked branches leave the
  // compiler unable to count the loads in flight, and it would wait for all of them.
  constexpr int NV4 = (2 * s3::MAT / 4 + 64 * s3::NHA - 1) / (64 * s3::NHA);
  struct Set {
    int cs[s3::NF];
    uint32_t cm[s3::NF];
    float g[s3::NF];
    f32x4 v[NV4];
    float xs[s3::NJ], xc[s3::NJ];  // dense columns of the chunk scattered / margined
    unsigned long long rg;         // RARE, helper 0: the row's rare-slot margin granule
  };
  uint32_t p1[s3::NF], p2[s3::NF];  // meta of chunk k (scattered next) and k − 1
  // RARE: helper 0 loads each chunk's rare-slot margins (s3_rare's granules) with its words
  // — a chunk ahead, like every helper load, instead of the scanner waiting on L2 (measured:
  // a granule loaded by the scanner one chunk ahead still stalled it ≈ 2.2 K cycles per
  // chunk) — and folds them into its base-margin partial
  const unsigned long long want = (unsigned long long)cb.epoch;
  bool dead = false;
  auto load_rare = [&](int ch) -> unsigned long long {
    const int row = t0 + ch * s3::CH + r;
    const bool ok = RARE && q == 0 && ch >= 0 && ch < nch && row < t1;
    return ok ? __hip_atomic_load((s3_gu64*)(rgran + row), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT)
              : (want << 32);
  };
  auto load_words = [&](int ch, Set& S) {
    if constexpr (RARE) {  // 4-byte meta words; cs = 0 marks a table-slot occurrence
      S.rg = load_rare(ch);
#pragma unroll
      for (int i = 0; i < s3::NF; ++i) {
        const int f = q + s3::NHA * i;
        const int row = t0 + ch * s3::CH + r;
        const bool ok = ch >= 0 && ch < nch && f < dc && row < t1;
        const uint32_t mm = meta[ok ? (size_t)f * B + row : 0];
        S.cm[i] = ok ? mm : 0u;
        S.cs[i] = ok && (mm & (s3::F_TG | s3::F_INIT)) ? 0 : -1;
      }
      return;
    }
    // the helpers gather the non-table occurrences' w0 themselves: slot and meta word
#pragma unroll
    for (int i = 0; i < s3::NF; ++i) {
      const int f = q + s3::NHA * i;
      const int row = t0 + ch * s3::CH + r;
      const bool ok = ch >= 0 && ch < nch && f < dc && row < t1;
      const size_t at = ok ? (size_t)f * B + row : 0;
      const int sl = slotsT[at];
      const uint32_t mm = meta[at];
      S.cs[i] = ok ? sl : -1;
      S.cm[i] = ok ? mm : 0u;
    }
  };
  auto issue_gathers = [&](Set& S) {
    if constexpr (RARE) return;  // no gathers in the scan workgroup (s3_rare)
    if (cb.wbf) {
#pragma unroll
      for (int i = 0; i < s3::NF; ++i) {
        const bool glob = !RARE && S.cs[i] != -1 && !(S.cm[i] & s3::F_TG);
        S.g[i] = s3_w16(w, (glob && !dbg_gather) ? (S.cs[i] & 0x7fffffff) : 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < s3::NF; ++i) {
      // RARE: no gathers here (s3_rare sums every occurrence's w0)
      const bool glob = !RARE && S.cs[i] != -1 && !(S.cm[i] & s3::F_TG);
      S.g[i] = w[(glob && !dbg_gather) ? (S.cs[i] & 0x7fffffff) : 0];  // unused unless glob
    }
  };
  // aG_{ch} and aX1_{ch+1} (clamped reads past the round: never stored)
  auto issue_staging = [&](int ch, Set& S) {
#pragma unroll
    for (int u = 0; u < NV4; ++u) {
      const int i = min(hl + 64 * s3::NHA * u, 2 * s3::MAT / 4 - 1);
      const int mtx = i >> 10, e = i & 1023;
      const int kc = max(0, min(ch + mtx, nch - 1));
      S.v[u] = reinterpret_cast<const f32x4*>(chunk_prep(kc) + mtx * s3::MAT)[e];
    }
  };
  // dense columns of chunk ch (clamped chunk; 0 outside the round / past KN)
  constexpr int NJK = (KN + s3::NHA - 1) / s3::NHA;  // dense columns of this wave (≤ NJ)
  auto load_dense = [&](int ch, float* xd) {
#pragma unroll
    for (int i = 0; i < NJK; ++i) {
      const int j = qd + s3::NHA * i;
      const bool ok = j < KN && ch >= 0 && ch < nch;
      const int jc = j < KN ? j : 0, cc = max(0, min(ch, nch - 1));
      const float v = chunk_prep(cc)[2 * s3::MAT + s3::CH + jc * s3::CH + r];
      xd[i] = ok ? v : 0.f;
    }
  };
  // SPILL: the spoke's table outgrows the LDS (ids ≥ cap live in aglob). The two forms are
  // separate loops: a global table access anywhere in the loop made the compiler wait for
  // every load in flight (vmcnt(0)) before each field's margin, i.e. for the NXT set issued
  // at the top of the body — a memory round trip per chunk.
  auto body = [&](auto spill_tag, int k, Set& CUR, Set& NXT) {
    constexpr bool SPILL = decltype(spill_tag)::value;
    const int cn = k + 1, ks = k - 1;
    if (wave == swave) stamp(7);
    // ---- issue the NXT set (chunk cn + 1) but its gathers
    load_words(cn + 1, NXT);
    issue_staging(cn + 1, NXT);
    load_dense(ks + 1, NXT.xs);
    load_dense(cn + 1, NXT.xc);
    if (wave == swave) stamp(3);
    // ---- scatter chunk ks into the table and its dense update: one LDS atomic add per
    // occurrence (ds_add_f32; lanes on one entry are combined by the LDS unit inside the
    // instruction — a software loop over the ranks of equal slots cost 13 K cycles per
    // chunk, more than everything else of the chunk together)
    if (ks >= 0) {
      const float cv = sm.cb[ks & 1][r];
#pragma unroll
      for (int i = 0; i < s3::NF; ++i) {
        const uint32_t m = p2[i];
        // in-scan combine: every table occurrence into the table (an entry nobody reads
        // later takes the spoke's remaining deltas for the flush), the others to dacc
        const bool sc = (m & tmask) != 0u && cv != 0.f;
        const bool dr = inscan1 && (m & s3::F_PRES) != 0u && cv != 0.f;
        if (__builtin_amdgcn_ballot_w64(sc || dr) == 0ull) continue;
        const int lid = (int)(m >> s3::LID_SHIFT);
        const float val = (m & s3::F_SIGN) ? -cv : cv;
        if (dr) atomicAdd(&cb.dacc[lid], val * isc);  // lid = the slot (F_PRES)
        // (a branch-free form — every lane adding, the others 0 into a word of their own past
        // the table — measured slower: 961 → 1118 cycles per chunk)
        if (sc) {
          if constexpr (SPILL) {
            if (lid < cap) atomicAdd(&tab[lid], val);
            else atomicAdd(&ag[lid - cap], val);
          } else {
            atomicAdd(&tab[lid], val);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < NJK; ++i) {
        const int j = qd + s3::NHA * i;
        if (j < kd) wn[i] += wave_sum(cv * CUR.xs[i]);  // (padding columns are all zero)
      }
    }
    if (wave == swave) stamp(6);
    // ---- base margins of chunk cn: table entries (chunks ≤ k − 1 applied), w, dense
    if (cn < nch) {
      float base = 0.f;
#pragma unroll
      for (int i = 0; i < NJK; ++i) base = fmaf(CUR.xc[i], wn[i], base);
      if constexpr (RARE) {
        if (q == 0) {  // wave-uniform
          for (unsigned spins = 0;
               __builtin_amdgcn_ballot_w64((CUR.rg >> 32) != want) != 0ull;) {
            if (dead || ++spins > s3::SPIN_MAX) {  // bounded: the flag fails the round
              if (!dead && r == 0) atomicExch(&g_s3_comb_err, 2);
              dead = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            CUR.rg = load_rare(cn);
          }
          base += (CUR.rg >> 32) == want ? __uint_as_float((uint32_t)CUR.rg) : 0.f;
        }
      }
      if constexpr (!SPILL) {
        // every field's table reads first, then the first-occurrence writes: within a
        // chunk a table entry is either read (the slot was seen in an earlier chunk) or
        // written (its first occurrence), never both, and fields have disjoint slots — so
        // the reads need not wait for the previous field's write
        float tv[s3::NF];
#pragma unroll
        for (int i = 0; i < s3::NF; ++i) {
          const uint32_t m = CUR.cm[i];
          const bool tg = CUR.cs[i] != -1 && (m & s3::F_TG);
          tv[i] = 0.f;
          if (tg) tv[i] = tab[(int)(m >> s3::LID_SHIFT)];
        }
#pragma unroll
        for (int i = 0; i < s3::NF; ++i) {
          const uint32_t m = CUR.cm[i];
          const bool here = CUR.cs[i] != -1;
          const bool tg = here && (m & s3::F_TG), init = here && !tg && (m & s3::F_INIT);
          // RARE: the table holds the spoke's deltas (zeroed at the first occurrence)
          const float val = tg ? tv[i] : (RARE ? 0.f : CUR.g[i]);
          if (init) tab[(int)(m >> s3::LID_SHIFT)] = val;
          if (here && (!RARE || tg)) base += (m & s3::F_SIGN) ? -val : val;
        }
      }
#pragma unroll
      for (int i = 0; SPILL && i < s3::NF; ++i) {
        const uint32_t m = CUR.cm[i];
        const bool here = CUR.cs[i] != -1;
        const int lid = (int)(m >> s3::LID_SHIFT);
        const bool tg = here && (m & s3::F_TG), init = here && !tg && (m & s3::F_INIT);
        float val = RARE ? 0.f : CUR.g[i];
        // the table's global spill (lid ≥ cap) on its own wave-uniform path: a global
        // read merged into the LDS path would make every later use wait for all loads
        if (!SPILL || __builtin_amdgcn_ballot_w64((tg || init) && lid >= cap) == 0ull) {
          // exec-masked: the write needs the gathered w only on a slot's first occurrence (a
          // branch-free read + write per lane made every field's LDS write wait for its
          // gather: margins 1.6 K → 4.5 K cycles per chunk, scripts/scan3_probe.py)
          if (tg) val = tab[lid];
          if (init) tab[lid] = val;
        } else if constexpr (SPILL) {
          if (tg) val = lid < cap ? tab[lid] : __hip_atomic_load(&ag[lid - cap], __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
          if (init) {
            if (lid < cap) tab[lid] = val;
            else __hip_atomic_store(&ag[lid - cap], val, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (here && (!RARE || tg)) base += (m & s3::F_SIGN) ? -val : val;
      }
      sm.part[cn & 1][q][r] = base;
    }
    if (wave == swave) stamp(4);
    // ---- aG_{cn} → G[cn & 1], aX1_{cn+1} → X1[(cn+1) & 1]
#pragma unroll
    for (int u = 0; u < NV4; ++u) {
      const int i = hl + 64 * s3::NHA * u;
      const int mtx = i >> 10, e = i & 1023;
      if (i < 2 * s3::MAT / 4 && cn + mtx < nch) {
        const int row = e >> 4, col = (e & 15) * 4;
        float* dst = mtx == 0 ? &sm.G[cn & 1][row][col] : &sm.X1[(cn + 1) & 1][row][col];
        *reinterpret_cast<f32x4*>(dst) = CUR.v[u];
      }
    }
    // ---- the NXT gathers (its words have had the scatter and the margins to arrive)
    issue_gathers(NXT);
#pragma unroll
    for (int i = 0; i < s3::NF; ++i) {
      p2[i] = p1[i];
      p1[i] = CUR.cm[i];
    }
    if (wave == swave) stamp(5);
    __syncthreads();
  };

  Set A, Bs;
#pragma unroll
  for (int i = 0; i < s3::NF; ++i) p1[i] = p2[i] = 0u;
  load_words(0, A);
  issue_staging(0, A);
  load_dense(-2, A.xs);
  load_dense(0, A.xc);
  issue_gathers(A);
  if (cb.lidcount[s] <= cap) {  // the whole table in LDS (every spoke of the bench stream)
    for (int k = -1; k <= nch; k += 2) {
      body(S3Tag<false>{}, k, A, Bs);
      if (k + 1 <= nch) body(S3Tag<false>{}, k + 1, Bs, A);
    }
  } else {
    for (int k = -1; k <= nch; k += 2) {
      body(S3Tag<true>{}, k, A, Bs);
      if (k + 1 <= nch) body(S3Tag<true>{}, k + 1, Bs, A);
    }
  }
  if (stamps && lane == 0 && wave == swave)
    for (int k = 2; k < 8; ++k) atomicAdd(&stamps[(size_t)s * 16 + k], st_acc[k]);
  // round end: this wave's dense deltas
#pragma unroll
  for (int i = 0; i < s3::NJ; ++i) {
    const int j = qd + s3::NHA * i;
    if (lane == 0 && j < KN) wsd[(size_t)s * s3::DS + j] = wn[i] - w0[i];
  }
  if (q == 0 && lane >= KN && lane < s3::DS) wsd[(size_t)s * s3::DS + lane] = 0.f;
  if (cb.inscan) s3_inscan_flush<RARE>(cb, tab, ag, cap, w, s);
  s3_spoke_end(tail == 1, slotsT, dc, B, R, cb, ws, wsd, dn, dim, p, sm, s);
}

// Several pipelines that share one prep (the same batch and row scaling: BASELINE config 5's
// concurrent classifiers) in ONE launch, each with its own model, accumulator, granule
// buffers and rule constants (one pipeline is the M = 1 case). Blocks are pipeline-major and,
// within a pipeline, role-major — its w0-margin workgroups (RARE), its scan workgroups, its
// combiners — so the grid needs no co-residency: a block only waits on blocks dispatched
// before it (a scan on its w0 workgroup, a combiner on its scan), which never wait on it, and
// the later pipelines' blocks take the CUs the earlier ones free. One launch also sidesteps
// the four hardware queues per process that capped concurrent pipeline streams.
constexpr int kS3MaxPipes = 16;
struct S3Pipe {
  const float* w;
  float* aglob;
  float* ws;
  float* wsd;
  unsigned long long* rgran;
  S3Comb cb;
  SeqParams p;
};
struct S3Pipes {
  int M;
  int ncomb;  // combiner workgroups per spoke (0: none)
  int tail;   // 1: each scan workgroup combines its own spoke after its scan; 2: the
              // spoke's w0-margin workgroup combines it once its w0 pass is done (RARE)
  // the prep made on another stream: every workgroup waits for its ready word to reach
  // `wepoch` (omldm_scan3_signal at the prep's end) instead of the launch waiting on the
  // prep's event (null: no wait)
  const unsigned long long* wflag;
  unsigned long long wepoch;
  S3Pipe pipe[kS3MaxPipes];
};

// A prep's ready word: the prep made ahead on its own stream ends with this one-lane kernel
// (after the prep's kernels, stream order), and the round's launch waits for the word in
// its workgroups (s3_wait_prep) instead of a cross-stream wait on an event: the barrier
// packet released the scan ~11 µs after the previous round's apply and together with the
// next prep's kernels (~7 µs and ahead of them without it; 0.311 → 0.292 ms per round,
// profiles/round5/devgap/).
__global__ void s3_signal_kernel(unsigned long long* flag, unsigned long long epoch) {
  if (threadIdx.x == 0)
    __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// Bounded: a prep that never signals fails the round loudly (g_s3_comb_err = 3).
__device__ __forceinline__ void s3_wait_prep(const unsigned long long* flag,
                                             unsigned long long epoch) {
  if (flag == nullptr) return;
  if (threadIdx.x == 0) {
    for (unsigned spins = 0;
         __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch;) {
      if (++spins > s3::SPIN_MAX) {
        atomicExch(&g_s3_comb_err, 3);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the prep's data past stale lines
  }
  __syncthreads();
}

template <int RULE, int KN, bool RARE>
__global__ __launch_bounds__(s3::NT, s3::WPE) __attribute__((amdgpu_waves_per_eu(s3::WPE, s3::WPE))) void s3_scan_kernel(
    const int* __restrict__ slotsT, const uint32_t* __restrict__ meta, int dc, int dn,
    const void* __restrict__ yv, int B, int R, const float* __restrict__ prep, int nchs,
    int dim, int cap, long long gstride, int S_act, S3Pipes pp) {
  __shared__ S3Smem sm;
  extern __shared__ float tab[];  // [cap] + 64 scratch words (one per lane)
  const int nblk = s3_nper(S_act, RARE, pp.ncomb, pp.pipe[0].cb.cns);  // per pipeline
  const int pi = (int)blockIdx.x / nblk, local = (int)blockIdx.x % nblk;
  s3_wait_prep(pp.wflag, pp.wepoch);
  int bid;
  if (RARE && local < S_act) bid = S_act + local;  // its w0-margin workgroups first
  else if (RARE && local < 2 * S_act) bid = local - S_act;
  else bid = local;  // (!RARE: scan blocks [0, S_act), combiners after)
  const S3Pipe& P = pp.pipe[pi];
  s3_scan_body<RULE, KN, RARE>(bid, nblk, pp.tail, sm, tab, slotsT, meta,
                               dc, dn, yv, B, R, prep, nchs, P.w, dim, P.aglob, cap, gstride,
                               P.cb, P.ws, P.wsd, P.p, P.rgran);
}

// ------------------------------------------------------------------ pass 5: combine
// dacc[slot] = inv_p · Σ over the spokes' occurrences of c_row · sign. Grid (row blocks of
// SB rows, fields): a block first sums its occurrences per slot in an LDS hash table (a
// low-cardinality field puts thousands of occurrences on a handful of slots: one global
// atomic each serialised in L2 — 0.96 ms per round), then adds each distinct slot's sum
// to dacc with one fp32 atomic; occurrences that find no free entry within a few probes
// (high-cardinality fields: little repetition) go to dacc directly. c = 0 rows (most rows
// the PA rule leaves alone) are skipped. The spokes' sums meet in L2 in arrival order: the
// round's model is the replica average up to fp32 rounding of those sums.
// The dense columns (numerical, intercept) from the spokes' dense deltas, the
// accumulator's scalars and the round's statistics (one block of 256 threads; run as the extra row of the scatter grid).
__device__ void s3_dense_body(const float* __restrict__ ws,
                              const float* __restrict__ wsd, const float* __restrict__ sig,
                              int S_act, int dn, int dim, int bias, float inv_p,
                              float* __restrict__ dacc,
                              double* __restrict__ cum) {  // (blockDim ≥ 256; dn < 256)
  // shrinking rules: spoke s ends at σ_s·(w0 + δ_s): dacc gets Σ σ_s·δ_s and the apply's
  // coefficient of w0, dacc[dim] = Σ σ_s (linear_apply: w = (dacc[dim]·w + dacc)/dacc[dim+1])
  const int tid = threadIdx.x;
  // a round whose launch recorded a failed bounded wait (a prep that never signalled, a
  // combiner or helper that gave up) scanned stale or partial data: the apply discards it
  // (dacc[dim+1] < 0: w unchanged, dacc cleared; a large negative survives a cross-rank
  // sum, so every rank discards) and its statistics are not counted
  const bool bad = __hip_atomic_load(&g_s3_comb_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  for (int i = tid; i < dn; i += 256) {
    float v = 0.f;
    for (int s = 0; s < S_act; ++s) v += wsd[(size_t)s * s3::DS + i] * (sig ? sig[s] : 1.f);
    dacc[i] = v * inv_p;
  }
  if (tid == 0) {
    float v = 0.f, a = 0.f;
    if (bias)
      for (int s = 0; s < S_act; ++s) v += wsd[(size_t)s * s3::DS + dn] * (sig ? sig[s] : 1.f);
    for (int s = 0; s < S_act; ++s) a += sig ? sig[s] : 1.f;
    dacc[dim - 1] = v * inv_p;
    dacc[dim] = a * inv_p;
    dacc[dim + 1] = bad ? -1e30f : (float)S_act * inv_p;
  }
  if (cum && !bad && tid < 6 && tid != 4) {
    double t = 0.0;
    for (int s = 0; s < S_act; ++s) t += (double)ws[(size_t)s * s3::WS + tid];
    cum[tid] += t;
  }
}

namespace s3 {
constexpr int SB = 4096;     // rows per scatter block
constexpr int SH = 4096;     // LDS hash entries per block
constexpr int SPROBE = 8;
}  // namespace s3

__global__ __launch_bounds__(256) void s3_tail_kernel(const float* __restrict__ ws,
                                                      const float* __restrict__ wsd,
                                                      const float* __restrict__ sig, int S_act,
                                                      int dn, int dim, int bias, float inv_p,
                                                      float* __restrict__ dacc,
                                                      double* __restrict__ cum) {
  s3_dense_body(ws, wsd, sig, S_act, dn, dim, bias, inv_p, dacc, cum);
}

__global__ __launch_bounds__(256) void s3_scatter_kernel(const int* __restrict__ slotsT,
                                                         const unsigned long long* __restrict__ gran, int B,
                                                         int n_rows, float inv_p,
                                                         float* __restrict__ dacc, int dc,
                                                         const float* __restrict__ ws,
                                                         const float* __restrict__ wsd, int S_act,
                                                         int dn, int dim, int bias,
                                                         double* __restrict__ cum, int R,
                                                         const float* __restrict__ sig) {
  if ((int)blockIdx.y == dc) {  // the dense columns / scalars / statistics: one extra block
    if (blockIdx.x == 0) s3_dense_body(ws, wsd, sig, S_act, dn, dim, bias, inv_p, dacc, cum);
    return;
  }
  __shared__ int hk[s3::SH];
  __shared__ float hv[s3::SH];
  const int f = blockIdx.y, tid = threadIdx.x;
  const int r0 = blockIdx.x * s3::SB, r1 = min(n_rows, r0 + s3::SB);
  for (int i = tid; i < s3::SH; i += 256) {
    hk[i] = -1;
    hv[i] = 0.f;
  }
  __syncthreads();
  const int* col = slotsT + (size_t)f * B;
  for (int row = r0 + tid; row < r1; row += 256) {
    const int v = col[row];
    if (v == -1) continue;
    const float c = __uint_as_float((uint32_t)gran[row]);  // a kernel boundary after the scan
    if (c == 0.f) continue;
    const int key = v & 0x7fffffff;
    const float sc = sig ? inv_p * sig[row / R] : inv_p;
    const float val = v < 0 ? -c * sc : c * sc;
    uint32_t at = ((uint32_t)key * 0x9E3779B1u) >> (32 - 12);
    bool done = false;
    for (int probe = 0; probe < s3::SPROBE; ++probe) {
      const int prev = atomicCAS(&hk[at], -1, key);
      if (prev == -1 || prev == key) {
        atomicAdd(&hv[at], val);
        done = true;
        break;
      }
      at = (at + 1) & (s3::SH - 1);
    }
    if (!done) atomicAdd(&dacc[key], val);
  }
  __syncthreads();
  for (int i = tid; i < s3::SH; i += 256) {
    const int key = hk[i];
    if (key != -1) atomicAdd(&dacc[key], hv[i]);
  }
}

// ------------------------------------------------------------------ MultiClassPA on v3
// The reference's MultiClassPA (K prototypes; row t moves prototype y_t by +τ·x_t and the
// best wrong one r_t by −τ·x_t, τ = min(C, ℓ/(2‖x‖²)), ℓ = max(0, 1 − (s_y − s_r))) on the
// same prep as the binary scan (slots, occurrence flags, unscaled chunk Grams, a_t =
// 1/(2‖x‖² + kadd)). Per spoke one 12-wave workgroup: the scanner keeps the K scores of its
// row as u[k] = (base margin) + Σ_{s<t} c_s^k·G_ts, the step broadcasts (τ_t, r_t) and
// every lane adds ±τ_t·G[lane][t] to two of its K scores; the helpers assemble the K base
// margins from the slot table (K floats per table slot: w0 at the first occurrence, the
// spoke's updates added by the scatter) or the key-major prototypes, and stage the Grams.
// Each row's (τ, r) goes to a record; s3mc_scatter_kernel adds the spokes' updates after.
// K ∈ {2, 4, 8, 16} (nclass ≤ K; the classes past nclass cost uniform branches only): the
// helpers add their base-margin partials into one K × 64 array with LDS 64-bit integer
// atomics on 32.32 fixed point (the scanner reads K values per lane per chunk and clears
// them), so the LDS the scan needs grows by K·1 KB, not by K·NHA·512 B — and the sum is
// independent of the helpers' arrival order: with float atomics a near-tie between two
// classes could resolve differently from run to run (the argmax is discontinuous).
namespace s3 {
constexpr int MCK = 16;  // classes on the v3 multiclass scan (more: the spoke tables)
}

template <int K>
struct S3McSmem {
  alignas(16) float G[2][s3::CH][s3::GS];
  alignas(16) float X1[2][s3::CH][s3::GS];
  long long part[2][K][s3::CH];  // base margins by class, 32.32 fixed point (LDS atomics)
  float tau[2][s3::CH];      // τ of the chunk's rows, by parity
  int rr[2][s3::CH];         // r (the updated wrong class) of the chunk's rows
};

// Branch-free (selects only): on the scanner's chain, a data-dependent branch per class
// (exec-mask save / restore and a scalar branch) cost ~700 cycles per step at K = 4.
template <int K>
__device__ __forceinline__ void s3mc_decide(const float (&u)[K], int yi, int nclass, float a,
                                            float cmax, bool valid, float& tau, int& r,
                                            float& margin) {
  float sy = 0.f, best = -INFINITY;
  r = -1;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float v = u[k];
    const bool isy = k == yi;
    sy = isy ? v : sy;
    const bool gt = k < nclass && !isy && v > best;  // ties: the lowest index
    best = gt ? v : best;
    r = gt ? k : r;
  }
  margin = sy - best;
  const float loss = fmaxf(0.f, 1.f - margin);
  tau = (valid && r >= 0 && a > 0.f) ? fminf(cmax, loss * a) : 0.f;
}

// The scanner's form: w[c] = the row's score of class c with −inf at its own class (and
// past nclass), sy = its own class's score — both kept up to date by the steps, so the
// best wrong class is a max tree of depth log2 K (ties: the lowest index, as the scan in
// class order) instead of a K-long compare chain on the step's critical path.
template <int K>
__device__ __forceinline__ void s3mc_decide_w(const float (&w)[K], float sy, float a, float cmax,
                                              bool valid, float& tau, int& r, float& margin) {
  float v[K];
  int ix[K];
#pragma unroll
  for (int c = 0; c < K; ++c) v[c] = w[c], ix[c] = c;
#pragma unroll
  for (int st = 1; st < K; st <<= 1) {
#pragma unroll
    for (int i = 0; i + st < K; i += 2 * st) {
      const bool gt = v[i + st] > v[i];
      v[i] = gt ? v[i + st] : v[i];
      ix[i] = gt ? ix[i + st] : ix[i];
    }
  }
  r = v[0] == -INFINITY ? -1 : ix[0];
  margin = sy - v[0];
  const float loss = fmaxf(0.f, 1.f - margin);
  tau = (valid && r >= 0 && a > 0.f) ? fminf(cmax, loss * a) : 0.f;
}

#ifndef S3MC_PAIR_TREE_K
#define S3MC_PAIR_TREE_K 2  // (value, index) pair tree up to this K; the fmax / OR tree above
#endif
// K > S3MC_PAIR_TREE_K, the same form: the best wrong score by an fmax tree, its class as the lowest set
// bit of the classes equal to it (an OR tree of one-hot words): depth ~2·log2 K, and no
// (value, index) pair arrays (the wide templates' VGPR budget).
template <int N>
__device__ __forceinline__ float s3mc_tmax(const float* v) {
  if constexpr (N == 1) return v[0];
  else return fmaxf(s3mc_tmax<N / 2>(v), s3mc_tmax<N - N / 2>(v + N / 2));
}
template <int N>
__device__ __forceinline__ uint32_t s3mc_tbits(const float* v, float best, int c0) {
  if constexpr (N == 1) return v[0] == best ? (1u << c0) : 0u;
  else return s3mc_tbits<N / 2>(v, best, c0) | s3mc_tbits<N - N / 2>(v + N / 2, best, c0 + N / 2);
}
template <int K>
__device__ __forceinline__ void s3mc_decide_w2(const float (&w)[K], float sy, float a, float cmax,
                                               bool valid, float& tau, int& r, float& margin) {
  const float best = s3mc_tmax<K>(w);
  const uint32_t bits = s3mc_tbits<K>(w, best, 0);
  r = best == -INFINITY ? -1 : (int)__builtin_ctz(bits | 0x80000000u);
  margin = sy - best;
  const float loss = fmaxf(0.f, 1.f - margin);
  tau = (valid && r >= 0 && a > 0.f) ? fminf(cmax, loss * a) : 0.f;
}

// The coefficient of class c in a step that moves class yt by +τ and class rt by −τ:
// uniform operands, selected on the scalar unit (the sign through the bit pattern).
__device__ __forceinline__ float s3mc_coef(int c, int yt, int rt, uint32_t ctb) {
  const uint32_t v = c == yt ? ctb : (c == rt ? (ctb ^ 0x80000000u) : 0u);
  return __uint_as_float(v);
}

struct S3McArgs {
  const float* Wt;  // key-major prototypes [dim][kp] (fp32)
  int kp, nclass, variant;
  float cmax;       // C (PA-I), +inf otherwise
  float* ws;        // [S][WS] loss, rows, mistakes
  float* wsd;       // [S][K][DS] dense-column updates per class
  float* aglob;     // [S][gstride·K] the slot table past the LDS
  float* tau;       // [B] τ per row
  int* rr;          // [B] r per row
};

template <int K, int KN>
__global__ __launch_bounds__(s3::NT, s3::WPE) __attribute__((amdgpu_waves_per_eu(s3::WPE, s3::WPE))) void s3mc_scan_kernel(
    const int* __restrict__ slotsT, const uint32_t* __restrict__ meta,
    const int* __restrict__ lidcount, int dc, int dn, int bias, int B, int R,
    const float* __restrict__ prep, int nchs, int dim, int cap, long long gstride, S3McArgs A) {
  __shared__ S3McSmem<K> sm;
  extern __shared__ float tab[];  // [cap]: table slot i's class k at i·K + k
  constexpr int PF = s3_prep_floats<KN>();
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int s = blockIdx.x;
  int t0, t1;
  spoke_rows(s, R, B, t0, t1);
  if (t0 >= t1) {
    if (tid < s3::WS) A.ws[(size_t)s * s3::WS + tid] = 0.f;
    for (int i = tid; i < K * s3::DS; i += s3::NT) A.wsd[(size_t)s * K * s3::DS + i] = 0.f;
    return;
  }
  const int nch = (t1 - t0 + s3::CH - 1) / s3::CH;
  const float* P0 = prep + (size_t)s * nchs * PF;
  auto chunk_prep = [&](int k) { return P0 + (size_t)k * PF; };
  float* ag = A.aglob + (size_t)s * gstride * K;
  for (int i = tid; i < 2 * K * s3::CH; i += s3::NT) (&sm.part[0][0][0])[i] = 0;
  __syncthreads();

  if (wave == 0) {
    // ---------------------------------------------------------------- scanner
    __builtin_amdgcn_s_setprio(3);
    float loss = 0.f, nex = 0.f, mist = 0.f;
    float f1[K];
#pragma unroll
    for (int k = 0; k < K; ++k) f1[k] = 0.f;
    float ynx = chunk_prep(0)[s3_prep_y<KN>() + lane];
    float anx = chunk_prep(0)[2 * s3::MAT + lane];
    unsigned long long* const dbg = g_s3mc_dbg;
    unsigned long long t_chain = 0, t_wait = 0;
    for (int k = -1; k <= nch; ++k) {
      const unsigned long long ta = dbg ? __builtin_amdgcn_s_memtime() : 0;
      if (k >= 0 && k < nch) {
        const int b = k & 1;
        const int row = t0 + k * s3::CH + lane;
        const bool valid = row < t1 && ynx == ynx;
        const int yi = valid ? (int)ynx : -1;
        const float a = valid ? anx : 0.f;
        if (k + 1 < nch) {
          ynx = chunk_prep(k + 1)[s3_prep_y<KN>() + lane];
          anx = chunk_prep(k + 1)[2 * s3::MAT + lane];
        }
        // K ≤ 4: w[c] = the row's score of class c with −inf at its own class (and past
        // nclass), sy = its own class's score, both kept up to date by the steps, and the
        // best wrong class a max tree (s3mc_decide_w); K ≥ 8: the plain scores u = w and
        // the branch-free class scan (s3mc_decide) — measured per K (profiles/round6/mc/)
        constexpr bool TREE = true;  // the masked form at every K (decide_w / decide_w2)
        float w[K], n1[K], sy = 0.f;
#pragma unroll
        for (int c = 0; c < K; ++c) {
          const float v = (float)(__ll2double_rn(sm.part[b][c][lane]) * 0x1p-32) + f1[c];
          sm.part[b][c][lane] = 0;  // the helpers add chunk k + 2's partials here
          n1[c] = 0.f;
          sy = c == yi ? v : sy;
          w[c] = TREE && (c == yi || c >= A.nclass) ? -INFINITY : v;
        }
        // the lane's row of G_k in VGPRs; the chunk's steps are kept (τ_t, r_t, y_t) and
        // folded into chunk k+1 through X1 after the chain (off it, from LDS)
        const float* grow = &sm.G[b][lane][0];
        float gg[s3::CH];
#pragma unroll
        for (int t4 = 0; t4 < s3::CH; t4 += 4) {
          const float4 g4 = *reinterpret_cast<const float4*>(grow + t4);
          gg[t4] = g4.x, gg[t4 + 1] = g4.y, gg[t4 + 2] = g4.z, gg[t4 + 3] = g4.w;
        }
        float tl, mg;
        int rl;
#pragma unroll
        for (int t = 0; t < s3::CH; ++t) {
          if constexpr (K <= S3MC_PAIR_TREE_K) s3mc_decide_w<K>(w, sy, a, A.cmax, valid, tl, rl, mg);
          else s3mc_decide_w2<K>(w, sy, a, A.cmax, valid, tl, rl, mg);
          const uint32_t ctb = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(tl), t);
          const int rt = __builtin_amdgcn_readlane(rl, t);
          const int yt = __builtin_amdgcn_readlane(yi, t);
#pragma unroll
          for (int c = 0; c < K; ++c)  // G strictly lower: lane t frozen after step t
            w[c] = fmaf(s3mc_coef(c, yt, rt, ctb), gg[t], w[c]);  // −inf stays −inf
          if constexpr (TREE) sy = fmaf(s3mc_coef(yi, yt, rt, ctb), gg[t], sy);
        }
        if constexpr (K <= S3MC_PAIR_TREE_K) s3mc_decide_w<K>(w, sy, a, A.cmax, valid, tl, rl, mg);
        else s3mc_decide_w2<K>(w, sy, a, A.cmax, valid, tl, rl, mg);
        // chunk k+1's X1 fold: n1[c] = Σ_t c_t^c · X1_{k+1}[lane][t]
        {
          const float* xrow = &sm.X1[b ^ 1][lane][0];
#pragma unroll 8
          for (int t = 0; t < s3::CH; ++t) {
            const uint32_t ctb = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(tl), t);
            const int rt = __builtin_amdgcn_readlane(rl, t);
            const int yt = __builtin_amdgcn_readlane(yi, t);
            const float x = xrow[t];
#pragma unroll
            for (int c = 0; c < K; ++c) n1[c] = fmaf(s3mc_coef(c, yt, rt, ctb), x, n1[c]);
          }
        }
        sm.tau[b][lane] = tl;
        sm.rr[b][lane] = rl;
        if (row < t1) {
          A.tau[row] = tl;
          A.rr[row] = rl;
        }
        if (valid) {
          loss += fmaxf(0.f, 1.f - mg);
          nex += 1.f;
          mist += mg <= 0.f ? 1.f : 0.f;
        }
#pragma unroll
        for (int c = 0; c < K; ++c) f1[c] = n1[c];
      }
      if (dbg) {
        const unsigned long long tb = __builtin_amdgcn_s_memtime();
        __syncthreads();
        t_chain += tb - ta;
        t_wait += __builtin_amdgcn_s_memtime() - tb;
      } else {
        __syncthreads();
      }
    }
    loss = wave_sum(loss);
    nex = wave_sum(nex);
    mist = wave_sum(mist);
    if (lane == 0) {
      float* wr = A.ws + (size_t)s * s3::WS;
      wr[0] = loss, wr[1] = nex, wr[2] = mist;
      for (int i = 3; i < s3::WS; ++i) wr[i] = 0.f;
      if (dbg) {  // [s·8]: chunks, scanner chain, scanner barrier wait, helper phases (sums)
        atomicAdd(&dbg[s * 8 + 0], (unsigned long long)nch);
        atomicAdd(&dbg[s * 8 + 1], t_chain);
        atomicAdd(&dbg[s * 8 + 2], t_wait);
      }
    }
    return;
  }

  // ------------------------------------------------------------------- helpers
  const int q = wave - 1, r = lane;
  const int kd = dn + (bias ? 1 : 0);
  const int hl = q * 64 + lane;
  const int capid = cap / K;  // table slots in LDS; the rest in ag (global)
  constexpr int NJK0 = (KN + s3::NHA - 1) / s3::NHA;  // this wave's dense columns
  float wn[K][NJK0];  // the round-start values are re-read at the round end
  auto w0_at = [&](int i, int c) {
    const int j = q + s3::NHA * i;
    const int key = j < dn ? j : dim - 1;
    const bool real = j < KN && (j < dn || (bias && j == dn));
    return real ? A.Wt[(size_t)key * A.kp + c] : 0.f;
  };
#pragma unroll
  for (int i = 0; i < NJK0; ++i)
#pragma unroll
    for (int c = 0; c < K; ++c) wn[c][i] = w0_at(i, c);
  constexpr int NV4 = (2 * s3::MAT / 4 + 64 * s3::NHA - 1) / (64 * s3::NHA);
  constexpr int NJK = (KN + s3::NHA - 1) / s3::NHA;
  struct Set {
    int cs[s3::NF];
    uint32_t cm[s3::NF];
    float g[s3::NF][K];
    f32x4 v[NV4];
    float xs[s3::NJ], xc[s3::NJ];
  };
  uint32_t p1[s3::NF], p2[s3::NF];
  auto load_words = [&](int ch, Set& S) {
#pragma unroll
    for (int i = 0; i < s3::NF; ++i) {
      const int f = q + s3::NHA * i;
      const int row = t0 + ch * s3::CH + r;
      const bool ok = ch >= 0 && ch < nch && f < dc && row < t1;
      const size_t at = ok ? (size_t)f * B + row : 0;
      const int sl = slotsT[at];
      const uint32_t mm = meta[at];
      S.cs[i] = ok ? sl : -1;
      S.cm[i] = ok ? mm : 0u;
    }
  };
  auto issue_gathers = [&](Set& S) {
#pragma unroll
    for (int i = 0; i < s3::NF; ++i) {
      const bool glob = S.cs[i] != -1 && !(S.cm[i] & s3::F_TG);
      const float* src = A.Wt + (size_t)(glob ? (S.cs[i] & 0x7fffffff) : 0) * A.kp;
      if constexpr (K >= 4) {
#pragma unroll
        for (int c4 = 0; c4 < K; c4 += 4) {
          const float4 v = *reinterpret_cast<const float4*>(src + c4);
          S.g[i][c4] = v.x, S.g[i][c4 + 1] = v.y, S.g[i][c4 + 2] = v.z, S.g[i][c4 + 3] = v.w;
        }
      } else {
        const float2 v = *reinterpret_cast<const float2*>(src);
        S.g[i][0] = v.x, S.g[i][1] = v.y;
      }
    }
  };
  auto issue_staging = [&](int ch, Set& S) {
#pragma unroll
    for (int u = 0; u < NV4; ++u) {
      const int i = min(hl + 64 * s3::NHA * u, 2 * s3::MAT / 4 - 1);
      const int mtx = i >> 10, e = i & 1023;
      const int kc = max(0, min(ch + mtx, nch - 1));
      S.v[u] = reinterpret_cast<const f32x4*>(chunk_prep(kc) + mtx * s3::MAT)[e];
    }
  };
  auto load_dense = [&](int ch, float* xd) {
#pragma unroll
    for (int i = 0; i < NJK; ++i) {
      const int j = q + s3::NHA * i;
      const bool ok = j < KN && ch >= 0 && ch < nch;
      const int jc = j < KN ? j : 0, cc = max(0, min(ch, nch - 1));
      const float v = chunk_prep(cc)[2 * s3::MAT + s3::CH + jc * s3::CH + r];
      xd[i] = ok ? v : 0.f;
    }
  };
  // table slot `lid`, class c: LDS below capid slots, else the spoke's global spill area
  auto tab_add = [&](auto spill_tag, int lid, int c, float v) {
    constexpr bool SPILL = decltype(spill_tag)::value;
    if (!SPILL || lid < capid) atomicAdd(&tab[lid * K + c], v);
    else atomicAdd(&ag[(size_t)(lid - capid) * K + c], v);
  };
  unsigned long long* const hdbg = g_s3mc_dbg;
  unsigned long long h_sc = 0, h_mg = 0, h_st = 0, h_wt = 0;
  // K ≥ 8 (LEAN): the gathers and the Gram staging of a chunk are issued and consumed in
  // the same body (their latency under the scatter work) instead of a body ahead: the
  // K-wide gathers and the staged tiles are not live across the barrier (VGPR budget)
  constexpr bool LEAN = K >= 8;
  auto store_staging = [&](int cn, const Set& S) {
#pragma unroll
    for (int u = 0; u < NV4; ++u) {
      const int i = hl + 64 * s3::NHA * u;
      const int mtx = i >> 10, e = i & 1023;
      if (i < 2 * s3::MAT / 4 && cn + mtx < nch) {
        const int row = e >> 4, col = (e & 15) * 4;
        float* dst = mtx == 0 ? &sm.G[cn & 1][row][col] : &sm.X1[(cn + 1) & 1][row][col];
        *reinterpret_cast<f32x4*>(dst) = S.v[u];
      }
    }
  };
  auto body = [&](auto spill_tag, int k, Set& CUR, Set& NXT) {
    constexpr bool SPILL = decltype(spill_tag)::value;
    const int cn = k + 1, ks = k - 1;
    const unsigned long long ha = hdbg ? __builtin_amdgcn_s_memtime() : 0;
    load_words(cn + 1, NXT);
    if constexpr (LEAN) {
      issue_staging(cn, CUR);
      if constexpr (K < 16) issue_gathers(CUR);  // K = 16: loaded in the margin loop
    } else {
      issue_staging(cn + 1, NXT);
    }
    load_dense(ks + 1, NXT.xs);
    load_dense(cn + 1, NXT.xc);
    // ---- scatter chunk ks: +τ·sign into class y, −τ·sign into class r
    if (ks >= 0) {
      const float tv = sm.tau[ks & 1][r];
      const int rc = sm.rr[ks & 1][r];
      const float yf = chunk_prep(ks)[s3_prep_y<KN>() + r];
      const int yc = (yf == yf && yf >= 0.f && yf < (float)A.nclass) ? (int)yf : -1;
#pragma unroll
      for (int i = 0; i < s3::NF; ++i) {
        const uint32_t m = p2[i];
        const bool sc = (m & s3::F_SCAT) != 0u && tv != 0.f;
        if (__builtin_amdgcn_ballot_w64(sc) == 0ull) continue;
        const int lid = (int)(m >> s3::LID_SHIFT);
        const float val = (m & s3::F_SIGN) ? -tv : tv;
        if (sc) {
          if (yc >= 0) tab_add(spill_tag, lid, yc, val);
          if (rc >= 0) tab_add(spill_tag, lid, rc, -val);
        }
      }
      if constexpr (SPILL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < NJK; ++i) {
        const int j = q + s3::NHA * i;
        if (j < kd) {
#pragma unroll
          for (int c = 0; c < K; ++c) {
            if (K <= 4 || c < A.nclass) {
              const float cf = c == yc ? tv : (c == rc ? -tv : 0.f);
              wn[c][i] += wave_sum(cf * CUR.xs[i]);
            }
          }
        }
      }
    }
    if constexpr (LEAN) store_staging(cn, CUR);  // the staged tiles die before the gathers' use
    const unsigned long long hb = hdbg ? __builtin_amdgcn_s_memtime() : 0;
    // ---- base margins of chunk cn
    if (cn < nch) {
      float base[K];
#pragma unroll
      for (int c = 0; c < K; ++c) {
        base[c] = 0.f;
#pragma unroll
        for (int i = 0; i < NJK; ++i) base[c] = fmaf(CUR.xc[i], wn[c][i], base[c]);
      }
#pragma unroll
      for (int i = 0; i < s3::NF; ++i) {
        const uint32_t m = CUR.cm[i];
        const bool here = CUR.cs[i] != -1;
        const bool tg = here && (m & s3::F_TG), init = here && !tg && (m & s3::F_INIT);
        const int lid = (int)(m >> s3::LID_SHIFT);
        float val[K];
        if constexpr (K >= 16) {  // no prefetch at the widest template (VGPR budget): the
          // helpers wait less than the scanner's chunk period there
          const bool glob = here && !(m & s3::F_TG);
          const float* src = A.Wt + (size_t)(glob ? (CUR.cs[i] & 0x7fffffff) : 0) * A.kp;
#pragma unroll
          for (int c4 = 0; c4 < K; c4 += 4) {
            const float4 v = *reinterpret_cast<const float4*>(src + c4);
            val[c4] = v.x, val[c4 + 1] = v.y, val[c4 + 2] = v.z, val[c4 + 3] = v.w;
          }
        } else {
#pragma unroll
          for (int c = 0; c < K; ++c) val[c] = CUR.g[i][c];
        }
        if (!SPILL || __builtin_amdgcn_ballot_w64((tg || init) && lid >= capid) == 0ull) {
          if (tg) {
#pragma unroll
            for (int c = 0; c < K; ++c) val[c] = tab[lid * K + c];
          }
          if (init) {
#pragma unroll
            for (int c = 0; c < K; ++c) tab[lid * K + c] = val[c];
          }
        } else if constexpr (SPILL) {
          float* gp = ag + (size_t)(lid >= capid ? lid - capid : 0) * K;
          if (tg) {
#pragma unroll
            for (int c = 0; c < K; ++c)
              val[c] = lid < capid ? tab[lid * K + c]
                                   : __hip_atomic_load(gp + c, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          if (init) {
#pragma unroll
            for (int c = 0; c < K; ++c) {
              if (lid < capid) tab[lid * K + c] = val[c];
              else __hip_atomic_store(gp + c, val[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (here) {
#pragma unroll
          for (int c = 0; c < K; ++c) base[c] += (m & s3::F_SIGN) ? -val[c] : val[c];
        }
      }
#pragma unroll
      for (int c = 0; c < K; ++c)
        if (K <= 4 || c < A.nclass)
          atomicAdd(reinterpret_cast<unsigned long long*>(&sm.part[cn & 1][c][r]),
                    (unsigned long long)__double2ll_rn((double)base[c] * 0x1p32));
    }
    const unsigned long long hc = hdbg ? __builtin_amdgcn_s_memtime() : 0;
    // ---- aG_{cn} → G[cn & 1], aX1_{cn+1} → X1[(cn+1) & 1] (LEAN: before the margins)
    if constexpr (!LEAN) store_staging(cn, CUR);
    if constexpr (!LEAN) issue_gathers(NXT);
#pragma unroll
    for (int i = 0; i < s3::NF; ++i) {
      p2[i] = p1[i];
      p1[i] = CUR.cm[i];
    }
    if (hdbg) {
      const unsigned long long hd = __builtin_amdgcn_s_memtime();
      __syncthreads();
      h_sc += hb - ha;
      h_mg += hc - hb;
      h_st += hd - hc;
      h_wt += __builtin_amdgcn_s_memtime() - hd;
    } else {
      __syncthreads();
    }
  };
  Set Sa, Sb;
#pragma unroll
  for (int i = 0; i < s3::NF; ++i) p1[i] = p2[i] = 0u;
  load_words(0, Sa);
  if constexpr (!LEAN) issue_staging(0, Sa);
  load_dense(-2, Sa.xs);
  load_dense(0, Sa.xc);
  if constexpr (!LEAN) issue_gathers(Sa);
  if (lidcount[s] <= capid) {
    for (int k = -1; k <= nch; k += 2) {
      body(S3Tag<false>{}, k, Sa, Sb);
      if (k + 1 <= nch) body(S3Tag<false>{}, k + 1, Sb, Sa);
    }
  } else {
    for (int k = -1; k <= nch; k += 2) {
      body(S3Tag<true>{}, k, Sa, Sb);
      if (k + 1 <= nch) body(S3Tag<true>{}, k + 1, Sb, Sa);
    }
  }
  // round end: this wave's dense-column updates per class
#pragma unroll
  for (int i = 0; i < s3::NJ; ++i) {
    const int j = q + s3::NHA * i;
    if (lane == 0 && j < s3::DS)
#pragma unroll
      for (int c = 0; c < K; ++c)
        A.wsd[((size_t)s * K + c) * s3::DS + j] =
            (i < NJK0 && j < KN) ? wn[c][i < NJK0 ? i : 0] - w0_at(i, c) : 0.f;
  }
  if (hdbg && lane == 0) {  // helper phases summed over the helper waves
    atomicAdd(&hdbg[s * 8 + 3], h_sc);
    atomicAdd(&hdbg[s * 8 + 4], h_mg);
    atomicAdd(&hdbg[s * 8 + 5], h_st);
    atomicAdd(&hdbg[s * 8 + 6], h_wt);
    if (q == 0) atomicAdd(&hdbg[s * 8 + 7], (unsigned long long)(lidcount[s] > capid));
  }
}

// After the scan: dacc[k·dim + slot] += Σ over the spokes' occurrences of ±τ (class y: +,
// class r: −), LDS-aggregated per block as s3_scatter_kernel; the extra row of blocks adds the
// dense columns and the statistics (stats[0..3] += loss, rows, mistakes, active spokes).
__global__ __launch_bounds__(256) void s3mc_scatter_kernel(
    const int* __restrict__ slotsT, const float* __restrict__ tau, const int* __restrict__ rr,
    const void* __restrict__ yv, int y8, int nclass, int B, int n_rows, float* __restrict__ dacc,
    int dim, int dc, int dn, int bias, int K, int KN, const float* __restrict__ ws,
    const float* __restrict__ wsd, int S_act, float* __restrict__ stats) {
  if ((int)blockIdx.y == dc) {
    if (blockIdx.x != 0) return;
    const int tid = threadIdx.x;
    for (int i = tid; i < K * KN; i += 256) {
      const int c = i / KN, j = i - c * KN;
      // dacc holds nclass rows: the padded classes (K > nclass) have none
      if (j >= dn + (bias ? 1 : 0) || c >= nclass) continue;
      float v = 0.f;
      for (int s = 0; s < S_act; ++s) v += wsd[((size_t)s * K + c) * s3::DS + j];
      const int key = j < dn ? j : dim - 1;
      dacc[(size_t)c * dim + key] += v;
    }
    if (tid < 3) {
      float t = 0.f;
      for (int s = 0; s < S_act; ++s) t += ws[(size_t)s * s3::WS + tid];
      stats[tid] += t;
    }
    if (tid == 3) stats[3] += (float)S_act;
    return;
  }
  __shared__ int hk[s3::SH];
  __shared__ float hv[s3::SH];
  const int f = blockIdx.y, tid = threadIdx.x;
  const int r0 = blockIdx.x * s3::SB, r1 = min(n_rows, r0 + s3::SB);
  for (int i = tid; i < s3::SH; i += 256) {
    hk[i] = -1;
    hv[i] = 0.f;
  }
  __syncthreads();
  const int* col = slotsT + (size_t)f * B;
  auto add = [&](int key, float val) {
    uint32_t at = ((uint32_t)key * 0x9E3779B1u) >> (32 - 12);
    for (int probe = 0; probe < s3::SPROBE; ++probe) {
      const int prev = atomicCAS(&hk[at], -1, key);
      if (prev == -1 || prev == key) {
        atomicAdd(&hv[at], val);
        return;
      }
      at = (at + 1) & (s3::SH - 1);
    }
    atomicAdd(&dacc[key], val);
  };
  for (int row = r0 + tid; row < r1; row += 256) {
    const int v = col[row];
    const float t = tau[row];
    if (v == -1 || t == 0.f) continue;
    const int slot = v & 0x7fffffff;
    const float val = v < 0 ? -t : t;
    const float yf = load_y(yv, row, y8);
    const int yc = (yf == yf && yf >= 0.f && yf < (float)nclass) ? (int)yf : -1;
    if (yc >= 0) add(yc * dim + slot, val);
    if (rr[row] >= 0) add(rr[row] * dim + slot, -val);
  }
  __syncthreads();
  for (int i = tid; i < s3::SH; i += 256) {
    const int key = hk[i];
    if (key != -1) atomicAdd(&dacc[key], hv[i]);
  }
}

template <int RULE, int KN, bool RARE>
static int s3_launch_scan_t(const int* slotsT, const uint32_t* meta, int dc, int dn, const void* y,
                            int B, int R, int S_act, const float* prep, int nchs, int dim, int cap,
                            long long gstride, const S3Pipes& pp, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&s3_scan_kernel<RULE, KN, RARE>),
                        hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024 - (int)sizeof(S3Smem));
    attr_set = true;
  }
  // per pipeline: S_act rare-slot (RARE), S_act scan and ncomb·S_act combiner workgroups,
  // role-major across the pipelines (s3_scan_kernel)
  const int nblk = pp.M * s3_nper(S_act, RARE, pp.ncomb, pp.pipe[0].cb.cns);
  hipLaunchKernelGGL((s3_scan_kernel<RULE, KN, RARE>), dim3(nblk), dim3(s3::NT),
                     (size_t)(cap + 64) * sizeof(float), st, slotsT, meta, dc, dn, y, B, R, prep,
                     nchs, dim, cap, gstride, S_act, pp);
  return (int)hipGetLastError();
}

template <int KN>
static int s3_launch_scan(int rule, bool rare, const int* slotsT, const uint32_t* meta, int dc,
                          int dn, const void* y, int B, int R, int S_act, const float* prep,
                          int nchs, int dim, int cap, long long gstride, const S3Pipes& pp,
                          hipStream_t st) {
#define OMLDM_S3L(RL, RA) \
  return s3_launch_scan_t<RL, KN, RA>(slotsT, meta, dc, dn, y, B, R, S_act, prep, nchs, dim, cap, \
                                      gstride, pp, st)
  if (rare) {
    if (rule == kSeqHinge) OMLDM_S3L(kSeqHinge, true);
    if (rule == kSeqEps) OMLDM_S3L(kSeqEps, true);
    if (rule == kSeqPegasos) OMLDM_S3L(kSeqPegasos, true);
    OMLDM_S3L(kSeqLogistic, true);
  }
  if (rule == kSeqHinge) OMLDM_S3L(kSeqHinge, false);
  if (rule == kSeqEps) OMLDM_S3L(kSeqEps, false);
  if (rule == kSeqPegasos) OMLDM_S3L(kSeqPegasos, false);
  OMLDM_S3L(kSeqLogistic, false);
#undef OMLDM_S3L
}

}  // namespace omldm

using namespace omldm;

// ------------------------------------------------------------------ host API
namespace {
int s3_sact(int B, int R, int S) {
  const long long sact = ((long long)B + R - 1) / R;
  return sact < S ? (int)sact : S;
}
int s3_kn(int dn, int bias) { return dn + (bias ? 1 : 0) <= 16 ? 16 : 32; }
constexpr size_t kFlagsLds = (size_t)s3::HCAP * 12;
}  // namespace

static int g_s3_cap_override = -1;  // tests: a small LDS table forces the global spill path

// Round mode: 4 (default) = a rare-slot workgroup per spoke computes the round-start
// weights of the non-table occurrences ahead of the scan (s3_rare); 3 = the scan workgroup's
// helpers gather them themselves (the A/B reference). The granule buffer is 2·B words
// longer in mode 4 (set before a process's first prepare: it sizes the workspaces).
static int g_s3_mode = 4;
// the in-scan combine (S3Comb::inscan) in place of the combiner workgroups: 1 (auto) when
// the combiners' grid exceeds one workgroup per CU (16 pipelines: 1.20 → 0.84 ms; one
// pipeline: 0.311 vs 0.327-0.351 ms, profiles/round5/inscan/), 2 always, 0 never
static int g_s3_inscan = 1;
OMLDM_API void omldm_scan3_set_inscan(int v) { g_s3_inscan = v; }
OMLDM_API void omldm_scan3_set_mode(int m) { g_s3_mode = m == 3 ? 3 : 4; }
OMLDM_API int omldm_scan3_get_mode() { return g_s3_mode; }

// Max table entries the scan keeps in LDS.
OMLDM_API int omldm_scan3_lds_cap() {
  const int hw = (int)((160 * 1024 - sizeof(S3Smem)) / sizeof(float)) - 64;
  return g_s3_cap_override >= 0 && g_s3_cap_override < hw ? g_s3_cap_override : hw;
}

OMLDM_API void omldm_scan3_set_cap(int cap) { g_s3_cap_override = cap; }

// 1: pass 3 on the VALU reference kernel (tests: A/B against the MFMA kernel)
static int g_s3_gram_valu = 0;
OMLDM_API void omldm_scan3_set_gram_valu(int v) { g_s3_gram_valu = v; }
OMLDM_API int omldm_scan3_set_gram_ablate(int v) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_s3_gram_ablate), &v, sizeof(v));
}

// combiner workgroups per spoke in the scan's launch (0: the whole-GPU scatter kernel after
// the scan — the A/B reference); at most (MAXF + 11) / 12 parts do work
static int g_s3_comb = 1;
OMLDM_API void omldm_scan3_set_comb(int v) { g_s3_comb = v < 0 ? 0 : (v > 3 ? 3 : v); }
// launch form of a mode-4 round: 0 / 1 the latency form (pipelines beyond the GPU's CUs run
// in later waves of workgroups: the pipeline-major block order needs no co-residency), 2 the
// throughput form (one self-contained workgroup per spoke, helpers gather),
// 3 w0-margin workgroups with each scan workgroup combining its own spoke (no combiners),
// 4 two workgroups per spoke: the w0-margin workgroup combines the spoke after its w0 pass
static int g_s3_form = 0;
static int g_s3_cns = 0;  // spokes per combiner workgroup: 0 auto
OMLDM_API void omldm_scan3_set_cns(int v) { g_s3_cns = v < 0 || v > 16 ? 0 : v; }
OMLDM_API void omldm_scan3_set_form(int v) { g_s3_form = v < 0 || v > 4 ? 0 : v; }
OMLDM_API int omldm_scan3_get_comb() { return g_s3_comb; }

// 1 if a combiner gave up waiting for its spoke's granules since the last call (resets it;
// synchronises the device)
OMLDM_API int omldm_scan3_comb_err() {
  int v = 0, z = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_s3_comb_err), sizeof(v)) != hipSuccess) return -1;
  if (v) hipMemcpyToSymbol(HIP_SYMBOL(g_s3_comb_err), &z, sizeof(z));
  return v;
}

// The combiner-timeout flag OR-ed into out[0] (device-visible memory, e.g. the device alias
// of a pinned host word) and cleared, in stream order and without a host sync: the engine
// reads the word a tick later (utils/health.py) and fails the job if it is set.
__global__ void s3_err_drain_kernel(int* out) {
  if (threadIdx.x == 0) {  // (the highest code: the waits are 1 combiner, 2 helper, 3 prep)
    const int v = atomicExch(&g_s3_comb_err, 0);
    out[0] = v > out[0] ? v : out[0];
  }
}

OMLDM_API int omldm_scan3_comb_err_drain(int* out, void* stream) {
  hipLaunchKernelGGL(s3_err_drain_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
  return (int)hipGetLastError();
}

// 1 when the v3 round handles this shape (field-aware slots, R ≤ RMAX).
OMLDM_API int omldm_scan3_fits(int dn, int dc, int R, int bias) {
  return dc > 0 && dc <= s3::MAXF && dn >= 0 && dn + (bias ? 1 : 0) <= s3::KNMAX && R > 0 &&
         R <= s3::RMAX;
}

// Workspace sizes (4-byte words) for one round of S spokes × R rows, B rows in all, dc
// fields:  0 slotsT [dc·B]   1 occ [2·dc·B]   2 lidcount [S]   3 prep [S·nchs·PF]
//          4 granules [2·B]  5 ws [S·WS]     6 wsd [S·DS]     7 aglob [S·gstride]
// (the granule buffer must be zeroed when allocated: see S3Comb)
OMLDM_API long long omldm_scan3_ws_words(int which, int B, int R, int S, int dn, int dc,
                                         long long span, int bias) {
  (void)span;
  const long long nchs = (R + s3::CH - 1) / s3::CH;
  const int kn = s3_kn(dn, bias);
  const long long pf = kn == 16 ? s3_prep_floats<16>() : s3_prep_floats<32>();
  switch (which) {
    case 0: return (long long)dc * B;
    case 1:  // meta word per occurrence, then each table id's slot [S][R·dc/2 + 64]
      return (long long)dc * B + (long long)S * ((long long)R * dc / 2 + 64);
    case 2: return S;
    case 3: return (long long)S * nchs * pf + S + 64;  // + σ at each spoke's end
    case 4: return 4LL * B;  // c granules + the w0-margin granules (mode 4)
    case 5: return (long long)S * s3::WS;
    case 6: return (long long)S * s3::DS;
    case 7: return (long long)S * ((long long)R * dc / 2 + 64);
  }
  return 0;
}

OMLDM_API int omldm_scan3_nbufs() { return 8; }

struct S3Ws {
  int* slotsT;
  uint32_t* meta;
  int* lidcount;
  float* prep;
  unsigned long long* gran;
  float* ws;
  float* wsd;
  float* aglob;
};

static S3Ws s3_ws(void* const* ptrs) {
  return S3Ws{(int*)ptrs[0], (uint32_t*)ptrs[1], (int*)ptrs[2], (float*)ptrs[3],
              (unsigned long long*)ptrs[4], (float*)ptrs[5], (float*)ptrs[6], (float*)ptrs[7]};
}

// The Gram pass needs the slots but not the flags: it runs on a companion stream of the
// caller's (same CU mask) beside the flags pass, and the caller's stream waits for both.
static int g_s3_prep_split = 0;  // measured: 309.5 (on) vs 319.8 M ex/s (off)
OMLDM_API void omldm_scan3_set_prep_split(int v) { g_s3_prep_split = v; }
namespace {
struct S3Side {
  hipStream_t side;
  hipEvent_t fork, join;
};
std::mutex g_s3_side_mu;
std::unordered_map<hipStream_t, S3Side> g_s3_side;

S3Side* s3_side(hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_s3_side_mu);
  auto it = g_s3_side.find(st);
  if (it != g_s3_side.end()) return &it->second;
  S3Side sd{};
  uint32_t mask[32] = {};
  const bool masked = st != nullptr && hipExtStreamGetCUMask(st, 32, mask) == hipSuccess;
  if (!(masked && hipExtStreamCreateWithCUMask(&sd.side, 32, mask) == hipSuccess) &&
      hipStreamCreateWithFlags(&sd.side, hipStreamNonBlocking) != hipSuccess)
    return nullptr;
  if (hipEventCreateWithFlags(&sd.fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&sd.join, hipEventDisableTiming) != hipSuccess)
    return nullptr;
  return &g_s3_side.emplace(st, sd).first->second;
}
}  // namespace

// Explicit teardown of the HIP objects this library created on demand (the companion prep
// streams and their fork / join events): called from the Python loader's atexit hook, while
// the HIP runtime is still up — not left to static destructors at process exit.
OMLDM_API int omldm_scan3_teardown() {
  std::lock_guard<std::mutex> lk(g_s3_side_mu);
  int n = 0;
  for (auto& kv : g_s3_side) {
    hipStreamSynchronize(kv.second.side);
    hipEventDestroy(kv.second.fork);
    hipEventDestroy(kv.second.join);
    hipStreamDestroy(kv.second.side);
    ++n;
  }
  g_s3_side.clear();
  return n;
}

// Passes 1-3 (model-independent): slots, flags, Grams. `src` is the tokens (hashed = 0),
// row-major int32 field-aware slots (1) or the compact int16 slots (2). span: slots per
// field (0: (dim − dn − 1) / dc, the raw-token hashing's; the compact wire's cat_span
// otherwise — fields occupy [dn + f·span, dn + (f + 1)·span)).
OMLDM_API int omldm_scan3_prepare(const float* num, int dn, const void* src, int hashed, int dc,
                                  const void* y, int y8, int B, int R, int S, int dim, int bias,
                                  int rule, int variant, float C, long long span_in,
                                  int cbase, int shr, float shr_r, float tbase, float lr,
                                  void* const* ptrs, void* stream) {
  if (S <= 0 || B <= 0) return 0;
  if (!omldm_scan3_fits(dn, dc, R, bias)) return -3;
  if ((long long)(dim - dn - 1) / dc < 1) return -2;
  if (cbase < 0) cbase = dn;
  if (span_in < 0 || (long long)cbase + (long long)dc * span_in > (long long)dim - 1) return -2;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t span = span_in > 0 ? (uint32_t)span_in : (uint32_t)((dim - dn - 1) / dc);
  const S3Ws W = s3_ws(ptrs);
  const int S_act = s3_sact(B, R, S);
  hipLaunchKernelGGL(s3_slots_kernel, dim3((B + 255) / 256), dim3(256), 0, st, src, B, dc, dn,
                     span, hashed, cbase, W.slotsT);
  hipMemsetAsync(W.lidcount, 0, sizeof(int) * S, st);
  S3Side* sd = g_s3_prep_split ? s3_side(st) : nullptr;
  hipStream_t gst = st;  // the Gram pass's stream
  if (sd) {
    hipEventRecord(sd->fork, st);
    hipStreamWaitEvent(sd->side, sd->fork, 0);
    gst = sd->side;
  }
  hipLaunchKernelGGL(s3_flags_kernel, dim3(dc, S_act), dim3(s3::FT), 0, st, W.slotsT, B, R,
                     W.meta, W.lidcount, dim <= (1 << 22) ? 1 : 0,
                     reinterpret_cast<int*>(W.meta + (size_t)dc * B),
                     (long long)R * dc / 2 + 64);
  const int nchs = (R + s3::CH - 1) / s3::CH;
  // a per row: −1/(‖x‖² + kadd) (hinge, ε), 1 (logistic), y (Pegasos), 1/(2‖x‖² + kadd)
  // (MultiClassPA: rule 4)
  const int affine = rule == kSeqLogistic ? 0 : rule == kSeqPegasos ? 2 : rule == 4 ? 3 : 1;
  const float kadd = ((affine == 1 || affine == 3) && variant == 2) ? 0.5f / C : 0.f;
  if (rule == kSeqPegasos && shr != 2) return -2;
  // logistic without shrink: the Grams' columns carry lr·y (s3_gram_colscale)
  const float cscale = rule == kSeqLogistic && !shr ? lr : 0.f;
  if (g_s3_gram_valu) {
    if (s3_kn(dn, bias) == 16)
      hipLaunchKernelGGL(s3_gram_kernel<16>, dim3(nchs, S_act), dim3(256), 0, gst, W.slotsT, dc,
                         num, dn, y, y8, B, R, bias, affine, kadd, W.prep, nchs, shr, shr_r, cscale);
    else
      hipLaunchKernelGGL(s3_gram_kernel<32>, dim3(nchs, S_act), dim3(256), 0, gst, W.slotsT, dc,
                         num, dn, y, y8, B, R, bias, affine, kadd, W.prep, nchs, shr, shr_r, cscale);
  } else if (s3_kn(dn, bias) == 16) {
    hipLaunchKernelGGL(s3_gram_mfma_kernel<16>, dim3(nchs, S_act), dim3(256), 0, gst, W.slotsT,
                       dc, num, dn, y, y8, B, R, bias, affine, kadd, W.prep, nchs, shr, shr_r, cscale);
  } else {
    hipLaunchKernelGGL(s3_gram_mfma_kernel<32>, dim3(nchs, S_act), dim3(256), 0, gst, W.slotsT,
                       dc, num, dn, y, y8, B, R, bias, affine, kadd, W.prep, nchs, shr, shr_r, cscale);
  }
  if (shr) {  // σ per row from the targets the Gram pass wrote into the prep
    float* sig = W.prep + (size_t)S * nchs * (s3_kn(dn, bias) == 16 ? s3_prep_floats<16>()
                                                                    : s3_prep_floats<32>());
    if (s3_kn(dn, bias) == 16)
      hipLaunchKernelGGL(s3_sigma_kernel<16>, dim3(S_act), dim3(64), 0, gst, W.prep, nchs, B, R,
                         shr, shr_r, tbase, sig);
    else
      hipLaunchKernelGGL(s3_sigma_kernel<32>, dim3(S_act), dim3(64), 0, gst, W.prep, nchs, B, R,
                         shr, shr_r, tbase, sig);
  }
  if (sd) {
    hipEventRecord(sd->join, gst);
    hipStreamWaitEvent(st, sd->join, 0);
  }
  return (int)hipGetLastError();
}

// Pass 4 (the scan) + pass 5 (the combine) of M ≥ 1 pipelines on one prepared round, one
// launch (s3_scan_kernel). Pipeline m: model w[m], accumulator dacc[m] (zeroed here unless
// flags bit 0 says the caller keeps it zero), running totals cum[m] (or null), rule
// constants C / eps / lr / inv_p [m], its 8 workspace pointers ptrs[8m .. 8m+8) (the first four
// — slots, occurrences, table counts, prep — the shared prep's; granules, spoke rows, dense
// deltas and table spill its own), its granule epoch (≥ 1, one more than the last round on
// that granule buffer, zeroed when allocated) and arrival word (null: tail kernel after).
// The next run on this thread waits in its launch for a prep's ready word (see S3Pipes)
static thread_local const unsigned long long* t_s3_wflag = nullptr;
static thread_local unsigned long long t_s3_wepoch = 0;
OMLDM_API void omldm_scan3_wait_next(const void* flag, unsigned long long epoch) {
  t_s3_wflag = static_cast<const unsigned long long*>(flag);
  t_s3_wepoch = epoch;
}
OMLDM_API int omldm_scan3_signal(void* flag, unsigned long long epoch, void* stream) {
  hipLaunchKernelGGL(s3_signal_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     static_cast<unsigned long long*>(flag), epoch);
  return (int)hipGetLastError();
}

static int s3_run_impl(int M, const float* const* w, float* const* dacc, double* const* cum,
                       const float* C, const float* eps, const float* lr, const float* inv_p,
                       void* const* ptrs, const unsigned* epoch, void* const* arrive, int dn,
                       int dc, const void* y, int y8, int B, int R, int S, int dim, int rule,
                       int variant, int bias, long long span_in, int flags, int shr,
                       const float* lam, const float* tbase, hipStream_t st) {
  const unsigned long long* wflag = t_s3_wflag;  // consumed whatever this call does
  const unsigned long long wepoch = t_s3_wepoch;
  t_s3_wflag = nullptr;
  if (M < 1 || M > kS3MaxPipes) return -4;
  if (S <= 0 || B <= 0) return 0;
  if (!omldm_scan3_fits(dn, dc, R, bias)) return -3;
  if (span_in < 0) return -2;  // the slots' range was checked by the prepare
  const uint32_t span = span_in > 0 ? (uint32_t)span_in : (uint32_t)((dim - dn - 1) / dc);
  const S3Ws W0 = s3_ws(ptrs);
  const int S_act = s3_sact(B, R, S);
  const int nchs = (R + s3::CH - 1) / s3::CH;
  const int kn = s3_kn(dn, bias);
  const int cap = omldm_scan3_lds_cap();
  const long long gstride = (long long)R * dc / 2 + 64;
  if (rule == kSeqPegasos && shr != 2) return -2;
  // shrinking rules: σ at each spoke's end, after the prep blocks (s3_sigma_kernel)
  const float* sig = shr ? W0.prep + (size_t)S * nchs * (kn == 16 ? s3_prep_floats<16>()
                                                                  : s3_prep_floats<32>())
                         : nullptr;
  // latency form (mode 4): w0-margin workgroups + in-launch combiners beside the scans, the
  // grid in waves of workgroups when it exceeds the GPU; throughput form (OMLDM_S3_FORM=2):
  // one self-contained workgroup per spoke — helpers gather, the spoke combined by its own
  // workgroup after its scan. Mode 3: helpers gather, in-launch combiners.
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
  }
  int ncomb = g_s3_comb;
  bool rare = g_s3_mode == 4 && ncomb > 0;
  bool tail = false;
  int tailm = 0;
  // auto = the latency form at every pipeline count (profiles/round5/mp_form*.json: 16
  // pipelines 1.19 ms in three waves of workgroups vs 1.32 ms in the throughput form)
  if (rare && g_s3_form == 2) {
    rare = false;
    tail = true;
    ncomb = 0;
  } else if (rare && g_s3_form == 3) {
    tail = true;
    ncomb = 0;
  } else if (rare && g_s3_form == 4) {
    tailm = 2;
    ncomb = 0;
  }
  // spokes per combiner workgroup (OMLDM_S3_CNS, A/B): 1 — a combiner of 2 or 4 spokes falls
  // behind its scans (16 pipelines: 1.20 / 1.27 / 1.67 ms, profiles/round5/mp_cns*.json)
  int cns = g_s3_cns > 0 ? g_s3_cns : 1;
  if (!rare || ncomb != 1) cns = 1;
  // in-scan combine: no combiner workgroups. Auto (past one workgroup per CU): no w0-margin
  // workgroups either — the helpers gather w0 and add the non-table occurrences (16
  // pipelines: one wave of 256 workgroups instead of three); forced: the w0-margin
  // workgroups while they fit, folding the non-table occurrences after their pass
  const bool fits = (long long)M * s3_nper(S_act, rare, ncomb, cns) <= ncu;
  const bool inscan = ncomb > 0 && g_s3_form < 2 && dim <= (1 << 22) &&
                      (g_s3_inscan == 2 || (g_s3_inscan == 1 && !fits));
  if (inscan) {
    ncomb = 0;
    cns = 1;
    rare = g_s3_inscan == 2 && g_s3_mode == 4 && (long long)M * 2 * S_act <= ncu;
  }
  S3Pipes pp{};
  pp.M = M;
  // the in-launch wait for the prep's ready word only while the scan grid leaves most CUs
  // to the prep's kernels (otherwise spinning LDS-heavy workgroups could hold the CUs the
  // prep needs until the bounded wait gives up): past that, the stream waits on the word
  if (wflag && (long long)M * s3_nper(S_act, rare, ncomb, cns) > ncu / 2) {
    const hipError_t we = hipStreamWaitValue64(st, const_cast<unsigned long long*>(wflag),
                                               wepoch, hipStreamWaitValueGte, ~0ull);
    if (we != hipSuccess) return (int)we;
    wflag = nullptr;
  }
  pp.wflag = wflag;
  pp.wepoch = wepoch;
  pp.ncomb = ncomb > 0 ? ncomb : 0;
  pp.tail = tail ? 1 : tailm;
  for (int m = 0; m < M; ++m) {
    if (epoch[m] == 0u) return -2;
    const S3Ws Wm = s3_ws(ptrs + 8 * m);
    const SeqParams p{rule, variant, variant == 1 ? C[m] : INFINITY,
                      variant == 2 ? 0.5f / C[m] : 0.f, eps[m], lr[m], inv_p[m], bias, y8, span,
                      shr, lam ? lam[m] : 0.f, tbase ? tbase[m] : 0.f};
    // flags bit 1: w[m] points at a bf16 model (modelDtype bf16: margins on bf16 weights)
    // flags bit 0: dacc[:dim] is already zero (linear_apply clears it after every round), so
    // the combine adds straight into it (a memset beside the prep kernels took 15-20 us)
    if (!(flags & 1)) hipMemsetAsync(dacc[m], 0, sizeof(float) * (size_t)dim, st);
    // the tail in the scan's launch (last scan block) when the caller gave an arrival word;
    // mode 4: the rare-slot workgroups' margin granules follow the c granules
    pp.pipe[m] = S3Pipe{w[m], Wm.aglob, Wm.ws, Wm.wsd, rare ? Wm.gran + B : nullptr,
                        S3Comb{W0.lidcount, Wm.gran, epoch[m], S_act, dacc[m], inv_p[m],
                               static_cast<unsigned long long*>(arrive[m]), cum[m], sig,
                               (flags & 2) ? 1 : 0, cns,
                               reinterpret_cast<const int*>(W0.meta + (size_t)dc * B),
                               gstride, inscan ? (rare ? 2 : 1) : 0},
                        p};
  }
  const int e = kn == 16 ? s3_launch_scan<16>(rule, rare, W0.slotsT, W0.meta, dc, dn, y, B, R,
                                              S_act, W0.prep, nchs, dim, cap, gstride, pp, st)
                         : s3_launch_scan<32>(rule, rare, W0.slotsT, W0.meta, dc, dn, y, B, R,
                                              S_act, W0.prep, nchs, dim, cap, gstride, pp, st);
  if (e) return e;
  for (int m = 0; m < M; ++m) {
    const S3Ws Wm = s3_ws(ptrs + 8 * m);
    if (ncomb > 0 || tail || tailm || inscan) {  // the categorical slots were combined in the scan's launch
      if (!arrive[m])
        hipLaunchKernelGGL(s3_tail_kernel, dim3(1), dim3(256), 0, st, Wm.ws, Wm.wsd, sig, S_act,
                           dn, dim, bias, inv_p[m], dacc[m], cum[m]);
      continue;
    }
    const int n_rows = (int)((long long)S_act * R < B ? (long long)S_act * R : B);
    const int nblk = (n_rows + s3::SB - 1) / s3::SB;
    hipLaunchKernelGGL(s3_scatter_kernel, dim3(nblk > 0 ? nblk : 1, dc + (arrive[m] ? 0 : 1)),
                       dim3(256), 0, st, W0.slotsT, Wm.gran, B, n_rows, inv_p[m], dacc[m], dc,
                       Wm.ws, Wm.wsd, S_act, dn, dim, bias, cum[m], R, sig);
  }
  return (int)hipGetLastError();
}

// One pipeline (the M = 1 case). `parts` is kept for the pipelined-sync interface: part 0
// completes all of dacc (the combine is a few tens of µs of atomics), later parts launch
// nothing.
OMLDM_API int omldm_scan3_run(const float* w, int dn, int dc, const void* y, int y8, int B, int R,
                              int S, float* dacc, int dim, double* cum, int rule, int variant,
                              float C, float eps, float lr, float inv_p, int bias,
                              long long span_in, void* const* ptrs, int part, int parts,
                              int flags, unsigned epoch, void* arrive, int shr, float lam,
                              float tbase, void* stream) {
  if (part != 0) return 0;
  (void)parts;
  return s3_run_impl(1, &w, &dacc, &cum, &C, &eps, &lr, &inv_p, ptrs, &epoch, &arrive, dn, dc, y,
                     y8, B, R, S, dim, rule, variant, bias, span_in, flags, shr, &lam, &tbase,
                     (hipStream_t)stream);
}

// M pipelines sharing one prep, one launch (per-pipeline arrays as in s3_run_impl).
OMLDM_API int omldm_scan3_run_multi(int M, const float* const* w, float* const* dacc,
                                    double* const* cum, const float* C, const float* eps,
                                    const float* lr, const float* inv_p, void* const* ptrs,
                                    const unsigned* epoch, void* const* arrive, int dn, int dc,
                                    const void* y, int y8, int B, int R, int S, int dim,
                                    int rule, int variant, int bias, long long span_in, int flags,
                                    int shr, const float* lam, const float* tbase, void* stream) {
  return s3_run_impl(M, w, dacc, cum, C, eps, lr, inv_p, ptrs, epoch, arrive, dn, dc, y, y8, B, R,
                     S, dim, rule, variant, bias, span_in, flags, shr, lam, tbase,
                     (hipStream_t)stream);
}

OMLDM_API int omldm_scan3_max_pipes() { return kS3MaxPipes; }

// [lo, hi) of dacc that combine part `part` of `parts` completes: part 0 all of it.
OMLDM_API int omldm_scan3_part_bounds(int dim, int dn, int dc, long long span_in, int part,
                                      int parts, long long* lohi) {
  (void)dn, (void)dc, (void)span_in, (void)parts;
  lohi[0] = part == 0 ? 0 : (long long)dim + 2;
  lohi[1] = (long long)dim + 2;
  return 0;
}

OMLDM_API int omldm_scan3_hprio(int v) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_s3_hprio), &v, sizeof(v));
}

OMLDM_API int omldm_scan3_dense_order(int v) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_s3_dense_order), &v, sizeof(v));
}

OMLDM_API int omldm_scan3_debug(int v) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_s3_debug), &v, sizeof(v));
}

// MultiClassPA scan diagnostics: buf = u64 [S·8] (accumulated; null turns them off).
OMLDM_API int omldm_scan3mc_debug(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_s3mc_dbg), &buf, sizeof(buf));
}

OMLDM_API int omldm_scan3_stamps(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_s3_stamps), &buf, sizeof(buf));
}

// ------------------------------------------------------------------ MultiClassPA host API
// The LDS slot table of the multiclass scan (floats) and its global spill (floats per spoke).
template <int K>
static int s3mc_cap() {
  return (int)((160 * 1024 - sizeof(S3McSmem<K>)) / sizeof(float)) / K * K;
}
OMLDM_API int omldm_scan3mc_lds_cap(int K) {
  switch (K) {
    case 2: return s3mc_cap<2>();
    case 4: return s3mc_cap<4>();
    case 8: return s3mc_cap<8>();
    default: return s3mc_cap<16>();
  }
}
OMLDM_API long long omldm_scan3mc_spill_floats(int R, int dc, int K) {
  return ((long long)R * dc / 2 + 64) * K;
}

template <int K, int KN>
static int s3mc_launch(const S3Ws& W, int dc, int dn, int bias, int B, int R, int S_act,
                       int nchs, int dim, long long gstride, const S3McArgs& A, hipStream_t st) {
  const int cap = omldm_scan3mc_lds_cap(K);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&s3mc_scan_kernel<K, KN>),
                        hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024 - (int)sizeof(S3McSmem<K>));
    attr_set = true;
  }
  hipLaunchKernelGGL((s3mc_scan_kernel<K, KN>), dim3(S_act), dim3(s3::NT),
                     (size_t)cap * sizeof(float), st, W.slotsT, W.meta, W.lidcount, dc, dn, bias,
                     B, R, W.prep, nchs, dim, cap, gstride, A);
  return (int)hipGetLastError();
}

// One MultiClassPA round of S spokes on a prep made by omldm_scan3_prepare with rule 4:
// dacc [K][dim] += Σ_s Δ_s, stats[0..3] += (loss, rows, mistakes, active spokes). Wt: the
// key-major fp32 prototypes [dim][kp]; ptrs: the prep's 8 workspace pointers (slots, meta,
// table counts, prep used); ws [S·8], wsd [S·K·32], aglob [S·omldm_scan3mc_spill_floats],
// tau [B], rr [B] scratch. K ∈ {2, 4} (nclass ≤ K).
OMLDM_API int omldm_scan3mc_run(const float* Wt, int kp, int K, int nclass, int dn, int dc,
                                const void* y, int y8, int B, int R, int S, float* dacc, int dim,
                                float* stats, int variant, float C, int bias, void* const* ptrs,
                                float* ws, float* wsd, float* aglob, float* tau, int* rr,
                                void* stream) {
  if (S <= 0 || B <= 0) return 0;
  if ((K != 2 && K != 4 && K != 8 && K != 16) || nclass < 2 || nclass > K || kp < K) return -2;
  if (!omldm_scan3_fits(dn, dc, R, bias)) return -3;
  hipStream_t st = (hipStream_t)stream;
  const S3Ws W = s3_ws(ptrs);
  const int S_act = s3_sact(B, R, S);
  const int nchs = (R + s3::CH - 1) / s3::CH;
  const long long gstride = (long long)R * dc / 2 + 64;
  const S3McArgs A{Wt, kp, nclass, variant, variant == 1 ? C : INFINITY, ws, wsd, aglob, tau, rr};
  const bool k16 = s3_kn(dn, bias) == 16;
  int e;
  if (K == 2)
    e = k16 ? s3mc_launch<2, 16>(W, dc, dn, bias, B, R, S_act, nchs, dim, gstride, A, st)
            : s3mc_launch<2, 32>(W, dc, dn, bias, B, R, S_act, nchs, dim, gstride, A, st);
  else if (K == 4)
    e = k16 ? s3mc_launch<4, 16>(W, dc, dn, bias, B, R, S_act, nchs, dim, gstride, A, st)
            : s3mc_launch<4, 32>(W, dc, dn, bias, B, R, S_act, nchs, dim, gstride, A, st);
  else if (K == 8)
    e = k16 ? s3mc_launch<8, 16>(W, dc, dn, bias, B, R, S_act, nchs, dim, gstride, A, st)
            : s3mc_launch<8, 32>(W, dc, dn, bias, B, R, S_act, nchs, dim, gstride, A, st);
  else
    e = k16 ? s3mc_launch<16, 16>(W, dc, dn, bias, B, R, S_act, nchs, dim, gstride, A, st)
            : s3mc_launch<16, 32>(W, dc, dn, bias, B, R, S_act, nchs, dim, gstride, A, st);
  if (e) return e;
  const int n_rows = (int)((long long)S_act * R < B ? (long long)S_act * R : B);
  const int nblk = (n_rows + s3::SB - 1) / s3::SB;
  hipLaunchKernelGGL(s3mc_scatter_kernel, dim3(nblk > 0 ? nblk : 1, dc + 1), dim3(256), 0, st,
                     W.slotsT, tau, rr, y, y8, nclass, B, n_rows, dacc, dim, dc, dn, bias, K,
                     s3_kn(dn, bias), ws, wsd, S_act, stats);
  return (int)hipGetLastError();
}
