// NN learner: fused MLP training and inference on the fp32 matrix cores.
//
// Reference: the NN learner runs DL4J MultiLayerNetwork.fit on ND4J/OpenBLAS — GEMM,
// the row-wise bias broadcast that crashed (BaseLayer.preOutputWithPreNorm → doRowWise →
// execBroadcast, hs_err_pid77107.log:97-110), activations and an SGD step, each a
// separate native call per layer per mini-batch.
//
// Design (one kernel per protocol round):
// * one workgroup (4 waves) = one virtual spoke. It copies the round-start model into
//   LDS and runs plain mini-batch SGD over its row range: forward, loss gradient,
//   backward and the weight update never leave LDS/registers;
// * every GEMM-shaped step is v_mfma_f32_32x32x2_f32 on 32-row mini-batches:
//     forward   H_{l+1} = act(H_l · W_lᵀ + b_l)     (bias + activation fused in the
//                                                     epilogue: ReLU / tanh / sigmoid / identity)
//     backward  dH_l    = (dZ_{l+1} · W_l) ⊙ act'(H_l)  (derivative from the stored output)
//               W_l    -= η · dZ_{l+1}ᵀ · H_l       (applied straight from the MFMA
//                                                     accumulators — each element has
//                                                     exactly one owner lane)
//   widths are zero-padded to 32; padding stays exactly zero through every step;
// * LDS row strides are padded to an odd number of floats so the 32 lanes of an MFMA
//   operand column hit distinct banks;
// * round end: each spoke adds its model delta to a device accumulator and an apply
//   pass averages the deltas of the active spokes (omldm_multiclass_apply) — the
//   intra-GPU hub; across GPUs the protocol ships the flat parameter vector over RCCL.
#include "common.h"

namespace omldm {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kMB = 32;
constexpr int kMaxLayers = 4;

enum MlpAct : int { kRelu = 0, kTanh = 1, kSigmoid = 2, kIdentity = 3 };

struct MlpDesc {
  int L, task, K, act;  // act: hidden-layer activation (MlpAct)
  int bf16;             // 1: GEMM operands rounded to bf16 (v_mfma_f32_32x32x16_bf16)
  int n[kMaxLayers + 1], np[kMaxLayers + 1];
  int woff[kMaxLayers], boff[kMaxLayers];
  int lw[kMaxLayers], lb[kMaxLayers], ldw[kMaxLayers];
  int lh[kMaxLayers + 1], ldh[kMaxLayers + 1];
  int lg0, lg1, ldg, ly, total;
  // round kernel v2 (mlp_round2_kernel): bias-gradient accumulators per layer, three
  // rotating gradient buffers, a 4-float statistics scratch
  int lbg[kMaxLayers], lgb[3], lsc;
};

// C[32×32] = A[32×K]·B[K×32] with A(i,k) = a[i·ars + k·acs], B(k,j) = b[k·brs + j·bcs].
// Result reg q of lane is C(row(q, lane), lane&31). K is a multiple of 16 (widths padded to
// 32, mini-batches of 32 rows). An operand whose k index is contiguous in LDS (AK: acs ==
// 1, BK: brs == 1 — forward: H rows and W rows; backward dH: G rows) is read as two 16-byte
// ds_read_b128 per 8 k values: row strides are ≡ 4 floats mod 64 banks (make_desc), so the
// 16-lane groups of a b128 read hit disjoint banks, and every row start and k offset is a
// multiple of 4 floats. Strided operands are read one float per k.
//
// fp32 (v_mfma_f32_32x32x2_f32): for its 8 MFMAs of a 16-wide k step, lane half kh supplies
// the 8 contiguous k = k0 + 8·kh + u (u = MFMA index) of its row / column in both operands
// — a permutation of the k sum, so one half's values are one contiguous run.
template <bool AK, bool BK>
__device__ __forceinline__ f32x16 wave_gemm32_f32(const float* a, int ars, int acs,
                                                  const float* b, int brs, int bcs, int K) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, kh = lane >> 5;
  f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const float* ap = a + r * ars + 8 * kh * (AK ? 1 : acs);
  const float* bp = b + 8 * kh * (BK ? 1 : brs) + r * bcs;
  for (int k = 0; k < K; k += 16) {
    float av[8], bv[8];
    if constexpr (AK) {
      const float4 x0 = *reinterpret_cast<const float4*>(ap + k);
      const float4 x1 = *reinterpret_cast<const float4*>(ap + k + 4);
      av[0] = x0.x; av[1] = x0.y; av[2] = x0.z; av[3] = x0.w;
      av[4] = x1.x; av[5] = x1.y; av[6] = x1.z; av[7] = x1.w;
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) av[u] = ap[(k + u) * acs];
    }
    if constexpr (BK) {
      const float4 y0 = *reinterpret_cast<const float4*>(bp + k);
      const float4 y1 = *reinterpret_cast<const float4*>(bp + k + 4);
      bv[0] = y0.x; bv[1] = y0.y; bv[2] = y0.z; bv[3] = y0.w;
      bv[4] = y1.x; bv[5] = y1.y; bv[6] = y1.z; bv[7] = y1.w;
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) bv[u] = bp[(k + u) * brs];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
  }
  return acc;
}

// Mixed precision: the same product with operands rounded to bf16 (RNE) as they leave
// LDS and fp32 accumulation, on v_mfma_f32_32x32x16_bf16 — K/16 instructions instead
// of K/2. Operand map: lane l (r = l&31, h = l>>5) supplies A(r, k + 8h + j) and
// B(k + 8h + j, r), j = 0..7 (already one contiguous run per lane); the C layout is the
// fp32 form's.
typedef short bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ short bf16_bits(float v) {
  return __builtin_bit_cast(short, __float2bfloat16(v));
}
template <bool CONTIG>
__device__ __forceinline__ void load8_bf16(const float* p, int stride, int k, bf16x8& o) {
  if constexpr (CONTIG) {
    const float4 x0 = *reinterpret_cast<const float4*>(p + k);
    const float4 x1 = *reinterpret_cast<const float4*>(p + k + 4);
    o[0] = bf16_bits(x0.x); o[1] = bf16_bits(x0.y); o[2] = bf16_bits(x0.z); o[3] = bf16_bits(x0.w);
    o[4] = bf16_bits(x1.x); o[5] = bf16_bits(x1.y); o[6] = bf16_bits(x1.z); o[7] = bf16_bits(x1.w);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf16_bits(p[(k + j) * stride]);
  }
}
template <bool AK, bool BK>
__device__ __forceinline__ f32x16 wave_gemm32_bf16(const float* a, int ars, int acs,
                                                   const float* b, int brs, int bcs, int K) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, kh = lane >> 5;
  f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const float* ap = a + r * ars + 8 * kh * (AK ? 1 : acs);
  const float* bp = b + 8 * kh * (BK ? 1 : brs) + r * bcs;
#pragma unroll 2
  for (int k = 0; k < K; k += 16) {
    bf16x8 af, bfr;
    load8_bf16<AK>(ap, acs, k, af);
    load8_bf16<BK>(bp, brs, k, bfr);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc, 0, 0, 0);
  }
  return acc;
}

#ifndef OMLDM_MLP_VEC
#define OMLDM_MLP_VEC 3  // diagnostics: bit 0 vector reads of k-contiguous A, bit 1 of B
#endif
constexpr bool kVecA = (OMLDM_MLP_VEC & 1) != 0, kVecB = (OMLDM_MLP_VEC & 2) != 0;

template <bool AK, bool BK>
__device__ __forceinline__ f32x16 wave_gemm32(const float* a, int ars, int acs, const float* b,
                                              int brs, int bcs, int K, int bf16) {
  return bf16 ? wave_gemm32_bf16<AK, BK>(a, ars, acs, b, brs, bcs, K)
              : wave_gemm32_f32<AK, BK>(a, ars, acs, b, brs, bcs, K);
}

// 16×16 tiles (v_mfma_f32_16x16x4_f32 / v_mfma_f32_16x16x16_bf16): a 32-row mini-batch
// against 64-wide layers then has 8–16 output tiles per GEMM instead of 2–4, so all four
// waves of the spoke work in every phase rather than one or two. Lane l (i = l&15,
// g = l>>4) supplies, per 16-wide k step, the 4 consecutive k = k0 + 4g + u of its A row
// and B column (one b128 read when k is contiguous in LDS); fp32 MFMA u takes value u
// (a permutation of the k sum), bf16 takes all four at once. acc[j] = C(4g + j, i).
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
template <bool AK, bool BK>
__device__ __forceinline__ f32x4 wave_gemm16(const float* a, int ars, int acs, const float* b,
                                             int brs, int bcs, int K, int bf16) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* ap = a + r * ars + 4 * g * (AK ? 1 : acs);
  const float* bp = b + 4 * g * (BK ? 1 : brs) + r * bcs;
  for (int k = 0; k < K; k += 16) {
    float av[4], bv[4];
    if constexpr (AK) {
      const float4 x = *reinterpret_cast<const float4*>(ap + k);
      av[0] = x.x; av[1] = x.y; av[2] = x.z; av[3] = x.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) av[u] = ap[(k + u) * acs];
    }
    if constexpr (BK) {
      const float4 y = *reinterpret_cast<const float4*>(bp + k);
      bv[0] = y.x; bv[1] = y.y; bv[2] = y.z; bv[3] = y.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) bv[u] = bp[(k + u) * brs];
    }
    if (bf16) {
      const bf16x4 af = {bf16_bits(av[0]), bf16_bits(av[1]), bf16_bits(av[2]), bf16_bits(av[3])};
      const bf16x4 bfv = {bf16_bits(bv[0]), bf16_bits(bv[1]), bf16_bits(bv[2]), bf16_bits(bv[3])};
      acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(af, bfv, acc, 0, 0, 0);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
    }
  }
  return acc;
}

#ifndef OMLDM_MLP_TILE
#define OMLDM_MLP_TILE 16  // output tile of the round/forward GEMMs: 16 or 32
#endif
#if OMLDM_MLP_TILE == 16
typedef f32x4 AccT;
constexpr int kT = 16, kQ = 4;
__device__ __forceinline__ int trow(int q, int lane) { return 4 * (lane >> 4) + q; }
template <bool AK, bool BK>
__device__ __forceinline__ AccT tile_gemm(const float* a, int ars, int acs, const float* b, int brs,
                                          int bcs, int K, int bf16) {
  return wave_gemm16<AK, BK>(a, ars, acs, b, brs, bcs, K, bf16);
}
#else
typedef f32x16 AccT;
constexpr int kT = 32, kQ = 16;
__device__ __forceinline__ int trow(int q, int lane) {
  return (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
}
template <bool AK, bool BK>
__device__ __forceinline__ AccT tile_gemm(const float* a, int ars, int acs, const float* b, int brs,
                                          int bcs, int K, int bf16) {
  return wave_gemm32<AK, BK>(a, ars, acs, b, brs, bcs, K, bf16);
}
#endif

// Activation and its derivative expressed through the activation's OUTPUT h (what the
// forward pass keeps in LDS): relu' = [h > 0], tanh' = 1 − h², σ' = h(1 − h).
__device__ __forceinline__ float act_fwd(float v, int act) {
  switch (act) {
    case kTanh: return tanhf(v);
    case kSigmoid: return 1.f / (1.f + __expf(-v));
    case kIdentity: return v;
    default: return fmaxf(v, 0.f);
  }
}

__device__ __forceinline__ float act_grad(float h, int act) {
  switch (act) {
    case kTanh: return 1.f - h * h;
    case kSigmoid: return h * (1.f - h);
    case kIdentity: return 1.f;
    default: return h > 0.f ? 1.f : 0.f;
  }
}

__device__ void load_model(const float* __restrict__ w, float* sm, const MlpDesc& g) {
  for (int l = 0; l < g.L; ++l) {
    const int rows = g.np[l + 1], ld = g.ldw[l], nin = g.n[l], nout = g.n[l + 1];
    float* W = sm + g.lw[l];
    for (int i = threadIdx.x; i < rows * ld; i += blockDim.x) {
      const int o = i / ld, c = i - o * ld;
      W[i] = (o < nout && c < nin) ? w[g.woff[l] + o * nin + c] : 0.f;
    }
    for (int o = threadIdx.x; o < rows; o += blockDim.x)
      sm[g.lb[l] + o] = o < nout ? w[g.boff[l] + o] : 0.f;
  }
}

// Forward of one 32-row tile already staged in H_0; H_L holds the logits.
__device__ void forward(float* sm, const MlpDesc& g) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int l = 0; l < g.L; ++l) {
    const float* H = sm + g.lh[l];
    float* Ho = sm + g.lh[l + 1];
    const float* W = sm + g.lw[l];
    const float* bs = sm + g.lb[l];
    const int ntc = g.np[l + 1] / kT, nt = (kMB / kT) * ntc, ldo = g.ldh[l + 1];
    const bool hidden = l + 1 < g.L;
    for (int t = wave; t < nt; t += 4) {
      const int rt = t / ntc, ct = t - rt * ntc;
      const AccT acc = tile_gemm<kVecA, kVecB>(H + rt * kT * g.ldh[l], g.ldh[l], 1,
                                               W + ct * kT * g.ldw[l], 1, g.ldw[l], g.np[l], g.bf16);
      const int col = ct * kT + (lane & (kT - 1));
      const float bias = bs[col];
      const bool pad = col >= g.n[l + 1];  // padding columns stay exactly zero
#pragma unroll
      for (int q = 0; q < kQ; ++q) {
        float v = acc[q] + bias;
        if (hidden) v = pad ? 0.f : act_fwd(v, g.act);
        Ho[(rt * kT + trow(q, lane)) * ldo + col] = v;
      }
    }
    __syncthreads();
  }
}

__device__ void stage_rows(const float* __restrict__ x, long long r0, long long r1, float* sm,
                           const MlpDesc& g) {
  const int np0 = g.np[0], n0 = g.n[0], ld = g.ldh[0];
  float* H = sm + g.lh[0];
  for (int i = threadIdx.x; i < kMB * np0; i += blockDim.x) {
    const int r = i / np0, c = i - r * np0;
    const long long row = r0 + r;
    H[r * ld + c] = (row < r1 && c < n0) ? x[row * n0 + c] : 0.f;
  }
}

// Diagnostics only (csrc/tests/mlp_stamp_probe.hip builds with OMLDM_MLP_STAMPS): per
// spoke, clock64 sums of the mini-batch phases (staging+barrier, forward, loss, backward).
// The sums stay in registers until the round's end (a global read-modify-write per stamp
// would put a memory round trip into every phase it measures).
#ifdef OMLDM_MLP_STAMPS
__device__ unsigned long long* g_mlp_stamps;
#define MLP_STAMP(k)                                                                  \
  do {                                                                                \
    const unsigned long long now_ = clock64();                                        \
    if ((k) > 0) mlp_acc_[(k) & 7] += now_ - mlp_t_;                                    \
    mlp_t_ = now_;                                                                    \
  } while (0)
#define MLP_STAMP_FLUSH()                                                             \
  do {                                                                                \
    if (tid == 0)                                                                     \
      for (int k_ = 1; k_ < 8; ++k_) g_mlp_stamps[(size_t)blockIdx.x * 8 + k_] += mlp_acc_[k_]; \
  } while (0)
#else
#define MLP_STAMP_FLUSH() \
  do {                    \
  } while (0)
#define MLP_STAMP(k) \
  do {               \
  } while (0)
#endif

__global__ __launch_bounds__(256) void mlp_round_kernel(const float* __restrict__ w,
                                                        const float* __restrict__ x,
                                                        const float* __restrict__ yv, long long B,
                                                        int R, float lr, float* __restrict__ dacc,
                                                        float* __restrict__ stats,
                                                        float* __restrict__ nact, MlpDesc g,
                                                        float* __restrict__ ws, int nparams) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long r0 = (long long)blockIdx.x * R;
  const long long r1 = min(B, r0 + R);
  if (r0 >= B) return;
  load_model(w, sm, g);
  float loss = 0.f, corr = 0.f, nv = 0.f;
  const int L = g.L, npL = g.np[L];
  // Row staging with the NEXT mini-batch's loads in flight while the current one trains
  // (np0 ≤ 64: ≤ 8 slots of the 32 × np0 tile per thread, fixed (row, col) per slot);
  // wider inputs stage synchronously.
  constexpr int kSlots = 8;
  const int np0 = g.np[0], n0 = g.n[0], ld0 = g.ldh[0];
  const bool pf = np0 <= 64;
  int soff[kSlots], srow[kSlots], scol[kSlots];
#pragma unroll
  for (int j = 0; j < kSlots; ++j) {
    const int i = tid + 256 * j;
    const bool in = pf && i < kMB * np0;
    srow[j] = in ? i / np0 : -1;
    scol[j] = in ? i - srow[j] * np0 : 0;
    soff[j] = in ? srow[j] * ld0 + scol[j] : 0;
  }
  float xr[kSlots];
  float yr = 0.f;
  auto fetch = [&](long long m) {  // unconditional loads from clamped rows
#pragma unroll
    for (int j = 0; j < kSlots; ++j) {
      const long long row = min(m + (srow[j] < 0 ? 0 : srow[j]), r1 - 1);
      xr[j] = x[row * n0 + (scol[j] < n0 ? scol[j] : 0)];
    }
    yr = yv[min(m + (tid < kMB ? tid : 0), r1 - 1)];
  };
  if (pf) fetch(r0);
#ifdef OMLDM_MLP_STAMPS
  unsigned long long mlp_t_ = clock64();
  unsigned long long mlp_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  for (long long m0 = r0; m0 < r1; m0 += kMB) {
    MLP_STAMP(0);
    if (pf) {
      float* H = sm + g.lh[0];
#pragma unroll
      for (int j = 0; j < kSlots; ++j)
        if (srow[j] >= 0) H[soff[j]] = (m0 + srow[j] < r1 && scol[j] < n0) ? xr[j] : 0.f;
      if (tid < kMB) sm[g.ly + tid] = m0 + tid < r1 ? yr : __builtin_nanf("");
      if (m0 + kMB < r1) fetch(m0 + kMB);
    } else {
      stage_rows(x, m0, r1, sm, g);
      if (tid < kMB) {
        const long long row = m0 + tid;
        sm[g.ly + tid] = row < r1 ? yv[row] : __builtin_nanf("");
      }
    }
    __syncthreads();
    MLP_STAMP(1);
    forward(sm, g);
    MLP_STAMP(2);
    // ---- loss gradient dZ_L (one thread per row)
    bool valid = false;
    if (tid < kMB) {
      const float y = sm[g.ly + tid];
      valid = !__builtin_isnan(y);
      const float* o = sm + g.lh[L] + tid * g.ldh[L];
      float* G = sm + g.lg0 + tid * g.ldg;
      for (int k = 0; k < npL; ++k) G[k] = 0.f;
      if (valid) {
        if (g.task == 0) {  // regression, squared error (sum)
          const float e = o[0] - y;
          G[0] = 2.f * e;
          loss += e * e;
        } else if (g.task == 1) {  // binary logistic on ±1 / {0,1} labels
          const float t = y > 0.f ? 1.f : 0.f, z = o[0];
          G[0] = 1.f / (1.f + __expf(-z)) - t;
          loss += fmaxf(z, 0.f) - z * t + log1pf(__expf(-fabsf(z)));
          corr += ((z >= 0.f) == (t > 0.f)) ? 1.f : 0.f;
        } else {  // multiclass softmax cross-entropy
          int yi = (int)y;
          yi = yi < 0 ? 0 : (yi >= g.K ? g.K - 1 : yi);
          float m = o[0];
          int am = 0;
          for (int k = 1; k < g.K; ++k)
            if (o[k] > m) {
              m = o[k];
              am = k;
            }
          float se = 0.f;
          for (int k = 0; k < g.K; ++k) se += __expf(o[k] - m);
          const float inv = 1.f / se;
          for (int k = 0; k < g.K; ++k) G[k] = __expf(o[k] - m) * inv - (k == yi ? 1.f : 0.f);
          loss += -(o[yi] - m - __logf(se));
          corr += am == yi ? 1.f : 0.f;
        }
        nv += 1.f;
      }
    }
    const int cnt = __syncthreads_count(valid ? 1 : 0);
    MLP_STAMP(3);
    if (cnt == 0) continue;
    const float eta = lr / (float)cnt;
    int gcur = g.lg0, gnext = g.lg1;
    for (int l = L - 1; l >= 0; --l) {
      const float* Gc = sm + gcur;
      float* W = sm + g.lw[l];
      const float* H = sm + g.lh[l];
      const int ldw = g.ldw[l], ldh = g.ldh[l], nin = g.np[l], nout = g.np[l + 1];
      if (l > 0) {  // dH_l = (dZ · W_l) ⊙ act'(H_l)
        float* Gn = sm + gnext;
        const int ntc = nin / kT;
        for (int t = wave; t < (kMB / kT) * ntc; t += 4) {
          const int rt = t / ntc, ct = t - rt * ntc;
          const AccT acc = tile_gemm<kVecA, false>(Gc + rt * kT * g.ldg, g.ldg, 1, W + ct * kT, ldw,
                                                   1, nout, g.bf16);
          const int col = ct * kT + (lane & (kT - 1));
#pragma unroll
          for (int q = 0; q < kQ; ++q) {
            const int row = rt * kT + trow(q, lane);
            Gn[row * g.ldg + col] = acc[q] * act_grad(H[row * ldh + col], g.act);
          }
        }
      }
      __syncthreads();  // W_l fully read before it is updated
      MLP_STAMP(5);
      const int ntc = nin / kT, nto = nout / kT;
      for (int t = wave; t < nto * ntc; t += 4) {
        const int to = t / ntc, tc = t - to * ntc;
        const AccT acc =
            tile_gemm<false, false>(Gc + to * kT, 1, g.ldg, H + tc * kT, ldh, 1, kMB, g.bf16);
        const int c = tc * kT + (lane & (kT - 1));
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
          const int o = to * kT + trow(q, lane);
          W[o * ldw + c] -= eta * acc[q];
        }
      }
      MLP_STAMP(6);
      for (int o = tid; o < nout; o += blockDim.x) {
        float s = 0.f;
        for (int i = 0; i < kMB; ++i) s += Gc[i * g.ldg + o];
        sm[g.lb[l] + o] -= eta * s;
      }
      __syncthreads();
      MLP_STAMP(7);
      const int tmp = gcur;
      gcur = gnext;
      gnext = tmp;
    }
    MLP_STAMP(4);
  }
  MLP_STAMP_FLUSH();
  // ---- round end: Δ = W_spoke − W_0. With a workspace: the spoke's own row, plain
  // coalesced stores (mlp_colsum_kernel sums the rows); without: atomics into the
  // accumulator (every spoke hits the same nparams addresses — the slow fallback).
  float* wrow = ws ? ws + (size_t)blockIdx.x * nparams : nullptr;
  for (int l = 0; l < L; ++l) {
    const int nin = g.n[l], nout = g.n[l + 1], ld = g.ldw[l];
    const float* W = sm + g.lw[l];
    for (int i = tid; i < nout * nin; i += blockDim.x) {
      const int o = i / nin, c = i - o * nin;
      const float d = W[o * ld + c] - w[g.woff[l] + i];
      if (wrow) wrow[g.woff[l] + i] = d;
      else if (d != 0.f) atomicAdd(&dacc[g.woff[l] + i], d);
    }
    for (int o = tid; o < nout; o += blockDim.x) {
      const float d = sm[g.lb[l] + o] - w[g.boff[l] + o];
      if (wrow) wrow[g.boff[l] + o] = d;
      else if (d != 0.f) atomicAdd(&dacc[g.boff[l] + o], d);
    }
  }
  if (wave == 0) {
    loss = wave_sum(loss);
    corr = wave_sum(corr);
    nv = wave_sum(nv);
    if (lane == 0 && nv > 0.f) {
      atomicAdd(&stats[0], loss);
      atomicAdd(&stats[1], nv);
      atomicAdd(&stats[2], corr);
      atomicAdd(&stats[3], 1.f);
      if (nact) atomicAdd(nact, 1.f);  // the apply kernel's divisor (its own buffer)
    }
  }
}

// ------------------------------------------------------------------ round kernel v2
// The same mini-batch SGD, restructured for step latency (one 32-row step of a
// [13, 64, 64, 1] spoke is a chain of ~10 small GEMMs on one CU; the v1 kernel spent
// ~15 µs per step there, mostly in barriers, zero-padded work and serial loops):
// * widths padded to 16, not 32 (13 → 16 inputs, 1 → 16 outputs: half the MFMAs of the
//   first and last layers; row strides stay ≡ 4 floats mod 64 banks);
// * the loss is the last layer's epilogue: a row's ≤ 16 logits sit in one 16-lane DPP
//   row of the accumulator, so softmax max / sum / argmax are row_ror reductions and the
//   output gradient goes straight to LDS (no loss phase, no barrier);
// * bias gradients are column sums taken in the epilogue that produces each gradient
//   (LDS float atomics), not a 32-row serial loop per layer;
// * backward phase l computes dH_l (reads W_l) together with the update of W_{l+1} (whose
//   dH was the previous phase) from three rotating gradient buffers, and the last phase
//   updates W_1 and W_0 together: one barrier per layer instead of two;
// * the valid-row count of a step comes from a ballot over the staged labels in every
//   wave (no block-wide count);
// * operand loads of the next 16-wide k step are issued before the current MFMAs.
// Same arithmetic as v1 (fp32 MFMA, same mini-batch order); sums may associate
// differently.
// One 16×16 tile, K a multiple of 16: operands read at the top of each 16-wide k step
// (issued while the previous step's MFMAs are in the pipe), the accumulator chained through
// the MFMAs in place — no register copies of it between steps (a copy waits for the
// matrix pipe to drain). fp32 and bf16 are separate instantiations (no branch in the loop).
template <bool AK, bool BK, bool BF16>
__device__ __forceinline__ f32x4 gemm16t(const float* a, int ars, int acs, const float* b,
                                         int brs, int bcs, int K) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* ap = a + r * ars + 4 * g * (AK ? 1 : acs);
  const float* bp = b + 4 * g * (BK ? 1 : brs) + r * bcs;
  for (int k = 0; k < K; k += 16) {
    float av[4], bv[4];
    if constexpr (AK) {
      const float4 t = *reinterpret_cast<const float4*>(ap + k);
      av[0] = t.x; av[1] = t.y; av[2] = t.z; av[3] = t.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) av[u] = ap[(k + u) * acs];
    }
    if constexpr (BK) {
      const float4 t = *reinterpret_cast<const float4*>(bp + k);
      bv[0] = t.x; bv[1] = t.y; bv[2] = t.z; bv[3] = t.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) bv[u] = bp[(k + u) * brs];
    }
    if constexpr (BF16) {
      const bf16x4 af = {bf16_bits(av[0]), bf16_bits(av[1]), bf16_bits(av[2]), bf16_bits(av[3])};
      const bf16x4 bfv = {bf16_bits(bv[0]), bf16_bits(bv[1]), bf16_bits(bv[2]), bf16_bits(bv[3])};
      acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(af, bfv, acc, 0, 0, 0);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
    }
  }
  return acc;
}
template <bool AK, bool BK>
__device__ __forceinline__ f32x4 gemm16p(const float* a, int ars, int acs, const float* b,
                                         int brs, int bcs, int K, int bf16) {
  return bf16 ? gemm16t<AK, BK, true>(a, ars, acs, b, brs, bcs, K)
              : gemm16t<AK, BK, false>(a, ars, acs, b, brs, bcs, K);
}

// 16-lane DPP row reductions (every lane of the row gets the result)
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x124>(v));
  return fmaxf(v, dpp_mov<0x128>(v));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x124>(v);
  return v + dpp_mov<0x128>(v);
}
__device__ __forceinline__ float row16_min(float v) {
  v = fminf(v, dpp_mov<0xB1>(v));
  v = fminf(v, dpp_mov<0x4E>(v));
  v = fminf(v, dpp_mov<0x124>(v));
  return fminf(v, dpp_mov<0x128>(v));
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void mlp_round2_kernel(
    const float* __restrict__ w, const float* __restrict__ x, const float* __restrict__ yv,
    long long B, int R, float lr, float* __restrict__ dacc, float* __restrict__ stats,
    float* __restrict__ nact, MlpDesc g, float* __restrict__ ws, int nparams) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int NT = NW * 64;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int ci = lane & 15, cg = lane >> 4;  // accumulator column / row group
  const long long r0 = (long long)blockIdx.x * R;
  const long long r1 = min(B, r0 + R);
  if (r0 >= B) return;
  load_model(w, sm, g);
  const int L = g.L;
  for (int l = 0; l < L; ++l)
    for (int o = tid; o < g.np[l + 1]; o += NT) sm[g.lbg[l] + o] = 0.f;
  if (tid < 4) sm[g.lsc + tid] = 0.f;
  float loss = 0.f, corr = 0.f, nv = 0.f;
  auto gb = [&](int j) { return sm + g.lgb[j % 3]; };
  // staging: the next mini-batch's rows in registers while the current one trains
  constexpr int kSlots = (kMB * 64 + NT - 1) / NT;
  const int np0 = g.np[0], n0 = g.n[0], ld0 = g.ldh[0];
  const bool pf = np0 <= 64;
  int soff[kSlots], srow[kSlots], scol[kSlots];
#pragma unroll
  for (int j = 0; j < kSlots; ++j) {
    const int i = tid + NT * j;
    const bool in = pf && i < kMB * np0;
    srow[j] = in ? i / np0 : -1;
    scol[j] = in ? i - srow[j] * np0 : 0;
    soff[j] = in ? srow[j] * ld0 + scol[j] : 0;
  }
  float xr[kSlots];
  float yr = 0.f;
  auto fetch = [&](long long m) {
#pragma unroll
    for (int j = 0; j < kSlots; ++j) {
      const long long row = min(m + (srow[j] < 0 ? 0 : srow[j]), r1 - 1);
      xr[j] = x[row * n0 + (scol[j] < n0 ? scol[j] : 0)];
    }
    yr = yv[min(m + (tid < kMB ? tid : 0), r1 - 1)];
  };
  if (pf) fetch(r0);
  __syncthreads();
#ifdef OMLDM_MLP_STAMPS
  unsigned long long mlp_t_ = clock64();
  unsigned long long mlp_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  for (long long m0 = r0; m0 < r1; m0 += kMB) {
    MLP_STAMP(0);
    if (pf) {
      float* H = sm + g.lh[0];
#pragma unroll
      for (int j = 0; j < kSlots; ++j)
        if (srow[j] >= 0) H[soff[j]] = (m0 + srow[j] < r1 && scol[j] < n0) ? xr[j] : 0.f;
      if (tid < kMB) sm[g.ly + tid] = m0 + tid < r1 ? yr : __builtin_nanf("");
      if (m0 + kMB < r1) fetch(m0 + kMB);
    } else {
      stage_rows(x, m0, r1, sm, g);
      if (tid < kMB) {
        const long long row = m0 + tid;
        sm[g.ly + tid] = row < r1 ? yv[row] : __builtin_nanf("");
      }
    }
    __syncthreads();
    // valid rows of the step: every wave counts them itself
    const float yl = sm[g.ly + (lane & 31)];
    const int cnt = __builtin_popcountll(__builtin_amdgcn_ballot_w64(lane < 32 && yl == yl));
    if (cnt == 0) {
      __syncthreads();
      continue;
    }
    const float eta = lr / (float)cnt;
    MLP_STAMP(1);
    // ---- hidden layers: H_{l+1} = act(H_l · W_lᵀ + b_l)
    for (int l = 0; l + 1 < L; ++l) {
      const float* H = sm + g.lh[l];
      float* Ho = sm + g.lh[l + 1];
      const float* W = sm + g.lw[l];
      const float* bs = sm + g.lb[l];
      const int ntc = g.np[l + 1] / 16, nt = 2 * ntc, ldo = g.ldh[l + 1];
      for (int t = wave; t < nt; t += NW) {
        const int rt = t / ntc, ct = t - rt * ntc;
        const f32x4 acc = gemm16p<true, true>(H + rt * 16 * g.ldh[l], g.ldh[l], 1,
                                              W + ct * 16 * g.ldw[l], 1, g.ldw[l], g.np[l], g.bf16);
        const int col = ct * 16 + ci;
        const float bias = bs[col];
        const bool pad = col >= g.n[l + 1];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = acc[q] + bias;
          Ho[(rt * 16 + 4 * cg + q) * ldo + col] = pad ? 0.f : act_fwd(v, g.act);
        }
      }
      __syncthreads();
    }
    MLP_STAMP(2);
    // ---- output layer + loss (np_L = 16: one column tile, a row's logits in one DPP row)
    {
      const int l = L - 1;
      float* GL = gb(L);
      for (int rt = wave; rt < 2; rt += NW) {
        const f32x4 acc = gemm16p<true, true>(sm + g.lh[l] + rt * 16 * g.ldh[l], g.ldh[l], 1,
                                              sm + g.lw[l], 1, g.ldw[l], g.np[l], g.bf16);
        const float bias = sm[g.lb[l] + ci];
        float csum = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = rt * 16 + 4 * cg + q;
          const float o = acc[q] + bias;
          const float y = sm[g.ly + row];
          const bool valid = y == y;
          float gr = 0.f;
          if (g.task == 2) {
            const bool live = ci < g.K;
            int yi = valid ? (int)y : 0;
            yi = yi < 0 ? 0 : (yi >= g.K ? g.K - 1 : yi);
            const float m = row16_max(live ? o : -INFINITY);
            const float e = live ? __expf(o - m) : 0.f;
            const float se = row16_sum(e);
            const float am = row16_min(live && o == m ? (float)ci : 64.f);
            gr = valid && live ? e / se - (ci == yi ? 1.f : 0.f) : 0.f;
            if (valid && ci == yi) {
              loss += -(o - m - __logf(se));
              corr += (int)am == yi ? 1.f : 0.f;
            }
          } else if (ci == 0 && valid) {
            if (g.task == 0) {
              const float e = o - y;
              gr = 2.f * e;
              loss += e * e;
            } else {
              const float tt = y > 0.f ? 1.f : 0.f;
              gr = 1.f / (1.f + __expf(-o)) - tt;
              loss += fmaxf(o, 0.f) - o * tt + __logf(1.f + __expf(-fabsf(o)));  // statistic
              corr += ((o >= 0.f) == (tt > 0.f)) ? 1.f : 0.f;
            }
          }
          if (ci == 0 && valid) nv += 1.f;
          GL[row * g.ldg + ci] = gr;
          csum += gr;
        }
        atomicAdd(&sm[g.lbg[l] + ci], csum);
      }
      __syncthreads();
    }
    MLP_STAMP(3);
    // ---- backward: phase l = dH_l (l ≥ 1) + update of W_{l+1} (l + 1 ≤ L − 1), and the
    // last phase (l = 0) updates W_1 and W_0
    for (int l = L - 1; l >= 0; --l) {
      const int na = l >= 1 ? 2 * (g.np[l] / 16) : 0;
      const int ub = l + 1 <= L - 1 ? l + 1 : -1;  // W_{l+1}
      const int nb = ub >= 0 ? (g.np[ub + 1] / 16) * (g.np[ub] / 16) : 0;
      const int nc = l == 0 ? (g.np[1] / 16) * (g.np[0] / 16) : 0;
      for (int t = wave; t < na + nb + nc; t += NW) {
        if (t < na) {  // dH_l = (G_{l+1} · W_l) ⊙ act'(H_l)
          const float* Gc = gb(l + 1);
          float* Gn = gb(l);
          const float* W = sm + g.lw[l];
          const float* H = sm + g.lh[l];
          const int ntc = g.np[l] / 16, rt = t / ntc, ct = t - rt * ntc;
          const f32x4 acc = gemm16p<true, false>(Gc + rt * 16 * g.ldg, g.ldg, 1, W + ct * 16,
                                                 g.ldw[l], 1, g.np[l + 1], g.bf16);
          const int col = ct * 16 + ci;
          float csum = 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int row = rt * 16 + 4 * cg + q;
            const float v = acc[q] * act_grad(H[row * g.ldh[l] + col], g.act);
            Gn[row * g.ldg + col] = v;
            csum += v;
          }
          atomicAdd(&sm[g.lbg[l - 1] + col], csum);
        } else {  // W_u −= η · G_{u+1}ᵀ · H_u
          const int u = t < na + nb ? ub : 0;
          const int tt = t < na + nb ? t - na : t - na - nb;
          const float* Gc = gb(u + 1);
          float* W = sm + g.lw[u];
          const float* H = sm + g.lh[u];
          const int ntc = g.np[u] / 16, to = tt / ntc, tc = tt - to * ntc;
          const f32x4 acc = gemm16p<false, false>(Gc + to * 16, 1, g.ldg, H + tc * 16, g.ldh[u], 1,
                                                  kMB, g.bf16);
          const int c = tc * 16 + ci;
#pragma unroll
          for (int q = 0; q < 4; ++q) W[(to * 16 + 4 * cg + q) * g.ldw[u] + c] -= eta * acc[q];
        }
      }
      auto bias_step = [&](int u) {
        for (int o = tid; o < g.np[u + 1]; o += NT) {
          sm[g.lb[u] + o] -= eta * sm[g.lbg[u] + o];
          sm[g.lbg[u] + o] = 0.f;
        }
      };
      if (ub >= 0) bias_step(ub);
      if (l == 0) bias_step(0);
      __syncthreads();
      MLP_STAMP(4 + (l < 3 ? l : 3));  // 4: phase 0 (W_1, W_0), 5: phase 1, 6: phase 2
    }
  }
  MLP_STAMP_FLUSH();
  // ---- round end: Δ = W_spoke − W_0 (as v1)
  float* wrow = ws ? ws + (size_t)blockIdx.x * nparams : nullptr;
  for (int l = 0; l < L; ++l) {
    const int nin = g.n[l], nout = g.n[l + 1], ld = g.ldw[l];
    const float* W = sm + g.lw[l];
    for (int i = tid; i < nout * nin; i += NT) {
      const int o = i / nin, c = i - o * nin;
      const float d = W[o * ld + c] - w[g.woff[l] + i];
      if (wrow) wrow[g.woff[l] + i] = d;
      else if (d != 0.f) atomicAdd(&dacc[g.woff[l] + i], d);
    }
    for (int o = tid; o < nout; o += NT) {
      const float d = sm[g.lb[l] + o] - w[g.boff[l] + o];
      if (wrow) wrow[g.boff[l] + o] = d;
      else if (d != 0.f) atomicAdd(&dacc[g.boff[l] + o], d);
    }
  }
  loss = wave_sum(loss);
  corr = wave_sum(corr);
  nv = wave_sum(nv);
  if (lane == 0 && nv > 0.f) {
    atomicAdd(&sm[g.lsc + 0], loss);
    atomicAdd(&sm[g.lsc + 1], nv);
    atomicAdd(&sm[g.lsc + 2], corr);
  }
  __syncthreads();
  if (tid == 0 && sm[g.lsc + 1] > 0.f) {
    atomicAdd(&stats[0], sm[g.lsc + 0]);
    atomicAdd(&stats[1], sm[g.lsc + 1]);
    atomicAdd(&stats[2], sm[g.lsc + 2]);
    atomicAdd(&stats[3], 1.f);
    if (nact) atomicAdd(nact, 1.f);
  }
}

// Inference: every block stages the model once and walks 32-row tiles (grid-stride).
__global__ __launch_bounds__(256) void mlp_forward_kernel(const float* __restrict__ w,
                                                          const float* __restrict__ x,
                                                          long long B, float* __restrict__ out,
                                                          MlpDesc g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  load_model(w, sm, g);
  const int L = g.L;
  for (long long m0 = (long long)blockIdx.x * kMB; m0 < B; m0 += (long long)gridDim.x * kMB) {
    __syncthreads();  // previous tile's H_L consumed
    stage_rows(x, m0, B, sm, g);
    __syncthreads();
    forward(sm, g);
    const float* o = sm + g.lh[L];
    for (int i = threadIdx.x; i < kMB * g.K; i += blockDim.x) {
      const int r = i / g.K, k = i - r * g.K;
      if (m0 + r < B) out[(m0 + r) * g.K + k] = o[r * g.ldh[L] + k];
    }
  }
}

static int make_desc(int L, const int* widths, int task, int act, MlpDesc* g, int pad = 32) {
  if (L < 1 || L > kMaxLayers || (act & 0xff) > kIdentity || (act & ~0x1ff)) return -1;
  *g = MlpDesc{};
  g->L = L;
  g->task = task;
  g->act = act & 0xff;        // low byte: hidden activation
  g->bf16 = (act >> 8) & 1;   // bit 8: bf16 GEMM operands
  g->K = widths[L];
  int off = 0;
  for (int l = 0; l <= L; ++l) {
    if (widths[l] < 1) return -1;
    g->n[l] = widths[l];
    g->np[l] = (widths[l] + pad - 1) / pad * pad;
  }
  for (int l = 0; l < L; ++l) {  // flat parameter layout: W_l [n_{l+1} × n_l], b_l
    g->woff[l] = off;
    off += g->n[l + 1] * g->n[l];
    g->boff[l] = off;
    off += g->n[l + 1];
  }
  // row strides ≡ 4 floats mod 64 banks (np is a multiple of 32): a 16-lane group reading
  // 16 bytes each from 16 rows covers all 64 banks once, and a lane reading one float per
  // row (the strided operands) sees rows 4 banks apart; region starts 16-byte aligned
  int p = 0, maxnp = 0;
  auto al4 = [](int v) { return (v + 3) & ~3; };
  for (int l = 0; l < L; ++l) {
    g->ldw[l] = g->np[l] + 4;
    g->lw[l] = p;
    p = al4(p + g->np[l + 1] * g->ldw[l]);
    g->lb[l] = p;
    p = al4(p + g->np[l + 1]);
  }
  for (int l = 0; l <= L; ++l) {
    g->ldh[l] = g->np[l] + 4;
    g->lh[l] = p;
    p = al4(p + kMB * g->ldh[l]);
    if (g->np[l] > maxnp) maxnp = g->np[l];
  }
  g->ldg = maxnp + 4;
  g->lg0 = p;
  p += kMB * g->ldg;
  g->lg1 = p;
  p += kMB * g->ldg;
  g->ly = p;
  p += kMB;
  if (pad == 16) {  // v2 layout: three gradient buffers (lg0, lg1 + one more), bias grads
    g->lgb[0] = g->lg0;
    g->lgb[1] = g->lg1;
    g->lgb[2] = p;
    p += kMB * g->ldg;
    for (int l = 0; l < L; ++l) {
      g->lbg[l] = p;
      p = al4(p + g->np[l + 1]);
    }
    g->lsc = p;
    p += 4;
  }
  g->total = p;
  return 0;
}

// dacc[c] += Σ_{s in this block's 64-spoke slab} ws[s][c]: one atomic per (column, slab)
// instead of one per (column, spoke).
constexpr int kMlpSlab = 64;
__global__ __launch_bounds__(256) void mlp_colsum_kernel(const float* __restrict__ ws, int S,
                                                         int n, float* __restrict__ dacc) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n) return;
  const int s0 = blockIdx.y * kMlpSlab, s1 = min(S, s0 + kMlpSlab);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = s0;
  for (; s + 3 < s1; s += 4) {
    a0 += ws[(size_t)s * n + c];
    a1 += ws[(size_t)(s + 1) * n + c];
    a2 += ws[(size_t)(s + 2) * n + c];
    a3 += ws[(size_t)(s + 3) * n + c];
  }
  for (; s < s1; ++s) a0 += ws[(size_t)s * n + c];
  const float t = (a0 + a1) + (a2 + a3);
  if (t != 0.f) atomicAdd(&dacc[c], t);
}

}  // namespace omldm

using namespace omldm;

// Round kernel form: 0 v1 (mlp_round_kernel), 1 / 2 / 3 v2 with 4 / 8 / 16 waves (v2 takes
// output widths ≤ 16). `set` ≥ 0 sets it; the default comes from OMLDM_MLP_FORM (3).
OMLDM_API int omldm_mlp_form(int set) {
  static int form = [] {
    const char* e = getenv("OMLDM_MLP_FORM");
    return e ? atoi(e) : 3;
  }();
  if (set >= 0) form = set;
  return form;
}

// LDS bytes the fused kernels need for this layer stack (host-side feasibility check).
OMLDM_API long long omldm_mlp_lds_bytes(int L, const int* widths) {
  MlpDesc g;
  if (make_desc(L, widths, 0, 0, &g)) return -1;
  return (long long)g.total * 4;
}

// One protocol round: S spokes × R rows (spoke s owns rows [sR, sR+R)); task 0 regression,
// 1 binary logistic, 2 softmax. dacc[nparams] += Σ_s Δ_s; stats[0..3] += loss, n, correct,
// active spokes (spokes with ≥ 1 labelled row); nact (optional, zeroed beforehand) += active
// spokes too. Follow with omldm_multiclass_apply(w, dacc, nparams, ..., nact, ...): the
// apply kernel clears stats, so its divisor must live in a separate buffer.
// ws: optional S × nparams scratch (spoke deltas by plain stores + slab column sums).
OMLDM_API int omldm_mlp_round(const float* w, const float* x, const float* y, long long B, int R,
                              int S, int L, const int* widths, int task, int act, float lr,
                              float* dacc, float* stats, float* nact, float* ws, void* stream) {
  if (B <= 0 || S <= 0) return 0;
  if (R <= 0 || (long long)R * S < B) return -3;
  MlpDesc g;
  const int form = omldm_mlp_form(-1);
  if (form > 0 && widths[L] <= 16 && make_desc(L, widths, task, act, &g, 16) == 0 &&
      (size_t)g.total * 4 <= 160 * 1024) {
    const size_t lds = (size_t)g.total * 4;
    const int nparams = g.boff[g.L - 1] + g.n[g.L];
    int e;
    if (form == 3) {
      if ((e = check_dyn_lds((const void*)mlp_round2_kernel<16>, lds))) return e;
      hipLaunchKernelGGL(mlp_round2_kernel<16>, dim3(S), dim3(1024), lds, (hipStream_t)stream, w,
                         x, y, B, R, lr, dacc, stats, nact, g, ws, nparams);
    } else if (form == 2) {
      if ((e = check_dyn_lds((const void*)mlp_round2_kernel<8>, lds))) return e;
      hipLaunchKernelGGL(mlp_round2_kernel<8>, dim3(S), dim3(512), lds, (hipStream_t)stream, w, x,
                         y, B, R, lr, dacc, stats, nact, g, ws, nparams);
    } else {
      if ((e = check_dyn_lds((const void*)mlp_round2_kernel<4>, lds))) return e;
      hipLaunchKernelGGL(mlp_round2_kernel<4>, dim3(S), dim3(256), lds, (hipStream_t)stream, w, x,
                         y, B, R, lr, dacc, stats, nact, g, ws, nparams);
    }
  } else {
    if (make_desc(L, widths, task, act, &g)) return -1;
    const size_t lds = (size_t)g.total * 4;
    if (lds > 160 * 1024) return -2;
    int e = check_dyn_lds((const void*)mlp_round_kernel, lds);
    if (e) return e;
    const int nparams = g.boff[g.L - 1] + g.n[g.L];
    hipLaunchKernelGGL(mlp_round_kernel, dim3(S), dim3(256), lds, (hipStream_t)stream, w, x, y, B,
                       R, lr, dacc, stats, nact, g, ws, nparams);
  }
  const int nparams = g.boff[g.L - 1] + g.n[g.L];
  if (ws)
    hipLaunchKernelGGL(mlp_colsum_kernel, dim3((nparams + 255) / 256, (S + kMlpSlab - 1) / kMlpSlab),
                       dim3(256), 0, (hipStream_t)stream, ws, S, nparams, dacc);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_mlp_forward(const float* w, const float* x, long long B, int L,
                                const int* widths, int act, float* out, void* stream) {
  if (B <= 0) return 0;
  MlpDesc g;
  if (make_desc(L, widths, 0, act, &g)) return -1;
  const size_t lds = (size_t)g.total * 4;
  if (lds > 160 * 1024) return -2;
  int e = check_dyn_lds((const void*)mlp_forward_kernel, lds);
  if (e) return e;
  long long tiles = (B + kMB - 1) / kMB;
  int blocks = (int)(tiles < 1024 ? tiles : 1024);
  hipLaunchKernelGGL(mlp_forward_kernel, dim3(blocks), dim3(256), lds, (hipStream_t)stream, w, x,
                     B, out, g);
  return (int)hipGetLastError();
}
