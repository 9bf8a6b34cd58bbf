// HT learner: Hoeffding tree (VFDT) with Gaussian numeric-attribute observers, fully on
// the device (no host round trip per split decision).
//
// Reference: learner "HT" (omldm/utils/parsers/requestStream/PipelineMap.scala:68), run in
// SingleLearner mode (FlinkSpoke.scala:203-209); algorithm SURVEY.md Appendix D / K13:
// per-leaf sufficient statistics, split when ΔG > ε = sqrt(R² ln(1/δ) / (2n)) (or ε < τ).
//
// Tree = flat arrays (feature, threshold, left, right per node; class counts per node;
// per (node, feature, class) Gaussian moments n, Σx, Σx²; per (node, feature) range).
// * ht_update_kernel — one thread per row: route to the leaf through the (L2-resident)
//   node arrays; the wave aggregates its rows per (leaf, class) with ballots and DPP
//   reductions, then one lane per pair adds them to the leaf's statistics (float
//   atomics; range via the sign-split integer atomic min/max trick);
// * ht_split_kernel  — one workgroup per node; leaves that saw ≥ gracePeriod points
//   score nBins candidate thresholds per feature (class mass split by the Gaussian
//   CDFs, information gain) in parallel, reduce best / second-best attribute, apply the
//   Hoeffding test, and allocate two children with one atomic on the node counter;
// * ht_predict_kernel — route + majority class of the leaf.
#include "common.h"

namespace omldm {

constexpr int kHtMaxC = 32;
constexpr int kHtRegF = 8;  // features reduced per unrolled step of the wave aggregation

__device__ __forceinline__ void atomic_min_f(float* a, float v) {
  if (v >= 0.f)
    atomicMin(reinterpret_cast<int*>(a), __float_as_int(v));
  else
    atomicMax(reinterpret_cast<unsigned int*>(a), __float_as_uint(v));
}

__device__ __forceinline__ void atomic_max_f(float* a, float v) {
  if (v >= 0.f)
    atomicMax(reinterpret_cast<int*>(a), __float_as_int(v));
  else
    atomicMin(reinterpret_cast<unsigned int*>(a), __float_as_uint(v));
}

__device__ __forceinline__ int ht_route(const float* __restrict__ xr, const float* __restrict__ feat,
                                        const float* __restrict__ thr,
                                        const float* __restrict__ left,
                                        const float* __restrict__ right, int depth) {
  int node = 0;
  for (int it = 0; it <= depth; ++it) {
    const int f = (int)feat[node];
    if (f < 0) break;
    node = (int)(xr[f] <= thr[node] ? left[node] : right[node]);
  }
  return node;
}

__device__ __forceinline__ float wave_min(float v) { return -wave_max(-v); }

// One thread per row routes it to its leaf; the rows of a wavefront are then aggregated
// per distinct (leaf, class) pair before touching global memory: the wave repeatedly
// takes the first pending pair, ballots the lanes that share it, reduces their
// per-feature Σ1 (popcount), Σx, Σx², min and max with DPP wave reductions, and one
// lane issues the pair's atomics. Early in the stream every row of a wave lands in the
// same one or few leaves, so this turns ~64·(5d+2) same-address atomics per wave into
// (5d+2) per distinct pair (the previous per-row version serialised on them).
__global__ __launch_bounds__(256) void ht_update_kernel(
    const float* __restrict__ x, const float* __restrict__ yv, int B, int d, int C, int depth,
    const float* __restrict__ feat, const float* __restrict__ thr, const float* __restrict__ left,
    const float* __restrict__ right, float* __restrict__ cc, float* __restrict__ S0,
    float* __restrict__ S1, float* __restrict__ S2, float* __restrict__ lo, float* __restrict__ hi,
    float* __restrict__ since, float* __restrict__ nfit) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int key = -1, node = 0, yi = 0;
  const float* xr = x;
  if (row < B && !__builtin_isnan(yv[row])) {
    yi = (int)yv[row];
    yi = yi < 0 ? 0 : (yi >= C ? C - 1 : yi);
    xr = x + (size_t)row * d;
    node = ht_route(xr, feat, thr, left, right, depth);
    key = node * C + yi;
  }
  unsigned long long pending = __ballot(key >= 0);
  const float n = (float)__popcll(pending);
  if (lane == 0 && n > 0.f && nfit) atomicAdd(nfit, n);
  while (pending) {  // wave-uniform
    const int leader = __ffsll((long long)pending) - 1;
    const int k = __shfl(key, leader);
    const bool mine = key == k;
    const unsigned long long grp = __ballot(mine);
    pending &= ~grp;
    const float cnt = (float)__popcll(grp);
    const int nd = k / C, yc = k - nd * C;
    if (lane == leader) {
      atomicAdd(&cc[nd * C + yc], cnt);
      atomicAdd(&since[nd], cnt);
    }
    for (int f0 = 0; f0 < d; f0 += kHtRegF) {
      // features [f0, f0 + kHtRegF) of this lane's row, loaded once per chunk and pair
#pragma unroll
      for (int u = 0; u < kHtRegF; u += 2) {
        const int fa = f0 + u, fb = f0 + u + 1;
        const float va = (mine && fa < d) ? xr[fa] : 0.f;
        const float vb = (mine && fb < d) ? xr[fb] : 0.f;
        float s1a = va, s2a = va * va, s1b = vb, s2b = vb * vb;
        wave_sum2(s1a, s1b);
        wave_sum2(s2a, s2b);
        const float mna = wave_min(mine ? va : INFINITY), mxa = wave_max(mine ? va : -INFINITY);
        const float mnb = wave_min(mine ? vb : INFINITY), mxb = wave_max(mine ? vb : -INFINITY);
        if (lane == leader) {
          if (fa < d) {
            const size_t b = ((size_t)nd * d + fa) * C + yc;
            atomicAdd(&S0[b], cnt);
            atomicAdd(&S1[b], s1a);
            atomicAdd(&S2[b], s2a);
            atomic_min_f(&lo[nd * d + fa], mna);
            atomic_max_f(&hi[nd * d + fa], mxa);
          }
          if (fb < d) {
            const size_t b = ((size_t)nd * d + fb) * C + yc;
            atomicAdd(&S0[b], cnt);
            atomicAdd(&S1[b], s1b);
            atomicAdd(&S2[b], s2b);
            atomic_min_f(&lo[nd * d + fb], mnb);
            atomic_max_f(&hi[nd * d + fb], mxb);
          }
        }
      }
    }
  }
}

__device__ __forceinline__ float entropy(const float* m, int C, float tot) {
  if (tot <= 1e-12f) return 0.f;
  float h = 0.f;
  for (int c = 0; c < C; ++c) {
    const float p = m[c] / tot;
    if (p > 1e-12f) h -= p * __log2f(p);
  }
  return h;
}

// Class mass left of threshold t for feature f of node (Gaussian CDF per class).
__device__ __forceinline__ void split_mass(const float* S0, const float* S1, const float* S2,
                                           size_t base, int C, float t, float* lm, float* rm) {
  for (int c = 0; c < C; ++c) {
    const float n = S0[base + c];
    const float nn = fmaxf(n, 1.f);
    const float mu = S1[base + c] / nn;
    const float var = fmaxf(S2[base + c] / nn - mu * mu, 1e-6f);
    const float z = (t - mu) * rsqrtf(var);
    const float cdf = 0.5f * (1.f + erff(z * 0.70710678f));
    lm[c] = n * cdf;
    rm[c] = n - lm[c];
  }
}

__global__ __launch_bounds__(256) void ht_split_kernel(
    int N, int d, int C, int nb, float grace, float delta, float tau, float* __restrict__ feat,
    float* __restrict__ thr, float* __restrict__ left, float* __restrict__ right,
    float* __restrict__ cc, const float* __restrict__ S0, const float* __restrict__ S1,
    const float* __restrict__ S2, const float* __restrict__ lo, const float* __restrict__ hi,
    float* __restrict__ since, float* __restrict__ nnodes) {
  extern __shared__ __attribute__((aligned(16))) float gains[];  // [d·nb]
  const int node = blockIdx.x;
  if (node >= (int)nnodes[0] || feat[node] >= 0.f || since[node] < grace) return;
  const float* cn = cc + (size_t)node * C;
  float ntot = 0.f;
  int nz = 0;
  for (int c = 0; c < C; ++c) {
    ntot += cn[c];
    nz += cn[c] > 0.f;
  }
  if (ntot < 2.f || nz < 2 || (int)nnodes[0] + 2 > N) {
    if (threadIdx.x == 0) since[node] = 0.f;
    return;
  }
  const float h0 = entropy(cn, C, ntot);
  float lm[kHtMaxC], rm[kHtMaxC];
  for (int p = threadIdx.x; p < d * nb; p += 256) {
    const int f = p / nb, b = p - f * nb;
    const float l = lo[node * d + f], span = hi[node * d + f] - l;
    float g = -1.f;
    if (span > 0.f) {
      const float t = l + span * (float)(b + 1) / (float)(nb + 1);
      split_mass(S0, S1, S2, ((size_t)node * d + f) * C, C, t, lm, rm);
      float nl = 0.f, nr = 0.f;
      for (int c = 0; c < C; ++c) {
        nl += lm[c];
        nr += rm[c];
      }
      g = h0 - (nl * entropy(lm, C, nl) + nr * entropy(rm, C, nr)) / fmaxf(nl + nr, 1e-12f);
    }
    gains[p] = g;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  float g1 = -2.f, g2 = -2.f;
  int f1 = 0, b1 = 0;
  for (int f = 0; f < d; ++f) {
    float gm = -2.f;
    int bm = 0;
    for (int b = 0; b < nb; ++b)
      if (gains[f * nb + b] > gm) {
        gm = gains[f * nb + b];
        bm = b;
      }
    if (gm > g1) {
      g2 = g1;
      g1 = gm;
      f1 = f;
      b1 = bm;
    } else if (gm > g2) {
      g2 = gm;
    }
  }
  if (d == 1) g2 = 0.f;
  since[node] = 0.f;
  const float R = __log2f((float)C);
  const float eps = sqrtf(R * R * logf(1.f / delta) / (2.f * ntot));
  if (!(g1 > 0.f && (g1 - g2 > eps || eps < tau))) return;
  const int old = (int)atomicAdd(nnodes, 2.f);
  if (old + 2 > N) {
    atomicAdd(nnodes, -2.f);
    return;
  }
  const float l = lo[node * d + f1], span = hi[node * d + f1] - l;
  const float t = l + span * (float)(b1 + 1) / (float)(nb + 1);
  split_mass(S0, S1, S2, ((size_t)node * d + f1) * C, C, t, lm, rm);
  for (int c = 0; c < C; ++c) {
    cc[(size_t)old * C + c] = lm[c];
    cc[(size_t)(old + 1) * C + c] = rm[c];
  }
  thr[node] = t;
  left[node] = (float)old;
  right[node] = (float)(old + 1);
  __threadfence();
  feat[node] = (float)f1;
}

__global__ __launch_bounds__(256) void ht_predict_kernel(
    const float* __restrict__ x, int B, int d, int C, int depth, const float* __restrict__ feat,
    const float* __restrict__ thr, const float* __restrict__ left, const float* __restrict__ right,
    const float* __restrict__ cc, float* __restrict__ out) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= B) return;
  const int node = ht_route(x + (size_t)row * d, feat, thr, left, right, depth);
  const float* cn = cc + (size_t)node * C;
  int best = 0;
  for (int c = 1; c < C; ++c)
    if (cn[c] > cn[best]) best = c;
  out[row] = (float)best;
}

}  // namespace omldm

using namespace omldm;

// tree: pointers in the order feat, thr, left, right, cc, S0, S1, S2, lo, hi, since, nnodes.
OMLDM_API int omldm_ht_update(const float* x, const float* y, int B, int d, int C, int depth,
                              float* const* tree, float* nfit, void* stream) {
  if (B <= 0) return 0;
  if (C < 1 || C > kHtMaxC) return -1;
  hipLaunchKernelGGL(ht_update_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     x, y, B, d, C, depth, tree[0], tree[1], tree[2], tree[3], tree[4], tree[5],
                     tree[6], tree[7], tree[8], tree[9], tree[10], nfit);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_ht_split(int N, int d, int C, int nb, float grace, float delta, float tau,
                             float* const* tree, void* stream) {
  if (C < 1 || C > kHtMaxC || nb < 1) return -1;
  const size_t lds = (size_t)d * nb * 4;
  if (lds > 150 * 1024) return -2;
  int e = check_dyn_lds((const void*)ht_split_kernel, lds);
  if (e) return e;
  hipLaunchKernelGGL(ht_split_kernel, dim3(N), dim3(256), lds, (hipStream_t)stream, N, d, C, nb,
                     grace, delta, tau, tree[0], tree[1], tree[2], tree[3], tree[4], tree[5],
                     tree[6], tree[7], tree[8], tree[9], tree[10], tree[11]);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_ht_predict(const float* x, int B, int d, int C, int depth,
                               float* const* tree, float* out, void* stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(ht_predict_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     x, B, d, C, depth, tree[0], tree[1], tree[2], tree[3], tree[4], out);
  return (int)hipGetLastError();
}
