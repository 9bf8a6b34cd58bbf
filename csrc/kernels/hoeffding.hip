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
    float* __restrict__ since, double* __restrict__ nfit) {
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
  if (lane == 0 && n > 0.f && nfit) atomicAdd(nfit, (double)n);
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

// ---- sort-based update (default): no atomics on the leaf statistics --------------------
// Rows are counting-sorted by key = leaf·C + class, then blocks reduce contiguous chunks
// of one key's rows and add each chunk's totals with one atomic per statistic. Four short
// launches:
//   1. route + per-block key histogram (LDS), keys[row] kept;
//   2. scan: per-(block, key) bases in key-major order, segment starts/lengths;
//   3. scatter row ids to their sorted positions (LDS cursors, no global atomics);
//   4. per-chunk segment reduce (Σ1, Σx, Σx², min, max per feature).
constexpr int kHtRowsPerBlock = 4096;  // rows per route/scatter block (1024 threads)
constexpr int kHtSegChunk = 1024;      // rows per segment-reduce block (a key may span many)

// The tree's (feature, threshold, left, right) are staged in LDS as one int4 per node when
// they fit (one ds_read_b128 per level instead of four dependent L2 reads), and each thread
// routes its kHtRowsPerBlock / 1024 rows level-synchronously, so the per-level latency is
// paid once for all of them rather than once per row.
constexpr int kHtRowsPerThread = kHtRowsPerBlock / 1024;

__global__ __launch_bounds__(1024) void ht_route_hist_kernel(
    const float* __restrict__ x, const float* __restrict__ yv, int B, int d, int C, int depth,
    const float* __restrict__ feat, const float* __restrict__ thr, const float* __restrict__ left,
    const float* __restrict__ right, int nbins, int nnodes, int* __restrict__ keys,
    int* __restrict__ hist, double* __restrict__ nfit) {
  extern __shared__ int h[];  // [nbins], then int4 tree[nnodes] when nnodes > 0
  int4* tree = reinterpret_cast<int4*>(h + ((nbins + 3) & ~3));
  for (int b = threadIdx.x; b < nbins; b += 1024) h[b] = 0;
  for (int n = threadIdx.x; n < nnodes; n += 1024)
    tree[n] = make_int4((int)feat[n], __float_as_int(thr[n]), (int)left[n], (int)right[n]);
  __syncthreads();
  const int r0 = blockIdx.x * kHtRowsPerBlock + threadIdx.x;
  int node[kHtRowsPerThread], yi[kHtRowsPerThread];
  bool ok[kHtRowsPerThread];
#pragma unroll
  for (int u = 0; u < kHtRowsPerThread; ++u) {
    const int r = r0 + u * 1024;
    const float yr = r < B ? yv[r] : __builtin_nanf("");
    ok[u] = !__builtin_isnan(yr);
    const int yc = ok[u] ? (int)yr : 0;
    yi[u] = yc < 0 ? 0 : (yc >= C ? C - 1 : yc);
    node[u] = 0;
  }
  for (int it = 0; it <= depth; ++it) {
    bool more = false;
#pragma unroll
    for (int u = 0; u < kHtRowsPerThread; ++u) {
      int4 t;
      if (nnodes > 0) {
        t = tree[node[u]];
      } else {
        t = make_int4((int)feat[node[u]], __float_as_int(thr[node[u]]), (int)left[node[u]],
                      (int)right[node[u]]);
      }
      const bool inner = ok[u] && t.x >= 0;
      // branch-free gather from a clamped address (row 0 / feature 0 for finished rows)
      const size_t r = inner ? (size_t)(r0 + u * 1024) : 0;
      const float v = x[r * d + (inner ? t.x : 0)];
      const int nx = v <= __int_as_float(t.y) ? t.z : t.w;
      node[u] = inner ? nx : node[u];
      more |= inner;
    }
    if (!more) break;
  }
  float cnt = 0.f;
#pragma unroll
  for (int u = 0; u < kHtRowsPerThread; ++u) {
    const int r = r0 + u * 1024;
    if (r >= B) break;
    int key = ok[u] ? node[u] * C + yi[u] : -1;
    if (key >= nbins) key = -1;
    keys[r] = key;
    if (key >= 0) {
      atomicAdd(&h[key], 1);
      cnt += 1.f;
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += 1024) hist[(size_t)blockIdx.x * nbins + b] = h[b];
  const float n = wave_sum(cnt);
  if ((threadIdx.x & 63) == 0 && n > 0.f && nfit) atomicAdd(nfit, (double)n);
}

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int u = __shfl_up(v, off);
    v += lane >= off ? u : 0;
  }
  return v;
}

// Inclusive scan of two ints per thread over a 1024-thread block: wave scans (no
// barriers), then each wave adds the totals of the waves before it (one barrier).
__device__ __forceinline__ void block_scan2_1024(int& a, int& b, int2* wtot) {
  a = wave_incl_scan(a);
  b = wave_incl_scan(b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) wtot[w] = make_int2(a, b);
  __syncthreads();
  int pa = 0, pb = 0;
  for (int i = 0; i < w; ++i) {
    const int2 t = wtot[i];
    pa += t.x;
    pb += t.y;
  }
  a += pa;
  b += pb;
}

constexpr int kHtScanReg = 32;  // per-bin column of block counts held in registers

// One block of 1024 threads. hist[blk][bin] (counts) → bases; seg[bin] = (start, length);
// cstart[bin] = first segment-reduce chunk of the bin, cstart[nbins] = chunk count;
// ckey[chunk] = the bin (key) the chunk belongs to. With one bin per thread and
// nblk ≤ kHtScanReg the column is loaded once, all loads in flight together.
__global__ __launch_bounds__(1024) void ht_scan_kernel(int nblk, int nbins, int* __restrict__ hist,
                                                       int2* __restrict__ seg,
                                                       int* __restrict__ cstart,
                                                       int* __restrict__ ckey) {
  __shared__ int2 wtot[16];
  const int per = (nbins + 1023) / 1024;
  const int b0 = threadIdx.x * per, b1 = min(nbins, b0 + per);
  const bool reg = per == 1 && nblk <= kHtScanReg;
  int col[kHtScanReg];
  int tot = 0, ch = 0;
  if (reg) {
    const int bb = b0 < nbins ? b0 : 0;
#pragma unroll
    for (int k = 0; k < kHtScanReg; ++k)
      col[k] = hist[(size_t)(k < nblk ? k : 0) * nbins + bb];
    int run = 0;
#pragma unroll
    for (int k = 0; k < kHtScanReg; ++k) run += k < nblk ? col[k] : 0;
    if (b0 < nbins) {
      tot = run;
      ch = (run + kHtSegChunk - 1) / kHtSegChunk;
    }
  } else {
    for (int b = b0; b < b1; ++b) {
      int run = 0;
#pragma unroll 8
      for (int k = 0; k < nblk; ++k) run += hist[(size_t)k * nbins + b];
      seg[b] = make_int2(0, run);
      tot += run;
      ch += (run + kHtSegChunk - 1) / kHtSegChunk;
    }
  }
  int start = tot, cs = ch;
  block_scan2_1024(start, cs, wtot);
  start -= tot;
  cs -= ch;
  if (threadIdx.x == 1023) cstart[nbins] = cs + ch;
  if (reg) {
    if (b0 < nbins) {
      seg[b0] = make_int2(start, tot);
      cstart[b0] = cs;
      for (int c = 0; c < ch; ++c) ckey[cs + c] = b0;
      int run = start;
#pragma unroll
      for (int k = 0; k < kHtScanReg; ++k) {
        if (k < nblk) hist[(size_t)k * nbins + b0] = run;
        run += k < nblk ? col[k] : 0;
      }
    }
    return;
  }
  for (int b = b0; b < b1; ++b) {
    const int len = seg[b].y;
    const int nch = (len + kHtSegChunk - 1) / kHtSegChunk;
    seg[b] = make_int2(start, len);
    cstart[b] = cs;
    for (int c = 0; c < nch; ++c) ckey[cs + c] = b;
    cs += nch;
    int run = start;
    for (int k0 = 0; k0 < nblk; k0 += 8) {  // 8 loads in flight, then their 8 stores
      int c[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        c[u] = k0 + u < nblk ? hist[(size_t)(k0 + u) * nbins + b] : 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (k0 + u < nblk) hist[(size_t)(k0 + u) * nbins + b] = run;
        run += c[u];
      }
    }
    start += len;
  }
}

__global__ __launch_bounds__(1024) void ht_scatter_kernel(int B, int nbins,
                                                          const int* __restrict__ keys,
                                                          const int* __restrict__ hist,
                                                          int* __restrict__ sorted) {
  extern __shared__ int cur[];  // [nbins]
  for (int b = threadIdx.x; b < nbins; b += 1024) cur[b] = hist[(size_t)blockIdx.x * nbins + b];
  __syncthreads();
  const int r0 = blockIdx.x * kHtRowsPerBlock;
  for (int r = r0 + threadIdx.x; r < r0 + kHtRowsPerBlock && r < B; r += 1024) {
    const int key = keys[r];
    if (key >= 0) sorted[atomicAdd(&cur[key], 1)] = r;
  }
}

// One block per chunk of ≤ kHtSegChunk rows of one key (leaf·C + class), found by a
// binary search over the chunk starts; the chunk's per-feature totals are added to the
// leaf statistics with one atomic each (a key with a single chunk — the common case once
// the tree has grown — is the only writer of its statistics).
// DM > 0 (d ≤ DM): one pass over the chunk's rows with every feature's Σx, Σx², min, max in
// registers (a row's features are one contiguous run of x), then one wave reduction per
// statistic and a single barrier. DM == 0 (any d): one pass per feature.
template <int DM>
__global__ __launch_bounds__(256) void ht_segment_kernel(
    const float* __restrict__ x, int d, int C, int nbins, const int2* __restrict__ seg,
    const int* __restrict__ cstart, const int* __restrict__ ckey, const int* __restrict__ sorted,
    float* __restrict__ cc, float* __restrict__ S0, float* __restrict__ S1,
    float* __restrict__ S2, float* __restrict__ lo, float* __restrict__ hi,
    float* __restrict__ since) {
  const int chunk = blockIdx.x;
  const int nch = cstart[nbins];
  const int key = ckey[chunk];  // ckey has gridDim.x entries; stale beyond nch
  if (chunk >= nch) return;
  const int2 sg = seg[key];
  const int off = (chunk - cstart[key]) * kHtSegChunk;
  const int len = min(kHtSegChunk, sg.y - off);
  if (len <= 0) return;
  const int node = key / C, yc = key - node * C;
  const float cnt = (float)len;
  const int* rows = sorted + sg.x + off;
  const int w = threadIdx.x >> 6;
  auto publish = [&](int f, float t1, float t2, float tmn, float tmx) {
    const size_t o = ((size_t)node * d + f) * C + yc;
    atomicAdd(&S0[o], cnt);
    atomicAdd(&S1[o], t1);
    atomicAdd(&S2[o], t2);
    atomic_min_f(&lo[node * d + f], tmn);
    atomic_max_f(&hi[node * d + f], tmx);
  };
  if constexpr (DM > 0) {
    __shared__ float red[4][DM][4];
    float s1[DM], s2[DM], mn[DM], mx[DM];
#pragma unroll
    for (int f = 0; f < DM; ++f) {
      s1[f] = 0.f;
      s2[f] = 0.f;
      mn[f] = INFINITY;
      mx[f] = -INFINITY;
    }
    // RPT rows per thread per step: their ids, then all RPT·DM features, in flight together
    constexpr int RPT = DM <= 16 ? 4 : 2;
    for (int i0 = threadIdx.x; i0 < len; i0 += 256 * RPT) {
      int rid[RPT];
#pragma unroll
      for (int u = 0; u < RPT; ++u) rid[u] = rows[i0 + u * 256 < len ? i0 + u * 256 : i0];
      float v[RPT][DM];
#pragma unroll
      for (int u = 0; u < RPT; ++u) {
        const float* xr = x + (size_t)rid[u] * d;
#pragma unroll
        for (int f = 0; f < DM; ++f) v[u][f] = xr[f < d ? f : 0];
      }
#pragma unroll
      for (int u = 0; u < RPT; ++u) {
        if (i0 + u * 256 >= len) break;
#pragma unroll
        for (int f = 0; f < DM; ++f) {
          if (f < d) {
            s1[f] += v[u][f];
            s2[f] = fmaf(v[u][f], v[u][f], s2[f]);
            mn[f] = fminf(mn[f], v[u][f]);
            mx[f] = fmaxf(mx[f], v[u][f]);
          }
        }
      }
    }
#pragma unroll
    for (int f = 0; f < DM; ++f) {
      if (f < d) {
        wave_sum2(s1[f], s2[f]);
        const float tmn = -wave_max(-mn[f]), tmx = wave_max(mx[f]);
        if ((threadIdx.x & 63) == 0) {
          red[w][f][0] = s1[f];
          red[w][f][1] = s2[f];
          red[w][f][2] = tmn;
          red[w][f][3] = tmx;
        }
      }
    }
    __syncthreads();
    if (threadIdx.x < d) {
      const int f = threadIdx.x;
      publish(f, (red[0][f][0] + red[1][f][0]) + (red[2][f][0] + red[3][f][0]),
              (red[0][f][1] + red[1][f][1]) + (red[2][f][1] + red[3][f][1]),
              fminf(fminf(red[0][f][2], red[1][f][2]), fminf(red[2][f][2], red[3][f][2])),
              fmaxf(fmaxf(red[0][f][3], red[1][f][3]), fmaxf(red[2][f][3], red[3][f][3])));
    }
  } else {
    __shared__ float red[4][4];
    for (int f = 0; f < d; ++f) {
      float s1 = 0.f, s2 = 0.f, mn = INFINITY, mx = -INFINITY;
      for (int i = threadIdx.x; i < len; i += 256) {
        const float v = x[(size_t)rows[i] * d + f];
        s1 += v;
        s2 = fmaf(v, v, s2);
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
      }
      wave_sum2(s1, s2);
      mn = -wave_max(-mn);
      mx = wave_max(mx);
      if ((threadIdx.x & 63) == 0) {
        red[w][0] = s1;
        red[w][1] = s2;
        red[w][2] = mn;
        red[w][3] = mx;
      }
      __syncthreads();
      if (threadIdx.x == 0)
        publish(f, (red[0][0] + red[1][0]) + (red[2][0] + red[3][0]),
                (red[0][1] + red[1][1]) + (red[2][1] + red[3][1]),
                fminf(fminf(red[0][2], red[1][2]), fminf(red[2][2], red[3][2])),
                fmaxf(fmaxf(red[0][3], red[1][3]), fmaxf(red[2][3], red[3][3])));
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    atomicAdd(&cc[key], cnt);
    atomicAdd(&since[node], cnt);
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
  // best / second-best attribute: wave 0, one feature per lane (best bin = first maximum),
  // then a butterfly reduction of (top gain, its feature and bin, runner-up gain) that
  // keeps the lowest feature index on ties — the order a serial scan would give.
  if (threadIdx.x >= 64) return;
  float g1 = -2.f, g2 = -2.f;
  int f1 = 0x7fffffff, b1 = 0;
  for (int f = threadIdx.x; f < d; f += 64) {
    float gm = -2.f;
    int bm = 0;
#pragma unroll 4
    for (int b = 0; b < nb; ++b) {
      const float g = gains[f * nb + b];
      bm = g > gm ? b : bm;
      gm = g > gm ? g : gm;
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
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const float og1 = __shfl_xor(g1, m), og2 = __shfl_xor(g2, m);
    const int of1 = __shfl_xor(f1, m), ob1 = __shfl_xor(b1, m);
    const bool take = og1 > g1 || (og1 == g1 && of1 < f1);
    g2 = take ? fmaxf(g1, og2) : fmaxf(g2, og1);
    g1 = take ? og1 : g1;
    f1 = take ? of1 : f1;
    b1 = take ? ob1 : b1;
  }
  if (threadIdx.x != 0) return;
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

// The leaf of every row (exact per-point checks: models/dense.py HT._fit_exact).
__global__ __launch_bounds__(256) void ht_route_kernel(
    const float* __restrict__ x, int B, int d, int depth, const float* __restrict__ feat,
    const float* __restrict__ thr, const float* __restrict__ left, const float* __restrict__ right,
    int* __restrict__ out) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= B) return;
  out[row] = ht_route(x + (size_t)row * d, feat, thr, left, right, depth);
}

// ---- exact per-point VFDT in one persistent launch (models/dense.py HT._fit_exact) -------
// The reference learner checks a leaf at the very point it reaches gracePeriod points since
// its last check (FlinkSpoke.scala:92-107: one point at a time). Between two such due points
// every row's update is an order-free sum into its leaf, so one workgroup of 256 threads
// walks the tick in chunks of 256 rows (one per thread):
//  * the chunk's rows are routed through the LDS copy of the tree;
//  * each row's rank among the chunk's training rows of its leaf, in stream order (per-wave
//    ballots, then a per-leaf prefix over the 4 waves);
//  * the first due row = the lowest row whose rank since the segment start reaches its
//    leaf's remaining grace (a ballot + one LDS atomic min);
//  * the segment [start, due row] is added to the leaves' statistics — held in LDS for the
//    whole launch (class counts, per-(feature, class) moments, ranges), LDS atomics per
//    row — then the due leaf is checked by the whole workgroup (nBins candidate thresholds
//    per feature, Hoeffding test) and, on a split, the chunk restarts after the due row
//    under the new tree.
// No host round trip per segment (the host loop it replaces did ~650 segments per
// 131072-row tick, each with .item() syncs) and no global atomics (a first form with L2
// atomics spent ~45 K cycles per segment on them). S0 is the same for every feature (each
// training row adds 1 to all of them), so the launch keeps it per (node, class) and writes
// the per-feature copies back at its end. Σx / Σx² stay in global memory (L2 atomics) when
// the tree is too large for the LDS (S12 = false).
constexpr int kHxNT = 256;  // threads = rows per chunk
constexpr int kHxNW = kHxNT / 64;

struct HxTree {
  float *feat, *thr, *left, *right, *cc, *S0, *S1, *S2, *lo, *hi, *since, *nnodes;
};

__device__ __forceinline__ float ld_l2(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS layout. Per node: tn (int4: feature, threshold, left, right), since, consumed, slot
// (node → leaf slot, -1: not a leaf), cntw[NW] (u8 per-wave counts). Per leaf slot (a tree
// of N nodes has ≤ (N + 1) / 2 leaves; a split hands its slot to the left child after
// writing the parent's statistics back): node, cc[C], S0[C], lo[d], hi[d] and, with S12,
// Σx[d·C], Σx²[d·C]. Then gains[d·nb] and the chunk's rows xs[NT][d].
struct HxLayout {
  size_t tn, since, consumed, slot, cntw, snode, cc, s0, lo, hi, s1, s2, gains, xs, lmask, bytes;
  int NS;
};

__host__ __device__ inline HxLayout ht_exact_layout(int N, int d, int C, int nb, bool s12) {
  HxLayout L{};
  L.NS = (N + 1) / 2 + 1;
  size_t o = 0;
  auto put = [&](size_t n) {
    const size_t at = o;
    o += (n + 15) & ~(size_t)15;
    return at;
  };
  const size_t ns = (size_t)L.NS;
  L.tn = put((size_t)N * 16);
  L.since = put((size_t)N * 4);
  L.consumed = put((size_t)N * 4);
  L.slot = put((size_t)N * 4);
  L.cntw = put((size_t)kHxNW * N);
  L.snode = put(ns * 4);
  L.cc = put(ns * C * 4);
  L.s0 = put(ns * C * 4);
  L.lo = put(ns * d * 4);
  L.hi = put(ns * d * 4);
  L.s1 = s12 ? put(ns * d * C * 4) : 0;
  L.s2 = s12 ? put(ns * d * C * 4) : 0;
  L.gains = put((size_t)d * nb * 4);
  L.xs = put((size_t)kHxNT * d * 4);
  L.lmask = put((size_t)kHxNW * ns * 8);
  L.bytes = o;
  return L;
}

__device__ __forceinline__ void lds_min_f(float* a, float v) {  // (range: sign-split ints)
  if (v >= 0.f)
    atomicMin(reinterpret_cast<int*>(a), __float_as_int(v));
  else
    atomicMax(reinterpret_cast<unsigned int*>(a), __float_as_uint(v));
}
__device__ __forceinline__ void lds_max_f(float* a, float v) {
  if (v >= 0.f)
    atomicMax(reinterpret_cast<int*>(a), __float_as_int(v));
  else
    atomicMin(reinterpret_cast<unsigned int*>(a), __float_as_uint(v));
}

template <bool S12>
__global__ __launch_bounds__(kHxNT) void ht_exact_kernel(
    const float* __restrict__ x, const float* __restrict__ yv, int B, int d, int C, int depth,
    int N, int nb, float grace, float delta, float tau, HxTree T, double* __restrict__ nfit,
    unsigned long long* __restrict__ dbg, int rank_masks) {
  // dbg (diagnostics, may be null): [0] chunks, [1] segments, [2] splits, [3..6] cycles in
  // chunk setup / due search / statistics / split checks (wave 0's clock)
  unsigned long long t_setup = 0, t_due = 0, t_stat = 0, t_split = 0, n_chunk = 0, n_seg = 0,
                     n_split = 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char hx_smem[];
  const HxLayout Ly = ht_exact_layout(N, d, C, nb, S12);
  int4* tn = reinterpret_cast<int4*>(hx_smem + Ly.tn);
  float* since_l = reinterpret_cast<float*>(hx_smem + Ly.since);
  int* consumed = reinterpret_cast<int*>(hx_smem + Ly.consumed);
  int* slot = reinterpret_cast<int*>(hx_smem + Ly.slot);
  unsigned char* cntw = hx_smem + Ly.cntw;
  int* snode = reinterpret_cast<int*>(hx_smem + Ly.snode);
  float* ccl = reinterpret_cast<float*>(hx_smem + Ly.cc);
  float* s0l = reinterpret_cast<float*>(hx_smem + Ly.s0);
  float* lol = reinterpret_cast<float*>(hx_smem + Ly.lo);
  float* hil = reinterpret_cast<float*>(hx_smem + Ly.hi);
  float* s1 = reinterpret_cast<float*>(hx_smem + Ly.s1);
  float* s2 = reinterpret_cast<float*>(hx_smem + Ly.s2);
  float* gains = reinterpret_cast<float*>(hx_smem + Ly.gains);
  float* xs = reinterpret_cast<float*>(hx_smem + Ly.xs);
  // per wave and leaf slot: the lanes of the chunk's rows at that leaf (zero between uses)
  unsigned long long* lmask = reinterpret_cast<unsigned long long*>(hx_smem + Ly.lmask);
  const int NS = Ly.NS;
  __shared__ int s_first, s_leaf, s_flag, s_nn, s_nslot;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // Σx / Σx² of slot k, feature f, class c: LDS (S12) or the node's global rows
  auto s1p = [&](int k, int f, int c) -> float* {
    return S12 ? s1 + ((size_t)k * d + f) * C + c : T.S1 + ((size_t)snode[k] * d + f) * C + c;
  };
  auto s2p = [&](int k, int f, int c) -> float* {
    return S12 ? s2 + ((size_t)k * d + f) * C + c : T.S2 + ((size_t)snode[k] * d + f) * C + c;
  };
  // the leaves get slots (thread 0, node order)
  if (tid == 0) {
    s_nn = (int)T.nnodes[0];
    int k = 0;
    for (int n = 0; n < N; ++n) {
      const bool leaf = n < s_nn && T.feat[n] < 0.f && k < NS;
      slot[n] = leaf ? k : -1;
      if (leaf) snode[k++] = n;
    }
    s_nslot = k;
  }
  for (int i = tid; i < kHxNW * NS; i += kHxNT) lmask[i] = 0ull;
  for (int n = tid; n < N; n += kHxNT) {
    tn[n] = make_int4((int)T.feat[n], __float_as_int(T.thr[n]), (int)T.left[n], (int)T.right[n]);
    since_l[n] = T.since[n];
  }
  __syncthreads();
  const int nslot0 = s_nslot;
  for (int i = tid; i < nslot0 * C; i += kHxNT) {
    const int k = i / C, c = i % C, n = snode[k];
    ccl[i] = T.cc[(size_t)n * C + c];
    s0l[i] = T.S0[(size_t)n * d * C + c];  // (feature 0: every feature's count)
  }
  for (int i = tid; i < nslot0 * d; i += kHxNT) {
    const int k = i / d, f = i % d, n = snode[k];
    lol[i] = T.lo[(size_t)n * d + f];
    hil[i] = T.hi[(size_t)n * d + f];
  }
  if constexpr (S12)
    for (int i = tid; i < nslot0 * d * C; i += kHxNT) {
      const int k = i / (d * C), r = i % (d * C), n = snode[k];
      s1[i] = T.S1[(size_t)n * d * C + r];
      s2[i] = T.S2[(size_t)n * d * C + r];
    }
  __syncthreads();
  float myfit = 0.f;
  int c0 = 0;
  while (c0 < B) {  // (uniform)
    unsigned long long tc = __builtin_amdgcn_s_memtime();
    ++n_chunk;
    const int r = c0 + tid;
    const bool inb = r < B;
    const float yr = inb ? yv[r] : 0.f;
    const bool valid = inb && !__builtin_isnan(yr);
    int yi = valid ? (int)yr : 0;
    yi = yi < 0 ? 0 : (yi >= C ? C - 1 : yi);
    const int cend = min(c0 + kHxNT, B);  // exclusive
    // the chunk's rows into LDS: one coalesced block, every load in flight before the
    // stores (a load → store loop waited out one memory latency per element), then
    // routing reads LDS
    {
      const int ne = (cend - c0) * d;
      const float* src = x + (size_t)c0 * d;
      for (int e0 = 0; e0 < ne; e0 += 16 * kHxNT) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int e = e0 + u * kHxNT + tid;
          v[u] = src[e < ne ? e : 0];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int e = e0 + u * kHxNT + tid;
          if (e < ne) xs[e] = v[u];
        }
      }
    }
    for (int e = tid; e < kHxNW * N; e += kHxNT) cntw[e] = 0;
    for (int n = tid; n < N; n += kHxNT) consumed[n] = 0;
    __syncthreads();
    const float* xr = xs + (size_t)tid * d;
    int leaf = 0;
    if (inb) {
      for (int it = 0; it <= depth; ++it) {
        const int4 t = tn[leaf];
        if (t.x < 0) break;
        leaf = xr[t.x] <= __int_as_float(t.y) ? t.z : t.w;
      }
    }
    // the row's rank among the chunk's training rows of its leaf (stream order)
    int rank = 0;
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int ks = valid ? slot[leaf] : 0;
    if (rank_masks && !__ballot(valid && ks < 0)) {
      // every row's leaf has a slot: each row ORs its lane bit into its (wave, slot) mask,
      // reads the mask back (one wave's LDS instructions complete in order, so the read sees
      // every lane's OR) — rank = lanes below at the same leaf, count = all of them — and the
      // leaf's first lane publishes the count and clears the mask for the next chunk. O(1)
      // per row instead of one pass per distinct leaf of the wave.
      unsigned long long* lm = lmask + (size_t)w * NS + ks;
      if (valid) atomicOr(lm, 1ull << lane);
      const unsigned long long m = valid ? *lm : 0ull;
      if (valid) {
        rank = __popcll(m & below);
        if (rank == 0) {
          cntw[w * N + leaf] = (unsigned char)__popcll(m);
          *lm = 0ull;
        }
      }
    } else {
      unsigned long long pending = __ballot(valid);
      while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const int L = __shfl(leaf, leader);
        const unsigned long long m = __ballot(valid && leaf == L);
        pending &= ~m;
        if (valid && leaf == L) rank = __popcll(m & below);
        if (lane == leader) cntw[w * N + L] = (unsigned char)__popcll(m);
      }
    }
    __syncthreads();
    if (valid)
      for (int w2 = 0; w2 < w; ++w2) rank += cntw[w2 * N + leaf];
    int base = c0;
    bool restart = false;
    t_setup += __builtin_amdgcn_s_memtime() - tc;
    while (true) {
      tc = __builtin_amdgcn_s_memtime();
      ++n_seg;
      bool due = false;
      if (valid && r >= base) {
        const float rem = ceilf(grace - since_l[leaf]);
        const int need = rem < 1.f ? 1 : (int)rem;
        due = rank - consumed[leaf] + 1 == need;
      }
      if (tid == 0) s_first = 0x7fffffff;
      __syncthreads();
      const unsigned long long dm = __ballot(due);
      if (dm && lane == 0) atomicMin(&s_first, c0 + w * 64 + __ffsll((long long)dm) - 1);
      __syncthreads();
      const int first = s_first;
      const int last = first == 0x7fffffff ? cend - 1 : first;  // inclusive
      const bool seg = valid && r >= base && r <= last;
      if (r == first) s_leaf = leaf;
      t_due += __builtin_amdgcn_s_memtime() - tc;
      tc = __builtin_amdgcn_s_memtime();
      // the segment's rows into their leaves' statistics (LDS atomics, one row per thread)
      if (seg) {
        myfit += 1.f;
        const int k = slot[leaf];
        if (k >= 0) {
          atomicAdd(&ccl[k * C + yi], 1.f);
          atomicAdd(&s0l[k * C + yi], 1.f);
          // the row's features first (one wait), then fire-and-forget LDS atomics: float
          // add for the moments, float min / max for the range (no waits, no branches)
          auto put = [&](int f, float v) {
            atomicAdd(s1p(k, f, yi), v);
            atomicAdd(s2p(k, f, yi), v * v);
            __hip_atomic_fetch_min(&lol[k * d + f], v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_max(&hil[k * d + f], v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
          };
          if (d <= 32) {
            float v[32];
#pragma unroll
            for (int f = 0; f < 32; ++f) v[f] = f < d ? xr[f] : 0.f;
#pragma unroll
            for (int f = 0; f < 32; ++f)
              if (f < d) put(f, v[f]);
          } else {
            for (int f = 0; f < d; ++f) put(f, xr[f]);
          }
        }
        atomicAdd(&since_l[leaf], 1.f);
        atomicAdd(&consumed[leaf], 1);
      }
      if constexpr (!S12) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (L2 atomics)
      __syncthreads();
      t_stat += __builtin_amdgcn_s_memtime() - tc;
      if (first == 0x7fffffff) break;
      tc = __builtin_amdgcn_s_memtime();
      // the due leaf's split check (ht_split_kernel's criterion, by the whole workgroup)
      const int L = s_leaf, kL = slot[L];
      bool split = false;
      float ntot = 0.f;
      int nz = 0;
      if (kL >= 0)
        for (int c = 0; c < C; ++c) {
          ntot += ccl[kL * C + c];
          nz += ccl[kL * C + c] > 0.f;
        }
      if (kL >= 0 && !(ntot < 2.f || nz < 2 || s_nn + 2 > N)) {
        const float h0 = entropy(ccl + (size_t)kL * C, C, ntot);
        float lm[kHtMaxC], rm[kHtMaxC];
        auto mass = [&](int f, float t) {  // class mass left / right of t (Gaussian CDFs)
          for (int c = 0; c < C; ++c) {
            const float n = s0l[kL * C + c];
            const float nn = fmaxf(n, 1.f);
            // (global Σ rows written by L2 atomics: agent-scope loads, no stale L1 lines)
            const float m1 = S12 ? *s1p(kL, f, c) : ld_l2(s1p(kL, f, c));
            const float m2 = S12 ? *s2p(kL, f, c) : ld_l2(s2p(kL, f, c));
            const float mu = m1 / nn;
            const float var = fmaxf(m2 / nn - mu * mu, 1e-6f);
            const float z = (t - mu) * rsqrtf(var);
            const float cdf = 0.5f * (1.f + erff(z * 0.70710678f));
            lm[c] = n * cdf;
            rm[c] = n - lm[c];
          }
        };
        for (int p2 = tid; p2 < d * nb; p2 += kHxNT) {
          const int f = p2 / nb, b = p2 - f * nb;
          const float l = lol[kL * d + f], span = hil[kL * d + f] - l;
          float g = -1.f;
          if (span > 0.f) {
            mass(f, l + span * (float)(b + 1) / (float)(nb + 1));
            float nl = 0.f, nr = 0.f;
            for (int c = 0; c < C; ++c) {
              nl += lm[c];
              nr += rm[c];
            }
            g = h0 - (nl * entropy(lm, C, nl) + nr * entropy(rm, C, nr)) / fmaxf(nl + nr, 1e-12f);
          }
          gains[p2] = g;
        }
        __syncthreads();
        if (w == 0) {
          float g1 = -2.f, g2 = -2.f;
          int f1 = 0x7fffffff, b1 = 0;
          for (int f = lane; f < d; f += 64) {
            float gm = -2.f;
            int bm = 0;
            if (nb <= 16) {  // every read in flight before the first compare
              float gv[16];
#pragma unroll
              for (int b = 0; b < 16; ++b) gv[b] = b < nb ? gains[f * nb + b] : -2.f;
#pragma unroll
              for (int b = 0; b < 16; ++b) {
                bm = gv[b] > gm ? b : bm;
                gm = gv[b] > gm ? gv[b] : gm;
              }
            } else {
              for (int b = 0; b < nb; ++b) {
                const float g = gains[f * nb + b];
                bm = g > gm ? b : bm;
                gm = g > gm ? g : gm;
              }
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
          // lanes ≥ d hold no candidate: the butterfly spans the next power of two ≥ d
          const int span = d >= 64 ? 64 : (d <= 1 ? 1 : 1 << (32 - __builtin_clz(d - 1)));
          for (int m = 1; m < span; m <<= 1) {
            const float og1 = __shfl_xor(g1, m), og2 = __shfl_xor(g2, m);
            const int of1 = __shfl_xor(f1, m), ob1 = __shfl_xor(b1, m);
            const bool take = og1 > g1 || (og1 == g1 && of1 < f1);
            g2 = take ? fmaxf(g1, og2) : fmaxf(g2, og1);
            g1 = take ? og1 : g1;
            f1 = take ? of1 : f1;
            b1 = take ? ob1 : b1;
          }
          int flag = 0;
          if (lane == 0) {
            if (d == 1) g2 = 0.f;
            const float R = __log2f((float)C);
            const float eps = sqrtf(R * R * logf(1.f / delta) / (2.f * ntot));
            if (g1 > 0.f && (g1 - g2 > eps || eps < tau) && s_nslot < NS) {
              const int old = s_nn;
              const float l = lol[kL * d + f1], span = hil[kL * d + f1] - l;
              const float t = l + span * (float)(b1 + 1) / (float)(nb + 1);
              mass(f1, t);
              T.thr[L] = t;
              T.left[L] = (float)old;
              T.right[L] = (float)(old + 1);
              T.feat[L] = (float)f1;
              T.nnodes[0] = (float)(old + 2);
              tn[L] = make_int4(f1, __float_as_int(t), old, old + 1);
              s_nn = old + 2;
              flag = 1;
            }
          }
          flag = __shfl(flag, 0);
          if (flag) {
            // the parent's statistics back to its node rows (it is no leaf any more), then
            // its slot to the left child and a fresh slot to the right one
            const int n = L;
            for (int i = lane; i < C; i += 64) {
              T.cc[(size_t)n * C + i] = ccl[kL * C + i];
              for (int f = 0; f < d; ++f) T.S0[((size_t)n * d + f) * C + i] = s0l[kL * C + i];
            }
            for (int i = lane; i < d; i += 64) {
              T.lo[(size_t)n * d + i] = lol[kL * d + i];
              T.hi[(size_t)n * d + i] = hil[kL * d + i];
            }
            if constexpr (S12)
              for (int i = lane; i < d * C; i += 64) {
                T.S1[(size_t)n * d * C + i] = s1[(size_t)kL * d * C + i];
                T.S2[(size_t)n * d * C + i] = s2[(size_t)kL * d * C + i];
              }
            const int old = s_nn - 2, kR = s_nslot;
            // (S12 false: the children's global Σ rows start at zero in the model state)
            if (lane == 0) {
              slot[L] = -1;
              slot[old] = kL;
              slot[old + 1] = kR;
              snode[kL] = old;
              snode[kR] = old + 1;
              s_nslot = kR + 1;
              for (int c = 0; c < C; ++c) {  // children start with the split class mass
                ccl[kL * C + c] = lm[c];
                ccl[kR * C + c] = rm[c];
              }
            }
            for (int i = lane; i < C; i += 64) {
              s0l[kL * C + i] = 0.f;
              s0l[kR * C + i] = 0.f;
            }
            for (int i = lane; i < d; i += 64) {
              lol[kL * d + i] = INFINITY;
              hil[kL * d + i] = -INFINITY;
              lol[kR * d + i] = INFINITY;
              hil[kR * d + i] = -INFINITY;
            }
            if constexpr (S12)
              for (int i = lane; i < d * C; i += 64) {
                s1[(size_t)kL * d * C + i] = 0.f;
                s2[(size_t)kL * d * C + i] = 0.f;
                s1[(size_t)kR * d * C + i] = 0.f;
                s2[(size_t)kR * d * C + i] = 0.f;
              }
          }
          if (lane == 0) s_flag = flag;
        }
        __syncthreads();
        split = s_flag != 0;
      }
      if (tid == 0) since_l[L] = 0.f;  // (checked: the grace count restarts)
      __syncthreads();
      t_split += __builtin_amdgcn_s_memtime() - tc;
      n_split += split;
      base = first + 1;
      if (split) {  // the rest of the chunk under the new tree
        c0 = first + 1;
        restart = true;
        break;
      }
    }
    if (!restart) c0 = cend;
  }
  // the leaves' statistics back to their nodes' rows
  const int nsl = s_nslot;
  for (int n = tid; n < N; n += kHxNT) T.since[n] = since_l[n];
  for (int i = tid; i < nsl * C; i += kHxNT) {
    const int k = i / C, c = i % C, n = snode[k];
    T.cc[(size_t)n * C + c] = ccl[i];
  }
  for (int i = tid; i < nsl * d * C; i += kHxNT) {
    const int k = i / (d * C), rr = i % (d * C), n = snode[k];
    T.S0[(size_t)n * d * C + rr] = s0l[k * C + rr % C];
    if constexpr (S12) {
      T.S1[(size_t)n * d * C + rr] = s1[i];
      T.S2[(size_t)n * d * C + rr] = s2[i];
    }
  }
  for (int i = tid; i < nsl * d; i += kHxNT) {
    const int k = i / d, f = i % d, n = snode[k];
    T.lo[(size_t)n * d + f] = lol[i];
    T.hi[(size_t)n * d + f] = hil[i];
  }
  if (dbg && tid == 0) {
    dbg[0] += n_chunk;
    dbg[1] += n_seg;
    dbg[2] += n_split;
    dbg[3] += t_setup;
    dbg[4] += t_due;
    dbg[5] += t_stat;
    dbg[6] += t_split;
  }
  const float f = wave_sum(myfit);
  if (lane == 0 && nfit && f > 0.f) atomicAdd(nfit, (double)f);
}

}  // namespace omldm

using namespace omldm;

OMLDM_API int omldm_ht_route(const float* x, int B, int d, int depth, float* const* tree, int* out,
                             void* stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(ht_route_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, x,
                     B, d, depth, tree[0], tree[1], tree[2], tree[3], out);
  return (int)hipGetLastError();
}

// tree: pointers in the order feat, thr, left, right, cc, S0, S1, S2, lo, hi, since, nnodes.
// N: node capacity. ws: int scratch of omldm_ht_update_ws_ints(B, N, C) (0 → the wave-
// aggregated atomic kernel, kept as the fallback / A-B reference).
OMLDM_API long long omldm_ht_update_ws_ints(int B, int N, int C) {
  const long long nblk = (B + kHtRowsPerBlock - 1) / kHtRowsPerBlock;
  const long long nchunk = (long long)N * C + (B + kHtSegChunk - 1) / kHtSegChunk;
  return 2LL * B + ((nblk * N * C + 1) & ~1LL) + 2LL * N * C + (N * C + 2) + nchunk;
}

OMLDM_API int omldm_ht_update(const float* x, const float* y, int B, int d, int C, int depth,
                              int N, float* const* tree, double* nfit, int* ws, void* stream) {
  if (B <= 0) return 0;
  if (C < 1 || C > kHtMaxC) return -1;
  hipStream_t st = (hipStream_t)stream;
  if (!ws) {
    hipLaunchKernelGGL(ht_update_kernel, dim3((B + 255) / 256), dim3(256), 0, st, x, y, B, d, C,
                       depth, tree[0], tree[1], tree[2], tree[3], tree[4], tree[5], tree[6],
                       tree[7], tree[8], tree[9], tree[10], nfit);
    return (int)hipGetLastError();
  }
  const int nbins = N * C;
  if ((size_t)nbins * 4 > 64 * 1024) return -2;
  const int nblk = (B + kHtRowsPerBlock - 1) / kHtRowsPerBlock;
  int* keys = ws;
  int* sorted = ws + B;
  int* hist = ws + 2 * (size_t)B;
  int2* seg = reinterpret_cast<int2*>(hist + (((size_t)nblk * nbins + 1) & ~(size_t)1));
  int* cstart = reinterpret_cast<int*>(seg + nbins);  // [nbins + 1]
  // chunk count ≤ nbins + B / kHtSegChunk; surplus blocks exit on cstart[nbins]
  const int nchunk = nbins + (B + kHtSegChunk - 1) / kHtSegChunk;
  int* ckey = cstart + nbins + 2;  // [nchunk]
  const size_t lds = (size_t)nbins * 4;
  // tree staged in LDS next to the histogram when both fit in 64 KB
  const size_t lds_tree = (size_t)((nbins + 3) & ~3) * 4 + (size_t)N * 16;
  const int nstage = lds_tree <= 64 * 1024 ? N : 0;
  const size_t lds_route = nstage ? lds_tree : lds;
  int e = check_dyn_lds((const void*)ht_route_hist_kernel, lds_route);
  if (!e) e = check_dyn_lds((const void*)ht_scatter_kernel, lds);
  if (e) return e;
  hipLaunchKernelGGL(ht_route_hist_kernel, dim3(nblk), dim3(1024), lds_route, st, x, y, B, d, C,
                     depth, tree[0], tree[1], tree[2], tree[3], nbins, nstage, keys, hist, nfit);
  hipLaunchKernelGGL(ht_scan_kernel, dim3(1), dim3(1024), 0, st, nblk, nbins, hist, seg, cstart,
                     ckey);
  hipLaunchKernelGGL(ht_scatter_kernel, dim3(nblk), dim3(1024), lds, st, B, nbins, keys, hist,
                     sorted);
#define OMLDM_HT_SEG(DM)                                                                      \
  hipLaunchKernelGGL(ht_segment_kernel<DM>, dim3(nchunk), dim3(256), 0, st, x, d, C, nbins, seg, \
                     cstart, ckey, sorted, tree[4], tree[5], tree[6], tree[7], tree[8], tree[9],       \
                     tree[10])
  if (d <= 8) OMLDM_HT_SEG(8);
  else if (d <= 16) OMLDM_HT_SEG(16);
  else if (d <= 32) OMLDM_HT_SEG(32);
  else OMLDM_HT_SEG(0);
#undef OMLDM_HT_SEG
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

// The exact per-point VFDT over a tick in one launch (x [B, d] contiguous fp32, y [B]:
// NaN = not a training point). -2: the LDS layout does not fit (the host falls back).
OMLDM_API int omldm_ht_exact(const float* x, const float* y, int B, int d, int C, int depth,
                             int N, int nb, float grace, float delta, float tau,
                             float* const* tree, double* nfit, unsigned long long* dbg,
                             void* stream) {
  if (B <= 0) return 0;
  if (C < 1 || C > kHtMaxC || nb < 1 || d < 1) return -1;
  constexpr size_t kMax = 160 * 1024 - 256;
  const bool s12 = ht_exact_layout(N, d, C, nb, true).bytes <= kMax;
  const size_t lds = ht_exact_layout(N, d, C, nb, s12).bytes;
  if (lds > kMax) return -2;
  const void* fn = s12 ? (const void*)ht_exact_kernel<true> : (const void*)ht_exact_kernel<false>;
  static int rank_masks = -1;  // OMLDM_HT_RANK=0: the per-leaf ballot loop (the A/B)
  if (rank_masks < 0) {
    const char* ev = getenv("OMLDM_HT_RANK");
    rank_masks = (ev && ev[0] == '0') ? 0 : 1;
  }
  const int e = check_dyn_lds(fn, lds);
  if (e) return e;
  HxTree T{tree[0], tree[1], tree[2], tree[3], tree[4], tree[5],
           tree[6], tree[7], tree[8], tree[9], tree[10], tree[11]};
  if (s12)
    hipLaunchKernelGGL(ht_exact_kernel<true>, dim3(1), dim3(kHxNT), lds, (hipStream_t)stream, x,
                       y, B, d, C, depth, N, nb, grace, delta, tau, T, nfit, dbg, rank_masks);
  else
    hipLaunchKernelGGL(ht_exact_kernel<false>, dim3(1), dim3(kHxNT), lds, (hipStream_t)stream, x,
                       y, B, d, C, depth, N, nb, grace, delta, tau, T, nfit, dbg, rank_masks);
  return (int)hipGetLastError();
}
