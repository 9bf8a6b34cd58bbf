// Streaming preprocessors on the dense feature block of a micro-batch:
// StandardScaler (running moments, Chan merge), MinMaxScaler (running extrema),
// PolynomialFeatures (monomial expansion). Reference: the three preprocessor names the
// request validator accepts (omldm/utils/parsers/requestStream/PipelineMap.scala:67).
//
// x is row-major [B, d] (d ≤ a few hundred, B up to ~10^6). Column moments are taken
// with a shifted single pass (shift = running mean, so the f32 sums do not cancel) on
// 256-thread blocks that each own a slab of rows and accumulate per-column partials in
// LDS (ds_add_f32), then one block per column merges the slab partials into the
// running f64 state — no host round trip, no same-address global atomics.
#include "common.h"

namespace omldm {

constexpr int kPPThreads = 256;

// partial[blk][c][0..3] = Σ(x−shift), Σ(x−shift)², min, max over the block's rows.
__global__ __launch_bounds__(kPPThreads) void colmoments_kernel(
    const float* __restrict__ x, int B, int d, const double* __restrict__ shift,
    int rows_per_block, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* s1 = reinterpret_cast<float*>(smem);
  float* s2 = s1 + d;
  int* mn = reinterpret_cast<int*>(s2 + d);  // order-preserving int encoding of floats
  int* mx = mn + d;
  for (int c = threadIdx.x; c < d; c += kPPThreads) {
    s1[c] = 0.f;
    s2[c] = 0.f;
    mn[c] = 0x7fffffff;
    mx[c] = (int)0x80000000;
  }
  __syncthreads();
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min((long long)B, r0 + rows_per_block);
  const long long n = (r1 - r0) * d;
  const float* base = x + r0 * d;
  for (long long e = threadIdx.x; e < n; e += kPPThreads) {
    const int c = (int)(e % d);
    const float v = base[e];
    const float z = shift ? v - (float)shift[c] : v;  // extrema-only mode passes no shift
    atomicAdd(&s1[c], z);
    atomicAdd(&s2[c], z * z);
    const int iv = __float_as_int(v);
    const int key = iv >= 0 ? iv : (iv ^ 0x7fffffff);  // monotone in v
    atomicMin(&mn[c], key);
    atomicMax(&mx[c], key);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += kPPThreads) {
    float* o = partial + ((size_t)blockIdx.x * d + c) * 4;
    o[0] = s1[c];
    o[1] = s2[c];
    const int a = mn[c], b = mx[c];
    o[2] = __int_as_float(a >= 0 ? a : (a ^ 0x7fffffff));
    o[3] = __int_as_float(b >= 0 ? b : (b ^ 0x7fffffff));
  }
}

// One block per column: reduce the slab partials, then merge into the running state.
// mode bit0: update mean/M2 (Chan), bit1: update min/max.
__global__ __launch_bounds__(kPPThreads) void colmoments_merge_kernel(
    const float* __restrict__ partial, int nblk, int d, int B, double count,
    double* __restrict__ mean, double* __restrict__ m2, const double* __restrict__ shift,
    float* __restrict__ lo, float* __restrict__ hi, int mode) {
  __shared__ double r1[kPPThreads], r2[kPPThreads];
  __shared__ float rmn[kPPThreads], rmx[kPPThreads];
  const int c = blockIdx.x;
  double a1 = 0.0, a2 = 0.0;
  float amn = INFINITY, amx = -INFINITY;
  for (int b = threadIdx.x; b < nblk; b += kPPThreads) {
    const float* o = partial + ((size_t)b * d + c) * 4;
    a1 += o[0];
    a2 += o[1];
    amn = fminf(amn, o[2]);
    amx = fmaxf(amx, o[3]);
  }
  r1[threadIdx.x] = a1;
  r2[threadIdx.x] = a2;
  rmn[threadIdx.x] = amn;
  rmx[threadIdx.x] = amx;
  __syncthreads();
  for (int s = kPPThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      r1[threadIdx.x] += r1[threadIdx.x + s];
      r2[threadIdx.x] += r2[threadIdx.x + s];
      rmn[threadIdx.x] = fminf(rmn[threadIdx.x], rmn[threadIdx.x + s]);
      rmx[threadIdx.x] = fmaxf(rmx[threadIdx.x], rmx[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && B > 0) {
    if (mode & 1) {
      const double nb = (double)B;
      const double mb = shift[c] + r1[0] / nb;
      double m2b = r2[0] - r1[0] * r1[0] / nb;
      if (m2b < 0.0) m2b = 0.0;
      const double tot = count + nb;
      const double delta = mb - mean[c];
      mean[c] += delta * nb / tot;
      m2[c] += m2b + delta * delta * count * nb / tot;
    }
    if (mode & 2) {
      lo[c] = fminf(lo[c], rmn[0]);
      hi[c] = fmaxf(hi[c], rmx[0]);
    }
  }
}

// y = (x − μ)/σ (σ = sqrt(M2/N), 1 where 0) or (x − lo)/(hi − lo) (range 0 → 0).
__global__ __launch_bounds__(kPPThreads) void scale_kernel(
    const float* __restrict__ x, float* __restrict__ y, long long n, int d, int mode,
    const double* __restrict__ mean, const double* __restrict__ m2, double count,
    const float* __restrict__ lo, const float* __restrict__ hi) {
  for (long long e = (long long)blockIdx.x * kPPThreads + threadIdx.x; e < n;
       e += (long long)gridDim.x * kPPThreads) {
    const int c = (int)(e % d);
    const float v = x[e];
    float r;
    if (mode == 0) {
      const double var = count > 0.0 ? m2[c] / count : 0.0;
      const float sd = var > 0.0 ? (float)sqrt(var) : 1.f;
      r = (v - (float)mean[c]) / sd;
    } else {
      const float rg = hi[c] - lo[c];
      r = rg > 0.f ? (v - lo[c]) / rg : 0.f;
    }
    y[e] = r;
  }
}

// out[b] = [x[b, 0:d], Π_k x[b, idx[r][k]] for r in combos] ; idx −1 = no factor.
__global__ __launch_bounds__(kPPThreads) void poly_kernel(const float* __restrict__ x, int B, int d,
                                                          const int* __restrict__ idx, int ncomb,
                                                          int deg, float* __restrict__ out) {
  const int dout = d + ncomb;
  const long long n = (long long)B * dout;
  for (long long e = (long long)blockIdx.x * kPPThreads + threadIdx.x; e < n;
       e += (long long)gridDim.x * kPPThreads) {
    const long long b = e / dout;
    const int j = (int)(e - b * dout);
    const float* xr = x + b * d;
    float v;
    if (j < d) {
      v = xr[j];
    } else {
      const int* ir = idx + (size_t)(j - d) * deg;
      v = 1.f;
      for (int k = 0; k < deg; ++k)
        if (ir[k] >= 0) v *= xr[ir[k]];
    }
    out[e] = v;
  }
}

}  // namespace omldm

using namespace omldm;

static int grid_for(long long n) {
  long long g = (n + kPPThreads - 1) / kPPThreads;
  if (g > 4096) g = 4096;
  return g < 1 ? 1 : (int)g;
}

// Updates the running state with x [B, d]; mode bit0 moments, bit1 extrema.
// partial must hold ceil(B / rows_per_block) * d * 4 floats.
OMLDM_API int omldm_colstats_update(const float* x, int B, int d, double count, double* mean,
                                    double* m2, float* lo, float* hi, int mode, float* partial,
                                    int rows_per_block, void* stream) {
  if (B <= 0) return 0;
  if (((mode & 1) && (!mean || !m2)) || ((mode & 2) && (!lo || !hi)) || !partial) return -4;
  hipStream_t st = (hipStream_t)stream;
  const int nblk = (B + rows_per_block - 1) / rows_per_block;
  const size_t lds = (size_t)d * 16;
  if (lds > 160 * 1024) return -1;
  int e = check_dyn_lds((const void*)colmoments_kernel, lds);
  if (e) return e;
  hipLaunchKernelGGL(colmoments_kernel, dim3(nblk), dim3(kPPThreads), lds, st, x, B, d, mean,
                     rows_per_block, partial);
  hipLaunchKernelGGL(colmoments_merge_kernel, dim3(d), dim3(kPPThreads), 0, st, partial, nblk, d,
                     B, count, mean, m2, mean, lo, hi, mode);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_scale(const float* x, float* y, int B, int d, int mode, const double* mean,
                          const double* m2, double count, const float* lo, const float* hi,
                          void* stream) {
  const long long n = (long long)B * d;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(kPPThreads), 0, (hipStream_t)stream,
                     x, y, n, d, mode, mean, m2, count, lo, hi);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_poly(const float* x, int B, int d, const int* idx, int ncomb, int deg,
                         float* out, void* stream) {
  const long long n = (long long)B * (d + ncomb);
  if (n <= 0) return 0;
  hipLaunchKernelGGL(poly_kernel, dim3(grid_for(n)), dim3(kPPThreads), 0, (hipStream_t)stream, x,
                     B, d, idx, ncomb, deg, out);
  return (int)hipGetLastError();
}
