// Hub merge ops of the synchronisation protocols: drift norms for the
// GM / FGM safe zones, the elastic move of EASGD and the "fold the merged increment into
// the estimate and reload the model" step of every full sync — each one streaming pass
// over the flat parameter vector (HBM-bound) instead of 3-5 separate elementwise kernels
// and temporaries. They bracket the RCCL collective on the same stream.
#include "common.h"

namespace omldm {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// out[0] += Σ ((x − E)·scale)², out[1] += Σ E²  (n4 = n/4 vectors, tail handled by block 0)
__global__ __launch_bounds__(256) void drift_norms_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ E, long long n,
                                                          float scale, float* __restrict__ out) {
  __shared__ float part[8];
  float a = 0.f, b = 0.f;
  const long long n4 = n >> 2;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  const f32x4* e4 = reinterpret_cast<const f32x4*>(E);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4;
       i += (long long)gridDim.x * 256) {
    const f32x4 xv = x4[i], ev = e4[i];
    const f32x4 dv = (xv - ev) * scale;
    a += dv.x * dv.x + dv.y * dv.y + dv.z * dv.z + dv.w * dv.w;
    b += ev.x * ev.x + ev.y * ev.y + ev.z * ev.z + ev.w * ev.w;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    const float d = (x[i] - E[i]) * scale;
    a += d * d;
    b += E[i] * E[i];
  }
  wave_sum2(a, b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[w] = a;
    part[4 + w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&out[0], (part[0] + part[1]) + (part[2] + part[3]));
    atomicAdd(&out[1], (part[4] + part[5]) + (part[6] + part[7]));
  }
}

// E += alpha·d ; x = E   (full sync: fold the reduced increment, reload the model)
__global__ __launch_bounds__(256) void fold_reload_kernel(float* __restrict__ E,
                                                          const float* __restrict__ d, float alpha,
                                                          float* __restrict__ x, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const float e = fmaf(alpha, d[i], E[i]);
    E[i] = e;
    x[i] = e;
  }
}

// diff = x − c ; s = diff·pre  (EASGD before the all-reduce of s)
__global__ __launch_bounds__(256) void elastic_pre_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ c,
                                                          float* __restrict__ diff,
                                                          float* __restrict__ s, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const float v = x[i] - c[i];
    diff[i] = v;
    s[i] = v;
  }
}

// x −= α·diff ; c += α·s   (EASGD after the all-reduce: worker and centre moves)
__global__ __launch_bounds__(256) void elastic_post_kernel(float* __restrict__ x,
                                                           float* __restrict__ c,
                                                           const float* __restrict__ diff,
                                                           const float* __restrict__ s,
                                                           float alpha, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    x[i] = fmaf(-alpha, diff[i], x[i]);
    c[i] = fmaf(alpha, s[i], c[i]);
  }
}

// sent = x − E − shipped ; buf = sent ; shipped += sent   (asynchronous push)
__global__ __launch_bounds__(256) void async_push_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ E,
                                                         float* __restrict__ shipped,
                                                         float* __restrict__ sent,
                                                         float* __restrict__ buf, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const float v = x[i] - E[i] - shipped[i];
    sent[i] = v;
    buf[i] = v;
    shipped[i] += v;
  }
}

// x += merged·scale − sent ; shipped −= sent ; E += merged·scale   (asynchronous pull)
__global__ __launch_bounds__(256) void async_pull_kernel(float* __restrict__ x,
                                                         float* __restrict__ E,
                                                         float* __restrict__ shipped,
                                                         const float* __restrict__ sent,
                                                         const float* __restrict__ merged,
                                                         float scale, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const float m = merged[i] * scale, s = sent[i];
    x[i] += m - s;
    shipped[i] -= s;
    E[i] += m;
  }
}

static inline int grid_for(long long n) {
  long long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  return b < 1 ? 1 : (int)b;
}

}  // namespace omldm

using namespace omldm;

OMLDM_API int omldm_drift_norms(const float* x, const float* E, long long n, float scale,
                                float* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipMemsetAsync(out, 0, 2 * sizeof(float), s);
  if (n <= 0) return (int)hipGetLastError();
  if (((uintptr_t)x | (uintptr_t)E) & 15) return -1;
  hipLaunchKernelGGL(drift_norms_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, x, E, n,
                     scale, out);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_fold_reload(float* E, const float* d, float alpha, float* x, long long n,
                                void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fold_reload_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, E,
                     d, alpha, x, n);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_elastic_pre(const float* x, const float* c, float* diff, float* s,
                                long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(elastic_pre_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x,
                     c, diff, s, n);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_elastic_post(float* x, float* c, const float* diff, const float* s,
                                 float alpha, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(elastic_post_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     x, c, diff, s, alpha, n);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_async_push(const float* x, const float* E, float* shipped, float* sent,
                               float* buf, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(async_push_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x,
                     E, shipped, sent, buf, n);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_async_pull(float* x, float* E, float* shipped, const float* sent,
                               const float* merged, float scale, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(async_pull_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x,
                     E, shipped, sent, merged, scale, n);
  return (int)hipGetLastError();
}
