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

// ---------------------------------------------------------------------------------------
// GM / FGM monitoring decisions on the device (one lane): the per-round safe-zone test and
// the replicated hub logic read the 2-float drift norms where drift_norms_kernel left them
// and write the message to reduce / the sync decision — no host round-trip inside a round.
// The host reads the decision one round later through a pinned copy (protocols.py).
//
// FGM state st[8] (fp64): 0 c_prev (this worker's counter), 1 csum (Σ increments, hub),
// 2 theta (quantum; 0 ⇔ E == 0), 3 phi0 = −ε‖E‖², 4 phi (this worker's last φ),
// 5 decision latch (1 = full sync due), 6 subrounds.
constexpr double kFgmBig = 1e12;  // counter of a worker that drifted while E == 0

__device__ inline double fgm_counter(double phi, double phi0, double theta) {
  const double num = phi - phi0;
  if (theta <= 0.0) return num > 0.0 ? kFgmBig : 0.0;
  return fmin(kFgmBig, fmax(0.0, floor(num / theta)));
}

// GM: msg[0] = 1 when ‖X_i‖² > θ·max(‖E‖², 1) (max-reduced over workers)
__global__ void gm_local_kernel(const float* __restrict__ nrm, float thr, double* __restrict__ msg) {
  if (threadIdx.x == 0) msg[0] = nrm[0] > thr * fmaxf(nrm[1], 1.f) ? 1.0 : 0.0;
}

// FGM worker: φ = ‖X_i‖² − ε‖E‖²; counter increment since the last report; msg = (Δc, φ)
__global__ void fgm_local_kernel(const float* __restrict__ nrm, double* __restrict__ st,
                                 double eps, double* __restrict__ msg) {
  if (threadIdx.x != 0) return;
  const double phi = (double)nrm[0] - eps * (double)nrm[1];
  const double c = fgm_counter(phi, st[3], st[2]);
  msg[0] = c - st[0];
  msg[1] = phi;
  st[0] = c;
  st[4] = phi;
}

// FGM hub (replicated on every rank from the reduced msg): Σ counters > G ends the
// subround; ψ = Σφ ≥ ε_ψ·G·φ(0) ends the round (full sync due), otherwise θ = −ψ/(2G).
__global__ void fgm_hub_kernel(double* __restrict__ st, const double* __restrict__ msg,
                               double eps_psi, int G, double* __restrict__ flag) {
  if (threadIdx.x != 0) return;
  if (st[5] == 0.0) {
    st[1] += msg[0];
    if (st[1] > (double)G) {
      st[6] += 1.0;
      const double psi = msg[1];
      if (psi >= eps_psi * (double)G * st[3]) {
        st[5] = 1.0;
      } else {
        st[2] = -psi / (2.0 * G);
        st[1] = 0.0;
        st[0] = fgm_counter(st[4], st[3], st[2]);  // counters restart in the new subround
      }
    }
  }
  flag[0] = st[5];
}

// FGM round start (after a full sync, E = x): φ(0) = −ε‖E‖², θ = −ψ/(2G) = −φ(0)/2
__global__ void fgm_begin_kernel(const float* __restrict__ nrm, double* __restrict__ st,
                                 double eps) {
  if (threadIdx.x != 0) return;
  const double phi0 = -eps * (double)nrm[1];
  st[0] = 0.0;
  st[1] = 0.0;
  st[2] = phi0 < 0.0 ? -phi0 / 2.0 : 0.0;
  st[3] = phi0;
  st[4] = 0.0;
  st[5] = 0.0;
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

OMLDM_API int omldm_gm_local(const float* nrm, float thr, double* msg, void* stream) {
  hipLaunchKernelGGL(gm_local_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, nrm, thr, msg);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_fgm_local(const float* nrm, double* st, double eps, double* msg,
                              void* stream) {
  hipLaunchKernelGGL(fgm_local_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, nrm, st, eps,
                     msg);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_fgm_hub(double* st, const double* msg, double eps_psi, int G, double* flag,
                            void* stream) {
  hipLaunchKernelGGL(fgm_hub_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, st, msg, eps_psi,
                     G, flag);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_fgm_begin(const float* nrm, double* st, double eps, void* stream) {
  hipLaunchKernelGGL(fgm_begin_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, nrm, st, eps);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_async_pull(float* x, float* E, float* shipped, const float* sent,
                               const float* merged, float scale, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(async_pull_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x,
                     E, shipped, sent, merged, scale, n);
  return (int)hipGetLastError();
}
