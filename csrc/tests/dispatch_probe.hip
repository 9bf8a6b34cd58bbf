// Workgroup-dispatch cost probe (standalone, diagnostics): how long does a grid of
// one-wave workgroups with a per-workgroup LDS table take when each workgroup does
// almost nothing, versus the same work done by fewer waves that loop over several
// "spokes"? Answers whether the linear round kernel's fixed cost (≈ 52 µs at 8192
// one-wave workgroups, profiles/round1_ablation.md) is dispatch / LDS-allocation bound.
//
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/dispatch_probe csrc/tests/dispatch_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// Each "spoke": zero a table of `tsz` int2 in LDS, read 16 rows × 80 B of input, write one
// 8-KiB table image (like the round kernel's flush) and one float.
__global__ __launch_bounds__(64) void spoke_kernel(const int4* __restrict__ in, int2* __restrict__ tables,
                                                   float* __restrict__ out, int S, int tsz, int flush) {
  extern __shared__ int2 tab[];
  for (int s = blockIdx.x; s < S; s += gridDim.x) {
    for (int i = threadIdx.x; i < tsz; i += 64) tab[i] = make_int2(-1, 0);
    __syncthreads();
    // 16 rows × 80 B = 1280 B = 80 int4 per spoke
    float acc = 0.f;
    for (int i = threadIdx.x; i < 80; i += 64) {
      const int4 v = in[(size_t)s * 80 + i];
      acc += (float)(v.x + v.y + v.z + v.w);
    }
    atomicAdd(&tab[threadIdx.x].y, (int)acc);
    __syncthreads();
    if (flush)
      for (int i = threadIdx.x; i < tsz - 64; i += 64) tables[(size_t)s * (tsz - 64) + i] = tab[i];
    if (threadIdx.x == 0) out[s] = acc;
    __syncthreads();
  }
}

int main(int argc, char** argv) {
  const int S = 8192, tsz = 1024 + 64;
  int4* in;
  int2* tables;
  float* out;
  CK(hipMalloc(&in, (size_t)S * 80 * 16));
  CK(hipMalloc(&tables, (size_t)S * 1024 * 8));
  CK(hipMalloc(&out, S * 4));
  CK(hipMemset(in, 0, (size_t)S * 80 * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grids[] = {8192, 4096, 2048, 1024, 512};
  for (int flush = 0; flush < 2; ++flush) {
    for (int gi = 0; gi < 5; ++gi) {
      const int G = grids[gi];
      for (int w = 0; w < 5; ++w)
        hipLaunchKernelGGL(spoke_kernel, dim3(G), dim3(64), tsz * 8, 0, in, tables, out, S, tsz, flush);
      CK(hipDeviceSynchronize());
      const int iters = 50;
      CK(hipEventRecord(a, 0));
      for (int it = 0; it < iters; ++it)
        hipLaunchKernelGGL(spoke_kernel, dim3(G), dim3(64), tsz * 8, 0, in, tables, out, S, tsz, flush);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("flush=%d grid=%5d spokes/wave=%2d : %8.2f us/launch\n", flush, G, S / G,
             ms * 1000.f / iters);
    }
  }
  return 0;
}
