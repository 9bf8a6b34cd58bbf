// In-kernel clock of a lone wave (one CU busy, the rest of the chip idle) vs a full grid:
// Δs_memtime (shader cycles) / Δs_memrealtime (100 MHz) around a dependent fma chain.
// Build: hipcc --offload-arch=gfx950 -O3 clock_probe.hip -o clock_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chain(float* out, unsigned long long* st, int iters) {
  float a = threadIdx.x * 1e-3f, b = 0.999f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) a = fmaf(a, b, 1e-7f);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    st[0] = t1 - t0;
    st[1] = r1 - r0;
  }
}

int main() {
  float* out;
  unsigned long long* st;
  hipMalloc(&out, 1024 * 256 * 4);
  hipMallocManaged(&st, 16);
  for (int grid : {1, 1, 256, 1024}) {
    const int iters = 200000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(chain, dim3(grid), dim3(64), 0, 0, out, st, iters);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double cyc = (double)st[0], rt = (double)st[1];
    printf("grid %4d: %.0f cycles, %.3f ms realtime -> clock %.3f GHz; %.2f cycles per dependent fma; event %.3f ms\n",
           grid, cyc, rt / 1e5, cyc / (rt * 10.0), cyc / (iters * 16.0), ms);
  }
  return 0;
}
