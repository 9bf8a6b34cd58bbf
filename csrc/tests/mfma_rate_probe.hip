// Matrix-core issue rate on this part (diagnostics, standalone): one wave per SIMD runs
// N rounds of A independent v_mfma_f32_32x32x2_f32 (or 32x32x16 bf16) chains and reports
// shader-clock cycles per instruction, plus the whole-chip rate over all CUs.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/mfr csrc/tests/mfma_rate_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int A, bool BF16>
__global__ __launch_bounds__(256) void rate_kernel(float* out, unsigned long long* cyc, int n) {
  f32x16 acc[A];
#pragma unroll
  for (int a = 0; a < A; ++a)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[a][q] = 0.f;
  const float x = threadIdx.x * 1e-3f, y = 1.f + threadIdx.x * 1e-4f;
  bf16x8 xb, yb;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    xb[j] = (short)(threadIdx.x + j);
    yb[j] = (short)(threadIdx.x * 3 + j);
  }
  const unsigned long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int a = 0; a < A; ++a) {
      if constexpr (BF16) acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xb, yb, acc[a], 0, 0, 0);
      else acc[a] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[a], 0, 0, 0);
    }
  }
  const unsigned long long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < A; ++a)
#pragma unroll
    for (int q = 0; q < 16; ++q) s += acc[a][q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int A, bool BF16>
void run(const char* name, int blocks, float* out, unsigned long long* cyc) {
  const int n = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((rate_kernel<A, BF16>), dim3(blocks), dim3(256), 0, 0, out, cyc, n);
  hipDeviceSynchronize();
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL((rate_kernel<A, BF16>), dim3(blocks), dim3(256), 0, 0, out, cyc, n);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const double instr = (double)n * A;
  const double flop = instr * (BF16 ? 32.0 * 32 * 16 * 2 : 32.0 * 32 * 2 * 2) * blocks * 4;
  printf("%-28s blocks=%4d chains=%2d: %.1f clk/instr (wave 0), %.1f TFLOP/s whole launch\n", name,
         blocks, A, (double)c / instr, flop / (ms * 1e-3) / 1e12);
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 4096 * 256 * 4);
  hipMalloc(&cyc, 8);
  run<1, false>("f32 32x32x2 dependent", 256, out, cyc);
  run<4, false>("f32 32x32x2", 256, out, cyc);
  run<10, false>("f32 32x32x2", 256, out, cyc);
  run<4, false>("f32 32x32x2 2 waves/SIMD", 512, out, cyc);
  run<1, true>("bf16 32x32x16 dependent", 256, out, cyc);
  run<4, true>("bf16 32x32x16", 256, out, cyc);
  run<4, true>("bf16 32x32x16 2 waves/SIMD", 512, out, cyc);
  return 0;
}
