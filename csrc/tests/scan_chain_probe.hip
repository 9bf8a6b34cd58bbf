// Cycles per step of the exact scan's dependency chain (diagnostics, standalone).
//
// One 512-thread workgroup; wave 0 runs the 64-step recurrence of a chunk NCH times with
// the chunk's Gram rows in LDS, in one of these forms:
//   0  m-form (linear_scan.hip as of round 3): c = med3(fma(a, m, b)); readlane; m += c·G;
//      plus the two off-chain folds n1 += c·X1, n2 += c·X2 (3 LDS rows per lane)
//   1  u-form: the row's affine candidate kept directly, u = a·m + b, with G pre-scaled by
//      a (prep's job): c = med3(u); readlane; u += c·(aG); plus n1 += c·(aX1) (2 rows)
//   2  u-form alone (1 row)
//   3  u-form + n1 with both rows held in VGPRs for the whole chunk (no LDS in the chain)
// Waves 1-7 either idle at the barrier (load 0) or keep the LDS and VALU busy (load 1),
// like the helper waves of the scan kernel.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/scp csrc/tests/scan_chain_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int CH = 64, GS = 68;

__device__ __forceinline__ float rl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

template <int V>
__global__ __launch_bounds__(512, 1) void chain(const float* __restrict__ g, int nch, int load,
                                                float* __restrict__ out,
                                                unsigned long long* __restrict__ cyc) {
  __shared__ alignas(16) float G[3][CH][GS];
  __shared__ float junk[8][64];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int i = tid; i < 3 * CH * GS; i += 512) (&G[0][0][0])[i] = g[i % (CH * GS)] * (1 + i / (CH * GS));
  __syncthreads();
  if (wave == 0) {
    __builtin_amdgcn_s_setprio(3);
    const float a = -0.03f - 0.0001f * lane, b = (lane & 1) ? 0.03f : -0.03f;
    const float lo = (lane & 1) ? 0.f : -1.f, hi = (lane & 1) ? 1.f : 0.f;
    float m = 0.1f * lane, u = a * m + b, n1 = 0.f, n2 = 0.f, acc = 0.f;
    float gr[CH], xr[CH];
    if constexpr (V == 3) {
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        gr[s] = G[0][lane][s];
        xr[s] = G[1][lane][s];
      }
    }
    const unsigned long long t0 = clock64();
    for (int k = 0; k < nch; ++k) {
      if constexpr (V == 0) {
        const float* g0 = &G[0][lane][0];
        const float* g1 = &G[1][lane][0];
        const float* g2 = &G[2][lane][0];
#pragma unroll
        for (int t4 = 0; t4 < CH; t4 += 4) {
          const float4 a4 = *reinterpret_cast<const float4*>(g0 + t4);
          const float4 b4 = *reinterpret_cast<const float4*>(g1 + t4);
          const float4 c4 = *reinterpret_cast<const float4*>(g2 + t4);
          const float ga[4] = {a4.x, a4.y, a4.z, a4.w}, gb[4] = {b4.x, b4.y, b4.z, b4.w},
                      gc[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float ct = rl(__builtin_amdgcn_fmed3f(fmaf(a, m, b), lo, hi), t4 + q);
            m = fmaf(ct, ga[q], m);
            n1 = fmaf(ct, gb[q], n1);
            n2 = fmaf(ct, gc[q], n2);
          }
        }
        acc += m;
        m = n1 + 0.5f * m;
        n1 = n2;
        n2 = 0.f;
      } else if constexpr (V == 1 || V == 2) {
        const float* g0 = &G[0][lane][0];
        const float* g1 = &G[1][lane][0];
#pragma unroll
        for (int t4 = 0; t4 < CH; t4 += 4) {
          const float4 a4 = *reinterpret_cast<const float4*>(g0 + t4);
          float4 b4 = make_float4(0, 0, 0, 0);
          if constexpr (V == 1) b4 = *reinterpret_cast<const float4*>(g1 + t4);
          const float ga[4] = {a4.x, a4.y, a4.z, a4.w}, gb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float ct = rl(__builtin_amdgcn_fmed3f(u, lo, hi), t4 + q);
            u = fmaf(ct, ga[q], u);
            if constexpr (V == 1) n1 = fmaf(ct, gb[q], n1);
          }
        }
        acc += u;
        u = n1 + 0.5f * u;
        n1 = 0.f;
      } else {
#pragma unroll
        for (int s = 0; s < CH; ++s) {
          const float ct = rl(__builtin_amdgcn_fmed3f(u, lo, hi), s);
          u = fmaf(ct, gr[s], u);
          n1 = fmaf(ct, xr[s], n1);
        }
        acc += u;
        u = n1 + 0.5f * u;
        n1 = 0.f;
      }
      __syncthreads();
    }
    const unsigned long long t1 = clock64();
    out[lane] = acc;
    if (lane == 0) cyc[0] = t1 - t0;
  } else {
    float x = (float)tid;
    for (int k = 0; k < nch; ++k) {
      if (load) {
        for (int i = 0; i < 24; ++i) {
          x = fmaf(x, 1.0001f, junk[wave][(lane + i) & 63]);
          junk[wave][(lane * 7 + i) & 63] = x;
        }
      }
      __syncthreads();
    }
    if (x == 12345.f) out[64 + tid] = x;
  }
}

template <int V>
static double run(const float* dg, int nch, int load, float* dout, unsigned long long* dc) {
  hipLaunchKernelGGL(chain<V>, dim3(1), dim3(512), 0, 0, dg, nch, load, dout, dc);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(chain<V>, dim3(1), dim3(512), 0, 0, dg, nch, load, dout, dc);
  CK(hipDeviceSynchronize());
  unsigned long long c = 0;
  CK(hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost));
  return double(c) / (double(nch) * CH);
}

int main() {
  const int nch = 256;
  std::vector<float> g(CH * GS);
  srand(25);
  for (int t = 0; t < CH; ++t)
    for (int s = 0; s < GS; ++s) g[t * GS + s] = s < t ? 0.01f * ((rand() % 200) - 100) / 100.f : 0.f;
  float *dg, *dout;
  unsigned long long* dc;
  CK(hipMalloc(&dg, g.size() * 4));
  CK(hipMalloc(&dout, 4096 * 4));
  CK(hipMalloc(&dc, 8));
  CK(hipMemcpy(dg, g.data(), g.size() * 4, hipMemcpyHostToDevice));
  for (int load = 0; load < 2; ++load) {
    printf("{\"load\": %d, \"m_form_cyc_per_step\": %.2f, \"u_form_x1\": %.2f, \"u_form\": %.2f, "
           "\"u_form_x1_vgpr\": %.2f}\n",
           load, run<0>(dg, nch, load, dout, dc), run<1>(dg, nch, load, dout, dc),
           run<2>(dg, nch, load, dout, dc), run<3>(dg, nch, load, dout, dc));
  }
  return 0;
}
