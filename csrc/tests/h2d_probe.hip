// H2D probe: is hipMemcpyAsync from pinned host memory asynchronous for the calling
// thread, which engine does it use, and how fast is it alone and next to a kernel that
// keeps the CUs and HBM busy? Standalone (hipcc --offload-arch=gfx950 -O2).
//
//   ./h2d_probe [MB]
// Prints one line per variant: host enqueue µs, copy µs (event timed), GB/s, and the
// same with a concurrent compute kernel on another stream.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

// Memory-latency-bound busy kernel (random-ish gathers over a 256 MB table), bounded
// iteration count so it always finishes.
__global__ void busy_kernel(const float* __restrict__ t, float* __restrict__ out, int iters,
                            unsigned mask) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  unsigned h = i * 2654435761u;
  for (int k = 0; k < iters; ++k) {
    h = h * 1664525u + 1013904223u;
    acc += t[h & mask];
  }
  out[i] = acc;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? std::atoi(argv[1]) : 11;
  const size_t n = mb << 20;
  CK(hipSetDevice(0));
  void* d = nullptr;
  CK(hipMalloc(&d, n));
  const size_t tn = size_t(64) << 20;  // 64 M floats = 256 MB
  float* table = nullptr;
  float* out = nullptr;
  CK(hipMalloc(&table, tn * sizeof(float)));
  CK(hipMemset(table, 0, tn * sizeof(float)));
  const int busy_blocks = 2048, busy_threads = 256;
  CK(hipMalloc(&out, size_t(busy_blocks) * busy_threads * sizeof(float)));
  hipStream_t cs, ks;
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  struct Var {
    const char* name;
    unsigned flags;
    bool registered;
  } vars[] = {{"hipHostMalloc(default)", hipHostMallocDefault, false},
              {"hipHostMalloc(coherent)", hipHostMallocCoherent, false},
              {"hipHostMalloc(noncoherent)", hipHostMallocNonCoherent, false},
              {"hipHostMalloc(numa_user)", hipHostMallocNumaUser, false},
              {"malloc+hipHostRegister", 0, true}};
  for (const Var& v : vars) {
    void* h = nullptr;
    if (v.registered) {
      h = std::aligned_alloc(4096, n);
      CK(hipHostRegister(h, n, hipHostRegisterDefault));
    } else {
      CK(hipHostMalloc(&h, n, v.flags));
    }
    std::memset(h, 1, n);
    for (int with_busy = 0; with_busy < 2; ++with_busy) {
      double enq = 0, dev_ms = 0;
      const int reps = 10;
      for (int r = 0; r < reps + 2; ++r) {
        if (with_busy)
          hipLaunchKernelGGL(busy_kernel, dim3(busy_blocks), dim3(busy_threads), 0, ks, table,
                             out, 4000, unsigned(tn - 1));
        CK(hipEventRecord(e0, cs));
        const double t0 = now_us();
        CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, cs));
        const double t1 = now_us();
        CK(hipEventRecord(e1, cs));
        CK(hipStreamSynchronize(cs));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipStreamSynchronize(ks));
        if (r >= 2) {
          enq += t1 - t0;
          dev_ms += ms;
        }
      }
      std::printf("%-28s busy=%d  enqueue %8.1f us  copy %8.1f us  %6.1f GB/s\n", v.name,
                  with_busy, enq / reps, dev_ms / reps * 1e3, n / (dev_ms / reps * 1e-3) / 1e9);
    }
    if (v.registered) {
      CK(hipHostUnregister(h));
      std::free(h);
    } else {
      CK(hipHostFree(h));
    }
  }
  // busy kernel alone, for reference
  CK(hipEventRecord(e0, ks));
  hipLaunchKernelGGL(busy_kernel, dim3(busy_blocks), dim3(busy_threads), 0, ks, table, out, 4000,
                     unsigned(tn - 1));
  CK(hipEventRecord(e1, ks));
  CK(hipStreamSynchronize(ks));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::printf("busy kernel alone: %.1f us\n", ms * 1e3);
  return 0;
}
