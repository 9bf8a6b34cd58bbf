// Host <-> persistent-wave ping-pong latency: where should the request line live?
//   mode 0: request in coherent pinned HOST memory (the wave polls it over PCIe)
//   mode 1: request in fine-grained DEVICE memory written by the CPU through the BAR
//           (the host's store is posted; the wave polls its local HBM)
// The response always goes to coherent host memory. Bounded: the wave exits after
// `iters` pings or ~2 s of wall time. Standalone: hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e = (x);                                                                   \
    if (e != hipSuccess) {                                                                \
      std::printf("HIP error %s at line %d\n", hipGetErrorString(e), __LINE__);           \
      std::exit(2);                                                                       \
    }                                                                                     \
  } while (0)

__global__ void pong(unsigned* req, unsigned* resp, int iters, unsigned long long max_ticks) {
  const unsigned long long t_end = __builtin_amdgcn_s_memrealtime() + max_ticks;
  unsigned last = 0;
  for (int i = 0; i < iters; ++i) {
    unsigned v;
    while (true) {
      v = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v != last) break;
      if (__builtin_amdgcn_s_memrealtime() > t_end) return;
      __builtin_amdgcn_s_sleep(1);
    }
    last = v;
    if (threadIdx.x == 0) __hip_atomic_store(resp, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const int iters = 20000;
  CK(hipSetDevice(0));
  unsigned* resp = nullptr;
  CK(hipHostMalloc((void**)&resp, 256, hipHostMallocCoherent | hipHostMallocMapped));
  *resp = 0;
  unsigned *req_host = nullptr, *req_dev = nullptr;
  if (mode == 0) {
    CK(hipHostMalloc((void**)&req_host, 256, hipHostMallocCoherent | hipHostMallocMapped));
    *req_host = 0;
    CK(hipHostGetDevicePointer((void**)&req_dev, req_host, 0));
  } else {
    CK(hipExtMallocWithFlags((void**)&req_dev, 256, hipDeviceMallocFinegrained));
    CK(hipMemset(req_dev, 0, 256));
    CK(hipDeviceSynchronize());
    req_host = req_dev;  // the CPU writes through the same virtual address (BAR)
    volatile unsigned* probe = req_host;
    *probe = 0;  // faults here when VRAM is not CPU-mapped
  }
  unsigned* resp_dev = nullptr;
  CK(hipHostGetDevicePointer((void**)&resp_dev, resp, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, s, req_dev, resp_dev, iters,
                     200000000ull /* 2 s at 100 MHz */);
  std::vector<double> lat;
  lat.reserve(iters);
  volatile unsigned* vreq = req_host;
  volatile unsigned* vresp = resp;
  for (int i = 1; i <= iters; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(const_cast<unsigned*>(vreq), (unsigned)i, __ATOMIC_RELEASE);
    if (mode == 1) __builtin_ia32_sfence();  // drain the write-combining buffer (BAR)
    bool ok = false;
    for (long spin = 0; spin < 200000000L; ++spin) {
      if (__atomic_load_n(const_cast<unsigned*>(vresp), __ATOMIC_ACQUIRE) == (unsigned)i) {
        ok = true;
        break;
      }
    }
    if (!ok) {
      std::printf("mode %d: no answer at ping %d\n", mode, i);
      break;
    }
    lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  CK(hipStreamSynchronize(s));
  if (!lat.empty()) {
    std::sort(lat.begin() + 0, lat.end());
    std::printf("mode %d (%s): pings %zu  p50 %.2f us  p90 %.2f us  p99 %.2f us\n", mode,
                mode == 0 ? "request in host memory" : "request in device memory (BAR)",
                lat.size(), lat[lat.size() / 2], lat[lat.size() * 9 / 10], lat[lat.size() * 99 / 100]);
  }
  return 0;
}
