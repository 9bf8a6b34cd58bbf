// Device data plane of the Asynchronous / SSP parameter server (omldm_amd/parallel/p2p.py).
//
// Reference: a worker pushes its model to the parameter server and the server answers THAT
// worker only (omldm/network/FlinkNetwork.scala:262-271). Here the model bytes never leave
// HBM: every hub h owns one PUSH mailbox per worker (h's HBM, shard_h floats) and every
// worker one REPLY mailbox per hub (its HBM); the buffers are hipMalloc'd, exported as IPC
// handles and opened by the peer, which writes into them with peer copies over xGMI. The
// only host traffic is a 4-int header on the gloo control group after the copy's event
// completes (the reader launches its kernels after the header, so it sees the data).
//
//   worker push   : stage = x − base, xpush = x (one pass)  → peer copy into PUSH[h][me]
//   hub merge     : glob += scale · PUSH[h][r]                (the hub's PS stream)
//   hub reply     : peer copy glob → REPLY[r][h]
//   worker install: x = reply + (x − xpush), base = reply     (per hub shard)
#include "common.h"

namespace omldm {
namespace {

int grid_n(long long n) {
  long long b = (n + 255) / 256;
  b = b > 4096 ? 4096 : b;
  return (int)(b < 1 ? 1 : b);
}

__global__ __launch_bounds__(256) void p2p_delta_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ base,
                                                        float* __restrict__ xpush,
                                                        float* __restrict__ stage, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const float v = x[i];
    stage[i] = v - base[i];
    xpush[i] = v;
  }
}

__global__ __launch_bounds__(256) void p2p_axpy_kernel(float* __restrict__ y,
                                                       const float* __restrict__ x, float a,
                                                       long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    y[i] = fmaf(a, x[i], y[i]);
}

__global__ __launch_bounds__(256) void p2p_install_kernel(float* __restrict__ x,
                                                          const float* __restrict__ xpush,
                                                          float* __restrict__ base,
                                                          const float* __restrict__ r,
                                                          long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const float g = r[i];
    x[i] = g + (x[i] - xpush[i]);
    base[i] = g;
  }
}

}  // namespace
}  // namespace omldm

using namespace omldm;

// ---- mailboxes: plain hipMalloc allocations (an IPC handle names a whole allocation)
OMLDM_API void* omldm_ipc_alloc(long long bytes) {
  void* p = nullptr;
  if (bytes <= 0 || hipMalloc(&p, (size_t)bytes) != hipSuccess) return nullptr;
  hipMemset(p, 0, (size_t)bytes);
  return p;
}

OMLDM_API int omldm_ipc_free(void* p) { return p ? (int)hipFree(p) : 0; }

// 64-byte handle of an omldm_ipc_alloc buffer into `out`.
OMLDM_API int omldm_ipc_handle(void* p, void* out) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(h) == HIP_IPC_HANDLE_SIZE, "handle size");
  __builtin_memcpy(out, &h, sizeof(h));
  return 0;
}

OMLDM_API int omldm_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// A peer's buffer mapped into this process (same or another GPU of the node).
OMLDM_API void* omldm_ipc_open(const void* handle) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return nullptr;
  return p;
}

OMLDM_API int omldm_ipc_close(void* p) { return p ? (int)hipIpcCloseMemHandle(p) : 0; }

// dst ← src (either may be a peer mapping): the runtime's copy path handles the
// cross-device coherence of the written bytes.
OMLDM_API int omldm_copy_d2d(void* dst, const void* src, long long bytes, void* stream) {
  if (bytes <= 0) return 0;
  return (int)hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice,
                             (hipStream_t)stream);
}

OMLDM_API int omldm_p2p_delta(const float* x, const float* base, float* xpush, float* stage,
                              long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(p2p_delta_kernel, dim3(grid_n(n)), dim3(256), 0, (hipStream_t)stream, x,
                     base, xpush, stage, n);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_p2p_axpy(float* y, const float* x, float a, long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(p2p_axpy_kernel, dim3(grid_n(n)), dim3(256), 0, (hipStream_t)stream, y, x,
                     a, n);
  return (int)hipGetLastError();
}

OMLDM_API int omldm_p2p_install(float* x, const float* xpush, float* base, const float* r,
                                long long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(p2p_install_kernel, dim3(grid_n(n)), dim3(256), 0, (hipStream_t)stream, x,
                     xpush, base, r, n);
  return (int)hipGetLastError();
}
