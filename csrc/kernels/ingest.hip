// Ingest: pull a micro-batch from pinned host memory into HBM with a kernel.
//
// The reference feeds every spoke through Kafka consumers and Flink network buffers
// (omldm/Job.scala:42-57, omldm/job/FlinkLearning.scala:83). Here the host parser packs a
// micro-batch into a pinned, device-mapped buffer and the GPU pulls it over PCIe: many
// workgroups each keep several 16-byte loads in flight against host memory, which
// sustains more PCIe read bandwidth than one SDMA copy engine, and the same pass can
// unpack the compact wire format into the kernel layout (no second HBM pass).
#include "common.h"

#include <cstdlib>
#include <cstring>
#include <sys/mman.h>

namespace omldm {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Plain 16-byte-per-lane streaming copy (host-mapped src → device dst), 4 loads in
// flight per lane before the stores.
__global__ __launch_bounds__(256) void pull_copy_kernel(const u32x4* __restrict__ src,
                                                        u32x4* __restrict__ dst, long long n16) {
  const long long tid = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long stride = (long long)gridDim.x * 256;
  long long i = tid;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4 a = __builtin_nontemporal_load(src + i);
    const u32x4 b = __builtin_nontemporal_load(src + i + stride);
    const u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
    const u32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = __builtin_nontemporal_load(src + i);
}

// The same copy with write-through (sc1) buffer stores: the copied lines leave the copying
// XCD's L2 instead of staying there (a plain 20-MB store pass evicts what the training
// kernels on that XCD keep in its 4-MB L2; the batch is read next by every XCD anyway, from
// HBM). nbytes < 2^31 (one buffer descriptor).
__global__ __launch_bounds__(256) void pull_copy_wt_kernel(const u32x4* __restrict__ src,
                                                           u32x4* __restrict__ dst, long long n16) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(n16 * 16), 0x00020000);
  const int tid = blockIdx.x * 256 + threadIdx.x;
  const int stride = gridDim.x * 256;
  const int n = (int)n16;
  int i = tid;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const u32x4 a = __builtin_nontemporal_load(src + i);
    const u32x4 b = __builtin_nontemporal_load(src + i + stride);
    const u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
    const u32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
    __builtin_amdgcn_raw_buffer_store_b128(a, rs, i * 16, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(b, rs, (i + stride) * 16, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(c, rs, (i + 2 * stride) * 16, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(d, rs, (i + 3 * stride) * 16, 0, 16);
  }
  for (; i < n; i += stride)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_nontemporal_load(src + i), rs, i * 16, 0, 16);
}

// U loads in flight per lane before the stores (few waves, deep queues: long-latency PCIe
// reads from many waves clog the memory pipeline shared with the training kernels).
template <int U>
__global__ __launch_bounds__(256) void pull_copy_u_kernel(const u32x4* __restrict__ src,
                                                          u32x4* __restrict__ dst, long long n16) {
  const long long tid = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long stride = (long long)gridDim.x * 256;
  long long i = tid;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * stride] = v[u];
  }
  for (; i < n16; i += stride) dst[i] = __builtin_nontemporal_load(src + i);
}

// Several (host src → device dst, bytes) segments in one launch: blockIdx.y = segment
// (the engine's staging slot is one region per partition, plus the record offsets — a
// launch per segment cost the staging thread a HIP call each). src / dst 16-B aligned; a
// segment's last partial vector is copied bytewise by block 0.
struct PullSegs {
  static constexpr int kMax = 64;
  const unsigned char* src[kMax];
  unsigned char* dst[kMax];
  long long n[kMax];
};

__global__ __launch_bounds__(256) void pull_copy_segs_kernel(PullSegs d) {
  const int sg = blockIdx.y;
  const u32x4* src = reinterpret_cast<const u32x4*>(d.src[sg]);
  u32x4* dst = reinterpret_cast<u32x4*>(d.dst[sg]);
  const long long n = d.n[sg], n16 = n >> 4;
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4 a = __builtin_nontemporal_load(src + i);
    const u32x4 b = __builtin_nontemporal_load(src + i + stride);
    const u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
    const u32x4 e = __builtin_nontemporal_load(src + i + 3 * stride);
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = e;
  }
  for (; i < n16; i += stride) dst[i] = __builtin_nontemporal_load(src + i);
  const int tail = (int)(n & 15);
  if (blockIdx.x == 0 && (int)threadIdx.x < tail)
    d.dst[sg][n16 * 16 + threadIdx.x] = d.src[sg][n16 * 16 + threadIdx.x];
}

__global__ void pull_tail_kernel(const unsigned char* __restrict__ src,
                                 unsigned char* __restrict__ dst, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

}  // namespace omldm

using namespace omldm;

// A stream whose kernels may only run on `ncu` CUs spread over all XCDs (every
// (256/ncu)-th CU), so the ingest pull kernel never competes with the training kernels
// for more than that slice of the chip. Returns the hipStream_t (0 on failure).
// layout 0: every (total/ncu)-th CU; layout 1: CUs [0, ncu) (a contiguous block).
OMLDM_API void* omldm_stream_create_cumask_ex(int ncu, int invert, int layout) {
  hipDeviceProp_t prop;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
    return nullptr;
  const int total = prop.multiProcessorCount;
  if (ncu <= 0 || ncu >= total) ncu = total;
  uint32_t mask[16] = {0};
  const int step = total / ncu;
  if (layout == 1) {
    for (int c = 0; c < ncu; ++c) mask[c >> 5] |= 1u << (c & 31);
  } else {
    for (int i = 0, c = total - 1; i < ncu && c >= 0; ++i, c -= step) mask[c >> 5] |= 1u << (c & 31);
  }
  const int words = (total + 31) / 32;
  if (invert) {  // the complement: every CU the slice above does not own
    for (int w = 0; w < words; ++w) mask[w] = ~mask[w];
    if (total & 31) mask[words - 1] &= (1u << (total & 31)) - 1u;
  }
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask) != hipSuccess) return nullptr;
  return (void*)s;
}

// A stream restricted to the CUs whose bits are set in mask[0..words) (bit c = the c-th
// CU in the runtime's CU-mask order).
OMLDM_API void* omldm_stream_create_cumask_words(const uint32_t* mask, int words) {
  hipStream_t s = nullptr;
  if (words <= 0 || hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask) != hipSuccess)
    return nullptr;
  return (void*)s;
}

// Where a workgroup launched on `stream` runs: out[0] = XCC id, out[1] = HW_ID (CU, SH,
// SE fields) — maps CU-mask bits to XCDs (scripts/cumask_probe.py).
__global__ void cu_probe_kernel(int* out) {
  if (threadIdx.x == 0) {
    out[0] = (int)__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    out[1] = (int)__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
  }
}

OMLDM_API int omldm_cu_probe(int* out, void* stream) {
  hipLaunchKernelGGL(cu_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
  return (int)hipGetLastError();
}

OMLDM_API void* omldm_stream_create_cumask(int ncu) { return omldm_stream_create_cumask_ex(ncu, 0, 0); }

OMLDM_API int omldm_stream_destroy(void* s) { return (int)hipStreamDestroy((hipStream_t)s); }

// Plain async SDMA copy, issued straight to the runtime (no framework bookkeeping).
OMLDM_API int omldm_h2d_async(void* dst, const void* src, long long nbytes, void* stream) {
  return (int)hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyHostToDevice, (hipStream_t)stream);
}

// Device-side alias of a pinned host pointer (kernels may then read/write host memory
// directly over PCIe: zero-copy ingest of single-use rows, zero-copy predict results).
OMLDM_API void* omldm_host_device_ptr(void* host) {
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, host, 0) != hipSuccess) return nullptr;
  return dev;
}

// Pinned host buffer backed by transparent huge pages: 2 MiB-aligned anonymous memory
// with MADV_HUGEPAGE, faulted in, then registered (pinned + device-mapped). The GPU then
// reaches it through 2 MiB translations instead of 4 KiB ones, which matters for a copy
// kernel streaming host memory next to training kernels that share the GPU's address
// translation caches. Returns nullptr on failure; free with omldm_host_free_thp.
OMLDM_API void* omldm_host_alloc_thp(long long nbytes) {
  const size_t huge = size_t(2) << 20;
  const size_t n = ((size_t)nbytes + huge - 1) / huge * huge;
  void* p = nullptr;
  if (posix_memalign(&p, huge, n) != 0) return nullptr;
  madvise(p, n, MADV_HUGEPAGE);
  memset(p, 0, n);
  if (hipHostRegister(p, n, hipHostRegisterMapped) != hipSuccess) {
    free(p);
    return nullptr;
  }
  return p;
}

OMLDM_API void omldm_host_free_thp(void* p) {
  if (!p) return;
  hipHostUnregister(p);
  free(p);
}

// Registers an existing host allocation as pinned+mapped (for buffers not allocated pinned).
OMLDM_API int omldm_host_register(void* p, long long nbytes) {
  return (int)hipHostRegister(p, (size_t)nbytes, hipHostRegisterMapped);
}

// Copies nbytes from a pinned (device-mapped) host buffer to device memory by kernel.
// nseg (host src, device dst, bytes) segments in one launch (seg = 3 int64 each), about
// `blocks` workgroups in all. Host sources are mapped to their device addresses here.
OMLDM_API int omldm_pull_copy_segs(const long long* seg, int nseg, int blocks, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (blocks <= 0) blocks = 128;
  for (int base = 0; base < nseg; base += PullSegs::kMax) {
    const int cnt = nseg - base < PullSegs::kMax ? nseg - base : PullSegs::kMax;
    PullSegs d{};
    long long big = 0;
    for (int k = 0; k < cnt; ++k) {
      const long long* q = seg + 3 * (base + k);
      const void* src = reinterpret_cast<const void*>(q[0]);
      void* alias = nullptr;
      if (hipHostGetDevicePointer(&alias, const_cast<void*>(src), 0) == hipSuccess && alias)
        src = alias;
      if (((uintptr_t)src & 15) || (q[1] & 15)) return -1;
      d.src[k] = static_cast<const unsigned char*>(src);
      d.dst[k] = reinterpret_cast<unsigned char*>(q[1]);
      d.n[k] = q[2];
      big = q[2] > big ? q[2] : big;
    }
    if (!big) continue;
    int per = blocks / cnt;
    per = per < 1 ? 1 : per;
    hipLaunchKernelGGL(pull_copy_segs_kernel, dim3(per, cnt), dim3(256), 0, st, d);
  }
  return (int)hipGetLastError();
}

// 1: the default pull copy stores write-through (pull_copy_wt_kernel)
static int g_pull_wt = 1;
OMLDM_API void omldm_pull_copy_set_wt(int v) { g_pull_wt = v; }

OMLDM_API int omldm_pull_copy(const void* host_src, void* dst, long long nbytes, int blocks,
                              void* stream) {
  if (nbytes <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const void* src = host_src;
  void* dev_alias = nullptr;
  if (hipHostGetDevicePointer(&dev_alias, const_cast<void*>(host_src), 0) == hipSuccess && dev_alias)
    src = dev_alias;
  const long long n16 = nbytes / 16;
  if (((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) return -1;
  if (n16) {
    if (blocks <= 0) blocks = 1024;
    // blocks < 0 is not used; the high bits of `blocks` select the unroll depth:
    // blocks = nblk | (U << 16), U ∈ {8, 16} (default 4).
    const int U = blocks >> 16;
    const int nblk = blocks & 0xFFFF;
    if (U == 8)
      hipLaunchKernelGGL(pull_copy_u_kernel<8>, dim3(nblk), dim3(256), 0, st, (const u32x4*)src,
                         (u32x4*)dst, n16);
    else if (U == 16)
      hipLaunchKernelGGL(pull_copy_u_kernel<16>, dim3(nblk), dim3(256), 0, st,
                         (const u32x4*)src, (u32x4*)dst, n16);
    else if (g_pull_wt && n16 * 16 < (1LL << 31))
      hipLaunchKernelGGL(pull_copy_wt_kernel, dim3(nblk), dim3(256), 0, st, (const u32x4*)src,
                         (u32x4*)dst, n16);
    else
      hipLaunchKernelGGL(pull_copy_kernel, dim3(nblk), dim3(256), 0, st, (const u32x4*)src,
                         (u32x4*)dst, n16);
  }
  const long long tail = nbytes - n16 * 16;
  if (tail)
    hipLaunchKernelGGL(pull_tail_kernel, dim3(1), dim3(64), 0, st,
                       (const unsigned char*)src + n16 * 16, (unsigned char*)dst + n16 * 16,
                       tail);
  return (int)hipGetLastError();
}
