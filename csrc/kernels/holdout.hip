// Holdout routing of a training micro-batch, on the device.
//
// Reference (omldm/operators/spoke/FlinkSpoke.scala:95-104): a counter runs 0..9 over
// the training points; points 8 and 9 of every ten go to a FIFO test set of
// testSetSize; when the FIFO is full, the point it evicts is trained on instead.
//
// For a micro-batch of B training rows with the counter at c (0..9) the held rows are
// the ones with (i + c) % 10 >= 8 — pure index arithmetic, so the host passes only
// scalars (engine/holdout.py) and two kernels do the data movement:
//   gather : out = [non-held batch rows] ++ [ring rows (r1 + k) % size, k < n1]
//                  ++ [held batch rows of hold-ordinal s2 + k, k < n2]
//   scatter: ring[(rw + k) % size] = held batch row of hold-ordinal hs + k, k < ns
// The gather runs first on the stream, so evicted ring rows are read before the
// scatter overwrites them. One thread per (row, column) of the row layout
// num[dn] | cat[dc] | y: element sizes are runtime (fp32/bf16 num, int16/int32 cat).
#include "common.h"

namespace omldm {
namespace {

// i-th batch row of the non-held / held subsequence, counter at c.
__host__ __device__ __forceinline__ long long nonheld_row(long long r, int c) {
  const long long q = (c < 8 ? c : 8) + r;
  return (q / 8) * 10 + (q % 8) - c;
}
__host__ __device__ __forceinline__ long long held_row(long long r, int c) {
  const long long q = (c > 8 ? c - 8 : 0) + r;
  return (q / 2) * 10 + 8 + (q % 2) - c;
}

struct Rows {
  const unsigned char* num;
  const unsigned char* cat;
  const float* y;
};
struct RowsOut {
  unsigned char* num;
  unsigned char* cat;
  float* y;
};

__device__ __forceinline__ void copy_col(const Rows& s, long long si, const RowsOut& d,
                                         long long di, int col, int dn, int dc, int nes,
                                         int ces) {
  if (col < dn) {
    if (nes == 4)
      reinterpret_cast<float*>(d.num)[di * dn + col] =
          reinterpret_cast<const float*>(s.num)[si * dn + col];
    else
      reinterpret_cast<unsigned short*>(d.num)[di * dn + col] =
          reinterpret_cast<const unsigned short*>(s.num)[si * dn + col];
  } else if (col < dn + dc) {
    const int k = col - dn;
    if (ces == 4)
      reinterpret_cast<int*>(d.cat)[di * dc + k] = reinterpret_cast<const int*>(s.cat)[si * dc + k];
    else
      reinterpret_cast<unsigned short*>(d.cat)[di * dc + k] =
          reinterpret_cast<const unsigned short*>(s.cat)[si * dc + k];
  } else {
    d.y[di] = s.y[si];
  }
}

__global__ __launch_bounds__(256) void holdout_gather_kernel(
    Rows batch, Rows ring, RowsOut out, int c, long long n0, long long n1, long long r1,
    long long n2, long long s2, int size, int dn, int dc, int nes, int ces) {
  const int cols = dn + dc + 1;
  const long long total = (n0 + n1 + n2) * cols;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (long long)gridDim.x * 256) {
    const long long row = t / cols;
    const int col = (int)(t - row * cols);
    if (row < n0) {
      copy_col(batch, nonheld_row(row, c), out, row, col, dn, dc, nes, ces);
    } else if (row < n0 + n1) {
      copy_col(ring, (r1 + (row - n0)) % size, out, row, col, dn, dc, nes, ces);
    } else {
      copy_col(batch, held_row(s2 + (row - n0 - n1), c), out, row, col, dn, dc, nes, ces);
    }
  }
}

__global__ __launch_bounds__(256) void holdout_scatter_kernel(
    Rows batch, RowsOut ring, int c, long long ns, long long hs, long long rw, int size, int dn,
    int dc, int nes, int ces) {
  const int cols = dn + dc + 1;
  const long long total = ns * cols;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (long long)gridDim.x * 256) {
    const long long k = t / cols;
    const int col = (int)(t - k * cols);
    copy_col(batch, held_row(hs + k, c), ring, (rw + k) % size, col, dn, dc, nes, ces);
  }
}

int grid_for(long long work) {
  long long b = (work + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace
}  // namespace omldm

using namespace omldm;

// All pointers are device pointers. Batch: B rows; ring: `size` rows; out: n0+n1+n2 rows.
// Index ranges are validated on the host (engine/holdout.py) and re-checked here.
OMLDM_API int omldm_holdout_route(const void* bnum, const void* bcat, const float* by,
                                  long long B, void* rnum, void* rcat, float* ry, int size,
                                  void* onum, void* ocat, float* oy, int c, long long n0,
                                  long long n1, long long r1, long long n2, long long s2,
                                  long long ns, long long hs, long long rw, int dn, int dc,
                                  int nes, int ces, void* stream) {
  if (c < 0 || c > 9 || size < 0 || (nes != 2 && nes != 4) || (ces != 2 && ces != 4)) return -1;
  if ((n1 || ns) && size <= 0) return -1;
  // every batch row touched must exist: the last non-held / held rows of the ranges
  if (n0 > 0 && nonheld_row(n0 - 1, c) >= B) return -2;
  if (n2 > 0 && held_row(s2 + n2 - 1, c) >= B) return -2;
  if (ns > 0 && held_row(hs + ns - 1, c) >= B) return -2;
  if (n1 > 0 && (r1 < 0 || n1 > size)) return -2;
  if (ns > size || rw < 0) return -2;
  hipStream_t st = (hipStream_t)stream;
  Rows batch{(const unsigned char*)bnum, (const unsigned char*)bcat, by};
  Rows ring{(const unsigned char*)rnum, (const unsigned char*)rcat, ry};
  RowsOut out{(unsigned char*)onum, (unsigned char*)ocat, oy};
  RowsOut ringw{(unsigned char*)rnum, (unsigned char*)rcat, ry};
  const int cols = dn + dc + 1;
  const long long g = (n0 + n1 + n2) * cols;
  if (g > 0)
    hipLaunchKernelGGL(holdout_gather_kernel, dim3(grid_for(g)), dim3(256), 0, st, batch, ring,
                       out, c, n0, n1, r1, n2, s2, size, dn, dc, nes, ces);
  if (ns > 0)
    hipLaunchKernelGGL(holdout_scatter_kernel, dim3(grid_for(ns * cols)), dim3(256), 0, st,
                       batch, ringw, c, ns, hs, rw, size, dn, dc, nes, ces);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ per-spoke rings
// Every virtual spoke owns its own counter and FIFO ring (FlinkSpoke.scala:41,95-104):
// spoke s receives batch rows [b0, b0 + Bs) and its ring is rows [s·size, (s+1)·size) of
// the ring arrays. The host computes one descriptor per spoke (engine/holdout.py:
// SpokeRoute); out is spoke-major, spoke s's rows from o0 on:
//   [non-held rows] ++ [evicted ring rows] ++ [held rows that never fit the ring].
namespace omldm {
namespace {
struct SpokeDesc {
  long long b0, n0, n1, r1, n2, s2, ns, hs, rw, o0;
  long long c;  // counter 0..9
  long long pad;
};
static_assert(sizeof(SpokeDesc) == 12 * 8, "descriptor layout is shared with the host");

__device__ __forceinline__ Rows shift_rows(const Rows& r, long long rows, int dn, int dc,
                                           int nes, int ces) {
  return Rows{r.num + rows * dn * nes, r.cat + rows * dc * ces, r.y + rows};
}
__device__ __forceinline__ RowsOut shift_rows(const RowsOut& r, long long rows, int dn, int dc,
                                              int nes, int ces) {
  return RowsOut{r.num + rows * dn * nes, r.cat + rows * dc * ces, r.y + rows};
}

// grid (x, S): block row y serves spoke y
__global__ __launch_bounds__(256) void holdout_gather_spokes_kernel(
    Rows batch, Rows ring, RowsOut out, const SpokeDesc* __restrict__ desc, int size, int dn,
    int dc, int nes, int ces) {
  const SpokeDesc d = desc[blockIdx.y];
  const int cols = dn + dc + 1;
  const long long total = (d.n0 + d.n1 + d.n2) * cols;
  const int c = (int)d.c;
  const Rows b = shift_rows(batch, d.b0, dn, dc, nes, ces);
  const Rows rg = shift_rows(ring, (long long)blockIdx.y * size, dn, dc, nes, ces);
  const RowsOut o = shift_rows(out, d.o0, dn, dc, nes, ces);
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (long long)gridDim.x * 256) {
    const long long row = t / cols;
    const int col = (int)(t - row * cols);
    if (row < d.n0)
      copy_col(b, nonheld_row(row, c), o, row, col, dn, dc, nes, ces);
    else if (row < d.n0 + d.n1)
      copy_col(rg, (d.r1 + (row - d.n0)) % size, o, row, col, dn, dc, nes, ces);
    else
      copy_col(b, held_row(d.s2 + (row - d.n0 - d.n1), c), o, row, col, dn, dc, nes, ces);
  }
}

__global__ __launch_bounds__(256) void holdout_scatter_spokes_kernel(
    Rows batch, RowsOut ring, const SpokeDesc* __restrict__ desc, int size, int dn, int dc,
    int nes, int ces) {
  const SpokeDesc d = desc[blockIdx.y];
  const int cols = dn + dc + 1;
  const long long total = d.ns * cols;
  const int c = (int)d.c;
  const Rows b = shift_rows(batch, d.b0, dn, dc, nes, ces);
  const RowsOut rg = shift_rows(ring, (long long)blockIdx.y * size, dn, dc, nes, ces);
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (long long)gridDim.x * 256) {
    const long long k = t / cols;
    const int col = (int)(t - k * cols);
    copy_col(b, held_row(d.hs + k, c), rg, (d.rw + k) % size, col, dn, dc, nes, ces);
  }
}
}  // namespace
}  // namespace omldm

// desc_host: S descriptors (validated here against B / size / the output length), desc_dev:
// their device copy (the caller uploads them on `stream` before this call). max_rows: the
// largest per-spoke gather length (sizes the grid).
OMLDM_API int omldm_holdout_route_spokes(const void* bnum, const void* bcat, const float* by,
                                         long long B, void* rnum, void* rcat, float* ry,
                                         int size, int S, void* onum, void* ocat, float* oy,
                                         long long n_out, const long long* desc_host,
                                         const void* desc_dev, int dn, int dc, int nes, int ces,
                                         void* stream) {
  if (S <= 0 || size <= 0 || (nes != 2 && nes != 4) || (ces != 2 && ces != 4)) return -1;
  long long gmax = 0, smax = 0, o = 0;
  for (int s = 0; s < S; ++s) {
    const long long* d = desc_host + 12 * s;
    const long long b0 = d[0], n0 = d[1], n1 = d[2], r1 = d[3], n2 = d[4], s2 = d[5], ns = d[6],
                    hs = d[7], rw = d[8], o0 = d[9], c = d[10];
    if (c < 0 || c > 9 || b0 < 0 || o0 != o) return -2;
    if (n0 > 0 && b0 + nonheld_row(n0 - 1, (int)c) >= B) return -2;
    if (n2 > 0 && b0 + held_row(s2 + n2 - 1, (int)c) >= B) return -2;
    if (ns > 0 && b0 + held_row(hs + ns - 1, (int)c) >= B) return -2;
    if (n1 < 0 || n1 > size || r1 < 0 || ns < 0 || ns > size || rw < 0) return -2;
    o += n0 + n1 + n2;
    gmax = gmax > n0 + n1 + n2 ? gmax : n0 + n1 + n2;
    smax = smax > ns ? smax : ns;
  }
  if (o != n_out) return -2;
  hipStream_t st = (hipStream_t)stream;
  const SpokeDesc* dd = (const SpokeDesc*)desc_dev;
  Rows batch{(const unsigned char*)bnum, (const unsigned char*)bcat, by};
  Rows ring{(const unsigned char*)rnum, (const unsigned char*)rcat, ry};
  RowsOut out{(unsigned char*)onum, (unsigned char*)ocat, oy};
  RowsOut ringw{(unsigned char*)rnum, (unsigned char*)rcat, ry};
  const int cols = dn + dc + 1;
  auto gx = [](long long work) {
    long long b = (work + 255) / 256;
    b = b > 1024 ? 1024 : b;
    return (unsigned)(b < 1 ? 1 : b);
  };
  if (gmax > 0)
    hipLaunchKernelGGL(holdout_gather_spokes_kernel, dim3(gx(gmax * cols), S), dim3(256), 0, st,
                       batch, ring, out, dd, size, dn, dc, nes, ces);
  if (smax > 0)
    hipLaunchKernelGGL(holdout_scatter_spokes_kernel, dim3(gx(smax * cols), S), dim3(256), 0, st,
                       batch, ringw, dd, size, dn, dc, nes, ces);
  return (int)hipGetLastError();
}
