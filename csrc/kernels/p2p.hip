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

// ---------------------------------------------------------------------------------------
// Signal plane: the Asynchronous / SSP exchange with NO host message per push.
//
// The header plane above still sends a 4-int gloo header after every peer copy (a host
// thread per request). Here the control travels in HBM too: a worker's push is one kernel
// that writes δ straight into the hub's PUSH mailbox (peer stores over xGMI) and, from its
// last workgroup, releases the push word PUSHCTL[h][me] = (seq << 1) | final at system
// scope. The hub acquires the words at its next round (sig_hub_decide: one thread decides
// which pushes merge and which replies go out under the SSP bound), merges them and writes
// the replies into the workers' REPLY mailboxes in one pass (sig_hub_merge), and releases
// REPLYCTL[r][h] = the answered sequence. The worker's next step acquires its reply words
// (sig_worker_decide) and installs / pushes in one pass (sig_worker_apply). Every decision
// and every log entry (the deterministic replay's event order) is made on the device; the
// host launches four kernels per hub round and two per worker round, reads nothing back
// unless it must block (SSP, finalize), and has no thread per channel.
//
// Mailbox reads use system-scope loads (the writer is another agent, or another XCD of this
// one: a line this L2 cached at the previous round would be stale); writers end with a
// system-scope fence before the release store.
namespace omldm {
namespace sig {

enum : int {  // worker words
  W_SEQ = 0, W_INFLIGHT, W_INSTALL, W_PUSH, W_STATUS, W_NEV, W_INSTALLS, W_PUSHES, W_COUNT,
  W_FINAL,
  H_NMERGE = 16, H_NREPLY, H_MAXLEAD, H_COUNT, H_ANYM, H_ANYR, H_NDONE, H_PENDING, H_MLOG_N,
  H_RLOG_N,
  ARR = 32  // seen[G] done[G] answered[G] mnow[G] rnow[G]
};
enum : int { EV_STEP = 1, EV_INSTALL = 2, EV_PUSH = 3, EV_FINAL = 4 };
enum : int { M_STEP = 0, M_FINAL = 1, M_DRAIN = 2, M_RETRY = 4 };
constexpr int kMaxRanks = 64;

struct Args {
  long long* st;
  const long long* push_ctl;   // [G] on this hub: worker r's push word
  const long long* reply_ctl;  // [H] on this worker: hub h's reply word
  float* const* push_box;      // [G] hub: PUSH[me][r] (local)
  float* const* reply_box;     // [G] hub: REPLY[r][me] (peer)
  long long* const* reply_ctlp;  // [G] hub: &REPLYCTL[r][me] (peer)
  float* const* wpush_box;     // [H] worker: PUSH[h][me] (peer)
  long long* const* wpush_ctl;   // [H] worker: &PUSHCTL[h][me] (peer)
  const float* const* wreply_box;  // [H] worker: REPLY[me][h] (local)
  long long* evlog;
  long long* mlog;
  long long* rlog;
  long long cap;
  int G, H, me, s;  // s < 0: Asynchronous
};

__device__ inline long long ld_acq(const long long* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline float ld_sys(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void st_rel(long long* p, long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Every thread's stores reach memory, then the grid's last workgroup (counter) runs `tail`.
template <class F>
__device__ inline void last_block(long long* counter, F tail) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const long long old =
        __hip_atomic_fetch_add(counter, 1LL, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (long long)gridDim.x - 1) {
      tail();
      __hip_atomic_store(counter, 0LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ __launch_bounds__(64) void hub_decide_kernel(Args a) {
  if (threadIdx.x != 0) return;
  long long* st = a.st;
  const int G = a.G;
  long long* seen = st + ARR;
  long long* done = seen + G;
  long long* answered = done + G;
  long long* mnow = answered + G;
  long long* rnow = mnow + G;
  long long nm = st[H_NMERGE], anym = 0, anyr = 0;
  for (int r = 0; r < G; ++r) {
    const long long w = ld_acq(a.push_ctl + r);
    const long long sq = w >> 1;
    mnow[r] = 0;
    if (sq > seen[r]) {  // one push in flight per worker: sq == seen + 1
      mnow[r] = 1;
      anym = 1;
      seen[r] = sq;
      if (w & 1) done[r] = 1;
      const long long k = st[H_MLOG_N]++;
      if (k < a.cap) {
        a.mlog[2 * k] = r;
        a.mlog[2 * k + 1] = sq;
      }
      ++nm;
    }
  }
  long long mn = LLONG_MAX, mx = 0;
  for (int r = 0; r < G; ++r) {
    if (!done[r] && seen[r] < mn) mn = seen[r];
    if (seen[r] > mx) mx = seen[r];
  }
  if (mn == LLONG_MAX) mn = mx;
  long long ndone = 0, pend = 0;
  for (int r = 0; r < G; ++r) {
    rnow[r] = 0;
    if (answered[r] < seen[r]) {
      const long long lead = seen[r] - mn;
      if (a.s < 0 || done[r] || r == a.me || lead <= a.s) {
        rnow[r] = 1;
        anyr = 1;
        answered[r] = seen[r];
        st[H_NREPLY]++;
        if (r != a.me && !done[r] && lead > st[H_MAXLEAD]) st[H_MAXLEAD] = lead;
        const long long k = st[H_RLOG_N]++;
        if (k < a.cap) {
          a.rlog[2 * k] = r;
          a.rlog[2 * k + 1] = nm;
        }
      }
    }
    ndone += done[r];
    pend += answered[r] < seen[r];
  }
  st[H_NMERGE] = nm;
  st[H_ANYM] = anym;
  st[H_ANYR] = anyr;
  st[H_NDONE] = ndone;
  st[H_PENDING] = pend;
}

// glob += scale · Σ_r PUSH[me][r] (r ascending: the merge log's order), then glob → every
// REPLY[r][me] being answered, then (last workgroup) the reply words.
__global__ __launch_bounds__(256) void hub_merge_kernel(Args a, float* __restrict__ glob,
                                                        long long n, float scale) {
  const long long* st = a.st;
  if (!st[H_ANYM] && !st[H_ANYR]) return;
  __shared__ const float* mb[kMaxRanks];
  __shared__ float* rb[kMaxRanks];
  __shared__ int nm, nr;
  const int G = a.G;
  const long long* mnow = st + ARR + 3 * G;
  const long long* rnow = mnow + G;
  if (threadIdx.x == 0) {
    int i = 0, j = 0;
    for (int r = 0; r < G; ++r) {
      if (mnow[r]) mb[i++] = a.push_box[r];
      if (rnow[r]) rb[j++] = a.reply_box[r];
    }
    nm = i;
    nr = j;
  }
  __syncthreads();
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    float acc = glob[i];
    for (int k = 0; k < nm; ++k) acc = fmaf(scale, ld_sys(mb[k] + i), acc);
    if (nm) glob[i] = acc;
    for (int k = 0; k < nr; ++k) rb[k][i] = acc;
  }
  last_block(a.st + H_COUNT, [&] {
    const long long* answered = st + ARR + 2 * G;
    for (int r = 0; r < G; ++r)
      if (rnow[r]) st_rel(a.reply_ctlp[r], answered[r]);
  });
}

__device__ inline void log_ev(Args& a, long long code) {
  const long long k = a.st[W_NEV]++;
  if (k < a.cap) a.evlog[k] = code;
}

__global__ __launch_bounds__(64) void worker_decide_kernel(Args a, int mode) {
  if (threadIdx.x != 0) return;
  long long* st = a.st;
  const int kind = mode & 3;
  if (kind == M_STEP && !(mode & M_RETRY)) log_ev(a, EV_STEP);
  long long seq = st[W_SEQ], inflight = st[W_INFLIGHT], inst = 0, push = 0, blocked = 0;
  if (inflight) {
    bool in = true;
    for (int h = 0; h < a.H; ++h) in = in && ld_acq(a.reply_ctl + h) >= seq;
    if (in) {
      inst = 1;
      inflight = 0;
      st[W_INSTALLS]++;
      log_ev(a, EV_INSTALL);
    } else if (!(kind == M_STEP && a.s < 0)) {
      blocked = 1;  // SSP waits for the reply; finalize drains it
    }
  }
  if (!inflight && !blocked && kind != M_DRAIN) {
    bool ok = true;
    if (kind == M_STEP && a.s >= 0 && a.me < a.H) {  // a hub's own clock obeys the bound too
      const long long* seen = st + ARR;
      const long long* done = seen + a.G;
      long long mn = seq;
      for (int r = 0; r < a.G; ++r)
        if (r != a.me && !done[r] && seen[r] < mn) mn = seen[r];
      ok = seq - mn <= a.s;
    }
    if (ok) {
      ++seq;
      push = 1;
      inflight = 1;
      st[W_FINAL] = kind == M_FINAL;
      st[W_PUSHES]++;
      log_ev(a, kind == M_FINAL ? EV_FINAL : EV_PUSH);
    } else {
      blocked = 1;
    }
  }
  if (kind == M_DRAIN) blocked = inflight;
  st[W_SEQ] = seq;
  st[W_INFLIGHT] = inflight;
  st[W_INSTALL] = inst;
  st[W_PUSH] = push;
  st[W_STATUS] = blocked;
}

// Per hub shard h: install x = g + (x − xpush), base = g from REPLY[me][h]; push
// δ = x − base into PUSH[h][me], xpush = x; then (last workgroup) the push words.
__global__ __launch_bounds__(256) void worker_apply_kernel(Args a, float* __restrict__ x,
                                                           float* __restrict__ xpush,
                                                           float* __restrict__ base, long long n,
                                                           long long step) {
  const long long* st = a.st;
  const bool inst = st[W_INSTALL] != 0, push = st[W_PUSH] != 0;
  if (!inst && !push) return;
  for (int h = 0; h < a.H; ++h) {
    const long long lo = (long long)h * step, hi = lo + step < n ? lo + step : n;
    const float* rb = a.wreply_box[h];
    float* pb = a.wpush_box[h];
    for (long long i = lo + (long long)blockIdx.x * 256 + threadIdx.x; i < hi;
         i += (long long)gridDim.x * 256) {
      float xv = x[i], bv;
      if (inst) {
        const float g = ld_sys(rb + (i - lo));
        xv = g + (xv - xpush[i]);
        x[i] = xv;
        base[i] = g;
        bv = g;
      } else {
        bv = base[i];
      }
      if (push) {
        xpush[i] = xv;
        pb[i - lo] = xv - bv;
      }
    }
  }
  last_block(a.st + W_COUNT, [&] {
    if (push) {
      const long long w = (st[W_SEQ] << 1) | (st[W_FINAL] ? 1 : 0);
      for (int h = 0; h < a.H; ++h) st_rel(a.wpush_ctl[h], w);
    }
  });
}

int grid_big(long long n) {
  long long b = (n + 255) / 256;
  b = b > 1024 ? 1024 : b;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace sig
}  // namespace omldm

// ptrs: device int64[3G + 3H] = push_box[G] reply_box[G] reply_ctlp[G] wpush_box[H]
// wpush_ctl[H] wreply_box[H]; ctl: this rank's IPC control words, PUSHCTL[G] then
// REPLYCTL[H]. Returns a host handle (omldm_sig_destroy frees it).
OMLDM_API void* omldm_sig_create(long long* st, long long* ctl, long long* ptrs,
                                 long long* evlog, long long* mlog, long long* rlog,
                                 long long cap, int G, int H, int me, int s) {
  if (G < 1 || G > sig::kMaxRanks || H < 1 || H > G || me < 0 || me >= G) return nullptr;
  auto* a = new sig::Args;
  a->st = st;
  a->push_ctl = ctl;
  a->reply_ctl = ctl + G;
  a->push_box = reinterpret_cast<float* const*>(ptrs);
  a->reply_box = reinterpret_cast<float* const*>(ptrs + G);
  a->reply_ctlp = reinterpret_cast<long long* const*>(ptrs + 2 * G);
  a->wpush_box = reinterpret_cast<float* const*>(ptrs + 3 * G);
  a->wpush_ctl = reinterpret_cast<long long* const*>(ptrs + 3 * G + H);
  a->wreply_box = reinterpret_cast<const float* const*>(ptrs + 3 * G + 2 * H);
  a->evlog = evlog;
  a->mlog = mlog;
  a->rlog = rlog;
  a->cap = cap;
  a->G = G;
  a->H = H;
  a->me = me;
  a->s = s;
  return a;
}

OMLDM_API void omldm_sig_destroy(void* h) { delete static_cast<sig::Args*>(h); }

OMLDM_API int omldm_sig_state_words(int G) { return sig::ARR + 5 * G; }

// Hub round: acquire the push words, merge, reply (two launches, no host read).
OMLDM_API int omldm_sig_hub(void* h, float* glob, long long n, float scale, void* stream) {
  const sig::Args& a = *static_cast<sig::Args*>(h);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sig::hub_decide_kernel, dim3(1), dim3(64), 0, s, a);
  hipLaunchKernelGGL(sig::hub_merge_kernel, dim3(sig::grid_big(n)), dim3(256), 0, s, a, glob,
                     n, scale);
  return (int)hipGetLastError();
}

// Worker round: decide (mode: 0 step, 1 final, 2 drain; +4 retry) and install / push.
OMLDM_API int omldm_sig_worker(void* h, int mode, float* x, float* xpush, float* base,
                               long long n, long long step, void* stream) {
  const sig::Args& a = *static_cast<sig::Args*>(h);
  if (step <= 0 || (long long)a.H * step < n) return -1;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sig::worker_decide_kernel, dim3(1), dim3(64), 0, s, a, mode);
  hipLaunchKernelGGL(sig::worker_apply_kernel, dim3(sig::grid_big(step)), dim3(256), 0, s, a,
                     x, xpush, base, n, step);
  return (int)hipGetLastError();
}
