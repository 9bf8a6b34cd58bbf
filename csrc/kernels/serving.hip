// Low-latency forecasting: a persistent predict wavefront fed through a host mailbox.
//
// Reference path: forecasting record → FlinkSpoke → learner predict → Prediction side
// output → predictions topic (omldm/operators/spoke/FlinkSpoke.scala:105,
// omldm/network/FlinkNetwork.scala:250); its latency is a Flink task hop + JVM call.
// Here one resident wavefront polls a 256-byte request line in fine-grained (coherent),
// pinned host memory. Every poll is ONE wave-wide PCIe read of the whole line (lane l
// loads dword l): sequence number, checksum and the point itself — so a new request is
// picked up together with its payload in a single round trip instead of "read sequence,
// then read payload". The host writes the payload, then a position-mixed checksum keyed
// by the sequence, then the sequence (release); a torn read (new sequence, stale payload)
// fails the checksum and is simply re-polled. The wave scores the point against M models
// (same feature decoding as the training kernel) and publishes scores + the completion
// sequence with system-scope stores. No kernel launch or stream sync per request.
// cspan < 0: the request carries raw 32-bit category tokens (the binary wire), hashed by
// the wave itself (hash_dev.h) — the same hash as the training round.
//
// Model versions: the wave reads one of two weight banks, chosen per request by the
// request line's last dword (lane 63, covered by the checksum). The engine publishes each
// round's models into the bank no request is reading and switches requests to it once the
// publishing copy has completed (engine/forecast_server.py), so a prediction never sees a
// model that is half-way through an update.
//
// Safety: the wave exits on the stop word or after `lifetime_us` of wall time
// (s_memrealtime, 100 MHz), whichever comes first; every spin is bounded by it.
#include "common.h"
#include "hash_dev.h"

#include <chrono>
#include <cstdlib>
#include <cstring>

namespace omldm {

constexpr int kReqWords = 64;  // request line: [seq, csum, payload (dn + dc dwords), …, bank]
constexpr int kBankWord = kReqWords - 1;

struct alignas(256) Mailbox {
  unsigned int req[kReqWords];  // host → device (one 256-B line)
  unsigned int seq_done;        // device → host: last completed sequence number
  unsigned int stop;            // host → device: exit request
  unsigned int alive;           // device → host: 1 while the wave is polling
  unsigned int exit_reason;     // device → host: 1 stop word, 2 lifetime expired
  float result[60];             // scores of up to 60 models
  unsigned long long t_start, t_exit, t_end;  // diagnostics (100 MHz clock)
};

template <typename T>
__device__ __forceinline__ T sys_load(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ void sys_store(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ unsigned long long rt_now() {
  return __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
}

__host__ __device__ __forceinline__ uint32_t line_mix(uint32_t d, uint32_t pos) {
  uint32_t h = d + pos * 0x9E3779B9u;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}

template <typename WT, bool GROUPED>
__global__ __launch_bounds__(64) void serve_kernel(const WT* __restrict__ w0,
                                                   const WT* __restrict__ w1, long long wstride,
                                                   int M, int dn, int dc, int dim, int bias,
                                                   int cspan, Mailbox* mb,
                                                   unsigned long long lifetime_ticks) {
  const int lane = threadIdx.x;
  const int nf = dn + dc;
  const unsigned long long t_end = rt_now() + lifetime_ticks;
  unsigned int last = sys_load(&mb->req[0]);
  if (lane == 0) {
    sys_store(&mb->t_start, t_end - lifetime_ticks);
    sys_store(&mb->t_end, t_end);
    sys_store(&mb->alive, 1u);
  }
  int polls = 0;
  while (true) {
    const unsigned int d = sys_load(&mb->req[lane]);  // the whole line in one read
    const unsigned int seq = __builtin_amdgcn_readfirstlane(d);
    if (seq == last) {
      if (++polls >= 64) {  // re-check the clock / stop word every 64 polls
        polls = 0;
        bool quit = false;
        if (lane == 0) {
          const bool st = sys_load(&mb->stop) != 0u;
          const bool late = rt_now() > t_end;
          quit = st || late;
          if (quit) {
            sys_store(&mb->exit_reason, st ? 1u : 2u);
            sys_store(&mb->t_exit, rt_now());
          }
        }
        if (__builtin_amdgcn_readfirstlane(quit ? 1 : 0)) break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    // checksum over the payload lanes (position-mixed), keyed by the sequence
    const bool pl = (lane >= 2 && lane < 2 + nf) || lane == kBankWord;
    const uint32_t x = wave_xor(pl ? line_mix(d, (uint32_t)lane) : 0u) ^ line_mix(seq, 0u);
    const uint32_t csum = (uint32_t)__shfl((int)d, 1, 64);
    if (__builtin_amdgcn_readfirstlane(x == csum ? 1 : 0) == 0) continue;  // torn: re-poll
    const WT* __restrict__ w = __builtin_amdgcn_readlane((int)d, kBankWord) ? w1 : w0;
    // lane j ← payload dword j (feature j)
    const unsigned int fj = (unsigned int)__shfl((int)d, (lane + 2) & 63, 64);
    int idx = -1;
    float v = 0.f;
    const int j = lane;
    if (j == nf && bias) {
      idx = dim - 1;
      v = 1.f;
    } else if (j < dn) {
      idx = j;
      v = __uint_as_float(fj);
    } else if (j < nf) {
      const int c = (int)fj;
      if (cspan < 0) {  // raw binary wire: the 32-bit category token, hashed here
        const int code = hash_token_dev(fj, j - dn, dn, (uint32_t)((dim - dn - 1) / dc));
        if (code != -1) {
          idx = code & 0x7fffffff;
          v = code < 0 ? -1.f : 1.f;
        }
      } else if (cspan > 0) {
        const unsigned u = (unsigned)c & 0xFFFFu;
        if (u != 0xFFFFu) {
          idx = dn + (j - dn) * cspan + (int)(u & 0x7fffu);
          v = (u & 0x8000u) ? -1.f : 1.f;
        }
      } else if (c != -1) {
        idx = c & 0x7fffffff;
        v = c < 0 ? -1.f : 1.f;
      }
    }
    if ((unsigned)idx >= (unsigned)dim) {
      idx = -1;
      v = 0.f;
    }
    if constexpr (GROUPED) {
      // Models in groups of 16: the group's 16 gathers are issued back to back (one HBM
      // round trip per group, not per model), then reduced; lane m keeps model m's
      // score and the wave publishes all M scores with ONE wave-wide store.
      float mine = 0.f;
      for (int m0 = 0; m0 < M; m0 += 16) {
        float g[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
          g[k] = (idx >= 0 && m0 + k < M) ? to_f(w[(size_t)(m0 + k) * wstride + idx]) : 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          if (m0 + k < M) {  // wave-uniform: no reductions for absent models
            const float sk = wave_sum(v * g[k]);
            if (lane == m0 + k) mine = sk;
          }
        }
      }
      if (lane < M) sys_store(&mb->result[lane], mine);
    } else {  // one model: gather, reduce, lane 0 publishes
      for (int m = 0; m < M; ++m) {
        float acc = idx >= 0 ? v * to_f(w[(size_t)m * wstride + idx]) : 0.f;
        acc = wave_sum(acc);
        if (lane == 0) sys_store(&mb->result[m], acc);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (lane == 0) sys_store(&mb->seq_done, seq);
    last = seq;
    polls = 0;
  }
  if (lane == 0) sys_store(&mb->alive, 0u);
}

}  // namespace omldm

using namespace omldm;

OMLDM_API void* omldm_mailbox_alloc() {
  void* p = nullptr;
  if (hipHostMalloc(&p, sizeof(Mailbox), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return nullptr;
  memset(p, 0, sizeof(Mailbox));
  return p;
}

OMLDM_API void omldm_mailbox_free(void* p) {
  if (p) hipHostFree(p);
}

// w1: the second weight bank (nullptr: the requests' bank 1 reads w as well).
OMLDM_API int omldm_serve_start(const void* w, const void* w1, int w_bf16, long long wstride,
                                int M, int dn, int dc, int dim, int bias, int cspan,
                                void* mailbox, long long lifetime_us, void* stream) {
  if (M < 1 || M > 60 || dn + dc > kReqWords - 3 || dn + dc + (bias ? 1 : 0) > 64) return -2;
  if (w1 == nullptr) w1 = w;
  Mailbox* hmb = (Mailbox*)mailbox;
  void* dmb = nullptr;
  if (hipHostGetDevicePointer(&dmb, mailbox, 0) != hipSuccess || !dmb) return -3;
  __atomic_store_n(&hmb->stop, 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(&hmb->exit_reason, 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(&hmb->alive, 0u, __ATOMIC_SEQ_CST);
  const unsigned long long ticks = (unsigned long long)lifetime_us * 100ull;  // 100 MHz
  // grouped gathers for several models; OMLDM_SERVE_GROUPED=0/1 forces a variant (A/B)
  bool grouped = M > 1;
  if (const char* e = getenv("OMLDM_SERVE_GROUPED")) grouped = e[0] == '1';
  hipStream_t st = (hipStream_t)stream;
#define OMLDM_SERVE(WT, G)                                                                   \
  hipLaunchKernelGGL((serve_kernel<WT, G>), dim3(1), dim3(64), 0, st, (const WT*)w,          \
                     (const WT*)w1, wstride, M,                                               \
                     dn, dc, dim, bias, cspan, (Mailbox*)dmb, ticks)
  if (w_bf16) {
    if (grouped) OMLDM_SERVE(__hip_bfloat16, true);
    else OMLDM_SERVE(__hip_bfloat16, false);
  } else {
    if (grouped) OMLDM_SERVE(float, true);
    else OMLDM_SERVE(float, false);
  }
#undef OMLDM_SERVE
  return (int)hipGetLastError();
}

// Host side of one request: payload → checksum → sequence (release), then a bounded spin
// on the completion sequence; copies the M scores out. Returns 0, or -1 on timeout.
OMLDM_API int omldm_serve_request(void* mailbox, const float* num, int dn, const int* cat, int dc,
                                  int M, float* out, long long timeout_us, int bank) {
  Mailbox* mb = (Mailbox*)mailbox;
  const unsigned int seq = __atomic_load_n(&mb->req[0], __ATOMIC_RELAXED) + 1u;
  uint32_t x = line_mix(seq, 0u);
  for (int j = 0; j < dn; ++j) {
    uint32_t u;
    std::memcpy(&u, &num[j], 4);
    __atomic_store_n(&mb->req[2 + j], u, __ATOMIC_RELAXED);
    x ^= line_mix(u, (uint32_t)(2 + j));
  }
  for (int j = 0; j < dc; ++j) {
    const uint32_t u = (uint32_t)cat[j];
    __atomic_store_n(&mb->req[2 + dn + j], u, __ATOMIC_RELAXED);
    x ^= line_mix(u, (uint32_t)(2 + dn + j));
  }
  const uint32_t bk = bank ? 1u : 0u;
  __atomic_store_n(&mb->req[kBankWord], bk, __ATOMIC_RELAXED);
  x ^= line_mix(bk, (uint32_t)kBankWord);
  __atomic_store_n(&mb->req[1], x, __ATOMIC_RELAXED);
  __atomic_store_n(&mb->req[0], seq, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(&mb->seq_done, __ATOMIC_ACQUIRE) != seq) {
    if (std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() -
                                                              t0).count() > timeout_us)
      return -1;
  }
  for (int m = 0; m < M; ++m) out[m] = mb->result[m];
  return 0;
}

OMLDM_API void omldm_serve_stop(void* mailbox) {
  __atomic_store_n(&((Mailbox*)mailbox)->stop, 1u, __ATOMIC_SEQ_CST);
}

OMLDM_API void omldm_serve_times(void* mailbox, unsigned long long* out3) {
  const Mailbox* m = (const Mailbox*)mailbox;
  out3[0] = m->t_start;
  out3[1] = m->t_exit;
  out3[2] = m->t_end;
}

OMLDM_API int omldm_serve_exit_reason(void* mailbox) {
  return (int)__atomic_load_n(&((Mailbox*)mailbox)->exit_reason, __ATOMIC_ACQUIRE);
}

OMLDM_API int omldm_serve_alive(void* mailbox) {
  return (int)__atomic_load_n(&((Mailbox*)mailbox)->alive, __ATOMIC_ACQUIRE);
}

// The published-bank word of the native forecast lane (csrc/host/fcst_lane.cpp): a pinned
// coherent host word the GPU writes after a publish copy, in stream order
// (hipStreamWriteValue32), so the lane switches banks only once the copy has completed.
OMLDM_API void* omldm_bank_word_alloc() {
  void* p = nullptr;
  if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return nullptr;
  memset(p, 0, 64);
  return p;
}

OMLDM_API void omldm_bank_word_free(void* p) {
  if (p) hipHostFree(p);
}

OMLDM_API int omldm_bank_word_set(void* word, unsigned int v, void* stream) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, word, 0) != hipSuccess || !d) return -3;
  return (int)hipStreamWriteValue32((hipStream_t)stream, d, v, 0);
}
