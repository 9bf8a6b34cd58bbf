// Native forecast lane for file topics: poll → parse → serve → format → produce in a C++
// thread, outside the Python interpreter.
//
// Reference: a forecasting point reaching a spoke is predicted at once and its Prediction
// emitted right away (omldm/operators/spoke/FlinkSpoke.scala:101-105,
// omldm/network/FlinkNetwork.scala:243-257). engine/forecast_server.py's Python lane does
// the same per record but competes for the GIL with the tick thread (the driver measured
// its p50 / p99 doubling next to a busy tick). This thread touches no Python object: it
// preads the forecasting topic's partition logs from their byte offsets, parses each
// complete line with the same native parser as the tick (ingest.cpp), hands the features
// to the resident serving wave through its pinned mailbox (serving.hip's
// omldm_serve_request, passed in as a function pointer: this library does not link HIP),
// renders one Prediction line per served pipeline (egress.cpp) and appends them to a
// predictions partition with one write(2). The weight bank a request reads is a pinned
// word the GPU sets after a publish copy (hipStreamWriteValue32), so a request never reads
// a half-copied bank. Offsets are published after the record's Predictions are written
// (the checkpoint view: every record below an offset is answered).
//
// When the serving wave is down (not started yet, or its lifetime ended), the lane raises
// need_wave and waits; the Python supervisor (forecast_server.py) starts a wave and clears
// the flag. Per-stage nanoseconds (poll, parse, wave, format, produce) and each answered
// record's completion time (steady clock = CLOCK_MONOTONIC, Python's perf_counter) are kept
// for the bench.
#include <fcntl.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#define OMLDM_HOST_API extern "C" __attribute__((visibility("default")))

extern "C" int64_t omldm_parse_instances(const char* buf, const int64_t* off, int n, int dnum,
                                         int ddisc, int dc, int64_t dim, int cspan, float* num,
                                         void* cat, float* y, int8_t* op, int nthreads);
extern "C" int64_t omldm_format_predictions(const uint8_t* buf, const int64_t* starts,
                                            const int64_t* ends, int64_t n, int mlp_id,
                                            const float* preds, uint8_t* out, int64_t cap,
                                            int64_t* out_offs);

namespace {

using ServeFn = int (*)(void* mailbox, const float* num, int dn, const int* cat, int dc, int M,
                        float* out, long long timeout_us, int bank);
using AliveFn = int (*)(void* mailbox);

constexpr int kOpForecasting = 1;
constexpr int kStages = 6;  // poll, parse, wave, format, produce, record total
constexpr size_t kRing = 1 << 16;

inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Lane {
  // topics
  std::vector<int> in_fd;
  std::vector<std::atomic<int64_t>> offs;
  std::vector<int> out_fd;
  unsigned rr = 0;
  // parse geometry
  int dnum = 0, ddisc = 0, dc = 0, cspan = 0;
  int64_t dim = 0;
  // serving
  ServeFn serve = nullptr;
  AliveFn alive = nullptr;
  std::atomic<void*> mailbox{nullptr};
  int M = 0;  // the wave's models (scores out[0..M))
  std::vector<int> pids, rows, cls;  // served pipelines: id, score index, classification
  const volatile uint32_t* bank_word = nullptr;
  // control
  std::atomic<int> stop{0}, pause{0}, paused{0}, need_wave{0};
  std::thread th;
  // statistics (written by the lane thread; read racily by the host — monotone counters)
  std::atomic<uint64_t> served{0}, invalid{0}, failed{0};
  std::atomic<int64_t> stage_ns[kStages];
  std::vector<int64_t> tout = std::vector<int64_t>(kRing);
  std::vector<int64_t> lat = std::vector<int64_t>(kRing);  // poll → produced, per record
  std::mutex mu;
  std::condition_variable cv;

  Lane(int nin) : offs(nin) {
    for (auto& s : stage_ns) s.store(0);
  }
};

void add(std::atomic<int64_t>& a, int64_t v) { a.fetch_add(v, std::memory_order_relaxed); }

// One complete record line [rec, rec + len): returns false when the lane must stop (it was
// asked to while waiting for a wave).
bool process(Lane& L, const char* rec, int64_t len, std::vector<float>& num,
             std::vector<uint8_t>& cat, std::vector<int>& cat32, std::vector<float>& out,
             std::vector<uint8_t>& obuf, int64_t t_poll) {
  const int64_t t0 = now_ns();
  const int dn = L.dnum + L.ddisc;
  int64_t off[2] = {0, len};
  float y = 0.f;
  int8_t op = 0;
  std::fill(num.begin(), num.end(), 0.f);
  omldm_parse_instances(rec, off, 1, L.dnum, L.ddisc, L.dc, L.dim, L.cspan, num.data(),
                        cat.data(), &y, &op, 1);
  if (op != kOpForecasting) {
    L.invalid.fetch_add(1, std::memory_order_relaxed);
    return true;
  }
  if (L.cspan > 0) {
    const uint16_t* c16 = reinterpret_cast<const uint16_t*>(cat.data());
    for (int j = 0; j < L.dc; ++j) cat32[j] = (int)c16[j];
  } else {
    std::memcpy(cat32.data(), cat.data(), sizeof(int) * (size_t)L.dc);
  }
  const int64_t t1 = now_ns();
  for (;;) {  // the wave: a bounded request; a down wave is restarted by the supervisor
    void* mb = L.mailbox.load(std::memory_order_acquire);
    if (mb && L.alive(mb)) {
      const int bank = L.bank_word ? (int)(*L.bank_word & 1u) : 0;
      if (L.serve(mb, num.data(), dn, cat32.data(), L.dc, L.M, out.data(), 200000, bank) == 0)
        break;
    }
    L.need_wave.store(1, std::memory_order_release);
    while (L.need_wave.load(std::memory_order_acquire)) {
      if (L.stop.load(std::memory_order_relaxed)) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  const int64_t t2 = now_ns();
  int64_t starts = 0, ends = len, lo[2];
  size_t pos = 0;
  for (size_t i = 0; i < L.pids.size(); ++i) {
    const float s = out[(size_t)L.rows[i]];
    const float pred = L.cls[i] ? (s >= 0.f ? 1.f : -1.f) : s;
    for (;;) {
      const int64_t n = omldm_format_predictions(reinterpret_cast<const uint8_t*>(rec), &starts,
                                                 &ends, 1, L.pids[i], &pred, obuf.data() + pos,
                                                 (int64_t)(obuf.size() - pos), lo);
      if (n >= 0) {
        pos += (size_t)n;
        break;
      }
      obuf.resize(obuf.size() * 2 + (size_t)(-n));
    }
  }
  const int64_t t3 = now_ns();
  if (!L.out_fd.empty()) {
    const int fd = L.out_fd[L.rr++ % L.out_fd.size()];
    size_t done = 0;
    while (done < pos) {
      const ssize_t w = ::write(fd, obuf.data() + done, pos - done);
      if (w <= 0) {
        L.failed.fetch_add(1, std::memory_order_relaxed);
        break;
      }
      done += (size_t)w;
    }
  }
  const int64_t t4 = now_ns();
  add(L.stage_ns[0], t0 - t_poll);
  add(L.stage_ns[1], t1 - t0);
  add(L.stage_ns[2], t2 - t1);
  add(L.stage_ns[3], t3 - t2);
  add(L.stage_ns[4], t4 - t3);
  add(L.stage_ns[5], t4 - t_poll);
  const uint64_t k = L.served.load(std::memory_order_relaxed);
  L.tout[k % kRing] = t4;
  L.lat[k % kRing] = t4 - t_poll;
  L.served.store(k + 1, std::memory_order_release);
  return true;
}

void run(Lane* Lp) {
  Lane& L = *Lp;
  const int dn = L.dnum + L.ddisc;
  std::vector<float> num((size_t)std::max(dn, 1)), out((size_t)std::max(L.M, 1));
  std::vector<uint8_t> cat((size_t)std::max(L.dc, 1) * 4), obuf(1 << 14);
  std::vector<int> cat32((size_t)std::max(L.dc, 1));
  std::vector<char> rbuf(1 << 16);
  int64_t last = now_ns();
  while (!L.stop.load(std::memory_order_relaxed)) {
    if (L.pause.load(std::memory_order_acquire)) {
      L.paused.store(1, std::memory_order_release);
      std::this_thread::sleep_for(std::chrono::microseconds(50));
      continue;
    }
    L.paused.store(0, std::memory_order_release);
    bool any = false;
    for (size_t p = 0; p < L.in_fd.size(); ++p) {
      const int64_t t_poll = now_ns();
      const int64_t base = L.offs[p].load(std::memory_order_relaxed);
      const ssize_t n = ::pread(L.in_fd[p], rbuf.data(), rbuf.size(), base);
      if (n <= 0) continue;
      size_t pos = 0;
      for (;;) {
        const char* nl =
            static_cast<const char*>(std::memchr(rbuf.data() + pos, '\n', (size_t)n - pos));
        if (!nl) break;
        const int64_t len = nl - (rbuf.data() + pos);
        if (len > 0 && !process(L, rbuf.data() + pos, len, num, cat, cat32, out, obuf,
                                pos == 0 ? t_poll : now_ns()))
          return;
        pos += (size_t)len + 1;
        L.offs[p].store(base + (int64_t)pos, std::memory_order_release);
      }
      if (pos == 0 && (size_t)n == rbuf.size()) rbuf.resize(rbuf.size() * 2);  // a long line
      if (pos > 0) {
        any = true;
        std::lock_guard<std::mutex> g(L.mu);
        L.cv.notify_all();
      }
    }
    const int64_t t = now_ns();
    if (any) {
      last = t;
      continue;
    }
    // idle: spin for 2 ms after traffic, then short sleeps, then 1 ms sleeps once quiet
    const int64_t quiet = t - last;
    if (quiet < 2'000'000) continue;
    std::this_thread::sleep_for(std::chrono::microseconds(quiet < 50'000'000 ? 20 : 1000));
  }
}

}  // namespace

// in_fds[nin]: the forecasting partitions' logs (read), offs0[nin] their start offsets;
// out_fds[nout]: predictions partitions (O_APPEND). serve / alive: serving.hip's
// omldm_serve_request / omldm_serve_alive. M: the wave's models; pids / rows / cls [np]:
// the served pipelines (score index into the wave's output, classification → ±1).
// bank_word: pinned word holding the bank requests read (null: bank 0).
OMLDM_HOST_API void* omldm_fcst_lane_start(const int* in_fds, const int64_t* offs0, int nin,
                                           const int* out_fds, int nout, int dnum, int ddisc,
                                           int dc, int64_t dim, int cspan, void* serve,
                                           void* alive, int M, const int* pids, const int* rows,
                                           const int* cls, int np, const void* bank_word) {
  if (nin < 0 || nout < 0 || !serve || !alive || M < 1 || np < 0) return nullptr;
  Lane* L = new Lane(nin);
  for (int i = 0; i < nin; ++i) {
    L->in_fd.push_back(in_fds[i]);
    L->offs[i].store(offs0[i]);
  }
  for (int i = 0; i < nout; ++i) L->out_fd.push_back(out_fds[i]);
  L->dnum = dnum;
  L->ddisc = ddisc;
  L->dc = dc;
  L->dim = dim;
  L->cspan = cspan;
  L->serve = reinterpret_cast<ServeFn>(serve);
  L->alive = reinterpret_cast<AliveFn>(alive);
  L->M = M;
  for (int i = 0; i < np; ++i) {
    if (rows[i] < 0 || rows[i] >= M) {
      delete L;
      return nullptr;
    }
    L->pids.push_back(pids[i]);
    L->rows.push_back(rows[i]);
    L->cls.push_back(cls[i]);
  }
  L->bank_word = static_cast<const volatile uint32_t*>(bank_word);
  L->th = std::thread(run, L);
  return L;
}

OMLDM_HOST_API void omldm_fcst_lane_set_mailbox(void* lane, void* mailbox) {
  Lane* L = static_cast<Lane*>(lane);
  L->mailbox.store(mailbox, std::memory_order_release);
  L->need_wave.store(0, std::memory_order_release);
}

OMLDM_HOST_API int omldm_fcst_lane_need_wave(void* lane) {
  return static_cast<Lane*>(lane)->need_wave.load(std::memory_order_acquire);
}

// pause = 1: returns once the lane is between records (it answers nothing until resumed).
OMLDM_HOST_API int omldm_fcst_lane_pause(void* lane, int pause, long long timeout_us) {
  Lane* L = static_cast<Lane*>(lane);
  L->pause.store(pause ? 1 : 0, std::memory_order_release);
  if (!pause) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  while (!L->paused.load(std::memory_order_acquire)) {
    if (std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() -
                                                              t0).count() > timeout_us)
      return -1;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  return 0;
}

OMLDM_HOST_API void omldm_fcst_lane_offsets(void* lane, int64_t* out) {
  Lane* L = static_cast<Lane*>(lane);
  for (size_t i = 0; i < L->offs.size(); ++i) out[i] = L->offs[i].load(std::memory_order_acquire);
}

// stats[0..2] = served, invalid, failed writes; stats[3..8] = nanoseconds summed per stage
// (poll, parse, wave, format, produce, record total).
OMLDM_HOST_API void omldm_fcst_lane_stats(void* lane, int64_t* stats) {
  Lane* L = static_cast<Lane*>(lane);
  stats[0] = (int64_t)L->served.load(std::memory_order_acquire);
  stats[1] = (int64_t)L->invalid.load();
  stats[2] = (int64_t)L->failed.load();
  for (int s = 0; s < kStages; ++s) stats[3 + s] = L->stage_ns[s].load();
}

// Completion time (steady-clock ns) of answered record k (k < served, within the last 65536).
OMLDM_HOST_API int64_t omldm_fcst_lane_tout(void* lane, int64_t k) {
  Lane* L = static_cast<Lane*>(lane);
  return L->tout[(size_t)k % kRing];
}

// Blocks (no GIL held by the ctypes caller) until `served` reaches `count`; 0, or -1 on
// timeout.
OMLDM_HOST_API int omldm_fcst_lane_wait(void* lane, int64_t count, long long timeout_us) {
  Lane* L = static_cast<Lane*>(lane);
  const auto dl = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us);
  // spin briefly (sub-10 µs answers), then sleep on the condition variable
  for (int i = 0; i < 20000; ++i)
    if ((int64_t)L->served.load(std::memory_order_acquire) >= count) return 0;
  std::unique_lock<std::mutex> g(L->mu);
  while ((int64_t)L->served.load(std::memory_order_acquire) < count) {
    if (L->cv.wait_until(g, dl) == std::cv_status::timeout &&
        (int64_t)L->served.load(std::memory_order_acquire) < count)
      return -1;
  }
  return 0;
}

OMLDM_HOST_API int64_t omldm_fcst_lane_now_ns() { return now_ns(); }

// The last min(n, served, 65536) records' lane latencies (ns, first poll of the record's
// read → its Predictions written) into out; returns how many.
OMLDM_HOST_API int64_t omldm_fcst_lane_latencies(void* lane, int64_t* out, int64_t n) {
  Lane* L = static_cast<Lane*>(lane);
  const int64_t k = (int64_t)L->served.load(std::memory_order_acquire);
  const int64_t m = std::min<int64_t>({n, k, (int64_t)kRing});
  for (int64_t i = 0; i < m; ++i) out[i] = L->lat[(size_t)(k - m + i) % kRing];
  return m;
}

OMLDM_HOST_API void omldm_fcst_lane_stop(void* lane) {
  Lane* L = static_cast<Lane*>(lane);
  if (!L) return;
  L->stop.store(1, std::memory_order_release);
  if (L->th.joinable()) L->th.join();
  delete L;
}
