// Native asynchronous H2D copy engine (ingest runtime component).
//
// Measured on MI355X (profiles/round1_ablation.md): a large hipMemcpyAsync from pinned
// memory keeps the *calling host thread* busy for roughly the transfer time, so issuing
// it from the training loop serialises host enqueue with PCIe and kills copy/compute
// overlap, while a copy *kernel* competes with the training kernels for CUs. This engine
// moves the SDMA submission to its own host thread: the training thread enqueues a copy
// request (dst, src, bytes, "buffer free" event) and continues launching kernels; the
// engine thread makes its streams wait for the buffer-free event, splits the copy over
// `nstreams` streams (several SDMA queues), joins them and records the "copied" event.
// The training thread later makes its compute stream wait for that event on the GPU
// (omldm_copy_engine_stream_wait), so no host thread ever waits for PCIe except the
// engine's own.
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"

namespace omldm {

struct CopyJob {
  void* dst;
  const void* src;
  size_t n;
  hipEvent_t wait;  // may be null: GPU-side precondition (destination buffer free)
  hipEvent_t done;  // recorded after the whole copy
  uint64_t ticket;
};

struct CopyEngine {
  std::vector<hipStream_t> streams;
  std::vector<hipEvent_t> joins;
  std::thread th;
  std::mutex m;
  std::condition_variable cv, cv_done;
  std::deque<CopyJob> q;
  uint64_t submitted = 0, issued = 0;
  int err = 0;
  bool stop = false;
  int device = 0;

  void run() {
    hipSetDevice(device);
    for (;;) {
      CopyJob j;
      {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return stop || !q.empty(); });
        if (q.empty()) return;
        j = q.front();
        q.pop_front();
      }
      int e = 0;
      const int k = (int)streams.size();
      const size_t chunk = ((j.n + k - 1) / k + 255) & ~(size_t)255;
      for (int s = 0; s < k; ++s) {
        const size_t off = (size_t)s * chunk;
        if (off >= j.n) break;
        const size_t len = j.n - off < chunk ? j.n - off : chunk;
        if (j.wait) e |= (int)hipStreamWaitEvent(streams[s], j.wait, 0);
        e |= (int)hipMemcpyAsync((char*)j.dst + off, (const char*)j.src + off, len,
                                 hipMemcpyHostToDevice, streams[s]);
        if (s > 0) {
          e |= (int)hipEventRecord(joins[s], streams[s]);
          e |= (int)hipStreamWaitEvent(streams[0], joins[s], 0);
        }
      }
      e |= (int)hipEventRecord(j.done, streams[0]);
      {
        std::lock_guard<std::mutex> lk(m);
        issued = j.ticket;
        if (e && !err) err = e;
      }
      cv_done.notify_all();
    }
  }
};

}  // namespace omldm

using namespace omldm;

OMLDM_API void* omldm_copy_engine_create(int nstreams) {
  auto* e = new CopyEngine();
  if (nstreams < 1) nstreams = 1;
  hipGetDevice(&e->device);
  for (int i = 0; i < nstreams; ++i) {
    hipStream_t s;
    hipEvent_t ev;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      delete e;
      return nullptr;
    }
    e->streams.push_back(s);
    e->joins.push_back(ev);
  }
  e->th = std::thread([e] { e->run(); });
  return e;
}

OMLDM_API void omldm_copy_engine_destroy(void* p) {
  auto* e = (CopyEngine*)p;
  {
    std::lock_guard<std::mutex> lk(e->m);
    e->stop = true;
  }
  e->cv.notify_all();
  e->th.join();
  for (auto s : e->streams) hipStreamSynchronize(s);
  for (auto s : e->streams) hipStreamDestroy(s);
  for (auto ev : e->joins) hipEventDestroy(ev);
  delete e;
}

OMLDM_API void* omldm_event_create() {
  hipEvent_t ev;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return nullptr;
  return (void*)ev;
}

OMLDM_API int omldm_event_destroy(void* ev) { return (int)hipEventDestroy((hipEvent_t)ev); }

OMLDM_API int omldm_event_record(void* ev, void* stream) {
  return (int)hipEventRecord((hipEvent_t)ev, (hipStream_t)stream);
}

// Enqueue a copy; returns its ticket (> 0).
OMLDM_API unsigned long long omldm_copy_engine_submit(void* p, void* dst, const void* src,
                                                      long long n, void* wait_event,
                                                      void* done_event) {
  auto* e = (CopyEngine*)p;
  uint64_t t;
  {
    std::lock_guard<std::mutex> lk(e->m);
    t = ++e->submitted;
    e->q.push_back(CopyJob{dst, src, (size_t)n, (hipEvent_t)wait_event, (hipEvent_t)done_event, t});
  }
  e->cv.notify_one();
  return t;
}

// Make `stream` wait (on the GPU) for the copy with this ticket: blocks the host only until
// the engine thread has *issued* that copy (its done event recorded), not until PCIe is done.
OMLDM_API int omldm_copy_engine_stream_wait(void* p, unsigned long long ticket, void* done_event,
                                            void* stream) {
  auto* e = (CopyEngine*)p;
  {
    std::unique_lock<std::mutex> lk(e->m);
    e->cv_done.wait(lk, [&] { return e->issued >= ticket; });
    if (e->err) return e->err;
  }
  return (int)hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)done_event, 0);
}
