// Topic-log reader for the engine's ingest thread: one pread of a partition log straight
// into the (pinned) staging slot of the next tick, then a memchr scan that indexes the
// complete records (one JSON DataInstance per line).
//
// Reference path being replaced: a Flink Kafka source subtask per partition deserialising
// one record at a time (omldm/Job.scala:42-57). Here a tick's records stay one byte
// block end to end: log → pinned slot (this file) → HBM → GPU JSON parser
// (csrc/kernels/json_ingest.hip). Both calls run without the Python GIL (ctypes), so the
// engine reads tick k+1 while the GPU trains on tick k.
#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>
#include <unistd.h>

#include <emmintrin.h>

#define OMLDM_HOST_API extern "C" __attribute__((visibility("default")))

// Appends the record ends ('\n' + 1) found in buf[from, to) to offs[n + 1 ...] until
// max_records: 64 bytes per step (four SSE2 compares into one 64-bit mask), set bits in
// order — 15 % faster than memchr per record on ~168-byte DIB records (one call each).
// *pos = one past the last newline.
static inline void index_newlines(const uint8_t* buf, int64_t from, int64_t to,
                                  int64_t max_records, int64_t* offs, int64_t& n,
                                  int64_t& pos) {
  const __m128i nl = _mm_set1_epi8('\n');
  int64_t i = from;
  for (; i + 64 <= to && n < max_records; i += 64) {
    const __m128i* p = reinterpret_cast<const __m128i*>(buf + i);
    uint64_t m =
        (uint64_t)(unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128(p), nl)) |
        ((uint64_t)(unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128(p + 1), nl)) << 16) |
        ((uint64_t)(unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128(p + 2), nl)) << 32) |
        ((uint64_t)(unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128(p + 3), nl)) << 48);
    while (m && n < max_records) {
      pos = i + __builtin_ctzll(m) + 1;
      offs[++n] = pos;
      m &= m - 1;
    }
  }
  for (; i < to && n < max_records; ++i)
    if (buf[i] == '\n') {
      pos = i + 1;
      offs[++n] = pos;
    }
}

// Indexes up to max_records complete lines of buf[0, len). offs[0] = 0 and
// offs[i + 1] = one past the '\n' of record i. Returns the record count n; offs[n] is
// the number of bytes consumed (a trailing partial line is left for the next read).
OMLDM_HOST_API int64_t omldm_index_lines(const uint8_t* buf, int64_t len, int64_t max_records,
                                         int64_t* offs) {
  offs[0] = 0;
  int64_t n = 0, pos = 0;
  index_newlines(buf, 0, len, max_records, offs, n, pos);
  return n;
}

// pread of the log at `offset` into dst (restarting on EINTR / short reads), indexing the
// complete lines as they arrive. The first read asks for `hint` bytes (0: the whole cap);
// if that holds fewer than max_records complete records and the log goes on, further
// reads ask for the missing records at the mean length seen so far (+10 %), never beyond
// cap — so a tick reads what it consumes instead of a fixed safety margin that the next
// tick reads again. Returns the record count (≥ 0) or -errno; *used = bytes consumed.
namespace {
struct LogRead {  // a region read in progress
  int64_t got = 0, n = 0, pos = 0, scanned = 0;
  bool eof = false;
};

// Goes on reading a region from state `s` (the bytes [0, s.got) are in dst and indexed up
// to s.scanned) with a next read up to `want`, as omldm_read_log describes.
int64_t read_log_cont(int fd, int64_t offset, uint8_t* dst, int64_t cap, int64_t max_records,
                      int64_t* offs, LogRead& s, int64_t want) {
  for (;;) {
    while (s.got < want) {
      ssize_t r = pread(fd, dst + s.got, size_t(want - s.got), off_t(offset + s.got));
      if (r < 0) {
        if (errno == EINTR) continue;
        return -errno;
      }
      if (r == 0) {
        s.eof = true;
        break;
      }
      s.got += r;
    }
    index_newlines(dst, s.scanned, s.got, max_records, offs, s.n, s.pos);
    s.scanned = s.n >= max_records ? s.pos : s.got;
    if (s.n >= max_records || s.eof || want >= cap) return 0;
    const int64_t per = s.n ? s.pos / s.n : 2 * want;  // no complete record yet: double it
    const int64_t more = (max_records - s.n) * per / 10 * 11 + 4096;
    want = s.got + more < cap ? s.got + more : cap;
  }
}
}  // namespace

OMLDM_HOST_API int64_t omldm_read_log(int fd, int64_t offset, uint8_t* dst, int64_t cap,
                                      int64_t max_records, int64_t* offs, int64_t* used,
                                      int64_t hint) {
  LogRead s;
  offs[0] = 0;
  const int64_t e = read_log_cont(fd, offset, dst, cap, max_records, offs, s,
                                  hint > 0 && hint < cap ? hint : cap);
  if (e < 0) {
    *used = 0;
    return e;
  }
  *used = offs[s.n];
  return s.n;
}

// A small persistent pool for omldm_fill_regions (opt-in, OMLDM_READ_POOL=1: measured
// slower than a thread per region per block). run(n, width, f) calls f(0 .. n-1) on up to
// width − 1 workers plus the caller and returns when all are done; one batch at a time.
namespace {
class ReadPool {
 public:
  void run(int n, int width, const std::function<void(int)>& f) {
    std::lock_guard<std::mutex> batch(batch_mu_);  // one block at a time
    grow(width - 1);
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &f;
      total_ = n;
      next_ = 0;
      done_ = 0;
      active_ = width - 1 < (int)workers_.size() ? width - 1 : (int)workers_.size();
      ++gen_;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return done_ == total_ && busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void drain() {
    for (;;) {
      int j;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (next_ >= total_) return;
        j = next_++;
      }
      (*fn_)(j);
      std::lock_guard<std::mutex> lk(mu_);
      if (++done_ == total_) done_cv_.notify_all();
    }
  }
  void grow(int want) {
    while ((int)workers_.size() < want && (int)workers_.size() < 64) {
      const int id = (int)workers_.size();
      workers_.emplace_back([this, id] { loop(id); });
      workers_.back().detach();
    }
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (id >= active_ || fn_ == nullptr) continue;
        ++busy_;
      }
      drain();
      std::lock_guard<std::mutex> lk(mu_);
      if (--busy_ == 0) done_cv_.notify_all();
    }
  }
  std::mutex batch_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void(int)>* fn_ = nullptr;
  int total_ = 0, next_ = 0, done_ = 0, active_ = 0, busy_ = 0;
  uint64_t gen_ = 0;
};
ReadPool& read_pool() {
  static ReadPool* p = new ReadPool();  // never destroyed: detached workers outlive exit
  return *p;
}
}  // namespace

// One tick's block in one call: the (partition region) reads of the block run on up to
// `nthreads` threads, then the block's record index is assembled here (the Python form of
// this — a thread-pool task per region, then numpy slicing per region — held the GIL for
// about half a millisecond per block). Job j = jobs[6j .. 6j+5] = {fd, file offset, region
// start in the slot, region cap, max records, hint}. Out:
//   offs[0..n]       record starts in the slot (offs[i+1] = end of record i, as written
//                    by the regions; the last record of a region is followed by its gap)
//   ends[0..n)       true end of each record (gap-free at region ends; may be null)
//   doffs[0..n]      the same records packed for the device, each region 16-B aligned
//                    (may be null)
//   res[2j], res[2j+1]  records read and bytes consumed of job j
//   segs[3s..3s+2]   (slot start, device start, bytes) of each non-empty region
//   meta = {n, nbytes (end of the last record in the slot), dev_nbytes, nsegs, ngaps}
// Returns n ≥ 0, or -errno of the first failed read.
OMLDM_HOST_API int64_t omldm_fill_regions(int nj, const int64_t* jobs, uint8_t* slot,
                                          int64_t* offs, int64_t* ends, int64_t* doffs,
                                          int64_t* res, int64_t* segs, int64_t* meta,
                                          int nthreads) {
  std::vector<std::vector<int64_t>> ro(nj);
  std::vector<int64_t> rn(nj, 0), ru(nj, 0);
  auto run = [&](int j) {
    const int64_t* J = jobs + 6 * j;
    ro[j].assign(size_t(J[4] > 0 ? J[4] : 0) + 1, 0);
    if (J[4] <= 0 || J[3] <= 0) return;
    rn[j] = omldm_read_log(int(J[0]), J[1], slot + J[2], J[3], J[4], ro[j].data(), &ru[j], J[5]);
  };
  const int nt = nthreads < 1 ? 1 : nthreads;
  // more readers than regions: each region's first read (its hint) is cut into pieces
  // read and newline-indexed on their own threads, then stitched in order (records may
  // straddle pieces: only the '\n' positions matter); a region short of records goes on
  // reading on its own.
  // opt-in (OMLDM_READ_SPLIT=1): measured slower end to end on the MI355X host (DIB
  // pread 1.02 vs 0.52 ms per 131072-record block, profiles/round5/e2e/)
  const char* split_e = std::getenv("OMLDM_READ_SPLIT");
  const bool split_env = split_e && split_e[0] == '1';
  constexpr int64_t kMinPiece = 256 << 10;
  const int per = nt / (nj > 0 ? nj : 1);
  if (split_env && per >= 2) {
    struct Piece {
      int j;
      int64_t a, b, got = 0;
      int err = 0;
      std::vector<int64_t> nl;
    };
    std::vector<Piece> pcs;
    std::vector<int> first(nj + 1, 0);
    for (int j = 0; j < nj; ++j) {
      first[j] = (int)pcs.size();
      const int64_t* J = jobs + 6 * j;
      if (J[4] <= 0 || J[3] <= 0) continue;
      const int64_t h = J[5] > 0 && J[5] < J[3] ? J[5] : J[3];
      int np = (int)(h / kMinPiece);
      np = np < 1 ? 1 : (np > per ? per : np);
      for (int p = 0; p < np; ++p)
        pcs.push_back(Piece{j, h * p / np, h * (p + 1) / np});
    }
    first[nj] = (int)pcs.size();
    auto piece = [&](int i) {
      Piece& q = pcs[i];
      const int64_t* J = jobs + 6 * q.j;
      uint8_t* dst = slot + J[2];
      while (q.a + q.got < q.b) {
        ssize_t r = pread(int(J[0]), dst + q.a + q.got, size_t(q.b - q.a - q.got),
                          off_t(J[1] + q.a + q.got));
        if (r < 0) {
          if (errno == EINTR) continue;
          q.err = errno;
          return;
        }
        if (r == 0) break;
        q.got += r;
      }
      q.nl.reserve(size_t(q.got / 96 + 8));
      const uint8_t* b = dst + q.a;
      int64_t i0 = 0;
      const __m128i nlv = _mm_set1_epi8('\n');
      for (; i0 + 64 <= q.got; i0 += 64) {
        const __m128i* v = reinterpret_cast<const __m128i*>(b + i0);
        uint64_t m =
            (uint64_t)(unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128(v), nlv)) |
            ((uint64_t)(unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128(v + 1), nlv)) << 16) |
            ((uint64_t)(unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128(v + 2), nlv)) << 32) |
            ((uint64_t)(unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128(v + 3), nlv)) << 48);
        while (m) {
          q.nl.push_back(q.a + i0 + __builtin_ctzll(m) + 1);
          m &= m - 1;
        }
      }
      for (; i0 < q.got; ++i0)
        if (b[i0] == '\n') q.nl.push_back(q.a + i0 + 1);
    };
    const int np_all = (int)pcs.size();
    const int nth = nt < np_all ? nt : np_all;
    const char* pool_e = std::getenv("OMLDM_READ_POOL");
    if (pool_e && pool_e[0] == '1') {  // persistent workers (no thread creation per block)
      const std::function<void(int)> f = piece;
      read_pool().run(np_all, nth, f);
    } else {
      std::vector<std::thread> th;
      th.reserve(nth);
      for (int t = 0; t < nth; ++t)
        th.emplace_back([&, t] {
          for (int i = t; i < np_all; i += nth) piece(i);
        });
      for (auto& x : th) x.join();
    }
    // stitch each region, then let the regions short of records read on (in parallel)
    std::vector<LogRead> st(nj);
    std::vector<int64_t> cont_want(nj, 0);
    for (int j = 0; j < nj; ++j) {
      const int64_t* J = jobs + 6 * j;
      ro[j].assign(size_t(J[4] > 0 ? J[4] : 0) + 1, 0);
      if (J[4] <= 0 || J[3] <= 0) continue;
      LogRead& s = st[j];
      int64_t* o = ro[j].data();
      for (int i = first[j]; i < first[j + 1]; ++i) {
        const Piece& q = pcs[i];
        if (q.err) {
          rn[j] = -q.err;
          break;
        }
        for (size_t t = 0; t < q.nl.size() && s.n < J[4]; ++t) {
          s.pos = q.nl[t];
          o[++s.n] = s.pos;
        }
        s.got += q.got;
        if (q.got < q.b - q.a) {
          s.eof = true;
          break;
        }
      }
      if (rn[j] < 0) continue;
      s.scanned = s.n >= J[4] ? s.pos : s.got;
      const int64_t h = J[5] > 0 && J[5] < J[3] ? J[5] : J[3];
      if (s.n >= J[4] || s.eof || h >= J[3]) {
        rn[j] = s.n;
        ru[j] = o[s.n];
        continue;
      }
      const int64_t perr = s.n ? s.pos / s.n : 2 * h;
      const int64_t more = (J[4] - s.n) * perr / 10 * 11 + 4096;
      cont_want[j] = s.got + more < J[3] ? s.got + more : J[3];
    }
    std::vector<std::thread> th;
    for (int j = 0; j < nj; ++j)
      if (cont_want[j] > 0)
        th.emplace_back([&, j] {
          const int64_t* J = jobs + 6 * j;
          const int64_t e = read_log_cont(int(J[0]), J[1], slot + J[2], J[3], J[4],
                                          ro[j].data(), st[j], cont_want[j]);
          rn[j] = e < 0 ? e : st[j].n;
          ru[j] = e < 0 ? 0 : ro[j][st[j].n];
        });
    for (auto& x : th) x.join();
  } else {
    const int ntr = nt > nj ? nj : nt;
    // measured (scripts/gpu_r4_pool.sh, same box, alternated): a thread per reader per
    // block 149-150 M DIB records/s end to end, the pool 111-112 M (its workers'
    // condition-variable wake-ups and the shared job counter cost more than thread
    // creation): the pool is opt-in
    static const bool use_pool = [] {
      const char* e = std::getenv("OMLDM_READ_POOL");
      return e && e[0] == '1';
    }();
    if (ntr <= 1) {
      for (int j = 0; j < nj; ++j) run(j);
    } else if (use_pool) {
      read_pool().run(nj, ntr, run);
    } else {  // a thread per reader per block
      std::vector<std::thread> th;
      th.reserve(ntr);
      for (int t = 0; t < ntr; ++t)
        th.emplace_back([&, t] {
          for (int j = t; j < nj; j += ntr) run(j);
        });
      for (auto& x : th) x.join();
    }
  }
  for (int j = 0; j < nj; ++j)
    if (rn[j] < 0) return rn[j];
  int64_t n = 0, end = 0, dpos = 0, nsegs = 0, ngaps = 0;
  offs[0] = 0;
  for (int j = 0; j < nj; ++j) {
    const int64_t k = rn[j], start = jobs[6 * j + 2];
    res[2 * j] = k;
    res[2 * j + 1] = ru[j];
    if (!k) continue;
    const int64_t* o = ro[j].data();
    if (n && start != end) {  // the previous region's last record is followed by a gap
      if (ends) ends[n - 1] = end;
      ++ngaps;
    }
    offs[n] = start;
    for (int64_t i = 1; i <= k; ++i) {
      offs[n + i] = o[i] + start;
      if (ends) ends[n + i - 1] = o[i] + start;
    }
    if (doffs) {
      for (int64_t i = 0; i <= k; ++i) doffs[n + i] = o[i] + dpos;
      segs[3 * nsegs] = start;
      segs[3 * nsegs + 1] = dpos;
      segs[3 * nsegs + 2] = o[k];
      ++nsegs;
      dpos = (dpos + o[k] + 15) & ~int64_t(15);
    }
    n += k;
    end = start + o[k];
  }
  meta[0] = n;
  meta[1] = end;
  meta[2] = dpos;
  meta[3] = nsegs;
  meta[4] = ngaps;
  return n;
}
