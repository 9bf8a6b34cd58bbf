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
#include <cstring>
#include <unistd.h>

#define OMLDM_HOST_API extern "C" __attribute__((visibility("default")))

// Indexes up to max_records complete lines of buf[0, len). offs[0] = 0 and
// offs[i + 1] = one past the '\n' of record i. Returns the record count n; offs[n] is
// the number of bytes consumed (a trailing partial line is left for the next read).
OMLDM_HOST_API int64_t omldm_index_lines(const uint8_t* buf, int64_t len, int64_t max_records,
                                         int64_t* offs) {
  offs[0] = 0;
  int64_t n = 0, pos = 0;
  while (n < max_records && pos < len) {
    const void* nl = std::memchr(buf + pos, '\n', size_t(len - pos));
    if (!nl) break;
    pos = static_cast<const uint8_t*>(nl) - buf + 1;
    offs[++n] = pos;
  }
  return n;
}

// pread of the log at `offset` into dst (restarting on EINTR / short reads), indexing the
// complete lines as they arrive. The first read asks for `hint` bytes (0: the whole cap);
// if that holds fewer than max_records complete records and the log goes on, further
// reads ask for the missing records at the mean length seen so far (+10 %), never beyond
// cap — so a tick reads what it consumes instead of a fixed safety margin that the next
// tick reads again. Returns the record count (≥ 0) or -errno; *used = bytes consumed.
OMLDM_HOST_API int64_t omldm_read_log(int fd, int64_t offset, uint8_t* dst, int64_t cap,
                                      int64_t max_records, int64_t* offs, int64_t* used,
                                      int64_t hint) {
  int64_t got = 0, n = 0, pos = 0;
  int64_t want = hint > 0 && hint < cap ? hint : cap;
  bool eof = false;
  offs[0] = 0;
  for (;;) {
    while (got < want) {
      ssize_t r = pread(fd, dst + got, size_t(want - got), off_t(offset + got));
      if (r < 0) {
        if (errno == EINTR) continue;
        *used = 0;
        offs[0] = 0;
        return -errno;
      }
      if (r == 0) {
        eof = true;
        break;
      }
      got += r;
    }
    while (n < max_records && pos < got) {
      const void* nl = std::memchr(dst + pos, '\n', size_t(got - pos));
      if (!nl) break;
      pos = static_cast<const uint8_t*>(nl) - dst + 1;
      offs[++n] = pos;
    }
    if (n >= max_records || eof || want >= cap) break;
    const int64_t per = n ? pos / n : 2 * want;  // no complete record yet: double the read
    const int64_t more = (max_records - n) * per / 10 * 11 + 4096;
    want = got + more < cap ? got + more : cap;
  }
  *used = offs[n];
  return n;
}
