"""Protocol-level fake Kafka broker for tests (no real broker exists in this sandbox).

Speaks the same request subset as omldm_amd.io.kafka (ApiVersions v0, Metadata v1/v4,
ListOffsets v1, Produce v3/v7, Fetch v4/v10, CreateTopics v0/v2) on 127.0.0.1, stores records in memory and
re-encodes RecordBatch v2 on fetch with the codec the partition was last written with —
so the client's framing, varints, CRC-32C and codecs are exercised in both directions.
Like a real broker it refuses to serve zstd batches to Fetch < v10 (error 76,
UNSUPPORTED_COMPRESSION_TYPE). ``control_every`` > 0 appends a transactional control
batch after every that many records. Compatibility with a real broker is "parity
unpinned".
"""
from __future__ import annotations

import socketserver
import struct
import threading
from collections import defaultdict

from omldm_amd.io.kafka import R, W, decode_batches, encode_batch


class FakeKafka:
    # ApiVersions answers: "classic" (every version this client implements), "modern"
    # (Kafka 4.0 ranges after KIP-896 removed the oldest versions) or "legacy" (a
    # pre-0.10 broker: ApiVersions unknown, the connection is dropped)
    VERSIONS = {
        "classic": {18: (0, 2), 3: (0, 8), 0: (0, 8), 1: (0, 11), 2: (0, 5), 19: (0, 4)},
        "modern": {18: (0, 4), 3: (4, 12), 0: (3, 11), 1: (4, 17), 2: (1, 9), 19: (2, 7)},
    }

    def __init__(self, default_partitions: int = 4, control_every: int = 0,
                 versions: str = "classic"):
        self.versions = versions
        self.calls = []                    # (api, version) of every request
        self.logs = defaultdict(list)      # (topic, p) -> [bytes]
        self.codec = defaultdict(int)      # (topic, p) -> codec of the last produce
        self.log_start = defaultdict(int)  # (topic, p) -> first offset retention kept
        self.control_every = control_every
        self.fetch_versions = []
        self.nparts = {}
        self.default_partitions = default_partitions
        self.lock = threading.Lock()
        outer = self

        class H(socketserver.BaseRequestHandler):
            def handle(self):
                s = self.request
                while True:
                    hdr = self._recv(4)
                    if not hdr:
                        return
                    n = struct.unpack(">i", hdr)[0]
                    req = R(self._recv(n))
                    api, ver, cid = req.i16(), req.i16(), req.i32()
                    req.s()
                    body = outer.dispatch(api, ver, req)
                    if body is None:  # unknown request: drop the connection
                        return
                    msg = struct.pack(">i", cid) + body
                    s.sendall(struct.pack(">i", len(msg)) + msg)

            def _recv(self, n):
                buf = bytearray()
                while len(buf) < n:
                    c = self.request.recv(n - len(buf))
                    if not c:
                        return None
                    buf += c
                return bytes(buf)

        class S(socketserver.ThreadingTCPServer):
            allow_reuse_address = True
            daemon_threads = True

        self.server = S(("127.0.0.1", 0), H)
        self.port = self.server.server_address[1]
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True)
        self.thread.start()

    @property
    def addr(self) -> str:
        return f"127.0.0.1:{self.port}"

    def close(self):
        self.server.shutdown()
        self.server.server_close()

    def _parts(self, topic):
        return self.nparts.setdefault(topic, self.default_partitions)

    def dispatch(self, api, ver, r: R) -> bytes:
        with self.lock:
            self.calls.append((api, ver))
            table = self.VERSIONS.get(self.versions)
            if api == 18:  # ApiVersions v0
                if table is None:
                    return None
                return bytes(W().i16(0).arr(sorted(table.items()), lambda w, kv: w.i16(kv[0]).i16(
                    kv[1][0]).i16(kv[1][1])).b)
            if table is not None and api in table and not (table[api][0] <= ver <= table[api][1]):
                raise ValueError(f"api {api} v{ver} outside the advertised range {table[api]}")
            if api == 3:  # Metadata v1 / v4
                topics = r.arr(lambda r: r.s())
                w = W()
                if ver >= 3:
                    w.i32(0)  # throttle
                w.arr([(0, "127.0.0.1", self.port)],
                      lambda w, b: w.i32(b[0]).s(b[1]).i32(b[2]).s(None))
                if ver >= 2:
                    w.s("fake-cluster")
                w.i32(0)
                w.arr(topics, lambda w, t: w.i16(0).s(t).i8(0).arr(
                    list(range(self._parts(t))),
                    lambda w, p: w.i16(0).i32(p).i32(0).arr([0], lambda w, x: w.i32(x)).arr(
                        [0], lambda w, x: w.i32(x))))
                return bytes(w.b)
            if api == 19:  # CreateTopics v0 / v2
                reqs = r.arr(lambda r: (r.s(), r.i32(), r.i16(),
                                        r.arr(lambda r: (r.i32(), r.arr(lambda r: r.i32()))),
                                        r.arr(lambda r: (r.s(), r.s()))))
                for name, n, *_ in reqs:
                    self.nparts[name] = max(1, n)
                w = W()
                if ver >= 2:
                    w.i32(0)  # throttle
                w.arr(reqs, lambda w, q: (w.s(q[0]).i16(0), w.s(None) if ver >= 1 else None))
                return bytes(w.b)
            if api == 0:  # Produce v3 / v7 (same request; v5+ answers log_start_offset)
                r.s(), r.i16(), r.i32()
                topics = r.arr(lambda r: (r.s(), r.arr(lambda r: (r.i32(), r.by()))))
                out = []
                for t, parts in topics:
                    po = []
                    for p, rs in parts:
                        log = self.logs[(t, p)]
                        base = len(log)
                        self.codec[(t, p)] = struct.unpack_from(">h", rs, 21)[0] & 7
                        log.extend(v for _, v in decode_batches(rs))
                        po.append((p, base))
                    out.append((t, po))
                w = W().arr(out, lambda w, tp: w.s(tp[0]).arr(
                    tp[1], lambda w, pb: (w.i32(pb[0]).i16(0).i64(pb[1]).i64(-1),
                                          w.i64(0) if ver >= 5 else None))).i32(0)
                return bytes(w.b)
            if api == 2:  # ListOffsets v1
                r.i32()
                topics = r.arr(lambda r: (r.s(), r.arr(lambda r: (r.i32(), r.i64()))))
                w = W().arr(topics, lambda w, tp: w.s(tp[0]).arr(
                    tp[1], lambda w, pt: w.i32(pt[0]).i16(0).i64(-1).i64(
                        len(self.logs[(tp[0], pt[0])]) if pt[1] == -1
                        else self.log_start[(tp[0], pt[0])])))
                return bytes(w.b)
            if api == 1:  # Fetch v4 / v10
                self.fetch_versions.append(ver)
                r.i32(), r.i32(), r.i32(), r.i32(), r.i8()
                if ver >= 7:
                    r.i32(), r.i32()  # session id / epoch
                topics = r.arr(lambda r: (r.s(), r.arr(lambda r: (
                    r.i32(), r.i32() if ver >= 9 else None, r.i64(),
                    r.i64() if ver >= 5 else None, r.i32()))))
                w = W().i32(0)
                if ver >= 7:
                    w.i16(0).i32(0)

                def part(w, pt, t):
                    p, _epoch, off, _lso, _mx = pt
                    log = self.logs[(t, p)]
                    codec = self.codec[(t, p)]
                    err = 76 if codec == 4 and ver < 10 else 0
                    if off < self.log_start[(t, p)] or off > len(log):
                        err = 1  # OFFSET_OUT_OF_RANGE
                    rs = b"" if err else self._record_set(log, off, codec)
                    w.i32(p).i16(err).i64(len(log)).i64(len(log))
                    if ver >= 5:
                        w.i64(0)
                    w.i32(0).by(rs)

                w.arr(topics, lambda w, tp: w.s(tp[0]).arr(tp[1], lambda w, pt: part(w, pt,
                                                                                     tp[0])))
                return bytes(w.b)
        raise ValueError(f"unsupported api {api}")

    def _record_set(self, log, off, codec) -> bytes:
        """Batches of ≤ 200 records from ``off`` (≤ 500 records). With ``control_every`` a
        control batch follows each data batch; a real log gives the marker its own offset,
        this log has none to give, so the marker reuses the batch's last offset."""
        out, o, end = b"", off, min(len(log), off + 500)
        while o < end:
            n = min(200, end - o)
            if self.control_every:
                n = min(n, self.control_every)
            out += encode_batch(log[o:o + n], base_offset=o, compression=codec)
            if self.control_every:
                out += encode_batch([b"\x00\x00\x00\x00"], base_offset=o + n - 1,
                                    control=True)
            o += n
        return out
