"""Minimal Kafka wire-protocol client (no client library is installed or fetchable).

Reference: every OMLDM input/output is a Kafka topic (FlinkKafkaConsumer/Producer,
omldm/Job.scala:42-105; omldm/utils/KafkaUtils.scala:13-18 sets bootstrap.servers — and
the misspelled ``group.flink_worker_id``; we track offsets ourselves and
need no consumer group). Implemented subset, enough for produce/consume of JSON records:

* ApiVersions v0 (api 18) — on every new connection; each request below then uses the
                          highest version both sides implement (brokers of Kafka 4.0
                          dropped the oldest versions, KIP-896; pre-0.10 brokers that do
                          not answer ApiVersions get the lowest versions listed)
* Metadata v1 / v4 (api 3)   — topic → partitions + leader brokers
* ListOffsets v1 (api 2) — earliest (-2) / latest (-1) offsets
* Produce v3 / v7 (api 0)    — RecordBatch v2, acks=1 (zstd batches need v7)
* Fetch v4 / v10 (api 1)      — RecordBatch v2 decoding (magic 2; older message sets and
                          transactional control batches skipped); v10 also once a broker
                          answers UNSUPPORTED_COMPRESSION_TYPE (zstd topics need ≥ v10)
* CreateTopics v0 / v2 (api 19) — best effort, for ``create_topic``
* compression: gzip / snappy / lz4 / zstd batches are read transparently and any of them
  can be written (``KafkaBroker(..., compression="lz4")`` or ``host:port?compression=lz4``)
CRC-32C of record batches is computed by the host library (csrc/host/crc32c.cpp); the
codecs and the record-set decoder that fills the pinned staging slot without a Python
object per record are csrc/host/kafka_wire.cpp.
Compatibility is at the level of the public protocol spec; tests exercise it against a
protocol-level fake broker (tests/fake_kafka.py) — there is no real broker here.
"""
from __future__ import annotations

import socket
import struct
import threading
import time

from omldm_amd.io.transport import Broker

# ------------------------------------------------------------------ primitives


def crc32c(data: bytes) -> int:
    from omldm_amd.ops import native

    return int(native.host().omldm_crc32c(data, len(data), 0))


def _zz(n: int) -> int:
    return (n << 1) ^ (n >> 63)


def _unzz(n: int) -> int:
    return (n >> 1) ^ -(n & 1)


def varint(n: int) -> bytes:
    n = _zz(n) & 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def read_varint(buf: bytes, pos: int) -> tuple[int, int]:
    shift = 0
    res = 0
    while True:
        b = buf[pos]
        pos += 1
        res |= (b & 0x7F) << shift
        if not b & 0x80:
            return _unzz(res), pos
        shift += 7


class W:
    def __init__(self):
        self.b = bytearray()

    def i8(self, v):
        self.b += struct.pack(">b", v)
        return self

    def i16(self, v):
        self.b += struct.pack(">h", v)
        return self

    def i32(self, v):
        self.b += struct.pack(">i", v)
        return self

    def i64(self, v):
        self.b += struct.pack(">q", v)
        return self

    def s(self, v: str | None):
        if v is None:
            return self.i16(-1)
        e = v.encode()
        self.i16(len(e))
        self.b += e
        return self

    def by(self, v: bytes | None):
        if v is None:
            return self.i32(-1)
        self.i32(len(v))
        self.b += v
        return self

    def arr(self, items, fn):
        self.i32(len(items))
        for it in items:
            fn(self, it)
        return self


class R:
    def __init__(self, b: bytes):
        self.b = b
        self.p = 0

    def _u(self, fmt, n):
        v = struct.unpack_from(fmt, self.b, self.p)[0]
        self.p += n
        return v

    def i8(self):
        return self._u(">b", 1)

    def i16(self):
        return self._u(">h", 2)

    def i32(self):
        return self._u(">i", 4)

    def i64(self):
        return self._u(">q", 8)

    def s(self):
        n = self.i16()
        if n < 0:
            return None
        v = self.b[self.p:self.p + n].decode()
        self.p += n
        return v

    def by(self):
        n = self.i32()
        if n < 0:
            return None
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def arr(self, fn):
        return [fn(self) for _ in range(self.i32())]


# ----------------------------------------------------------------- record batch


CODECS = {"none": 0, "gzip": 1, "snappy": 2, "lz4": 3, "zstd": 4}
UNSUPPORTED_COMPRESSION_TYPE = 76
OFFSET_OUT_OF_RANGE = 1


def codec_id(c) -> int:
    if isinstance(c, int):
        if c not in CODECS.values():
            raise ValueError(f"unknown Kafka compression codec {c}")
        return c
    key = (c or "none").lower()
    if key not in CODECS:
        raise ValueError(f"unknown Kafka compression codec {c!r} (one of {sorted(CODECS)})")
    return CODECS[key]


def _codec_call(fn, codec: int, data: bytes, *extra) -> bytes:
    import ctypes

    from omldm_amd.ops import native

    lib = native.host()
    out, n = ctypes.c_void_p(), ctypes.c_longlong()
    rc = getattr(lib, fn)(codec, data, len(data), *extra, ctypes.byref(out), ctypes.byref(n))
    if rc:
        what = {-1: "unknown codec", -2: "corrupt data", -3: "codec library not found",
                -4: "too large", -6: "out of memory"}.get(rc, str(rc))
        raise ValueError(f"kafka {fn.split('_')[-1]} ({codec}): {what}")
    try:
        return ctypes.string_at(out.value, n.value) if n.value else b""
    finally:
        lib.omldm_codec_free(out)


def compress(codec, data: bytes, level: int = -1) -> bytes:
    c = codec_id(codec)
    return data if c == 0 else _codec_call("omldm_codec_compress", c, data, level)


def decompress(codec, data: bytes) -> bytes:
    c = codec_id(codec)
    return data if c == 0 else _codec_call("omldm_codec_decompress", c, data)


def codec_available(codec) -> bool:
    from omldm_amd.ops import native

    return bool(native.host().omldm_codec_available(codec_id(codec)))


def encode_lines(buf, offs, compression=0, base_offset: int = 0, ts_ms: int | None = None,
                 strip_nl: bool = True) -> bytes:
    """Native encode_batch of the records buf[offs[i]:offs[i+1]] (trailing newlines dropped)."""
    import ctypes

    import numpy as np

    from omldm_amd.ops import native

    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    ts = int(time.time() * 1000) if ts_ms is None else ts_ms
    lib = native.host()
    out, n = ctypes.c_void_p(), ctypes.c_longlong()
    rc = lib.omldm_kafka_encode_lines(buf.ctypes.data, offs.ctypes.data, len(offs) - 1,
                                      int(strip_nl), base_offset, ts, codec_id(compression), -1,
                                      ctypes.byref(out), ctypes.byref(n))
    if rc:
        raise ValueError(f"kafka batch encode failed ({rc})")
    try:
        return ctypes.string_at(out.value, n.value)
    finally:
        lib.omldm_codec_free(out)


def encode_batch(values: list[bytes], base_offset: int = 0, ts_ms: int | None = None,
                 keys: list | None = None, compression=0, control: bool = False) -> bytes:
    """RecordBatch v2 of ``values``; ``compression`` (name or id) compresses the records
    section and sets attributes bits 0-2; ``control`` marks a transactional control batch."""
    codec = codec_id(compression)
    ts = int(time.time() * 1000) if ts_ms is None else ts_ms
    recs = bytearray()
    for i, v in enumerate(values):
        k = keys[i] if keys else None
        body = bytearray()
        body += struct.pack(">b", 0)       # attributes
        body += varint(0)                  # timestamp delta
        body += varint(i)                  # offset delta
        if k is None:
            body += varint(-1)
        else:
            body += varint(len(k)) + k
        body += varint(len(v)) + v
        body += varint(0)                  # headers
        recs += varint(len(body)) + body
    tail = W()
    attrs = codec | (0x20 if control else 0)
    tail.i16(attrs).i32(len(values) - 1).i64(ts).i64(ts).i64(-1).i16(-1).i32(-1).i32(len(values))
    payload = bytes(tail.b) + (compress(codec, bytes(recs)) if codec else bytes(recs))
    crc = crc32c(payload)
    head = W()
    head.i64(base_offset).i32(4 + 1 + 4 + len(payload)).i32(0).i8(2)
    head.b += struct.pack(">I", crc)
    return bytes(head.b) + payload


def decode_batches(data: bytes, verify: bool = True) -> list[tuple[int, bytes]]:
    """[(offset, value)] of every record in a (possibly truncated) record set."""
    out = []
    p = 0
    while p + 17 <= len(data):
        base, blen = struct.unpack_from(">qi", data, p)
        end = p + 12 + blen
        if end > len(data):
            break  # partial batch at the end of a fetch
        magic = data[p + 16]
        if magic != 2:
            p = end
            continue
        crc = struct.unpack_from(">I", data, p + 17)[0]
        body = data[p + 21:end]
        if verify and crc32c(body) != crc:
            raise ValueError("record batch CRC mismatch")
        attrs = struct.unpack_from(">h", body, 0)[0]
        if attrs & 0x20:  # transactional control batch (commit / abort marker)
            p = end
            continue
        count = struct.unpack_from(">i", body, 36)[0]
        q = 40
        if attrs & 0x7:
            body = decompress(attrs & 0x7, bytes(body[40:]))
            q = 0
        for _ in range(count):
            ln, q = read_varint(body, q)
            rend = q + ln
            q += 1
            _, q = read_varint(body, q)       # timestamp delta
            od, q = read_varint(body, q)      # offset delta
            kl, q = read_varint(body, q)
            if kl > 0:
                q += kl
            vl, q = read_varint(body, q)
            val = body[q:q + vl] if vl >= 0 else b""
            out.append((base + od, bytes(val)))
            q = rend
        p = end
    return out


# ---------------------------------------------------------------------- client


class _Conn:
    def __init__(self, host: str, port: int, timeout: float = 10.0):
        self.addr, self.timeout = (host, port), timeout
        self._open()
        self.versions = self._api_versions()  # api → (min, max); None: not answered

    def _open(self):
        self.sock = socket.create_connection(self.addr, timeout=self.timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.cid = 0
        self.lock = threading.Lock()

    def _api_versions(self):
        try:
            r = self.call(18, 0, b"")
            err = r.i16()
            vs = r.arr(lambda r: (r.i16(), r.i16(), r.i16()))
            if err == 0:
                return {k: (lo, hi) for k, lo, hi in vs}
        except (IOError, OSError, struct.error):
            pass
        self.close()  # a broker without ApiVersions drops the connection: reopen
        self._open()
        return None

    def version(self, api: int, ours: tuple) -> int:
        """Highest of ``ours`` (ascending) the broker accepts for ``api``."""
        if self.versions is None or api not in self.versions:
            return ours[0]
        lo, hi = self.versions[api]
        ok = [v for v in ours if lo <= v <= hi]
        if not ok:
            raise IOError(f"kafka broker {self.addr} supports api {api} v{lo}-v{hi}; "
                          f"this client implements {ours}")
        return ok[-1]

    def call(self, api: int, ver: int, body: bytes, client: str = "omldm-amd") -> R:
        with self.lock:
            self.cid += 1
            h = W().i16(api).i16(ver).i32(self.cid).s(client)
            msg = bytes(h.b) + body
            self.sock.sendall(struct.pack(">i", len(msg)) + msg)
            n = struct.unpack(">i", self._recv(4))[0]
            r = R(self._recv(n))
            if r.i32() != self.cid:
                raise IOError("kafka correlation id mismatch")
            return r

    def _recv(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise IOError("kafka connection closed")
            buf += chunk
        return bytes(buf)

    def close(self):
        self.sock.close()


class KafkaBroker(Broker):
    """transport.Broker over the Kafka protocol (bootstrap ``host:port[,host:port]``)."""

    def __init__(self, bootstrap: str, timeout: float = 10.0, compression=None):
        bootstrap, _, query = bootstrap.partition("?")
        opts = dict(kv.split("=", 1) for kv in query.split("&") if "=" in kv)
        self.codec = codec_id(compression if compression is not None
                              else opts.get("compression", "none"))
        self.bootstrap = [(h, int(p)) for h, p in (x.rsplit(":", 1) for x in bootstrap.split(","))]
        self.timeout = timeout
        self._fetch_v10: set = set()  # brokers that asked for Fetch ≥ v10 (zstd topics)
        self._conns: dict = {}
        self._meta: dict = {}     # topic -> {partition: leader}
        self._brokers: dict = {}  # node -> (host, port)
        self._rr: dict = {}

    # partitions may be fetched concurrently (engine.ingest.TickIngest reads every owned
    # partition on its own thread): each thread talks over its own connections, and the
    # native decode runs outside the GIL
    parallel_reads = True

    def _addr(self, node=None):
        return self._brokers.get(node, self.bootstrap[0]) if node is not None else self.bootstrap[0]

    def _conn(self, node=None) -> _Conn:
        key = (self._addr(node), threading.get_ident())
        c = self._conns.get(key)
        if c is None:
            c = self._conns[key] = _Conn(key[0][0], key[0][1], self.timeout)
        return c

    def _metadata(self, topic: str, refresh: bool = False) -> dict:
        if topic in self._meta and not refresh:
            return self._meta[topic]
        conn = self._conn()
        ver = conn.version(3, (1, 4))
        w = W().arr([topic], lambda w, t: w.s(t))
        if ver >= 4:
            w.i8(0)  # allow_auto_topic_creation: no (create_topic does that)
        r = conn.call(3, ver, bytes(w.b))
        if ver >= 3:
            r.i32()  # throttle
        for node, host, port, _ in r.arr(lambda r: (r.i32(), r.s(), r.i32(), r.s())):
            self._brokers[node] = (host, port)
        if ver >= 2:
            r.s()  # cluster id
        r.i32()  # controller
        for err, name, _internal, parts in r.arr(lambda r: (
                r.i16(), r.s(), r.i8(),
                r.arr(lambda r: (r.i16(), r.i32(), r.i32(), r.arr(lambda r: r.i32()),
                                 r.arr(lambda r: r.i32()))))):
            if name == topic and err == 0:
                self._meta[topic] = {p[1]: p[2] for p in parts}
        return self._meta.get(topic, {})

    def create_topic(self, topic: str, partitions: int) -> None:
        try:
            conn = self._conn()
            ver = conn.version(19, (0, 2))
            body = W().arr([topic], lambda w, t: w.s(t).i32(partitions).i16(1).i32(0).i32(0)).i32(
                int(self.timeout * 1000))
            if ver >= 1:
                body.i8(0)  # validate_only
            conn.call(19, ver, bytes(body.b))
        except (IOError, OSError):
            pass
        self._meta.pop(topic, None)

    def partitions(self, topic: str) -> int:
        return max(1, len(self._metadata(topic)))

    def produce(self, topic, value, partition=None, key=None):
        if isinstance(value, str):
            value = value.encode()
        n = self.partitions(topic)
        if partition is None:
            partition = self._rr.get(topic, 0) % n
            self._rr[topic] = partition + 1
        self.produce_batch(topic, partition, [value])

    def produce_batch(self, topic: str, partition: int, values: list[bytes]) -> int:
        return self._produce_raw(topic, partition, encode_batch(values, compression=self.codec))

    def _produce_raw(self, topic: str, partition: int, rs: bytes) -> int:
        body = W().s(None).i16(1).i32(int(self.timeout * 1000)).arr(
            [topic], lambda w, t: w.s(t).arr([partition], lambda w, p: w.i32(p).by(rs)))
        conn = self._conn(self._metadata(topic).get(partition))
        ver = conn.version(0, (3, 7))
        if self.codec == CODECS["zstd"] and conn.versions is None:
            ver = 7  # brokers accept zstd from Produce v7
        r = conn.call(0, ver, bytes(body.b))
        res = r.arr(lambda r: (r.s(), r.arr(lambda r: (
            r.i32(), r.i16(), r.i64(), r.i64(), *((r.i64(),) if ver >= 5 else ())))))
        err = res[0][1][0][1]
        if err:
            raise IOError(f"kafka produce error {err}")
        return res[0][1][0][2]

    max_batch_bytes = 900 << 10  # under the brokers' default message.max.bytes (1 MiB)

    def produce_lines(self, topic, block, offs, partition=None):
        """A tick's newline-terminated output records as RecordBatches built natively
        (csrc/host/kafka_wire.cpp), ≤ ``max_batch_bytes`` each, one Produce per batch
        (Produce v3+ takes exactly one batch per partition)."""
        import numpy as np

        n = len(offs) - 1
        if n <= 0:
            return
        if partition is None:
            nparts = self.partitions(topic)
            partition = self._rr.get(topic, 0) % nparts
            self._rr[topic] = partition + 1
        buf = np.frombuffer(block, dtype=np.uint8) if isinstance(block, (bytes, bytearray)) \
            else np.ascontiguousarray(block).view(np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        i = 0
        while i < n:
            j = int(np.searchsorted(offs, offs[i] + self.max_batch_bytes, side="right")) - 1
            j = min(n, max(j, i + 1))
            self._produce_raw(topic, partition, encode_lines(buf, offs[i:j + 1], self.codec))
            i = j

    def _list_offset(self, topic: str, partition: int, ts: int) -> int:
        body = W().i32(-1).arr([topic], lambda w, t: w.s(t).arr(
            [partition], lambda w, p: w.i32(p).i64(ts)))
        conn = self._conn(self._metadata(topic).get(partition))
        r = conn.call(2, conn.version(2, (1,)), bytes(body.b))
        res = r.arr(lambda r: (r.s(), r.arr(lambda r: (r.i32(), r.i16(), r.i64(), r.i64()))))
        return int(res[0][1][0][3])

    def end_offset(self, topic, partition):
        return self._list_offset(topic, partition, -1)

    def _fetch(self, topic: str, partition: int, offset: int,
               max_bytes: int = 4 << 20) -> tuple[bytes, int]:
        """(raw record set, offset actually fetched from) of one partition (Fetch v10 when
        the broker offers it, else v4 — switching to v10 if it answers
        UNSUPPORTED_COMPRESSION_TYPE, i.e. zstd data). An offset that retention already
        deleted (OFFSET_OUT_OF_RANGE below the log start) resumes at the log start, as a
        consumer with auto.offset.reset=earliest would; the caller decodes from, and
        advances past, the returned offset."""
        leader = self._metadata(topic).get(partition)
        conn = self._conn(leader)
        addr = self._addr(leader)
        best = conn.version(1, (4, 10))
        for _ in range(3):
            v10 = best >= 10 or addr in self._fetch_v10
            w = W().i32(-1).i32(100).i32(1).i32(max(8 << 20, max_bytes)).i8(0)
            if v10:
                w.i32(0).i32(-1)  # no fetch session
            w.arr([topic], lambda w, t: w.s(t).arr([partition], lambda w, p: (
                w.i32(p), w.i32(-1) if v10 else None, w.i64(offset),
                w.i64(-1) if v10 else None, w.i32(max_bytes))))
            if v10:
                w.i32(0)  # forgotten topics
            r = conn.call(1, 10 if v10 else 4, bytes(w.b))
            r.i32()  # throttle
            if v10:
                top_err = r.i16()
                r.i32()  # session id
                if top_err:
                    raise IOError(f"kafka fetch error {top_err}")
            res = r.arr(lambda r: (r.s(), r.arr(lambda r: (
                r.i32(), r.i16(), r.i64(), r.i64(), *((r.i64(),) if v10 else ()),
                r.arr(lambda r: (r.i64(), r.i64())), r.by()))))
            out, err = b"", 0
            for _t, parts in res:
                for part in parts:
                    err = err or part[1]
                    out += part[-1] or b""
            if err == UNSUPPORTED_COMPRESSION_TYPE and not v10:
                self._fetch_v10.add(addr)
                continue
            if err == OFFSET_OUT_OF_RANGE:
                start = self._list_offset(topic, partition, -2)
                if offset < start:
                    offset = start
                    continue
            if err:
                raise IOError(f"kafka fetch error {err}")
            return out, offset
        raise IOError(f"kafka fetch of {topic}/{partition} at {offset} failed")

    def consume(self, topic, partition, offset, max_records):
        # the native decoder also steps over transactional control batches (a record-less
        # fetch still moves the offset), which the per-record form needs as much
        buf, offs, nxt = self.consume_block(topic, partition, offset, max_records)
        return [buf[int(offs[i]):int(offs[i + 1])] for i in range(len(offs) - 1)], nxt

    @staticmethod
    def _decode_into(data: bytes, offset: int, max_records: int, dst, cap: int):
        import ctypes

        import numpy as np

        from omldm_amd.ops import native

        offs = np.zeros(max(0, int(max_records)) + 1, dtype=np.int64)
        nxt = ctypes.c_longlong(offset)
        n = native.host().omldm_kafka_decode_into(
            data, len(data), offset, int(max_records), native.ptr(dst), int(cap),
            offs.ctypes.data, ctypes.byref(nxt), 1)
        if n < 0:
            what = {-2: "corrupt record set", -3: "codec library missing",
                    -5: "CRC-32C mismatch"}.get(int(n), "error")
            raise IOError(f"kafka record set decode failed: {what} ({n})")
        return int(n), offs[:n + 1].copy(), int(nxt.value)

    def consume_into(self, topic, partition, offset, max_records, dst, cap):
        """Native path: the fetched record set is decoded (and decompressed) by
        csrc/host/kafka_wire.cpp straight into ``dst[:cap]`` — no per-record objects."""
        data, offset = self._fetch(topic, partition, offset, max_bytes=max(1 << 20, int(cap)))
        n, offs, nxt = self._decode_into(data, offset, max_records, dst, cap)
        if n == 0 and nxt == offset and data and max_records > 0:
            # nothing decoded, offset not moved, yet the broker returned records: the
            # first record alone is larger than the destination — fail loudly instead of
            # stalling the partition on the same fetch forever
            raise IOError(f"kafka record at {topic}/{partition}@{offset} does not fit the "
                          f"{cap}-byte ingest buffer (raise the staging capacity)")
        return n, offs, nxt

    def consume_block(self, topic, partition, offset, max_records):
        import numpy as np

        data, offset = self._fetch(topic, partition, offset)
        cap = max(len(data) * 4, 1 << 16)  # compressed sets inflate: grow if needed
        while True:
            buf = np.empty(cap, dtype=np.uint8)
            n, offs, nxt = self._decode_into(data, offset, max_records, buf, cap)
            # done unless the first record alone did not fit (nothing taken, offset not
            # moved past a control batch); a set that inflates > 256× is not plausible
            if n or nxt != offset or not data or cap > 256 * len(data) + (1 << 20):
                return buf[:int(offs[-1])].tobytes(), offs, nxt
            cap *= 4

    def flush(self):
        pass

    def close(self):
        for c in list(self._conns.values()):
            c.close()
        self._conns.clear()
