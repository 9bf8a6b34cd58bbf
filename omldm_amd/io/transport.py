"""Topic transports: the engine's user-facing I/O (Kafka-style topics of JSON records).

Reference: every input/output of the job is a Kafka topic (README.md:20-26; SURVEY.md
Appendix B): requests (1 partition), trainingData / forecastingData (36), responses (1),
predictions (36), performance; psMessages is gone (RCCL replaces it).

Brokers (selected by the ``*Addr`` flag):
* ``memory://name``        in-process broker (tests, single-process jobs)
* ``file:///dir``          one append-only JSONL log per (topic, partition); consumers keep
                           their own offsets — shared by all ranks of a node-local job
* ``host:port``            Kafka wire protocol (omldm_amd.io.kafka)
Partition assignment mirrors Flink's source subtasks: rank r of G consumes partitions
p with p % G == r (omldm/Job.scala:42-57).
"""
from __future__ import annotations

import os
import threading
from collections import defaultdict

import numpy as np


def join_block(recs: list) -> tuple[bytes, np.ndarray]:
    """list of records → (contiguous buffer, int64 offsets[n+1])."""
    offs = np.zeros(len(recs) + 1, dtype=np.int64)
    if recs:
        np.cumsum([len(r) for r in recs], out=offs[1:])
    return b"".join(recs), offs


class Broker:
    parallel_reads = False  # may consume_into run concurrently for different partitions?

    def partitions(self, topic: str) -> int:
        raise NotImplementedError

    def produce(self, topic: str, value: str | bytes, partition: int | None = None,
                key: str | None = None) -> None:
        raise NotImplementedError

    def consume(self, topic: str, partition: int, offset: int, max_records: int
                ) -> tuple[list[bytes], int]:
        """Returns (records, next_offset)."""
        raise NotImplementedError

    def end_offset(self, topic: str, partition: int) -> int:
        raise NotImplementedError

    def consume_block(self, topic: str, partition: int, offset: int, max_records: int
                      ) -> tuple[bytes, np.ndarray, int]:
        """Records as ONE buffer + offsets (the parser's input; no per-record objects
        on the fast path). Returns (buf, offsets[n+1], next_offset)."""
        recs, nxt = self.consume(topic, partition, offset, max_records)
        buf, offs = join_block(recs)
        return buf, offs, nxt

    def consume_into(self, topic: str, partition: int, offset: int, max_records: int,
                     dst: np.ndarray, cap: int) -> tuple[int, np.ndarray, int]:
        """Reads up to ``max_records`` whole records (≤ ``cap`` bytes) straight into
        ``dst[:cap]`` (a pinned staging slot). Returns (n, offs[n+1] relative to dst,
        next_offset). Generic form: consume_block + one copy; FileBroker reads the log
        into ``dst`` directly (csrc/host/logio.cpp)."""
        while max_records > 0:
            buf, offs, nxt = self.consume_block(topic, partition, offset, max_records)
            n = len(offs) - 1
            if n == 0 or offs[-1] <= cap:
                if n:
                    dst[:int(offs[-1])] = np.frombuffer(buf, dtype=np.uint8, count=int(offs[-1]))
                return n, offs, nxt
            max_records = int(np.searchsorted(offs, cap, side="right")) - 1  # what fits
        return 0, np.zeros(1, dtype=np.int64), offset

    def produce_lines(self, topic: str, block: bytes, offs: np.ndarray,
                      partition: int | None = None) -> None:
        """Appends the newline-terminated records block[offs[i]:offs[i+1]] (egress of a
        whole forecast batch). Generic form: one produce per record."""
        for i in range(len(offs) - 1):
            rec = block[int(offs[i]):int(offs[i + 1]) - 1]
            self.produce(topic, rec if isinstance(rec, bytes) else bytes(rec), partition=partition)

    def create_topic(self, topic: str, partitions: int) -> None:
        pass

    def flush(self) -> None:
        pass


class MemoryBroker(Broker):
    _registry: dict = {}
    _reg_lock = threading.Lock()

    def __init__(self):
        self._logs = defaultdict(list)     # (topic, p) -> list[bytes]
        self._nparts = {}
        self._lock = threading.Lock()
        self._rr = defaultdict(int)

    @classmethod
    def named(cls, name: str) -> "MemoryBroker":
        with cls._reg_lock:
            if name not in cls._registry:
                cls._registry[name] = MemoryBroker()
            return cls._registry[name]

    def create_topic(self, topic, partitions):
        with self._lock:
            self._nparts[topic] = max(self._nparts.get(topic, 0), int(partitions))

    def partitions(self, topic):
        return self._nparts.get(topic, 1)

    def produce(self, topic, value, partition=None, key=None):
        if isinstance(value, str):
            value = value.encode()
        with self._lock:
            n = self._nparts.setdefault(topic, 1)
            if partition is None:
                partition = self._rr[topic] % n
                self._rr[topic] += 1
            self._logs[(topic, partition % n)].append(value)

    def consume(self, topic, partition, offset, max_records):
        with self._lock:
            log = self._logs.get((topic, partition), [])
            recs = log[offset:offset + max_records]
        return recs, offset + len(recs)

    def end_offset(self, topic, partition):
        with self._lock:
            return len(self._logs.get((topic, partition), []))

    def records(self, topic) -> list[bytes]:
        """All records of a topic (partition order) — test helper."""
        with self._lock:
            out = []
            for p in range(self.partitions(topic)):
                out.extend(self._logs.get((topic, p), []))
            return out


class FileBroker(Broker):
    """Append-only JSONL logs: <root>/<topic>/<partition>.jsonl (one record per line).
    Consumer offsets are byte offsets, so every rank can tail its partitions."""

    parallel_reads = True  # consume_into is a GIL-free pread: partitions read concurrently

    def __init__(self, root: str):
        self.root = root
        os.makedirs(root, exist_ok=True)
        self._rr = defaultdict(int)
        self._lock = threading.Lock()
        self._fds: dict[str, int] = {}

    def _fd(self, path: str) -> int:
        fd = self._fds.get(path)
        if fd is None:
            fd = os.open(path, os.O_RDONLY)
            kept = self._fds.setdefault(path, fd)
            if kept != fd:  # another thread opened it first
                os.close(fd)
                fd = kept
        return fd

    def close(self) -> None:
        for fd in self._fds.values():
            try:
                os.close(fd)
            except OSError:
                pass
        self._fds.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def consume_into(self, topic, partition, offset, max_records, dst, cap, hint=0):
        """pread of the log straight into ``dst`` + memchr record index, without the GIL
        (csrc/host/logio.cpp: omldm_read_log). ``hint``: bytes the records are expected
        to take (the first read's size; more is read only if needed, up to ``cap``)."""
        from omldm_amd.ops import native

        path = os.path.join(self.root, topic, f"{partition}.jsonl")
        offs = np.empty(max(1, max_records) + 1, dtype=np.int64)
        if max_records <= 0 or cap <= 0 or not os.path.exists(path):
            offs[0] = 0
            return 0, offs[:1], offset
        used = np.zeros(1, dtype=np.int64)
        n = native.host().omldm_read_log(self._fd(path), offset, dst.ctypes.data, int(cap),
                                         int(max_records), offs.ctypes.data, used.ctypes.data,
                                         int(hint))
        if n < 0:
            raise OSError(-n, f"reading {path}")
        return int(n), offs[:n + 1], offset + int(used[0])

    def _dir(self, topic):
        d = os.path.join(self.root, topic)
        os.makedirs(d, exist_ok=True)
        return d

    def create_topic(self, topic, partitions):
        d = self._dir(topic)
        for p in range(int(partitions)):
            open(os.path.join(d, f"{p}.jsonl"), "ab").close()

    def partitions(self, topic):
        d = self._dir(topic)
        n = len([f for f in os.listdir(d) if f.endswith(".jsonl")])
        return max(1, n)

    def produce(self, topic, value, partition=None, key=None):
        if isinstance(value, str):
            value = value.encode()
        value = value.replace(b"\n", b" ")
        n = self.partitions(topic)
        with self._lock:
            if partition is None:
                partition = self._rr[topic] % n
                self._rr[topic] += 1
            with open(os.path.join(self._dir(topic), f"{partition % n}.jsonl"), "ab") as f:
                f.write(value + b"\n")

    def produce_block(self, topic: str, partition: int, block) -> None:
        """Bulk append of newline-terminated records (producers that batch, e.g. a
        Kafka producer's linger buffer); ``block``: bytes or a uint8 ndarray."""
        if isinstance(block, np.ndarray):
            block = memoryview(np.ascontiguousarray(block))
        elif block and not block.endswith(b"\n"):
            block += b"\n"
        n = self.partitions(topic)
        with self._lock:
            with open(os.path.join(self._dir(topic), f"{partition % n}.jsonl"), "ab") as f:
                f.write(block)

    def produce_lines(self, topic, block, offs, partition=None):
        if len(block) == 0:
            return
        if partition is None:
            with self._lock:
                partition = self._rr[topic] % self.partitions(topic)
                self._rr[topic] += 1
        self.produce_block(topic, partition, block)

    def consume(self, topic, partition, offset, max_records):
        path = os.path.join(self._dir(topic), f"{partition}.jsonl")
        if not os.path.exists(path):
            return [], offset
        with open(path, "rb") as f:
            left = os.fstat(f.fileno()).st_size - offset  # read() preallocates its size
            if left <= 0:
                return [], offset
            f.seek(offset)
            data = f.read(min(left, max(1, max_records) * 4096))
        if not data:
            return [], offset
        cut = data.rfind(b"\n")
        if cut < 0:
            return [], offset  # partial line still being written
        lines = data[:cut].split(b"\n")
        if len(lines) > max_records:
            lines = lines[:max_records]
            used = sum(len(x) + 1 for x in lines)
        else:
            used = cut + 1
        return [x for x in lines if x.strip()], offset + used

    def end_offset(self, topic, partition):
        # one fstat of the partition log's cached descriptor: the tick's forecast catch-up
        # and the forecast lane's poll ask for every partition, often (a stat of the path
        # plus the topic directory's makedirs cost ~15 µs per partition)
        path = os.path.join(self.root, topic, f"{partition}.jsonl")
        fd = self._fds.get(path)
        if fd is None:
            try:
                fd = self._fd(path)
            except FileNotFoundError:
                return 0
        return os.fstat(fd).st_size

    def consume_block(self, topic, partition, offset, max_records):
        """Reads a chunk of the log and indexes its lines with one vectorised newline
        scan — the records never become Python objects."""
        path = os.path.join(self.root, topic, f"{partition}.jsonl")
        empty = (b"", np.zeros(1, dtype=np.int64), offset)
        if max_records <= 0 or not os.path.exists(path):
            return empty
        cap = min(64 << 20, max(64 << 10, max_records * 768))
        with open(path, "rb") as f:
            f.seek(offset)
            data = f.read(cap)
            nl = np.flatnonzero(np.frombuffer(data, dtype=np.uint8) == 10)
            while nl.size == 0 and len(data) == cap:  # one record longer than the chunk
                more = f.read(cap)
                if not more:
                    break
                data += more
                nl = np.flatnonzero(np.frombuffer(data, dtype=np.uint8) == 10)
        if nl.size == 0:
            return empty
        nl = nl[:max_records]
        end = int(nl[-1]) + 1
        offs = np.empty(nl.size + 1, dtype=np.int64)
        offs[0] = 0
        offs[1:] = nl + 1
        return data[:end], offs, offset + end


def broker_for(addr: str) -> Broker:
    if addr.startswith("memory://"):
        return MemoryBroker.named(addr[len("memory://"):] or "default")
    if addr.startswith("file://"):
        return FileBroker(addr[len("file://"):])
    from omldm_amd.io.kafka import KafkaBroker

    return KafkaBroker(addr)


class Consumer:
    """Consumer of the partitions of one topic owned by this rank (p % world == rank).
    ``start`` = "earliest" | "latest" (reference: requests/data earliest, performance
    latest; omldm/Job.scala:42-57,127-142)."""

    def __init__(self, broker: Broker, topic: str, rank: int = 0, world: int = 1,
                 start: str = "earliest", all_partitions: bool = False):
        self.broker = broker
        self.topic = topic
        n = broker.partitions(topic)
        self.parts = list(range(n)) if all_partitions else [p for p in range(n)
                                                            if p % world == rank]
        self.offsets = {p: (broker.end_offset(topic, p) if start == "latest" else 0)
                        for p in self.parts}
        self._avg_len = 1024.0  # running bytes-per-record estimate (sizes poll_into reads)

    def poll(self, max_records: int) -> list[bytes]:
        out = []
        if not self.parts:
            return out
        share = max(1, max_records // len(self.parts))
        for p in self.parts:
            recs, nxt = self.broker.consume(self.topic, p, self.offsets[p], share)
            self.offsets[p] = nxt
            out.extend(recs)
        return out

    def poll_block(self, max_records: int) -> tuple[bytes, np.ndarray]:
        """Like ``poll`` but returns one buffer + offsets over all owned partitions."""
        if not self.parts:
            return b"", np.zeros(1, dtype=np.int64)
        share = max(1, max_records // len(self.parts))
        bufs, offs, base = [], [np.zeros(1, dtype=np.int64)], 0
        for p in self.parts:
            buf, o, nxt = self.broker.consume_block(self.topic, p, self.offsets[p], share)
            self.offsets[p] = nxt
            if len(o) > 1:
                bufs.append(buf)
                offs.append(o[1:] + base)
                base += len(buf)
        return b"".join(bufs), np.concatenate(offs)

    def read_plan(self, max_records: int) -> list[tuple[int, int, int]]:
        """(partition, max records, byte budget) of every owned partition for one block
        of ≤ ``max_records`` records — the regions of a staging slot that
        ``engine.ingest.TickIngest`` fills (in parallel when the broker allows)."""
        if not self.parts or max_records <= 0:
            return []
        share = max(1, max_records // len(self.parts))
        cap = int(share * self._avg_len * 1.5) + (64 << 10)
        return [(p, share, cap) for p in self.parts]

    def read_region(self, p: int, share: int, dst: np.ndarray) -> tuple[int, np.ndarray]:
        """Reads partition ``p`` into ``dst`` (its region); advances the offset and the
        bytes-per-record estimate. Returns (records, offsets relative to dst)."""
        if isinstance(self.broker, FileBroker):  # first read sized to the expected bytes
            k, o, nxt = self.broker.consume_into(self.topic, p, self.offsets[p], share, dst,
                                                 len(dst), hint=int(share * self._avg_len * 1.02)
                                                 + 4096)
        else:
            k, o, nxt = self.broker.consume_into(self.topic, p, self.offsets[p], share, dst,
                                                 len(dst))
        self.offsets[p] = nxt
        if k:
            self._avg_len = 0.8 * self._avg_len + 0.2 * (int(o[k]) / k)
        elif self.broker.end_offset(self.topic, p) > nxt:
            self._avg_len *= 2  # a record longer than the region: bigger regions next time
        return k, o

    def state_dict(self) -> dict:
        return {"offsets": dict(self.offsets)}

    def load_state_dict(self, sd: dict) -> None:
        for p, o in sd.get("offsets", {}).items():
            if int(p) in self.offsets:
                self.offsets[int(p)] = int(o)


def hub_message_partition(network_id: int, destination: int | None, n_partitions: int,
                          terminate: bool = False) -> int:
    """Reference FlinkHubMessagePartitioner (omldm/utils/kafkaPartitioners/
    FlinkHubMessagePartitioner.scala:7-20): terminate → 0; unicast → dest % n;
    broadcast → networkId % n. Kept for topic-compatible producers."""
    if terminate:
        return 0
    if destination is not None:
        return destination % n_partitions
    return network_id % n_partitions


def identity_partition(key: int, n: int) -> int:
    """Reference random_partitioner — actually the identity (random_partitioner.scala:7-15)."""
    if not 0 <= key < n:
        raise ValueError(f"partition key {key} out of range [0, {n})")
    return key
